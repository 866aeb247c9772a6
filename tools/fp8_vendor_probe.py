"""C4 encoder fp8 GEMM shapes: own fp8 kernel (MAECLIP_GEMM_LIB_FP8=0) vs the
vendor library with outer-vector scales (=1); median per-launch time."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")
M = 128 * 145
for name, N, Kd, epi, afmt in [("fc2 fwd+res", 1024, 4096, K.EPI_RESID, K.FP8_E4M3), ("qkv fwd", 3072, 1024, K.EPI_NONE, K.FP8_E4M3),
                               ("fc1 dgrad", 1024, 4096, K.EPI_NONE, K.FP8_E5M2), ("qkv dgrad", 1024, 3072, K.EPI_NONE, K.FP8_E5M2),
                               ("proj fwd+res", 1024, 1024, K.EPI_RESID, K.FP8_E4M3)]:
    A = K.quant_rows_fp8((torch.randn(M, Kd, device=dev)).to(torch.bfloat16), afmt)
    B = K.quant_rows_fp8(torch.randn(N, Kd, device=dev) * 0.05, K.FP8_E4M3)
    res = torch.randn(M, N, device=dev) if epi == K.EPI_RESID else None
    od = torch.float32 if epi == K.EPI_RESID else torch.bfloat16
    fn = lambda: K.linear_fp8(A, B, out_dtype=od, epilogue=epi, resid=res)
    t = {"0": [], "1": []}
    outs = {}
    for mode in ("0", "1"):
        os.environ["MAECLIP_GEMM_LIB_FP8"] = mode
        outs[mode] = fn().float()
    torch.cuda.synchronize()
    for r in range(5):
        for mode in ("0", "1"):
            os.environ["MAECLIP_GEMM_LIB_FP8"] = mode
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            t[mode].append(s.elapsed_time(e) / 10 * 1e3)
    d = (outs["0"] - outs["1"]).abs().max().item()
    print(json.dumps(dict(name=name, M=M, N=N, K=Kd, own_us=round(statistics.median(t["0"]), 1),
                          vendor_us=round(statistics.median(t["1"]), 1), max_diff=d,
                          max_ref=outs["0"].abs().max().item())), flush=True)
