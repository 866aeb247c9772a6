"""Race screen of a GEMM build (cdna_hip_programming.md §5: a sync-structure
edit makes a new template): every production shape (plus square ones) run
REPS times on fixed random operands; every output must be bitwise equal to the
first and within bf16 rounding of the fp32 torch product. Prints one JSON line
per shape; exits 1 on any mismatch. MAECLIP_LIB selects the build."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")
REPS = int(os.environ.get("REPS", "40"))
E, D = 128 * 50, 128 * 197
SHAPES = [("enc qkv fwd", E, 2304, 768, 0, 0, 0), ("enc fc1 fwd gelu'", E, 3072, 768, 0, 0, 4),
          ("enc fc2 fwd+res", E, 768, 3072, 0, 0, 2), ("enc fc1 dgrad", E, 768, 3072, 0, 1, 0),
          ("enc fc2 dgrad*gelu'", E, 3072, 768, 0, 1, 5), ("dec fc1 fwd gelu'", D, 2048, 512, 0, 0, 4),
          ("dec fc2 dgrad*gelu'", D, 2048, 512, 0, 1, 5), ("dec qkv dgrad", D, 512, 1536, 0, 1, 0),
          ("sq4096", 4096, 4096, 4096, 0, 0, 0), ("sq2048 RC", 2048, 2048, 2048, 0, 1, 0),
          ("ragged", 3000, 1000, 1024, 0, 0, 0)]
bad = 0
for name, M, N, Kd, la, lb, epi in SHAPES:
    g = torch.Generator(device=dev).manual_seed(M + N + Kd)
    A = (torch.randn(M, Kd, generator=g, device=dev) * 0.5).to(torch.bfloat16)
    B = (torch.randn((N, Kd) if lb == 0 else (Kd, N), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    out = torch.float32 if epi == K.EPI_RESID else torch.bfloat16
    C = torch.empty(M, N, device=dev, dtype=out)
    kw = {}
    if epi == K.EPI_RESID:
        kw = dict(resid=torch.randn(M, N, generator=g, device=dev), ldr=N)
    elif epi == K.EPI_GELU_D:
        kw = dict(aux_out=torch.empty(M, N, device=dev, dtype=torch.bfloat16), ldaux=N)
    elif epi == K.EPI_MUL_AUX:
        kw = dict(aux=torch.rand(M, N, generator=g, device=dev).to(torch.bfloat16), ldaux=N)
    fn = lambda: K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, la, lb, epilogue=epi, **kw)
    fn()
    torch.cuda.synchronize()
    first = C.clone()
    aux0 = kw["aux_out"].clone() if "aux_out" in kw else None
    diffs = 0
    for r in range(REPS):
        fn()
        if not torch.equal(C, first) or (aux0 is not None and not torch.equal(kw["aux_out"], aux0)):
            diffs += 1
    torch.cuda.synchronize()
    ref = (A.float() @ (B.float().t() if lb == 0 else B.float()))
    if epi == K.EPI_RESID:
        ref = ref + kw["resid"]
    elif epi == K.EPI_GELU_D:
        ref = torch.nn.functional.gelu(ref)
    elif epi == K.EPI_MUL_AUX:
        ref = ref * kw["aux"].float()
    err = ((first.float() - ref).abs().max() / ref.abs().max()).item()
    ok = diffs == 0 and err < 1e-2
    bad += not ok
    print(json.dumps(dict(name=name, M=M, N=N, K=Kd, reps=REPS, nondeterministic_reps=diffs, max_rel_err=err,
                          ok=ok)), flush=True)
sys.exit(1 if bad else 0)
