"""Per-shape GEMM throughput of libmaeclip vs torch.matmul (hipBLASLt) on the
production shapes of the C2 step (ViT-B/16 MAE+CLIP, B=256)."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")
E, D = 256 * 50, 256 * 197   # encoder / decoder token rows
SHAPES = [  # (name, M, N, K, a_layout, b_layout)
    ("enc qkv fwd", E, 2304, 768, 0, 0), ("enc fc1 fwd", E, 3072, 768, 0, 0), ("enc fc2 fwd", E, 768, 3072, 0, 0),
    ("enc proj fwd", E, 768, 768, 0, 0), ("dec qkv fwd", D, 1536, 512, 0, 0), ("dec fc1 fwd", D, 2048, 512, 0, 0),
    ("dec fc2 fwd", D, 512, 2048, 0, 0), ("dec pred fwd", D, 768, 512, 0, 0),
    ("enc fc2 dgrad", E, 3072, 768, 0, 1), ("enc fc1 dgrad", E, 768, 3072, 0, 1), ("dec fc2 dgrad", D, 2048, 512, 0, 1),
    ("dec fc1 dgrad", D, 512, 2048, 0, 1),
    ("enc fc1 wgrad", 3072, 768, E, 1, 1), ("enc fc2 wgrad", 768, 3072, E, 1, 1), ("enc qkv wgrad", 2304, 768, E, 1, 1),
    ("dec fc1 wgrad", 2048, 512, D, 1, 1), ("dec fc2 wgrad", 512, 2048, D, 1, 1), ("dec qkv wgrad", 1536, 512, D, 1, 1),
]

if os.environ.get("GEMM_SET") == "sq":   # the guide's reference shapes + K sweep at fixed M, N
    SHAPES = [("sq4096", 4096, 4096, 4096, 0, 0), ("sq8192", 8192, 8192, 8192, 0, 0),
              ("4096x4096 K768", 4096, 4096, 768, 0, 0), ("4096x4096 K1536", 4096, 4096, 1536, 0, 0),
              ("12800x3072 K768", E, 3072, 768, 0, 0), ("12800x3072 K3072", E, 3072, 3072, 0, 0),
              ("sq4096 RC", 4096, 4096, 4096, 0, 1)]


def mk(rows, cols):
    return (torch.randn(rows, cols, device=dev) * 0.5).to(torch.bfloat16)


def time_fn(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


if os.environ.get("GEMM_SET") == "epi":   # production epilogues (functions.py), no hipBLASLt leg
    SHAPES = [("dec fc2 dgrad*gelu'", D, 2048, 512, 0, 1, 5), ("enc fc2 dgrad*gelu'", E, 3072, 768, 0, 1, 5),
              ("dec fc1 fwd gelu", D, 2048, 512, 0, 0, 4), ("enc fc1 fwd gelu", E, 3072, 768, 0, 0, 4),
              ("dec fc2 fwd +res", D, 512, 2048, 0, 0, 2), ("enc fc2 fwd +res", E, 768, 3072, 0, 0, 2),
              ("dec proj fwd +res", D, 512, 512, 0, 0, 2), ("enc proj fwd +res", E, 768, 768, 0, 0, 2),
              ("dec proj dgrad", D, 512, 512, 0, 1, 0), ("enc proj dgrad", E, 768, 768, 0, 1, 0),
              ("dec qkv dgrad", D, 512, 1536, 0, 1, 0), ("enc qkv dgrad", E, 768, 2304, 0, 1, 0),
              ("enc fc1 dgrad", E, 768, 3072, 0, 1, 0), ("dec fc1 dgrad", D, 512, 2048, 0, 1, 0),
              ("enc qkv fwd", E, 2304, 768, 0, 0, 0), ("dec qkv fwd", D, 1536, 512, 0, 0, 0),
              ("L enc fc2 fwd +res", 128 * 145, 1024, 4096, 0, 0, 2), ("L enc qkv fwd", 128 * 145, 3072, 1024, 0, 0, 0),
              ("L enc fc1 dgrad", 128 * 145, 1024, 4096, 0, 1, 0)]


def epi_kwargs(epi, M, N):
    if epi == K.EPI_RESID:
        return dict(resid=torch.randn(M, N, device=dev), ldr=N)
    if epi in (K.EPI_GELU, K.EPI_GELU_D):
        return dict(aux_out=torch.empty(M, N, device=dev, dtype=torch.bfloat16), ldaux=N,
                    bias=torch.randn(N, device=dev))
    if epi in (K.EPI_MUL_AUX, K.EPI_DGELU):
        return dict(aux=torch.rand(M, N, device=dev).to(torch.bfloat16), ldaux=N)
    return {}


res = []
for shp in SHAPES:
    name, M, N, Kd, la, lb = shp[:6]
    epi = shp[6] if len(shp) > 6 else -1
    A = mk(M, Kd) if la == 0 else mk(Kd, M)
    B = mk(N, Kd) if lb == 0 else mk(Kd, N)
    C = torch.empty(M, N, device=dev, dtype=torch.float32 if (la, lb) == (1, 1) or epi == 2 else torch.bfloat16)
    S = 1
    ws = None
    if (la, lb) == (1, 1):  # production wgrad path: deterministic split-K
        from mae_clip_amd import _lib
        S = int(_lib.lib().maeclip_gemm_splitk(M, N, Kd))
        ws = torch.empty(S * M * N, device=dev) if S > 1 else None
    kw = epi_kwargs(epi, M, N) if epi >= 0 else {}
    f = lambda: K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, la, lb, splitk=S, workspace=ws,
                       epilogue=max(epi, 0), **kw)
    t = time_fn(f)
    if epi >= 0:
        fl = 2.0 * M * N * Kd
        r = dict(name=name, M=M, N=N, K=Kd, epi=epi, ours_tflops=round(fl / t / 1e12, 1), ours_us=round(t * 1e6, 1))
        print(json.dumps(r), flush=True)
        continue
    At = A if la == 0 else A.t()
    Bt = B.t() if lb == 0 else B
    tt = time_fn(lambda: torch.matmul(At, Bt))
    fl = 2.0 * M * N * Kd
    r = dict(name=name, M=M, N=N, K=Kd, ours_tflops=round(fl / t / 1e12, 1), hipblaslt_tflops=round(fl / tt / 1e12, 1),
             ours_us=round(t * 1e6, 1))
    res.append(r)
    print(json.dumps(r), flush=True)
