"""GEMM v6 (4-wave 128x128-per-wave tiles, csrc/gemm6.hip) against v4 on the
same inputs: bitwise equality of C and the time of each, for large square and
production shapes, plain (bf16 out) and RESID (fp32 out) epilogues.
usage: python tools/gemm6_probe.py          (spawns itself with MAECLIP_GEMM_V6=0/1)"""
import hashlib
import json
import os
import subprocess
import sys

SHAPES = [  # name, M, N, K, b_layout, epi (0 plain bf16 / 2 RESID f32 / 4 GELU_D / 5 MUL_AUX+colsum)
    # the C2 step's shapes per micro-batch (128 images: encoder 6400 rows, decoder 25216)
    ("enc qkv fwd", 6400, 2304, 768, 0, 0), ("enc proj fwd+res", 6400, 768, 768, 0, 2),
    ("enc fc1 fwd gelu'", 6400, 3072, 768, 0, 4), ("enc fc2 fwd+res", 6400, 768, 3072, 0, 2),
    ("dec qkv fwd", 25216, 1536, 512, 0, 0), ("dec proj fwd+res", 25216, 512, 512, 0, 2),
    ("dec fc1 fwd gelu'", 25216, 2048, 512, 0, 4), ("dec fc2 fwd+res", 25216, 512, 2048, 0, 2),
    ("enc fc2 dgrad*gelu'", 6400, 3072, 768, 1, 5), ("enc fc1 dgrad", 6400, 768, 3072, 1, 0),
    ("dec fc2 dgrad*gelu'", 25216, 2048, 512, 1, 5), ("dec fc1 dgrad", 25216, 512, 2048, 1, 0),
    ("dec qkv dgrad", 25216, 512, 1536, 1, 0), ("dec proj dgrad", 25216, 512, 512, 1, 0),
    ("sq8192", 8192, 8192, 8192, 0, 0),
    ("ragged M gelu'", 5000, 768, 1024, 0, 4), ("ragged M res", 777, 512, 640, 1, 2), ("ragged mulaux", 1000, 1024, 256, 1, 5),
]


def child():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    from mae_clip_amd import kernels as K
    dev = torch.device("cuda")
    out = {}
    for name, M, N, Kd, lb, epi in SHAPES:
        g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + Kd)
        A = (torch.randn(M, Kd, generator=g) * 0.5).to(dev, torch.bfloat16)
        B = (torch.randn(N, Kd, generator=g) * 0.5).to(dev, torch.bfloat16) if lb == 0 else \
            (torch.randn(Kd, N, generator=g) * 0.5).to(dev, torch.bfloat16)
        bias = torch.randn(N, generator=g).to(dev)
        extra = []
        if epi == 2:
            res = torch.randn(M, N, generator=g).to(dev)
            C = torch.empty(M, N, device=dev, dtype=torch.float32)
            kw = dict(epilogue=2, resid=res, ldr=N, bias=bias)
        elif epi == 4:
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ao = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            kw = dict(epilogue=4, aux_out=ao, ldaux=N, bias=bias)
            extra = [ao]
        elif epi == 5:
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            aux = torch.rand(M, N, generator=g).to(dev, torch.bfloat16)
            cs = torch.empty(K.gemm_colsum_rows(M), N, device=dev)
            kw = dict(epilogue=5, aux=aux, ldaux=N, colsum=cs)
            extra = [cs]
        else:
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            kw = dict(bias=bias)
        f = lambda: K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, 0, lb, **kw)
        f()
        torch.cuda.synchronize()
        hh = hashlib.sha1(C.cpu().view(torch.uint8).numpy().tobytes())
        for t in extra:
            hh.update(t.cpu().view(torch.uint8).numpy().tobytes())
        h = hh.hexdigest()[:16]
        torch.save([C.cpu()] + [t.cpu() for t in extra],
                   os.path.join(os.environ.get("TMPDIR", "/tmp"), f"v6probe_{os.environ['MAECLIP_GEMM_V6']}_{len(out)}.pt"))
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        s.record()
        for _ in range(reps):
            f()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        out[name] = dict(hash=h, us=round(us, 1), tflops=round(2.0 * M * N * Kd / us / 1e6, 1))
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
        sys.exit(0)
    res = {}
    for v in ("0", "1"):
        env = dict(os.environ, MAECLIP_GEMM_V6=v)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env, capture_output=True, text=True,
                           timeout=240)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-4000:])
            sys.exit(r.returncode)
        res[v] = json.loads(r.stdout.strip().splitlines()[-1])
    bad = 0
    for name, *_ in SHAPES:
        a, b = res["0"][name], res["1"][name]
        eq = a["hash"] == b["hash"]
        diff = {}
        if not eq:
            import torch
            k = list(res["0"]).index(name)
            ta = torch.load(os.path.join(os.environ.get("TMPDIR", "/tmp"), f"v6probe_0_{k}.pt"))
            tb = torch.load(os.path.join(os.environ.get("TMPDIR", "/tmp"), f"v6probe_1_{k}.pt"))
            for idx, (x, y) in enumerate(zip(ta, tb)):
                x, y = x.float(), y.float()
                d = (x - y).abs()
                nz = (d > 0).nonzero()
                diff[f"out{idx}"] = dict(max_abs=d.max().item(), max_ref=x.abs().max().item(),
                                         frac_diff=round((d > 0).float().mean().item(), 6),
                                         first=nz[:3].tolist(), rows=sorted(set(nz[:, 0].tolist()))[:8] if nz.numel() else [])
            # colsum partials are sums in another order: a rounding-level difference is expected
        bad += not eq and any(v["max_abs"] > 1e-3 * max(1.0, v["max_ref"]) for v in diff.values())
        print(json.dumps(dict(name=name, v4_us=a["us"], v6_us=b["us"], v4_tflops=a["tflops"], v6_tflops=b["tflops"],
                              speedup=round(a["us"] / b["us"], 3), bitwise_equal=eq, diff=diff)))
    sys.exit(1 if bad else 0)
