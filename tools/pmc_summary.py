"""Summarise tools/pmc_traffic.sh output into one JSON object (stdout and
<dir>/traffic.json): mean kernel duration (kernel trace), FETCH_SIZE x 2 +
WRITE_SIZE in bytes per launch, the algorithmic bytes and FLOPs of the shape.
usage: python tools/pmc_summary.py <dir> M N K la lb epi"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
WGRAD = sys.argv[2] == "--wgrad"   # tools/wgrad_pmc.sh: the grouped decoder weight gradients
if not WGRAD:
    M, N, K, la, lb, epi = (int(x) for x in sys.argv[2:8])
KNAME = "wgrad4_kernel" if WGRAD else "gemm"


def gemm_rows(pattern):
    rows = []
    for f in glob.glob(os.path.join(d, pattern), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if KNAME in r.get("Kernel_Name", "")]
    return rows


def counter(name):
    vals = {}
    for r in gemm_rows(f"{name}/**/*counter_collection.csv"):
        if r["Counter_Name"] == name:
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    v = sorted(vals.values())[2:]    # first launches are warm-up
    return sum(v) / max(1, len(v)), len(v)


tr = gemm_rows("trace/**/*kernel_trace.csv")
durs = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr)[2:]
dur_ns = sum(durs) / max(1, len(durs))
fetch, nf = counter("FETCH_SIZE")
write, nw = counter("WRITE_SIZE")
eb = 2
if WGRAD:   # tools/wgrad_one.py: 8 x (fc2, fc1, proj, qkv) at M = 50432, dW f32 written
    Mw, probs = 256 * 197, [(512, 2048), (2048, 512), (512, 512), (1536, 512)] * 8
    alg = sum(Mw * (n + k) * eb + n * k * 4 for n, k in probs)
    res = {"shape": f"wgrad_grouped M{Mw} x{len(probs)} N512 K2048 bf16>f32",
           "avg_launch_us": round(dur_ns / 1e3, 2),
           "fetch_bytes": fetch * 1024 * 2, "write_bytes": write * 1024,
           "hbm_bytes": fetch * 1024 * 2 + write * 1024,
           "algorithmic_bytes": alg, "flops": sum(2.0 * Mw * n * k for n, k in probs),
           "launches_counted": [nf, nw],
           "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (KB units); FETCH_SIZE doubled "
                   "(gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md §HBM); random bf16 operands, "
                   "tools/wgrad_one.py (the wgrad4_kernel launch; its stream-K reduce is a separate kernel)"}
    res["tflops"] = round(res["flops"] / (dur_ns * 1e-9) / 1e12, 1)
    res["hbm_gbs"] = round(res["hbm_bytes"] / (dur_ns * 1e-9) / 1e9, 1)
    json.dump(res, open(os.path.join(d, "traffic.json"), "w"), indent=1)
    print(json.dumps(res))
    sys.exit(0)
out_b = 4 if epi == 2 else 2
alg = M * K * eb + N * K * eb + M * N * out_b
if epi == 2:
    alg += M * N * 4                 # fp32 residual read
elif epi in (1, 4):
    alg += M * N * 2                 # bf16 aux_out written
elif epi in (3, 5):
    alg += M * N * 2                 # bf16 aux read
res = {"shape": f"M{M} N{N} K{K} {'KR'[la]}{'KR'[lb]} epi{epi} bf16",
       "avg_launch_us": round(dur_ns / 1e3, 2),
       "fetch_bytes": fetch * 1024 * 2, "write_bytes": write * 1024,
       "hbm_bytes": fetch * 1024 * 2 + write * 1024,
       "algorithmic_bytes": alg, "flops": 2.0 * M * N * K,
       "launches_counted": [nf, nw],
       "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (KB units); FETCH_SIZE doubled "
               "(gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md §HBM); random bf16 operands, "
               "tools/gemm_one.py"}
res["tflops"] = round(res["flops"] / (dur_ns * 1e-9) / 1e12, 1)
res["hbm_gbs"] = round(res["hbm_bytes"] / (dur_ns * 1e-9) / 1e9, 1)
json.dump(res, open(os.path.join(d, "traffic.json"), "w"), indent=1)
print(json.dumps(res))
