"""Summarise tools/pmc_instep.sh: per-launch kernel duration (trace pass) and
FETCH_SIZE x 2 + WRITE_SIZE bytes (PMC passes, KB units) of the dispatches of
one kernel (name substring, grid size) inside the C2 step; writes
<dir>/traffic.json in the format bench.py's pmc_traffic() reads.
usage: python tools/pmc_instep_summary.py <dir> KERNEL_SUBSTRING GRID_X "SHAPE KEY" [I/K]
I/K: of the matching dispatches in launch order keep those with index % K == I
(a kernel launched K times per step with one shape per position, e.g. the two
grouped weight-gradient launches: decoder first, then encoder)."""
import csv, glob, json, os, re, sys

d, kn, gx, key = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
pick = tuple(int(x) for x in sys.argv[5].split("/")) if len(sys.argv) > 5 and sys.argv[5] else None


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(d, pattern), recursive=True):
        for r in csv.DictReader(open(f)):
            if kn in r.get("Kernel_Name", "") and int(r.get("Grid_Size_X", r.get("Grid_Size", "0")) or 0) == gx:
                out.append(r)
    if pick:
        idk = "Dispatch_Id" if out and "Dispatch_Id" in out[0] else "Correlation_Id"
        ids = sorted({int(r[idk]) for r in out})
        keep = {x for j, x in enumerate(ids) if j % pick[1] == pick[0]}
        out = [r for r in out if int(r[idk]) in keep]
    return out


tr = rows("trace/**/*kernel_trace.csv")
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]


def counter(name):
    vals = {}
    for r in rows(f"{name}/**/*counter_collection.csv"):
        if r["Counter_Name"] == name:
            k = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    v = list(vals.values())
    return (sum(v) / len(v) if v else float("nan")), len(v)


fetch, nf = counter("FETCH_SIZE")
write, nw = counter("WRITE_SIZE")
if key.startswith("wgrad_grouped"):   # the C2 decoder group: 8 x (fc2, fc1, proj, qkv) at M = 50432, dW f32
    Mw, probs = 256 * 197, [(512, 2048), (2048, 512), (512, 512), (1536, 512)] * 8
    alg = sum(Mw * (n + k) * 2 + n * k * 4 for n, k in probs)
    flops = sum(2.0 * Mw * n * k for n, k in probs)
else:
    m = re.match(r"M(\d+) N(\d+) K(\d+) (\w)(\w) epi(\d+)", key)
    M, N, K, epi = int(m.group(1)), int(m.group(2)), int(m.group(3)), int(m.group(6))
    out_b = 4 if epi == 2 else 2
    alg = (M * K + N * K) * 2 + M * N * out_b
    alg += M * N * (4 if epi == 2 else 2 if epi in (1, 3, 4, 5) else 0)
    flops = 2.0 * M * N * K
dur_ns = sum(durs) / max(1, len(durs))
res = {"shape": key, "kernel": kn, "grid_x": gx, "avg_launch_us": round(dur_ns / 1e3, 2),
       "launches_traced": len(durs), "launches_counted": [nf, nw],
       "fetch_bytes": fetch * 1024 * 2, "write_bytes": write * 1024, "hbm_bytes": fetch * 1024 * 2 + write * 1024,
       "algorithmic_bytes": alg, "flops": flops,
       "note": "in-step: the C2 bench step itself (eager, bench.py --no-graph) under rocprofv3; FETCH_SIZE / "
               "WRITE_SIZE in separate passes (KB units), FETCH_SIZE doubled (gfx950 tallies 128-B requests at "
               "64 B, MI355X_MICROARCH.md §HBM); every dispatch of the kernel at this grid size in the run"}
res["traffic_over_algorithmic"] = round(res["hbm_bytes"] / alg, 3)
json.dump(res, open(os.path.join(d, "traffic.json"), "w"), indent=1)
print(json.dumps(res))
