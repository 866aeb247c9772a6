"""One training step out of a rocprofv3 kernel_trace.csv: busy vs wall time, the
largest idle gaps between kernels, and time per kernel group.
usage: python tools/trace_step.py run_kernel_trace.csv [step_index_from_end=1]"""
import csv, re, sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adamw_multi" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
a, b = ends[-k - 1] + 1, ends[-k]
step = rows[a:b + 1]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"kernels {len(step)}  wall {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(t1 - t0 - busy) / 1e6:.3f} ms")
gaps = []
for p, q in zip(step, step[1:]):
    g = int(q["Start_Timestamp"]) - int(p["End_Timestamp"])
    gaps.append((g, p["Kernel_Name"][:60], q["Kernel_Name"][:60]))
gaps.sort(reverse=True)
for g, p, q in gaps[:12]:
    print(f"  gap {g / 1e3:8.1f} us  after {re.sub(r'.anonymous namespace.::', '', p)}  before {re.sub(r'.anonymous namespace.::', '', q)}")
print(f"  gaps > 5us: {sum(g for g, _, _ in gaps if g > 5000) / 1e6:.3f} ms over {sum(1 for g, _, _ in gaps if g > 5000)}")
grp = {}
for r in step:
    n = r["Kernel_Name"]
    key = re.sub(r"\(maeclip.*|\(.*", "", re.sub(r".anonymous namespace.::", "", n))[:70]
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    e = grp.setdefault(key, [0, 0])
    e[0] += d
    e[1] += 1
for key, (d, c) in sorted(grp.items(), key=lambda x: -x[1][0])[:30]:
    print(f"{d / 1e3:9.1f} us {c:4d}x  {key}")
