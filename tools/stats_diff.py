"""Average kernel duration, two rocprofv3 kernel_stats.csv files side by side
(kernels matched by name; template arguments kept): python tools/stats_diff.py a.csv b.csv [filter]"""
import csv
import re
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        n = re.sub(r"\(anonymous namespace\)::|void ", "", r["Name"])
        out[n] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
flt = sys.argv[3] if len(sys.argv) > 3 else ""
for n in sorted(set(a) | set(b), key=lambda k: -(a.get(k, (0, 0))[1] * a.get(k, (0, 0))[0])):
    if flt and not re.search(flt, n):
        continue
    ca, ta = a.get(n, (0, float("nan")))
    cb, tb = b.get(n, (0, float("nan")))
    print(f"{ta:9.1f} {tb:9.1f} us  ({ca:4d}/{cb:4d})  {n[:110]}")
