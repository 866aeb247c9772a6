"""Kernel sequence of one training step from a rocprofv3 kernel_trace.csv, with
the neighbours of selected kernels (where do the torch copy / fill kernels of
the step come from?).
usage: python tools/step_seq.py run_kernel_trace.csv [pattern ...]"""
import csv, re, sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adamw_multi" in r["Kernel_Name"]]
a, b = ends[-3] + 1, ends[-2]
step = rows[a:b + 1]
pats = sys.argv[2:] or ["copyBuffer", "FillFunctor"]


def short(n):
    n = re.sub(r".anonymous namespace.::", "", n)
    return re.sub(r"\(maeclip.*|\(.*", "", n)[:60]


for i, r in enumerate(step):
    n = r["Kernel_Name"]
    if any(p in n for p in pats):
        prev = short(step[i - 1]["Kernel_Name"]) if i else "-"
        nxt = short(step[i + 1]["Kernel_Name"]) if i + 1 < len(step) else "-"
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"{i:5d} {short(n):40s} {d:6.1f}us  grid {r.get('Grid_Size', '?'):>8s}  after {prev:45s} before {nxt}")
