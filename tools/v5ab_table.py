"""Side-by-side table of two gemm_bench.py runs (v4 = MAECLIP_GEMM_V5=0, v5 = 1):
usage v5ab_table.py v4.jsonl v5.jsonl [v4epi.jsonl v5epi.jsonl]"""
import json
import sys


def load(path):
    out = {}
    for line in open(path):
        if line.startswith("{"):
            d = json.loads(line)
            out[(d["name"], d.get("epi", 0))] = d
    return out


args = sys.argv[1:]
for a, b in zip(args[0::2], args[1::2]):
    r4, r5 = load(a), load(b)
    for k in r4:
        if k in r5:
            x, y = r4[k]["ours_us"], r5[k]["ours_us"]
            print(f"{k[0]:22s} epi{k[1]}  v4 {x:8.1f} us  v5 {y:8.1f} us  {x / y:5.2f}x  "
                  f"({r5[k]['ours_tflops']:.0f} TF/s)")
