"""Summarise a rocprofv3 kernel_stats.csv per training step: kernel groups and top kernels."""
import csv, sys, re
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13.0
rows = list(csv.DictReader(open(path)))
groups = {}
for r in rows:
    n = r['Name']
    g = ('gemm wgrad' if 'wgrad' in n else 'gemm' if 'gemm' in n else 'attn' if 'attn_' in n else 'ln' if 'ln_' in n else
         'adamw/cast' if ('adamw' in n or 'cast_multi' in n) else 'colsum' if 'colsum' in n or 'vec_sum' in n else
         'torch' if 'at::native' in n or 'rocclr' in n else 'mae/other')
    groups[g] = groups.get(g, 0.0) + float(r['TotalDurationNs'])
tot = sum(groups.values())
print(f"total kernel time / step: {tot/steps/1e6:.2f} ms")
for g, v in sorted(groups.items(), key=lambda x: -x[1]):
    print(f"  {g:12s} {v/steps/1e6:7.2f} ms/step  {100*v/tot:5.1f}%")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    name = re.sub(r'\(anonymous namespace\)::', '', r['Name'])[:90]
    print(f"{float(r['TotalDurationNs'])/steps/1e3:8.1f}us/step n/step={int(r['Calls'])/steps:5.1f} avg={float(r['AverageNs'])/1e3:7.1f}us {name}")
