"""Steady-state per-step kernel summary from a rocprofv3 kernel trace.

usage: python tools/step_kernels.py run_kernel_trace.csv [last_steps] [top]

The trace is cut into training steps at every adamw_multi launch (the last
kernel of a step); only the last `last_steps` complete steps are used, so the
eager warm-up steps (and their torch kernels) do not pollute the per-step
figures the way the whole-run kernel_stats.csv does. Prints
  * kernel time per step by category,
  * the top kernels by time per step (name, launches per step, average),
  * one row per launch position for the grouped weight-gradient kernel
    (wgrad4_kernel: the decoder's launch, then the encoder's), so the
    bench's per-launch roofline figure can be recomputed from profiles/,
  * the torch / runtime kernels left inside the step.
"""
import csv
import re
import sys
from collections import defaultdict


def cat(n):
    return ('gemm wgrad' if 'wgrad' in n else 'gemm' if 'gemm' in n else
            'gemm (hipBLASLt)' if n.startswith(('Cijk_', 'Custom_Cijk')) else 'attn' if 'attn_' in n else
            'ln' if 'ln_' in n else 'adamw/cast' if ('adamw' in n or 'cast_multi' in n) else
            'colsum' if 'colsum' in n or 'vec_sum' in n else
            'torch' if 'at::native' in n or 'rocclr' in n else 'mae/other')


def short(n, w=90):
    n = re.sub(r'\(anonymous namespace\)::', '', n)
    n = re.sub(r'at::native::', '', n)
    return n[:w]


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if 'adamw_multi' in r['Kernel_Name']]
    if len(ends) < 2:
        sys.exit("fewer than two adamw_multi launches in the trace")
    pairs = list(zip(ends[:-1], ends[1:]))[-last:]
    nst = len(pairs)
    dur = lambda r: (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    groups = defaultdict(float)
    per = defaultdict(lambda: [0, 0.0])
    wg = defaultdict(list)
    torch_k = defaultdict(lambda: [0, 0.0])
    span = 0.0
    for a, b in pairs:
        step = rows[a + 1:b + 1]
        span += (int(step[-1]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e3
        k = 0
        for r in step:
            n, d = r['Kernel_Name'], dur(r)
            groups[cat(n)] += d
            per[n][0] += 1
            per[n][1] += d
            if 'wgrad4_kernel' in n:
                wg[k].append(d)
                k += 1
            if cat(n) == 'torch':
                torch_k[n][0] += 1
                torch_k[n][1] += d
    tot = sum(groups.values())
    print(f"steady-state steps: {nst} (of {len(ends) - 1}); adamw-to-adamw span {span / nst / 1e3:.2f} ms/step")
    print(f"kernel time / step: {tot / nst / 1e3:.2f} ms")
    for g, v in sorted(groups.items(), key=lambda x: -x[1]):
        print(f"  {g:12s} {v / nst / 1e3:7.2f} ms/step  {100 * v / tot:5.1f}%")
    print("top kernels (per step):")
    for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t / nst:9.1f}us/step n/step={c / nst:5.1f} avg={t / c:8.1f}us {short(n)}")
    print("grouped weight-gradient launches, per launch position in the step:")
    for k in sorted(wg):
        v = wg[k]
        print(f"  wgrad4 launch {k}: n={len(v)} avg={sum(v) / len(v):8.1f}us min={min(v):8.1f} max={max(v):8.1f}")
    print(f"torch / runtime kernels per step: {sum(c for c, _ in torch_k.values()) / nst:.1f}, "
          f"{sum(t for _, t in torch_k.values()) / nst:.1f} us")
    for n, (c, t) in sorted(torch_k.items(), key=lambda x: -x[1][1]):
        print(f"  n/step={c / nst:4.1f} {t / nst:7.1f}us {short(n, 120)}")


if __name__ == "__main__":
    main()
