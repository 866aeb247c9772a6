"""Per-step GPU occupancy from a rocprofv3 kernel_trace.csv with several streams:
wall time, time with >=1 kernel running (union), per-stream busy time, and the
idle intervals on the GPU (no kernel on any stream).
usage: python tools/trace_union.py run_kernel_trace.csv [step_from_end=1]"""
import csv, re, sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adamw_multi" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
step = rows[ends[-k - 1] + 1:ends[-k] + 1]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in step)
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
union, cur_s, cur_e, idle = 0, iv[0][0], iv[0][1], []
for s, e, r in iv[1:]:
    if s > cur_e:
        union += cur_e - cur_s
        idle.append((s - cur_e, cur_e - t0))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
print(f"kernels {len(step)}  wall {(t1 - t0) / 1e6:.3f} ms  union-busy {union / 1e6:.3f} ms  "
      f"GPU idle {(t1 - t0 - union) / 1e6:.3f} ms")
per = {}
for s, e, r in iv:
    q = (r.get("Queue_Id"), r.get("Stream_Id"))
    per[q] = per.get(q, 0) + e - s
for q, v in sorted(per.items(), key=lambda x: -x[1]):
    print(f"  queue/stream {q}: {v / 1e6:.3f} ms of kernels")
idle.sort(reverse=True)
print("largest idle gaps (us, at ms):", [(round(g / 1e3, 1), round(at / 1e6, 2)) for g, at in idle[:10]])
