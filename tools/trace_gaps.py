"""Per-stream timeline of back-to-back reruns from a rocprofv3 --kernel-trace CSV: for each exec
kernel, its average duration and the idle gap before it on its own queue, and how much of the
lanes kernel the concurrent spill kernel overlaps.  usage: python tools/trace_gaps.py trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
key_start = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start_Timestamp_ns"
key_end = "End_Timestamp" if "End_Timestamp" in rows[0] else "End_Timestamp_ns"
by_q = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    if "lanes" not in name and "cl_exec_kernel" not in name:
        continue
    q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
    by_q[(q, "lanes" if "lanes" in name else "exec")].append((int(r[key_start]), int(r[key_end])))
for (q, kind), ev in sorted(by_q.items()):
    ev.sort()
    ev = ev[len(ev) // 4:]  # steady state: drop the warm-up quarter
    dur = [e - s for s, e in ev]
    gaps = [ev[i + 1][0] - ev[i][1] for i in range(len(ev) - 1)]
    per = [ev[i + 1][0] - ev[i][0] for i in range(len(ev) - 1)]
    print(f"queue {q} {kind}: n={len(ev)} dur_us={sum(dur) / len(dur) / 1e3:.1f} "
          f"gap_us={sum(gaps) / max(len(gaps), 1) / 1e3:.1f} period_us={sum(per) / max(len(per), 1) / 1e3:.1f}")
lanes = sorted(v for (q, k), e in by_q.items() if k == "lanes" for v in e)
execs = sorted(v for (q, k), e in by_q.items() if k == "exec" for v in e)
if lanes and execs:
    ov = []
    for s, e in lanes[len(lanes) // 4:]:
        o = sum(max(0, min(e, e2) - max(s, s2)) for s2, e2 in execs)
        ov.append(o / (e - s))
    print(f"spill kernel overlap of the lanes kernel: {sum(ov) / len(ov):.2f} of its duration")
