"""Concurrency analysis of a rocprofv3 kernel trace: per queue, busy time (union of its kernels'
intervals) and the time during which >= 2 queues are busy at once, over a window.
  python tools/trace_overlap.py run_kernel_trace.csv [t_skip_ms]
(a negative t_skip_ms keeps only the last |t_skip_ms| ms of the trace)"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
if skip >= 0:
    t0 = min(int(r["Start_Timestamp"]) for r in rows) + skip * 1e6
else:
    t0 = max(int(r["End_Timestamp"]) for r in rows) + skip * 1e6
ev = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0:
        continue
    ev[r["Queue_Id"]].append((s, e, r["Kernel_Name"][:40]))
def union(iv):
    iv = sorted(iv)
    out = []
    for s, e, _ in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out
U = {q: union(v) for q, v in ev.items()}
t_end = max(e for v in ev.values() for _, e, _ in v)
span = t_end - t0
print(f"window {span/1e6:.2f} ms")
for q, u in sorted(U.items()):
    busy = sum(e - s for s, e in u)
    names = defaultdict(int)
    for _, _, n in ev[q]:
        names[n.split("<")[0].replace("void wcb::", "")] += 1
    top = sorted(names.items(), key=lambda kv: -kv[1])[:3]
    print(f"queue {q}: {len(ev[q])} kernels, busy {busy/1e6:.2f} ms ({100*busy/span:.1f}%), top {top}")
# time with k queues busy
pts = []
for q, u in U.items():
    for s, e in u:
        pts.append((s, 1)); pts.append((e, -1))
pts.sort()
cur, last = 0, pts[0][0]
hist = defaultdict(int)
for t, d in pts:
    hist[cur] += t - last
    cur += d
    last = t
for k in sorted(hist):
    print(f"{k} queues busy: {hist[k]/1e6:.2f} ms ({100*hist[k]/span:.1f}%)")
