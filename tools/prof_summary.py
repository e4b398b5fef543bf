"""Summarise a rocprofv3 kernel trace: per (kernel, grid) totals and averages."""
import collections
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
g = collections.defaultdict(list)
for r in rows:
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])   # total threads
    k = (r["Kernel_Name"].split("(")[0][:60], grid, r["Workgroup_Size_X"])
    g[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in g.values())
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{sum(v)/1e6:8.2f} ms {100*sum(v)/tot:5.1f}% n={len(v):6d} avg={sum(v)/len(v)/1e3:8.2f}us grid={k[1]:>9} wg={k[2]:>4} {k[0]}")
