"""Check a bench.py JSON line against a rocprofv3 kernel trace of the same command: the roofline kernel
must be the trace's top (kernel symbol, grid) by total time, and `frac` recomputed from the trace's
average duration for it must agree within 5 %.

usage: python tools/check_roofline.py <bench.json> <kernel_trace.csv>
"""
import collections
import csv
import json
import sys


def main():
    line = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1]
    roof = json.loads(line)["roofline"]
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[2])):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        g[f'{r["Kernel_Name"].split("(")[0]}|{grid}'].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    top = max(g, key=lambda k: sum(g[k]))
    key = f'{roof["kernel"]}|{roof["grid"]}'
    dur = g.get(key)
    out = {"bench_kernel": key, "trace_top": top, "match": key == top}
    if dur:
        avg_ms = sum(dur) / len(dur) / 1e6
        per = roof["flops_per_launch"] if roof["bound"] == "mfma" else roof["bytes_per_launch"]
        ach = per / (avg_ms * 1e-3) / (1e12 if roof["bound"] == "mfma" else 1e9)
        out.update(trace_avg_ms=round(avg_ms, 5), bench_avg_ms=roof["avg_launch_ms"], trace_launches=len(dur),
                   frac_bench=roof["frac"], frac_trace=round(ach / roof["peak"], 4),
                   rel_diff=round(abs(ach / roof["peak"] - roof["frac"]) / (ach / roof["peak"]), 4))
        out["within_5pct"] = out["rel_diff"] <= 0.05
    print(json.dumps(out, indent=1))
    return 0 if out["match"] and out.get("within_5pct") else 1


if __name__ == "__main__":
    sys.exit(main())
