"""Check a bench.py JSON line against rocprofv3 output of the same command: the roofline kernel must be
the top kernel symbol by total time (rocprofv3 --stats' grouping: kernel_stats.csv, or a kernel trace
grouped the same way), and `frac` recomputed from rocprof's average duration for it must agree
within 5 %.

usage: python tools/check_roofline.py <bench.json> <kernel_stats.csv | kernel_trace.csv>
"""
import collections
import csv
import json
import sys


def main():
    line = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1]
    roof = json.loads(line)["roofline"]
    rows = list(csv.DictReader(open(sys.argv[2])))
    tot, cnt = collections.defaultdict(float), collections.defaultdict(int)
    for r in rows:
        if "TotalDurationNs" in r:                      # --stats summary
            k = r["Name"].split("(")[0]
            tot[k] += float(r["TotalDurationNs"])
            cnt[k] += int(r["Calls"])
        else:                                            # kernel trace
            k = r["Kernel_Name"].split("(")[0]
            tot[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            cnt[k] += 1
    top = max(tot, key=tot.get)
    key = roof["kernel"]
    out = {"bench_kernel": key, "rocprof_top": top, "match": key == top}
    if key in tot:
        avg_ms = tot[key] / cnt[key] / 1e6
        per = roof["flops_per_launch"] if roof["bound"] == "mfma" else roof["bytes_per_launch"]
        ach = per / (avg_ms * 1e-3) / (1e12 if roof["bound"] == "mfma" else 1e9)
        out.update(rocprof_avg_ms=round(avg_ms, 5), bench_avg_ms=roof["avg_launch_ms"], rocprof_launches=cnt[key],
                   bench_launches_per_step=roof["launches_per_step"], frac_bench=roof["frac"],
                   frac_rocprof=round(ach / roof["peak"], 4),
                   rel_diff=round(abs(ach / roof["peak"] - roof["frac"]) / (ach / roof["peak"]), 4))
        out["within_5pct"] = out["rel_diff"] <= 0.05
    print(json.dumps(out, indent=1))
    return 0 if out["match"] and out.get("within_5pct") else 1


if __name__ == "__main__":
    sys.exit(main())
