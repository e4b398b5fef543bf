"""Decode-step anatomy from a rocprofv3 kernel trace: per step (select_finalize_kernel boundaries),
the wall time, the kernels of each queue back to back (sum of durations) and the gaps between
consecutive kernels of a queue (launch/dispatch latency on the critical path).

usage: python tools/step_timeline.py gpurun_out/.../run_kernel_trace.csv [n_steps_to_show]
"""
import collections
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["k"] = r["Kernel_Name"].split("(")[0].replace("void wcb::", "").replace("wcb::", "")[:48]
    rows.sort(key=lambda r: r["s"])
    fins = [r for r in rows if "select_finalize" in r["k"]]
    steps = []
    for a, b in zip(fins, fins[1:]):
        ks = [r for r in rows if a["e"] <= r["s"] and r["e"] <= b["e"]]
        if not ks:
            continue
        steps.append((a, b, ks))
    # keep steady-state steps whose wall is near the median (drops the encoder-overlap outliers too)
    walls = [b["e"] - a["e"] for a, b, _ in steps]
    med = statistics.median(walls)
    print(f"{len(steps)} steps, wall median {med / 1e3:.1f} us, min {min(walls) / 1e3:.1f}, max {max(walls) / 1e3:.1f}")
    per_kernel = collections.defaultdict(list)
    gaps = collections.defaultdict(list)
    busy_q = collections.defaultdict(list)
    for a, b, ks in steps:
        byq = collections.defaultdict(list)
        for r in ks:
            byq[r["Queue_Id"]].append(r)
            per_kernel[(r["k"], r["Grid_Size_X"], r["Grid_Size_Y"])].append(r["e"] - r["s"])
        for q, lst in byq.items():
            busy_q[q].append(sum(r["e"] - r["s"] for r in lst))
            prev = a["e"]
            for r in lst:
                gaps[q].append(r["s"] - prev)
                prev = r["e"]
    for q in sorted(busy_q):
        print(f"queue {q}: kernels/step {len(gaps[q]) / len(steps):.0f}, busy {statistics.median(busy_q[q]) / 1e3:.1f} us/step, "
              f"gap median {statistics.median(gaps[q]) / 1e3:.2f} us, gap sum/step {sum(gaps[q]) / len(steps) / 1e3:.1f} us")
    print("per kernel (median us, launches/step):")
    for k, v in sorted(per_kernel.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {statistics.median(v) / 1e3:7.2f} us  x{len(v) / len(steps):5.1f}  grid=({k[1]},{k[2]})  {k[0]}")


if __name__ == "__main__":
    main()
