"""Check a bench.py JSON line against rocprofv3 output of the same command: the roofline kernel must be
the top kernel symbol by total time (rocprofv3 --stats' grouping: kernel_stats.csv, or a kernel trace
grouped the same way), and `frac` recomputed from rocprof's average duration for it must agree
within 5 %. With a `roofline.step`, the step fraction is recomputed from the algorithmic
work the line states and each phase's fraction from the rocprof trace's kernel times.

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
        if roof.get("avg_launch_ms_serialised"):
            # rocprofv3's kernel trace serialises the replayed graph's kernels: its per-launch duration is the
            # bench's serialised profiling pass (HIP events), while the primary figure comes from device stamps
            # inside the pipelined graph (two decode chains and the next batch's encoder beside it)
            ser = roof["avg_launch_ms_serialised"]
            out["bench_avg_ms_serialised"] = ser
            out["serialised_rel_diff"] = round(abs(ser - avg_ms) / avg_ms, 4)
            out["serialised_within_5pct"] = out["serialised_rel_diff"] <= 0.05
            out["pipelined_over_serialised"] = round(roof["avg_launch_ms"] / ser, 4)
    step = roof.get("step")
    if step:
        # SURVEY §8(d) step fraction recomputed from the algorithmic work the line states (bytes / flops at
        # the peaks) over its ms_per_step, and each phase's ideal over the rocprof trace's GPU time of the
        # kernels of that phase (the bench's class -> kernel map: roofline + roofline_other)
        w = step["work"]
        peak_mfma = roof["peak"] if roof["bound"] == "mfma" else 2500.0
        ideal = {"front_end": w["front_end_bytes"] / 8000e9 * 1e3,
                 "encoder": w["encoder_flops"] / (peak_mfma * 1e12) * 1e3,
                 "decode": w["decode_bytes"] / 8000e9 * 1e3}
        frac = sum(ideal.values()) / step["measured_ms_per_step"]
        line_all = json.loads(line)
        cls_kernel = {c: v["kernel"] for c, v in (line_all.get("roofline_other") or {}).items()}
        for c in roof["class"].split("+"):
            cls_kernel[c] = roof["kernel"]
        phase_of = lambda c: ("front_end" if c in ("log_mel", "mel_to_conv_input")
                              else "encoder" if c.startswith("enc_") or c == "layernorm" else "decode")
        kern_phase = {}
        for c, k in cls_kernel.items():
            kern_phase.setdefault(k, phase_of(c))
        steps = max(1.0, cnt.get(roof["kernel"], 0) / max(roof["launches_per_step"], 1e-9))
        meas = collections.defaultdict(float)
        for k, t in tot.items():
            if k in kern_phase:
                meas[kern_phase[k]] += t / 1e6 / steps
        out["step"] = {"frac_bench": step["frac"], "frac_recomputed": round(frac, 4),
                       "rel_diff": round(abs(frac - step["frac"]) / frac, 4),
                       "rocprof_steps": round(steps, 2),
                       "phases_rocprof": {ph: {"ideal_ms": round(ideal[ph], 4), "rocprof_ms": round(meas[ph], 3),
                                               "frac": round(ideal[ph] / meas[ph], 4) if meas[ph] else None}
                                          for ph in ideal}}
        out["step"]["within_5pct"] = out["step"]["rel_diff"] <= 0.05
    print(json.dumps(out, indent=1))
    ok = (out["match"] and (out.get("within_5pct") or out.get("serialised_within_5pct"))
          and (not step or out["step"]["within_5pct"]))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
