"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.

MI355X_MICROARCH.md (HBM, gfx950): FETCH_SIZE counts half the bytes of wide coalesced streaming reads
(double it); WRITE_SIZE is exact for 16-B/lane stores. Launches are keyed "<kernel symbol>|<grid
threads>" — the names bench.py's roofline reports (wcb_profile_kernel) — so the bench can attach
`traffic` to whichever kernel dominates.

usage: python tools/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> <out.json> [top_n]
"""
import collections
import csv
import glob
import json
import os
import sys


def load(pass_dir: str, counter: str):
    files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {pass_dir}")
    per = collections.defaultdict(float)   # dispatch → counter sum
    meta = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (f, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per[key] += float(r["Counter_Value"])
            meta[key] = f'{r["Kernel_Name"].split("(")[0]}|{int(r.get("Grid_Size") or 0)}'
    out = collections.defaultdict(list)
    for k, v in per.items():
        out[meta[k]].append(v)
    return out


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of bench.py with the "
                     "bench's launch shapes (batch 32, fewer tokens)",
           "correction": "FETCH_SIZE(KB) x 1024 x 2 (gfx950 wide-read undercount) + WRITE_SIZE(KB) x 1024",
           "kernels": {}}
    # per symbol over every grid it runs at (bench.py's roofline groups as rocprofv3 --stats does)
    sym = collections.defaultdict(lambda: [[], []])
    for k in set(fetch) & set(write):
        sym[k.split("|")[0]][0].extend(fetch[k])
        sym[k.split("|")[0]][1].extend(write[k])
    res["symbols"] = {}
    for k, (f, w) in sorted(sym.items(), key=lambda kv: -sum(kv[1][0]))[:top]:
        fb = sum(f) / len(f) * 1024 * 2
        wb = sum(w) / len(w) * 1024
        res["symbols"][k] = {"launches": len(f), "read_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": fb + wb}
    keys = sorted(set(fetch) & set(write), key=lambda k: -sum(fetch[k]))[:top]
    for k in keys:
        f, w = fetch[k], write[k]
        fb = sum(f) / len(f) * 1024 * 2
        wb = sum(w) / len(w) * 1024
        res["kernels"][k] = {"launches_fetch_pass": len(f), "launches_write_pass": len(w),
                             "read_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": fb + wb}
    json.dump(res, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
