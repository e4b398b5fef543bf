"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.

MI355X_MICROARCH.md (HBM, gfx950): FETCH_SIZE counts half the bytes of wide coalesced streaming reads
(double it); WRITE_SIZE is exact for 16-B/lane stores. Kernel classes follow bench.py's roofline names:
  dec_xattn  attn_xenc_* launches (encoder-space cross-attention, 16-bit modes), else the
             attn_decode* launches with the largest grid (cross-attention over precomputed K/V)
  enc_gemm   gemm_ring_kernel / gemm_tile_kernel launches (encoder conv / QKV / out / fc1 / fc2)

usage: python tools/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> <out.json> [algorithmic bytes/launch json]
"""
import collections
import csv
import glob
import json
import os
import sys


def classify(name: str, grid: int, xattn_grid: int):
    if "attn_xenc" in name:
        return "dec_xattn"
    if "attn_decode" in name and grid == xattn_grid and xattn_grid > 0:
        return "dec_xattn"
    if "gemm_tile_kernel" in name or "gemm_ring_kernel" in name:
        return "enc_gemm"
    return None


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
            meta[key] = (r["Kernel_Name"], int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0))
    has_xenc = any("attn_xenc" in n for n, g in meta.values())
    xattn_grid = 0 if has_xenc else max([g for n, g in meta.values() if "attn_decode" in n] or [0])
    out = collections.defaultdict(list)
    for k, v in per.items():
        cls = classify(*meta[k], xattn_grid)
        if cls:
            out[cls].append(v)
    return out


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bench.py --steps 1 --warmup 1 --new-tokens 4 --no-overlap (batch 32: same launches as the bench)",
           "correction": "FETCH_SIZE(KB) x 1024 x 2 (gfx950 wide-read undercount) + WRITE_SIZE(KB) x 1024",
           "kernels": {}}
    for cls in sorted(set(fetch) | set(write)):
        f = fetch.get(cls, [])
        w = write.get(cls, [])
        if not f or not w:
            continue
        fb = sum(f) / len(f) * 1024 * 2
        wb = sum(w) / len(w) * 1024
        res["kernels"][cls] = {"launches_fetch_pass": len(f), "launches_write_pass": len(w),
                               "read_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                               "hbm_bytes_per_launch": fb + wb}
    json.dump(res, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
