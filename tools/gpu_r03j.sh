#!/bin/bash
# Round-3: tests, decode timing, C2 bench, and FETCH_SIZE PMC passes of a light bench run at two
# encoder tile rasters (encoder GEMM A/W re-fetch).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${OUT:-r03j}"; mkdir -p "$O"
OUT=${OUT:-r03j} TRACE=0 bash tools/gpu_r03i.sh || exit 1
PMC_ARGS="--steps 1 --warmup 1 --new-tokens 4 --no-overlap --no-cpu-baseline --no-profile --boost 0"
cd /tmp && export TMPDIR=/tmp
for r in ${RASTERS:-0 8}; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_r$r" -o run --output-format csv -- python3 "$R/bench.py" $PMC_ARGS --opt enc_raster=$r > "$O/pmc_r$r.out" 2> "$O/pmc_r$r.err" || { tail -5 "$O/pmc_r$r.err"; exit 1; }
done
cd "$R"
python3 - "$O" ${RASTERS:-0 8} <<'PY'
import csv, glob, os, sys, collections
O = sys.argv[1]
for r in sys.argv[2:]:
    per = collections.defaultdict(float); meta = {}
    for f in glob.glob(os.path.join(O, f"pmc_fetch_r{r}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != "FETCH_SIZE": continue
            k = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
            per[k] += float(row["Counter_Value"]); meta[k] = (row["Kernel_Name"].split("(")[0][-60:], int(row.get("Grid_Size") or 0))
    agg = collections.defaultdict(list)
    for k, v in per.items(): agg[meta[k]].append(v * 1024 * 2 / 1e6)   # KB units x 2 (gfx950 wide-read correction) -> MB
    print(f"raster {r}: FETCH_SIZE x2 per launch (MB)")
    for (name, grid), vs in sorted(agg.items(), key=lambda t: -sum(t[1]))[:8]:
        print(f"   {name:62s} grid {grid:9d} n {len(vs):4d} median {sorted(vs)[len(vs)//2]:9.1f}")
PY
echo done
