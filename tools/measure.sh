#!/bin/bash
# Round measurement on the GPU box: bench (driver defaults, with CPU baseline), bench without the
# in-bench profiling, rocprofv3 kernel trace + stats, and two PMC passes for HBM traffic.
# Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
TAG=${TAG:-r01}
O="$R/gpurun_out/meas"; mkdir -p "$O"
timeout -k 10 600 python bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -20 "$O/bench_default.err"; exit 1; }
cat "$O/bench_default.json"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > "$O/bench_noprof.json" 2> "$O/bench_noprof.err" || exit 1
cat "$O/bench_noprof.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/trace_bench.json" 2> "$O/trace_bench.err" || exit 1
# PMC passes on a light run of the same launches (4 tokens, serialised batches): one counter group each
PMC_ARGS="--steps 1 --warmup 1 --new-tokens 4 --no-overlap --no-cpu-baseline --no-profile"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" $PMC_ARGS > "$O/pmc_fetch.out" 2> "$O/pmc_fetch.err" || { tail -5 "$O/pmc_fetch.err"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" $PMC_ARGS > "$O/pmc_write.out" 2> "$O/pmc_write.err" || { tail -5 "$O/pmc_write.err"; exit 1; }
cd "$R"
python tools/prof_summary.py "$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)" 40 > "$O/kernel_summary.txt"
cat "$O/kernel_summary.txt" | head -25
python tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" "$O/pmc_traffic.json" > /dev/null
TRACE="$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)"
STATS="$(ls "$O"/trace/*kernel_stats.csv "$O"/trace/*/*kernel_stats.csv 2>/dev/null | head -1)"
cp "$STATS" "$O/kernel_stats.csv"
python tools/check_roofline.py "$O/bench_default.json" "$O/kernel_stats.csv" > "$O/check_default.json"; cat "$O/check_default.json"
