#!/bin/bash
# rocprofv3 kernel trace + per-kernel summary of one bench configuration (ARGS = bench.py arguments),
# written to gpurun_out/trace_$NAME/ and gpurun_out/trace_$NAME/kernel_summary.txt.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
N="${NAME:-cfg}"; O="$R/gpurun_out/trace_$N"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-profile $ARGS > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
cd "$R"
TR="$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)"
python tools/prof_summary.py "$TR" 40 > "$O/kernel_summary.txt" && head -30 "$O/kernel_summary.txt"
