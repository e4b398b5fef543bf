#!/bin/bash
# Probe: decode-chain concurrency (C2, C3) and a rocprofv3 kernel trace of the C3 bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/probe"; mkdir -p "$O"
timeout -k 10 200 python tools/decode_bench.py --model small --batch 32 --concurrent 2 > "$O/dec_c2.txt" 2>&1 && cat "$O/dec_c2.txt" || exit 1
timeout -k 10 200 python tools/decode_bench.py --model medium --batch 64 --beams 5 --short 4 --long 20 --reps 2 --concurrent 2 > "$O/dec_c3.txt" 2>&1 && cat "$O/dec_c3.txt" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace_c3" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-profile --steps 2 --warmup 1 --model medium --batch 64 --num-beams 5 > "$O/trace_c3.json" 2> "$O/trace_c3.err" || { tail -5 "$O/trace_c3.err"; exit 1; }
cd "$R"
python tools/prof_summary.py "$(ls "$O"/trace_c3/*kernel_trace.csv | head -1)" 40 > "$O/c3_summary.txt" && head -30 "$O/c3_summary.txt"
