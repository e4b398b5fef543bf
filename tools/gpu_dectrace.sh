#!/bin/bash
# rocprofv3 kernel trace + stats of the decode alone (tools/decode_bench.py: one 32-clip chain, no
# encoder overlap) → per-kernel summary of the decode step. Trace serialises kernels: use for relative
# costs, not for the overlapped bench timing.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/dectrace"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/tools/decode_bench.py" --long 40 --short 8 --reps 1 ${DB_ARGS:-} > "$O/db.txt" 2>&1 || { tail -5 "$O/db.txt"; exit 1; }
cd "$R"
TR="$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)"
python tools/prof_summary.py "$TR" 40 > "$O/kernel_summary.txt" && head -30 "$O/kernel_summary.txt"
