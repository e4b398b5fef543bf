#!/bin/bash
# Beam decode kernel traces (C3 medium 64x5 bf16, C5 large-v3 16x5 f16): rocprofv3 kernel trace of
# decode_bench, summarised per kernel.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${OUT:-beam}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/c3" -o run --output-format csv -- python3 "$R/tools/decode_bench.py" --model medium --batch 64 --beams 5 --short 4 --long 12 --reps 1 > "$O/c3.out" 2> "$O/c3.err" || { tail -5 "$O/c3.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/c5" -o run --output-format csv -- python3 "$R/tools/decode_bench.py" --model large-v3 --batch 16 --beams 5 --dtype f16 --phrases 5000 --short 4 --long 12 --reps 1 > "$O/c5.out" 2> "$O/c5.err" || { tail -5 "$O/c5.err"; exit 1; }
cd "$R"
for c in c3 c5; do
  TR="$(ls "$O"/$c/*kernel_trace.csv "$O"/$c/*/*kernel_trace.csv 2>/dev/null | head -1)"
  python tools/prof_summary.py "$TR" 30 > "$O/${c}_summary.txt" && echo "== $c" && head -22 "$O/${c}_summary.txt"
done
cat "$O/c3.out" "$O/c5.out" | grep token
echo done
