#!/bin/bash
# Decode-step baseline on the GPU box: standalone per-token decode time for C2 / C3 / C5 and a
# rocprofv3 kernel trace of the C2 decode alone. Each GPU step under its own limit, chained.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/dec"; mkdir -p "$O"
timeout -k 10 200 python -u tools/decode_bench.py --model small --batch 32 > "$O/c2.txt" 2>&1 || { tail -20 "$O/c2.txt"; exit 1; }
cat "$O/c2.txt"
if [ "${BEAMS:-1}" = "1" ]; then
timeout -k 10 300 python -u tools/decode_bench.py --model medium --batch 64 --beams 5 --short 4 --long 20 --reps 2 > "$O/c3.txt" 2>&1 || { tail -20 "$O/c3.txt"; exit 1; }
cat "$O/c3.txt"
timeout -k 10 300 python -u tools/decode_bench.py --model large-v3 --batch 16 --beams 5 --dtype f16 --phrases 5000 --short 4 --long 20 --reps 2 > "$O/c5.txt" 2>&1 || { tail -20 "$O/c5.txt"; exit 1; }
cat "$O/c5.txt"
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/tools/decode_bench.py" --model small --batch 32 --reps 1 > "$O/trace.out" 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
cd "$R"
python tools/prof_summary.py "$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)" 30 > "$O/kernel_summary.txt"
head -30 "$O/kernel_summary.txt"
