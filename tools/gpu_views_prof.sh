#!/bin/bash
# Kernel-level comparison of the two weight-loading paths (host f32 upload vs device bf16 views):
# rocprofv3 kernel trace of tools/overlap_probe.py --only-full for each, summarised per kernel.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/vp"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in host views; do
  F=""; [ $v = views ] && F="--views"
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/$v" -o run --output-format csv -- python3 "$R/tools/overlap_probe.py" --only-full --steps 4 $F ${ARGS:-} > "$O/$v.txt" 2>&1 || { tail -5 "$O/$v.txt"; exit 1; }
  grep pipelined "$O/$v.txt"
  TR="$(ls "$O"/$v/*kernel_trace.csv "$O"/$v/*/*kernel_trace.csv 2>/dev/null | head -1)"
  python "$R/tools/prof_summary.py" "$TR" 25 > "$O/${v}_summary.txt"; head -14 "$O/${v}_summary.txt"
done
