#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r06g"; mkdir -p "$O"
for o in "cu_split=0" "cu_split=8"; do
  timeout -k 10 300 python tools/split_probe.py --opt $o > "$O/probe_$o.txt" 2>&1 || { tail -20 "$O/probe_$o.txt"; exit 1; }
  grep variant "$O/probe_$o.txt"
done
