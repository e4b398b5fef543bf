#!/bin/bash
# cu_split diagnosis: decode alone (tools/decode_bench.py) and the C2 bench from a side stream
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r06c"; mkdir -p "$O"
for n in 0 8; do
  timeout -k 10 200 python tools/decode_bench.py --side-stream --opt cu_split=$n --reps 2 --concurrent 2 > "$O/dec_split$n.txt" 2>&1 || { tail -20 "$O/dec_split$n.txt"; exit 1; }
  tail -3 "$O/dec_split$n.txt"
done
for n in ${SPLITS:-0 8 12 16}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 20 --side-stream --opt cu_split=$n > "$O/c2_split$n.json" 2> "$O/c2_split$n.err" || { tail -20 "$O/c2_split$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c2_split$n.json'));print('cu_split $n side-stream',d['value'],d['ms_per_step'])"
done
