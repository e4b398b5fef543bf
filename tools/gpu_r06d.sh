#!/bin/bash
# cu_split (encoder-only CU mask) sweep of the C2 bench, interleaved with the default
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
export GPU_MAX_HW_QUEUES=${HWQ:-8}
O="$R/gpurun_out/r06d_q$GPU_MAX_HW_QUEUES"; mkdir -p "$O"
for n in ${SPLITS:-0 8 4 12 0 6 10}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 20 --opt cu_split=$n > "$O/c2_split$n.json" 2> "$O/c2_split$n.err" || { tail -20 "$O/c2_split$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c2_split$n.json'));print('cu_split $n',d['value'],d['ms_per_step'])"
done
