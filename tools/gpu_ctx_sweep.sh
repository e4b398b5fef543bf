#!/bin/bash
# Decode-context / hardware-queue sweep: overlapping decode calls (tools/decode_bench.py --concurrent,
# 200-token calls so the encoder is small beside the decode), then the C2 bench line (no CPU baseline,
# no profiling pass). Each variant: "<GPU_MAX_HW_QUEUES> <decode_contexts>".
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/ctx"; mkdir -p "$O"
for q in ${QUEUES:-4 8}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tools/decode_bench.py --long 200 --short 8 --reps 2 --concurrent 2 --opt decode_contexts=3 > "$O/db_q$q.txt" 2>&1 || { tail -20 "$O/db_q$q.txt"; exit 1; }
  echo "queues $q:"; cat "$O/db_q$q.txt"
done
for v in ${VARIANTS:-"4 2" "8 2" "4 3" "8 3" "16 4"}; do
  set -- $v
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile --steps ${STEPS:-20} --opt decode_contexts=$2 ${EXTRA:-} > "$O/q$1_c$2.json" 2> "$O/q$1_c$2.err" || { tail -20 "$O/q$1_c$2.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/q$1_c$2.json'));print('queues $1 contexts $2:',d['value'],'audio-s/s',d['ms_per_step'],'ms/step')"
done
