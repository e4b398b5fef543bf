#!/bin/bash
# bench.py under several env settings (BENCH_ENVS, ';'-separated), short runs, no CPU baseline.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/benv"; mkdir -p "$O"
IFS=';' read -ra ENVS <<< "${BENCH_ENVS:-WCB_DEC=1}"
for e in "${ENVS[@]}"; do
  env $e timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-profile ${BENCH_ARGS:-} > "$O/b.json" 2> "$O/b.err" || { tail -20 "$O/b.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/b.json')); print('$e', '->', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/step')"
done
