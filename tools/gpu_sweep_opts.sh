#!/bin/bash
# C2 bench over a list of option settings (OPTS="a=1 a=2 ..."), REPS passes interleaved; no CPU leg / profiling
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/sweep_${TAG:-x}"; mkdir -p "$O"
for i in ${REPS:-1 2}; do
  for o in $OPTS; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 20 --opt $o ${EXTRA:-} > "$O/c2_${o}_$i.json" 2> "$O/c2_${o}_$i.err" || { tail -20 "$O/c2_${o}_$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/c2_${o}_$i.json'));print('$o',d['value'],d['ms_per_step'])"
  done
done
