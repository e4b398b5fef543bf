#!/bin/bash
# A/B of one handle option on the C2 bench (interleaved, no CPU leg, no profiling pass); OPT="name=value"
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/ab_${TAG:-opt}"; mkdir -p "$O"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
  rc=$?; tail -5 "$O/pytest.log"; [ $rc = 0 ] || exit $rc
fi
for i in ${REPS:-1 2}; do
  for o in "${BASE:-lean_x=1}" "$OPT"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 20 --opt $o ${EXTRA:-} > "$O/c2_${o}_$i.json" 2> "$O/c2_${o}_$i.err" || { tail -20 "$O/c2_${o}_$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/c2_${o}_$i.json'));print('$o',d['value'],d['ms_per_step'])"
  done
done
