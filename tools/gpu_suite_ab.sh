#!/bin/bash
# full GPU suite (per-test limits) then an interleaved C2 A/B of one option (BASE vs OPT)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${TAG:-suite}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > "$O/pytest.log" 2>&1
rc=$?; tail -15 "$O/pytest.log"; [ $rc = 0 ] || exit $rc
for i in ${REPS:-1 2}; do
  for o in "$BASE" "$OPT"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 20 --opt $o > "$O/c2_${o}_$i.json" 2> "$O/c2_${o}_$i.err" || { tail -20 "$O/c2_${o}_$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/c2_${o}_$i.json'));print('$o',d['value'],d['ms_per_step'])"
  done
done
