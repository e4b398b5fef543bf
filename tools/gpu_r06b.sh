#!/bin/bash
# Round 6: step-wise / 8-rank shard / cu_split parity tests, then a C2 bench sweep over option cu_split.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r06b"; mkdir -p "$O"
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_stepwise.py tests/test_gpu_shard.py "tests/test_gpu_e2e.py::test_cu_split_is_bit_identical" -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > "$O/pytest.log" 2>&1
rc=$?; tail -22 "$O/pytest.log"; [ $rc = 0 ] || exit $rc
fi
for n in ${SPLITS:-0 8 4 12 16}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 20 --opt cu_split=$n > "$O/c2_split$n.json" 2> "$O/c2_split$n.err" || { tail -20 "$O/c2_split$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c2_split$n.json'));print('cu_split $n',d['value'],d['ms_per_step'])"
done
