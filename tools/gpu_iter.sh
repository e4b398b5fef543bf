#!/bin/bash
# One build-measure iteration on the GPU box: optional pytest subset (PYTEST_K / PYTEST_FILES),
# optional microbenchmark script (MB), the C2 bench line without CPU baseline / profiling pass.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/iter"; mkdir -p "$O"
if [ -n "${PYTEST_FILES:-}" ]; then
  timeout -k 10 ${PYT:-600} python -u -m pytest $PYTEST_FILES -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest.log" 2>&1 || { grep -E "FAILED|Error|assert" "$O/pytest.log" | head -30; tail -30 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
if [ -n "${MB:-}" ]; then
  timeout -k 10 300 python $MB > "$O/mb.txt" 2>&1 || { tail -20 "$O/mb.txt"; exit 1; }
  grep -v amdgpu.ids "$O/mb.txt"
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile ${C2_ARGS:-} > "$O/c2.json" 2> "$O/c2.err" || { tail -20 "$O/c2.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c2.json'));print('C2',d['value'],'audio-s/s',d['ms_per_step'],'ms/step')"
fi
