#!/bin/bash
# Round-3: decode-kernel microbench, the affected kernel / config tests, decode-alone timings, C2 bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${OUT:-r03h}"; mkdir -p "$O"
if [ "${MB:-1}" = 1 ]; then
  timeout -k 10 200 ./tools/dec_kernel_bench > "$O/dec_kernel.txt" 2>&1 || { echo "dec_kernel_bench failed"; tail -5 "$O/dec_kernel.txt"; exit 1; }
  cat "$O/dec_kernel.txt"
fi
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q -x --timeout 200 --timeout-method thread -k "$PYTEST_K" > "$O/pytest.log" 2>&1
  rc=$?
  tail -4 "$O/pytest.log"
  [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
fi
OUT=${OUT:-r03h} bash tools/gpu_r03d.sh
