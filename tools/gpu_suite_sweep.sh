#!/bin/bash
# full GPU suite, then the C2 option sweep (tools/gpu_sweep_opts.sh)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${TAG:-suite}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=5 > "$O/pytest.log" 2>&1
rc=$?; tail -4 "$O/pytest.log"; [ $rc = 0 ] || exit $rc
bash tools/gpu_sweep_opts.sh
