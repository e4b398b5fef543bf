#!/bin/bash
# GPU parity tests on the box (PYTEST_ARGS: extra pytest args, e.g. a file or -k filter), log under
# gpurun_out/tests/. One pytest process, per-test thread timeout.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/tests"; mkdir -p "$O"
timeout -k 10 ${T:-1000} python -u -m pytest tests -m gpu -x -v --timeout ${TT:-200} --timeout-method thread --durations=15 ${PYTEST_ARGS:-} > "$O/pytest.log" 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" "$O/pytest.log" | tail -60; tail -30 "$O/pytest.log" | grep -v PASSED; exit $rc
