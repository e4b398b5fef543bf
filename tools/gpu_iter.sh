#!/bin/bash
# Iteration on the GPU box: selected GPU tests (PYTEST_K filter, default all gpu tests), then a short
# bench (BENCH_ARGS). Each GPU step under its own limit, chained: the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K=${PYTEST_K:-}
if [ "$K" != "skip" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/pytest_iter.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { tail -20 gpurun_out/bench_iter.err; exit 1; }
  cat gpurun_out/bench_iter.json
fi
