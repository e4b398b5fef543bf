#!/bin/bash
# full GPU suite + smoke on the current library, then the C2 default bench line (no CPU leg)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${TAG:-suite}"; mkdir -p "$O"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$O/bench_c2.json" 2> "$O/bench_c2.err" || { tail -30 "$O/bench_c2.err"; exit 1; }
cut -c1-200 "$O/bench_c2.json"
