#!/bin/bash
# Round-6 closing run on the final library: GPU suite, smoke(), and the C3 / C5 beam bench lines.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r06_final"; mkdir -p "$O"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -3 "$O/smoke.log"
timeout -k 10 400 python -u bench.py --model medium --batch 64 --num-beams 5 --no-cpu-baseline > "$O/bench_c3.json" 2> "$O/bench_c3.err" \
  || { tail -30 "$O/bench_c3.err"; exit 1; }
cut -c1-300 "$O/bench_c3.json"
timeout -k 10 400 python -u bench.py --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 --no-cpu-baseline > "$O/bench_c5.json" 2> "$O/bench_c5.err" \
  || { tail -30 "$O/bench_c5.err"; exit 1; }
cut -c1-300 "$O/bench_c5.json"
