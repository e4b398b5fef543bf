#!/bin/bash
# beam_wide default: the configs suite (C3 / C5 parity, option formulations) and the C5 line
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/wide"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 400 python -u bench.py --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 --no-cpu-baseline > "$O/bench_c5.json" 2> "$O/bench_c5.err" \
  || { tail -30 "$O/bench_c5.err"; exit 1; }
cut -c1-200 "$O/bench_c5.json"
