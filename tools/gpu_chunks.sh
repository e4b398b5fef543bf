#!/bin/bash
# chunked beam top-K (default): beam parity suites, then C3 / C5 A/B against the per-row kernel
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/chunks"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_stepwise.py -m gpu -x -v --timeout 300 --timeout-method thread -k "beam or c3 or c5 or option or stepwise" > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
for o in beam_chunks=1 beam_chunks=0; do
  timeout -k 10 400 python -u bench.py --model medium --batch 64 --num-beams 5 --no-cpu-baseline --no-profile --opt $o > "$O/c3_$o.json" 2> "$O/c3_$o.err" || { tail -30 "$O/c3_$o.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c3_$o.json'));print('c3 $o',d['value'],d['ms_per_step'])"
  timeout -k 10 400 python -u bench.py --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 --no-cpu-baseline --no-profile --opt $o > "$O/c5_$o.json" 2> "$O/c5_$o.err" || { tail -30 "$O/c5_$o.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c5_$o.json'));print('c5 $o',d['value'],d['ms_per_step'])"
done
