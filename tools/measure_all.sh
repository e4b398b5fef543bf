#!/bin/bash
# Round-end measurement: full GPU parity suite, then tools/measure.sh (C2 bench with CPU baseline,
# bench without profiling, rocprofv3 trace, PMC passes), then C3 / C5 bench lines.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/meas"; mkdir -p "$O"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --durations=10 > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -3 "$O/pytest_gpu.log"
fi
bash tools/measure.sh || exit 1
cd "$R"
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --model medium --batch 64 --num-beams 5 > "$O/c3.json" 2> "$O/c3.err" || { tail -20 "$O/c3.err"; exit 1; }
python -c "import json;d=json.load(open('$O/c3.json'));print('C3',d['value'],d['ms_per_step'])"
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 > "$O/c5.json" 2> "$O/c5.err" || { tail -20 "$O/c5.err"; exit 1; }
python -c "import json;d=json.load(open('$O/c5.json'));print('C5',d['value'],d['ms_per_step'])"
