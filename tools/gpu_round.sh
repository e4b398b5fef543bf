#!/bin/bash
# One GPU round trip at HEAD: parity tests (optional), C2 / C3 / C5 bench lines without the CPU
# baseline, a rocprofv3 kernel trace of the C2 bench. Every GPU step has its own limit; the chain
# stops at the first failure. Env: TESTS=1 runs the GPU tests first, TRACE=1 adds the trace,
# BEAMS=0 skips C3/C5.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/round"; mkdir -p "$O"
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=10 ${PYTEST_ARGS:-} > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
  tail -3 "$O/pytest.log"
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${C2_ARGS:-} > "$O/c2.json" 2> "$O/c2.err" || { tail -20 "$O/c2.err"; exit 1; }
python -c "import json;d=json.load(open('$O/c2.json'));print('C2',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'])"
if [ "${BEAMS:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --model medium --batch 64 --num-beams 5 > "$O/c3.json" 2> "$O/c3.err" || { tail -20 "$O/c3.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c3.json'));print('C3',d['value'],d['ms_per_step'])"
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 > "$O/c5.json" 2> "$O/c5.err" || { tail -20 "$O/c5.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c5.json'));print('C5',d['value'],d['ms_per_step'])"
fi
if [ "${TRACE:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline ${C2_ARGS:-} > "$O/trace_c2.json" 2> "$O/trace_c2.err" || { tail -5 "$O/trace_c2.err"; exit 1; }
  cd "$R"
  TR="$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)"
  python tools/prof_summary.py "$TR" 40 > "$O/kernel_summary.txt" && head -25 "$O/kernel_summary.txt"
fi
