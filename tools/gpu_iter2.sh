#!/bin/bash
# Iteration: selected GPU tests (PYTEST_ARGS), C3 (+C5, C2) bench lines, optional C3 kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/iter"; mkdir -p "$O"
if [ -n "$PYTEST_ARGS" ]; then
  timeout -k 10 700 python -u -m pytest $PYTEST_ARGS -m gpu -x -q --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
timeout -k 10 400 python bench.py --no-cpu-baseline --no-profile --steps 5 --warmup 2 --model medium --batch 64 --num-beams 5 > "$O/c3.json" 2> "$O/c3.err" || { tail -20 "$O/c3.err"; exit 1; }
python -c "import json;d=json.load(open('$O/c3.json'));print('C3',d['value'],d['ms_per_step'])"
timeout -k 10 400 python bench.py --no-cpu-baseline --no-profile --steps 5 --warmup 2 --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 > "$O/c5.json" 2> "$O/c5.err" || { tail -20 "$O/c5.err"; exit 1; }
python -c "import json;d=json.load(open('$O/c5.json'));print('C5',d['value'],d['ms_per_step'])"
if [ "${C2:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > "$O/c2.json" 2> "$O/c2.err" || { tail -20 "$O/c2.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c2.json'));print('C2',d['value'],d['ms_per_step'])"
fi
if [ "${TRACE:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace_c3" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-profile --steps 2 --warmup 1 --model medium --batch 64 --num-beams 5 > "$O/trace_c3.json" 2> "$O/trace_c3.err" || { tail -5 "$O/trace_c3.err"; exit 1; }
  cd "$R"
  python tools/prof_summary.py "$(ls "$O"/trace_c3/*kernel_trace.csv | head -1)" 40 > "$O/c3_summary.txt" && head -24 "$O/c3_summary.txt"
fi
if [ "${TRACE5:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace_c5" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-profile --steps 2 --warmup 1 --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 > "$O/trace_c5.json" 2> "$O/trace_c5.err" || { tail -5 "$O/trace_c5.err"; exit 1; }
  cd "$R"
  python tools/prof_summary.py "$(ls "$O"/trace_c5/*kernel_trace.csv | head -1)" 40 > "$O/c5_summary.txt" && head -24 "$O/c5_summary.txt"
fi
