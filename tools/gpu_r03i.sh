#!/bin/bash
# Round-3: lean/fragment-major tests, decode-alone timings, C2 bench, rocprofv3 kernel trace of the C2 decode.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${OUT:-r03i}"; mkdir -p "$O"
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q -x --timeout 200 --timeout-method thread -k "$PYTEST_K" > "$O/pytest.log" 2>&1
  rc=$?
  tail -4 "$O/pytest.log"
  [ $rc -eq 0 ] || { echo "pytest rc $rc: stopping"; exit 1; }
fi
OUT=${OUT:-r03i} bash tools/gpu_r03d.sh || exit 1
if [ "${TRACE:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/tools/decode_bench.py" --model small --batch 32 --reps 2 > "$O/trace.out" 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
  cd "$R"
  TR="$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)"
  python tools/prof_summary.py "$TR" 40 > "$O/kernel_summary.txt" && head -24 "$O/kernel_summary.txt"
fi
echo done
