#!/bin/bash
# Decode-alone timings (graphs captured once per length) + a rocprofv3 kernel trace of the C2 decode.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03c"; mkdir -p "$O"
db() { timeout -k 10 300 python tools/decode_bench.py "$@" >> "$O/decode.txt" 2>> "$O/decode.err" || { echo "decode_bench $* failed"; tail -20 "$O/decode.err"; exit 1; }; tail -1 "$O/decode.txt"; }
IFS=';' read -ra DBS <<< "${DB_LIST:---model small --batch 32;--model small --batch 32 --opt xqk=1}"
for a in "${DBS[@]}"; do db $a; done
if [ "${TRACE:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/tools/decode_bench.py" --model small --batch 32 --reps 2 > "$O/trace.out" 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
  cd "$R"
  TR="$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)"
  python tools/prof_summary.py "$TR" 40 > "$O/kernel_summary.txt" && head -30 "$O/kernel_summary.txt"
fi
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -v --timeout 300 --timeout-method thread -k "$PYTEST_K" > "$O/pytest.log" 2>&1
  grep -E "FAILED|ERROR|passed|failed" "$O/pytest.log" | tail -12
fi
echo done
