#!/bin/bash
# Decode-kernel iteration on the GPU box: GPU parity tests (PYTEST_K filter, "skip" to skip), then
# standalone decode timing of C2 under a few env settings (DEC_ENVS, ';'-separated), then an optional
# rocprofv3 kernel trace of the C2 decode (PROF=1). Each GPU step under its own limit, chained.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/iter"; mkdir -p "$O"
K=${PYTEST_K:-}
if [ "$K" != "skip" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > "$O/pytest.log" 2>&1
  rc=$?; tail -15 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra ENVS <<< "${DEC_ENVS:-WCB_DEC=1}"
for e in "${ENVS[@]}"; do
  echo "== $e"
  env $e timeout -k 10 200 python -u tools/decode_bench.py ${DEC_ARGS:---model small --batch 32} > "$O/dec.txt" 2>&1 || { tail -20 "$O/dec.txt"; exit 1; }
  grep ms/token "$O/dec.txt"
done
if [ "${PROF:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  env ${PROF_ENV:-WCB_DEC=1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/tools/decode_bench.py" --model small --batch 32 --reps 1 > "$O/trace.out" 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
  cd "$R"
  python tools/prof_summary.py "$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)" 30 > "$O/kernel_summary.txt"
  head -24 "$O/kernel_summary.txt"
fi
