#!/bin/bash
# Encoder / decode co-residency experiment (C2): the bench line at several encoder CU reservations
# (option enc_cu_reserve), then a rocprofv3 kernel trace of the default for tools/trace_overlap.py.
# Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/cu"; mkdir -p "$O"
for v in ${VALS:-0 4 8}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --opt enc_cu_reserve=$v ${ARGS:-} > "$O/c2_r$v.json" 2> "$O/c2_r$v.err" || { tail -20 "$O/c2_r$v.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c2_r$v.json'));print('reserve $v', d['value'], d['ms_per_step'])"
done
if [ "${TRACE:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-profile --steps 6 --warmup 2 --boost 0 ${TRACE_ARGS:-} > "$O/trace.json" 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
  cd "$R"
  TR="$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)"
  python tools/trace_overlap.py "$TR" -250 > "$O/overlap.txt"; cat "$O/overlap.txt"
fi
