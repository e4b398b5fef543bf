#!/bin/bash
# The driver's bench command (default args, CPU leg included) plus a rocprofv3 kernel trace of the same
# command and the roofline cross-check; outputs under gpurun_out/$TAG.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${TAG:-full}"; mkdir -p "$O"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('C2',d['value'],d['ms_per_step'],r['frac'],r['traffic'],r['step']['frac'],r['step']['ideal_ms'],d['cpu_baseline'] and d['cpu_baseline']['value'])"
if [ "${TRACE:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/trace_bench.json" 2> "$O/trace_bench.err" || { tail -5 "$O/trace_bench.err"; exit 1; }
  cd "$R"
  TR="$(ls "$O"/trace/*kernel_trace.csv "$O"/trace/*/*kernel_trace.csv 2>/dev/null | head -1)"
  ST="$(ls "$O"/trace/*kernel_stats.csv "$O"/trace/*/*kernel_stats.csv 2>/dev/null | head -1)"
  python tools/prof_summary.py "$TR" 40 > "$O/kernel_summary.txt" && head -12 "$O/kernel_summary.txt"
  cp "$ST" "$O/kernel_stats.csv"
  python tools/check_roofline.py "$O/trace_bench.json" "$TR" > "$O/check.json"; cat "$O/check.json"
fi
