#!/bin/bash
# Round-3: beam tests, C3 / C5 bench lines (beam search now asynchronous: encoder / decode overlap).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${OUT:-r03k}"; mkdir -p "$O"
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "$PYTEST_K" > "$O/pytest.log" 2>&1
  rc=$?; tail -4 "$O/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc $rc: stopping"; exit 1; }
fi
run_bench() {   # name, args...
  local name=$1; shift
  timeout -k 10 500 python bench.py --no-cpu-baseline "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "bench $name failed"; tail -20 "$O/$name.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/$name.json'));r=d.get('roofline') or {};print('$name',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'))"
}
[ "${C3:-1}" = 1 ] && { run_bench c3 --steps 5 --warmup 2 --model medium --batch 64 --num-beams 5 ${C3_ARGS:-} || exit 1; }
[ "${C5:-1}" = 1 ] && { run_bench c5 --steps 5 --warmup 2 --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 ${C5_ARGS:-} || exit 1; }
[ "${C2:-0}" = 1 ] && { run_bench c2 || exit 1; }
echo done
