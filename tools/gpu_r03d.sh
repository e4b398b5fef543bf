#!/bin/bash
# Round-3 GPU round trip: decode-alone per-token times (DB_LIST), C2 bench lines (default + C2_OPTS
# sweeps), then the GPU suite (TESTS=1). A crash or timeout ends the call.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/${OUT:-r03d}"; mkdir -p "$O"
export WCB_GATE_LOG="$O/gates.txt"
db() { timeout -k 10 300 python tools/decode_bench.py "$@" >> "$O/decode.txt" 2>> "$O/decode.err" || { echo "decode_bench $* failed"; tail -20 "$O/decode.err"; exit 1; }; tail -1 "$O/decode.txt"; }
if [ -n "${DB_LIST:-}" ]; then
  IFS=';' read -ra DBS <<< "$DB_LIST"
  for a in "${DBS[@]}"; do db $a; done
fi
run_bench() {   # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "bench $name failed"; tail -20 "$O/$name.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/$name.json'));r=d.get('roofline') or {};print('$name',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'))"
}
if [ "${BENCH:-1}" = 1 ]; then
  run_bench c2 ${C2_ARGS:-}
  IFS=';' read -ra C2S <<< "${C2_OPTS:-}"
  i=0; for a in "${C2S[@]}"; do i=$((i+1)); run_bench c2_opt$i --no-profile $a; done
fi
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 ${TT:-900} python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread --durations=25 ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" "$O/pytest.log" | tail -30
  [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; tail -20 "$O/pytest.log"; exit $rc; }
fi
echo done
