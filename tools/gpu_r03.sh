#!/bin/bash
# Round-3 GPU round trip: the GPU suite (continues past ordinary test failures, stops the chain on a
# crash / timeout), then C2 / C3 / C5 bench lines (no CPU baseline) and optional option sweeps.
# Env: TESTS=0 skips the suite, PYTEST_ARGS extra pytest args, BEAMS=0 skips C3/C5, C2_OPTS / BEAM_OPTS:
# ";"-separated extra bench argument sets for sweeps.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03"; mkdir -p "$O"
export WCB_GATE_LOG="$O/gates.txt"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TT:-1000} python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread --durations=25 ${PYTEST_ARGS:-} > "$O/pytest.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" "$O/pytest.log" | tail -30
  # 0 ok, 1 test failures: go on; anything else (timeout, crash, interrupted) ends the call
  [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; tail -20 "$O/pytest.log"; exit $rc; }
fi
run_bench() {   # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "bench $name failed"; tail -20 "$O/$name.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/$name.json'));r=d.get('roofline') or {};print('$name',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'))"
}
run_bench c2
IFS=';' read -ra C2S <<< "${C2_OPTS:-}"
i=0; for a in "${C2S[@]}"; do i=$((i+1)); run_bench c2_opt$i $a; done
if [ "${BEAMS:-1}" = 1 ]; then
  run_bench c3 --steps 5 --warmup 2 --model medium --batch 64 --num-beams 5
  run_bench c5 --steps 5 --warmup 2 --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000
  IFS=';' read -ra BS <<< "${BEAM_OPTS:-}"
  i=0; for a in "${BS[@]}"; do i=$((i+1)); run_bench c3_opt$i --steps 5 --warmup 2 --model medium --batch 64 --num-beams 5 $a; run_bench c5_opt$i --steps 5 --warmup 2 --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000 $a; done
fi
echo done
