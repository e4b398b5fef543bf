#!/bin/bash
# Round-3 GPU round trip, most informative first: decode-alone per-token times (C2 default / xqk 0;
# C3 / C5 beam rows with the folded LayerNorm on and off), then the GPU suite, then the C2 bench line.
# A crash or timeout ends the call; ordinary test failures do not stop the bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r03"; mkdir -p "$O"
export WCB_GATE_LOG="$O/gates.txt"
db() {   # decode_bench args... (appends to decode.txt)
  timeout -k 10 300 python tools/decode_bench.py "$@" >> "$O/decode.txt" 2>> "$O/decode.err" || { echo "decode_bench $* failed rc=$?"; tail -20 "$O/decode.err"; exit 1; }
  tail -1 "$O/decode.txt"
}
if [ "${DECODE:-1}" = 1 ]; then
  C3A="--model medium --batch 64 --beams 5 --short 4 --long 20"
  C5A="--model large-v3 --batch 16 --beams 5 --dtype f16 --phrases 5000 --short 4 --long 20"
  IFS=';' read -ra DBS <<< "${DB_LIST:---model small --batch 32;--model small --batch 32 --opt xqk=0;$C3A;$C3A --opt beam_xattn=0;$C3A --opt ln_fold=0;$C5A;$C5A --opt beam_xattn=0;$C5A --opt ln_fold=0}"
  for a in "${DBS[@]}"; do db $a; done
fi
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TT:-900} python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread --durations=25 ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" "$O/pytest.log" | tail -30
  [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; tail -20 "$O/pytest.log"; exit $rc; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline ${C2_ARGS:-} > "$O/c2.json" 2> "$O/c2.err" || { echo "bench failed"; tail -20 "$O/c2.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c2.json'));r=d.get('roofline') or {};print('C2',d['value'],d['ms_per_step'],r.get('kernel'),r.get('frac'))"
fi
echo done
