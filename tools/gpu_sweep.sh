#!/bin/bash
# Tests (PYTEST_ARGS) then bench lines for each "--opt" setting in SWEEP (space-separated, "-" = none)
# on the C3 and C5 configurations (CONFIGS="c3 c5 c2").
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/sweep"; mkdir -p "$O"
if [ -n "$PYTEST_ARGS" ]; then
  timeout -k 10 700 python -u -m pytest $PYTEST_ARGS -m gpu -x -q --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
for cfg in ${CONFIGS:-c3 c5}; do
  case $cfg in
    c3) A="--steps 5 --warmup 2 --model medium --batch 64 --num-beams 5";;
    c5) A="--steps 5 --warmup 2 --model large-v3 --batch 16 --num-beams 5 --dtype f16 --bias-phrases 5000";;
    c2) A="";;
  esac
  for o in ${SWEEP:--}; do
    OA=""; [ "$o" != "-" ] && OA="--opt $o"
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-profile $A $OA > "$O/$cfg.$o.json" 2> "$O/$cfg.$o.err" || { tail -20 "$O/$cfg.$o.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/$cfg.$o.json'));print('$cfg','$o',d['value'],d['ms_per_step'])"
  done
done
