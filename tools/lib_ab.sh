#!/bin/bash
# A/B of two builds of libwcb.so on one box: the tree's library (new) against gpurun_ab_old.so (old,
# built from the previous commit), alternated, each bench a fresh process. Optional TESTS first.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/lab"; mkdir -p "$O"
L=whisper_context_biasing_amd/libwcb.so
cp "$L" "$O/new.so" && cp gpurun_ab_old.so "$O/old.so" || exit 1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS ${K:+-k "$K"} > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
  tail -2 "$O/tests.log"
fi
for i in $(seq 1 ${REPS:-3}); do
  for v in new old; do
    cp "$O/$v.so" "$L" || exit 1
    timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$O/b_$v.$i.json" 2> "$O/b.err" || { tail -20 "$O/b.err"; cp "$O/new.so" "$L"; exit 1; }
    python -c "
import json;d=json.load(open('$O/b_$v.$i.json'));ph=d.get('phases') or {}
print('$v', d['value'], d['ms_per_step'], {k: round(ph[k]['ms_per_step'],3) for k in ${PHASES:-['dec_xmerge','dec_xattn']} if k in ph})"
  done
done
cp "$O/new.so" "$L"
