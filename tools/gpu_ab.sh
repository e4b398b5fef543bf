#!/bin/bash
# GPU check + A/B of one handle option (C2 bench): the named test selection (TESTS, optional -k K), then the bench line with
# the defaults (profiling pass on: per-class phases) and with OPT (e.g. OPT="merge_v=0"), then the
# overlap probe. Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/ab"; mkdir -p "$O"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS ${K:+-k "$K"} > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
  tail -3 "$O/tests.log"
fi
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -20 "$O/bench_default.err"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['ms_per_step'])"
for o in ${OPT:-}; do   # one run per word; NAME=V,NAME2=V2 sets several options in one run
  a=""; for kv in ${o//,/ }; do a="$a --opt $kv"; done
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile ${BENCH_ARGS:-} $a > "$O/bench_$o.json" 2> "$O/bench_$o.err" || { tail -20 "$O/bench_$o.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$o.json'));print('$o', d['value'], d['ms_per_step'])"
done
if [ "${PROBE:-0}" = 1 ]; then
  timeout -k 10 300 python tools/overlap_probe.py --views > "$O/probe.txt" 2>&1 || { tail -20 "$O/probe.txt"; exit 1; }
  cat "$O/probe.txt"
fi
