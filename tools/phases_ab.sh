#!/bin/bash
# The C2 bench's serialised per-class phases (profiling pass on) for the defaults and each OPT
# (e.g. OPT="merge_v=2 merge_v=4"): prints value, ms/step and the decode / encoder classes per run.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/phases"; mkdir -p "$O"
for o in default ${OPT:-}; do
  a=""; [ "$o" != default ] && a="--opt $o"
  timeout -k 10 400 python bench.py --no-cpu-baseline $a ${BENCH_ARGS:-} > "$O/$o.json" 2> "$O/$o.err" || { tail -20 "$O/$o.err"; exit 1; }
  python - "$O/$o.json" "$o" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ph = d.get("phases", {})
cls = " ".join(f"{k}={v['ms_per_step']:.2f}" for k, v in ph.items() if isinstance(v, dict) and "ms_per_step" in v and v["ms_per_step"] > 0.3)
print(sys.argv[2], d["value"], d["ms_per_step"], cls, flush=True)
PY
done
