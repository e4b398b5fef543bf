#!/bin/bash
# Bench a list of env variants (one line each): value, ms/step and the per-phase table.
# usage: VARIANTS="A=1;A=2 B=3" bash tools/variants.sh [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:-X=0}"
for v in "${VS[@]}"; do
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline "$@" > gpurun_out/v.json 2> gpurun_out/v.err || { tail -20 gpurun_out/v.err; exit 1; }
  python - "$v" <<'PY'
import json, sys
d = json.load(open("gpurun_out/v.json"))
ph = {k: v["ms_per_step"] for k, v in d.get("phases", {}).items()}
r = d.get("roofline") or {}
print(f"{sys.argv[1]:40s} {d['value']:9.1f} aud-s/s {d['ms_per_step']:7.2f} ms  xattn {r.get('avg_launch_ms')} ms frac {r.get('frac')}  {ph}", flush=True)
PY
done
