#!/bin/bash
# masked-stream diagnosis: overlapping generate calls (tools/decode_bench.py --concurrent 2) and the C2 bench
# with the encoder stream unmasked / masked to every CU / masked to 24 CUs per XCD
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r06f"; mkdir -p "$O"
for o in "cu_split=0" "enc_mask_all=1" "cu_split=8"; do
  timeout -k 10 200 python tools/decode_bench.py --opt $o --reps 2 --concurrent 2 > "$O/dec_$o.txt" 2>&1 || { tail -20 "$O/dec_$o.txt"; exit 1; }
  grep -v amdgpu.ids "$O/dec_$o.txt" | tail -2
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 20 --opt $o > "$O/c2_$o.json" 2> "$O/c2_$o.err" || { tail -20 "$O/c2_$o.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/c2_$o.json'));print('$o',d['value'],d['ms_per_step'])"
done
