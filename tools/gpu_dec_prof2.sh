#!/bin/bash
# rocprofv3 kernel traces of the standalone C2 decode under several env settings (PROF_ENVS, ';'-separated).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/prof2"; mkdir -p "$O"
IFS=';' read -ra ENVS <<< "${PROF_ENVS:-WCB_DEC=1}"
i=0
for e in "${ENVS[@]}"; do
  i=$((i+1))
  cd /tmp && export TMPDIR=/tmp
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/t$i" -o run --output-format csv -- python3 "$R/tools/decode_bench.py" ${DEC_ARGS:---model small --batch 32} --reps 1 > "$O/t$i.out" 2> "$O/t$i.err" || { tail -5 "$O/t$i.err"; exit 1; }
  cd "$R"
  echo "== $e"; grep ms/token "$O/t$i.out"
  python tools/prof_summary.py "$(ls "$O"/t$i/*kernel_trace.csv "$O"/t$i/*/*kernel_trace.csv 2>/dev/null | head -1)" 30 | grep -v "ring\|flash\|layernorm_kernel\|rocclr\|logmel\|mel_to" | head -${TOPN:-16}
done
