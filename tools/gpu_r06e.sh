#!/bin/bash
# kernel trace of the C2 bench with option cu_split (queue concurrency)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r06e"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for n in ${SPLITS:-8 0}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/tr$n" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-profile --steps 4 --warmup 2 --opt cu_split=$n > "$O/b$n.json" 2> "$O/b$n.err" || { tail -5 "$O/b$n.err"; exit 1; }
  TR="$(ls "$O"/tr$n/*kernel_trace.csv "$O"/tr$n/*/*kernel_trace.csv 2>/dev/null | head -1)"
  python3 "$R/tools/trace_overlap.py" "$TR" -150 > "$O/overlap$n.txt" 2>&1; cat "$O/overlap$n.txt" | head -20
  python3 "$R/tools/prof_summary.py" "$TR" 12 > "$O/summary$n.txt"; head -12 "$O/summary$n.txt"
  python3 -c "
import csv,collections
rows=list(csv.DictReader(open('$TR')))
q=collections.Counter(r['Queue_Id'] for r in rows); print('queues',dict(q))
" 
done
