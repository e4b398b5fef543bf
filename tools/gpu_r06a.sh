#!/bin/bash
# Round-6 first GPU trip: CU-mask mapping probe, the new step-wise / 8-rank shard tests, a C2 bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r06a"; mkdir -p "$O"
timeout -k 10 60 ./tools/cumask_probe > "$O/cumask.txt" 2>&1 || { cat "$O/cumask.txt" | tail -20; exit 1; }
head -5 "$O/cumask.txt"
timeout -k 10 900 python -u -m pytest tests/test_gpu_stepwise.py tests/test_gpu_shard.py -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > "$O/pytest.log" 2>&1
rc=$?; tail -25 "$O/pytest.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > "$O/c2.json" 2> "$O/c2.err" || { tail -20 "$O/c2.err"; exit 1; }
python -c "import json;d=json.load(open('$O/c2.json'));print('C2',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['traffic'],d['roofline']['step']['frac'])"
