#!/bin/bash
# Round-4 decode experiments in one call: the cross-attention stream floor and access patterns, parity
# tests of the new layouts / fusions, decode-alone per-token times per option, overlapping decode
# contexts (with and without CU-split streams), the C2 bench line. Every GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/exp1"; mkdir -p "$O"
timeout -k 10 120 ./tools/xattn_floor > "$O/floor.txt" 2>&1 || { tail -5 "$O/floor.txt"; exit 1; }
head -6 "$O/floor.txt"
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_kernels.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "xenc or cross or fused or small_bf16 or c2_small or c2_timed or lean" > "$O/pytest.log" 2>&1 || { grep -E "FAILED|Error" "$O/pytest.log" | head -20; tail -20 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
DB="timeout -k 10 200 python tools/decode_bench.py --long 72 --short 8 --reps 3"
$DB > "$O/db_default.txt" 2>&1 && grep -v amdgpu.ids "$O/db_default.txt" || exit 1
$DB --opt xenc_fm=0 > "$O/db_nofm.txt" 2>&1 && grep -v amdgpu.ids "$O/db_nofm.txt" || exit 1
$DB --opt steps_per_graph=32 > "$O/db_spg32.txt" 2>&1 && grep -v amdgpu.ids "$O/db_spg32.txt" || exit 1
$DB --batch 64 > "$O/db_b64.txt" 2>&1 && grep -v amdgpu.ids "$O/db_b64.txt" || exit 1
DC="timeout -k 10 300 python tools/decode_bench.py --long 200 --short 8 --reps 2 --concurrent 2 --side-stream"
$DC > "$O/dc_default.txt" 2>&1 && grep -v amdgpu.ids "$O/dc_default.txt" || exit 1
$DC --opt decode_cu_split=1 > "$O/dc_cusplit.txt" 2>&1 && grep -v amdgpu.ids "$O/dc_cusplit.txt" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > "$O/c2.json" 2> "$O/c2.err" || { tail -20 "$O/c2.err"; exit 1; }
python -c "import json;d=json.load(open('$O/c2.json'));print('C2',d['value'],'audio-s/s',d['ms_per_step'],'ms/step')"
