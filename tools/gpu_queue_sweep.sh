set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/q
for cfg in "8 3" "8 2" "16 4"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --opt decode_contexts=$2 > gpurun_out/q/q$1_c$2.json 2> gpurun_out/q/q$1_c$2.err || { tail -5 gpurun_out/q/q$1_c$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/q/q$1_c$2.json'));print('q$1 c$2', d['value'], d['ms_per_step'])"
done
