set -o pipefail
mkdir -p gpurun_out/fl
timeout -k 10 200 python -u -c "
import sys; sys.path.insert(0,'tools'); sys.path.insert(0,'tests')
import torch; torch.manual_seed(0)
from microbench import attn_case
from test_gpu_kernels import _attn, _attn_ref
for S in (1500, 200):
  q=(torch.randn(4,S,768)*0.3).bfloat16().cuda(); k=torch.randn(4,S,768).bfloat16().cuda(); v=torch.randn(4,S,768).bfloat16().cuda()
  o5=_attn('bf16',q,k,v,105); o6=_attn('bf16',q,k,v,106); o4=_attn('bf16',q,k,v,100); r=_attn_ref(q,k,v)
  print('S',S,'105==106', torch.equal(o5,o6), 'err 106', (o6.double()-r).abs().max().item(), 'err 100', (o4.double()-r).abs().max().item())
for c in (106,105,100,106,105,100,1): attn_case(32,12,1500,1500,c)
" > gpurun_out/fl/micro.txt 2>&1 || { tail -20 gpurun_out/fl/micro.txt; exit 1; }
cat gpurun_out/fl/micro.txt
for i in 1 2; do
for o in ${OPTS:-enc_flash=6 enc_flash=5}; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --opt $o > gpurun_out/fl/b_$o.$i.json 2> gpurun_out/fl/b.err || { tail -20 gpurun_out/fl/b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/fl/b_$o.$i.json'));print('$o', d['value'], d['ms_per_step'])"
done; done
