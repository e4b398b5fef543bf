"""Bit-identity of a handle option against the defaults: C2-shaped greedy decode (whisper-small bf16, 32 clips,
1000-phrase boost, 24 tokens) and the encoder output. usage: python tools/opt_identity.py name=value [...]"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import whisper_np as W
from whisper_context_biasing_amd.config import get_dims
from whisper_context_biasing_amd.model import WhisperCB
from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list
from whisper_context_biasing_amd.weights import make_weights
dims = get_dims("small")
sd = make_weights(dims, seed=1, recipe="margin")
x = torch.from_numpy(W.log_mel(synth_batch(32), dims.n_mel))
kw = dict(max_length=24, min_new_tokens=24, bias_list=synth_bias_list(1000, eot=dims.eos_token_id), bias_boost=2.0)
m = WhisperCB.from_state_dict(dims, sd, dtype="bf16")
ref_e, ref = m.encode(x).clone(), m.generate(x, **kw).cpu()
for o in sys.argv[1:]:
    k, v = o.split("=")
    m.set_option(k, int(v))
ok = torch.equal(m.encode(x), ref_e) and torch.equal(m.generate(x, **kw).cpu(), ref)
print("identical" if ok else "DIFFERENT", sys.argv[1:], flush=True)
sys.exit(0 if ok else 1)
