"""Is the decode loop host-bound? Time generate(block=False) host return vs completion."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisper_context_biasing_amd.model import WhisperCB  # noqa: E402
from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list  # noqa: E402

m = WhisperCB.from_seed(sys.argv[1] if len(sys.argv) > 1 else "small")
pcm = torch.from_numpy(synth_batch(32)).cuda()
phr = synth_bias_list(1000, eot=m.dims.eos_token_id)
for graph in (True, False):
    for rep in range(3):
        mel = m.log_mel(pcm)
        m.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ids = m.generate(mel, max_length=64, min_new_tokens=64, bias_list=phr, bias_boost=2.0, block=False,
                         use_graph=graph)
        t1 = time.perf_counter()
        m.synchronize()
        t2 = time.perf_counter()
        print(f"graph={graph} host-return {1e3 * (t1 - t0):8.2f} ms   complete {1e3 * (t2 - t0):8.2f} ms", flush=True)
