"""Pipelined C2 step variants under a handle option (measurement tool): (a) the bench's step, log_mel(pcm)
then generate(mel, block=False); (b) generate(mel) only, mel computed once; (c) like (a) from a torch side
stream. Prints ms per step for each.

  python tools/split_probe.py --opt cu_split=8 [--opt ...] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisper_context_biasing_amd.config import get_dims  # noqa: E402
from whisper_context_biasing_amd.model import WhisperCB  # noqa: E402
from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list  # noqa: E402
from whisper_context_biasing_amd.weights import make_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--variants", default="abc")
    a = ap.parse_args()
    dims = get_dims("small")
    opts = {k: int(v) for k, v in (o.split("=", 1) for o in a.opt)}
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0), dtype="bf16", options=opts or None)
    pcm = torch.from_numpy(synth_batch(32)).cuda()
    phrases = synth_bias_list(1000, eot=dims.eos_token_id)
    kw = dict(max_length=64, min_new_tokens=64, bias_list=phrases, bias_boost=2.0, block=False)
    mel0 = m.log_mel(pcm)

    def run(variant):
        keep = []
        def step():
            mel = m.log_mel(pcm) if variant in "ac" else mel0
            keep.append((mel, m.generate(mel, **kw)))
        for _ in range(3):
            step()
        m.synchronize(); torch.cuda.synchronize(); keep.clear()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        m.synchronize(); torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    for v in a.variants:
        if v == "c":
            with torch.cuda.stream(torch.cuda.Stream()):
                ms = run(v)
        else:
            ms = run(v)
        print(f"{opts} variant {v}: {ms:.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
