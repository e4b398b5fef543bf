"""Interleaved A/B of decode-step options in ONE process (run-to-run noise of separate processes on the
GPU box is +-3 %): one model per option set, the same clips, rounds alternating over the sets; per set
the minimum over rounds of (long call - short call) / (long - short tokens).

  python tools/decode_ab.py --model small --batch 32 --sets "lean=1;lean=0" [--rounds 6]
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
    ap.add_argument("--model", default="small")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--beams", type=int, default=1)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--phrases", type=int, default=1000)
    ap.add_argument("--short", type=int, default=8)
    ap.add_argument("--long", type=int, default=72)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--sets", required=True, help='";"-separated option sets, each "name=v,name=v" (empty: defaults)')
    a = ap.parse_args()
    dims = get_dims(a.model)
    sd = make_weights(dims, seed=0)
    sets = [s.strip() for s in a.sets.split(";")]
    models = []
    for st in sets:
        opts = {k: int(v) for k, v in (o.split("=", 1) for o in st.split(",") if o)}
        models.append(WhisperCB.from_state_dict(dims, sd, dtype=a.dtype, options=opts or None))
    del sd
    pcm = torch.from_numpy(synth_batch(a.batch)).cuda()
    mel = models[0].log_mel(pcm)
    phrases = synth_bias_list(a.phrases, eot=dims.eos_token_id) if a.phrases else None

    def run(m, n):
        m.generate(mel, max_length=n, min_new_tokens=n, num_beams=a.beams, bias_list=phrases,
                   bias_boost=2.0 if phrases else 0.0)
        m.synchronize()
        torch.cuda.synchronize()

    def timed(m, n):
        t0 = time.perf_counter()
        run(m, n)
        return time.perf_counter() - t0

    # one call length only (a decode graph is keyed by the length: alternating lengths would re-capture it
    # every call); the front end + encoder part of a call is the same for every set, so differences of
    # the call time are decode differences. Per set: short-call floor measured once, after the rounds.
    for m in models:   # capture the graphs of both decode contexts
        for _ in range(2):
            run(m, a.long)
    best = [1e9 for _ in models]
    for _ in range(a.rounds):
        for i, m in enumerate(models):
            for _ in range(2):   # both decode contexts
                best[i] = min(best[i], timed(m, a.long))
    short = []
    for m in models:
        for _ in range(2):
            run(m, a.short)
        short.append(min(timed(m, a.short) for _ in range(4)))
    for st, tl, ts in zip(sets, best, short):
        per = (tl - ts) / (a.long - a.short) * 1e3
        print(f"{a.model} B={a.batch} beams={a.beams} {a.dtype} [{st or 'defaults'}]: {a.long}-token call "
              f"{tl * 1e3:.2f} ms ({per:.3f} ms/token against the {a.short}-token call {ts * 1e3:.2f} ms)", flush=True)


if __name__ == "__main__":
    main()
