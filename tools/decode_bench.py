"""Standalone decode-step timing: per-token GPU time of the greedy / beam decode loop alone (no
encoder overlap, one call in flight), from the difference of two fixed-length generate() calls.

  python tools/decode_bench.py --model small --batch 32 [--beams 5] [--dtype bf16] [--phrases 1000]
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--concurrent", type=int, default=0,
                    help="also time this many overlapping async calls of --long tokens (decode contexts in flight)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE", help="wcb_set_option")
    ap.add_argument("--side-stream", action="store_true",
                    help="issue every call from a non-default torch stream (CU-masked decode streams are "
                         "blocking streams: work on the legacy null stream would serialise them)")
    a = ap.parse_args()
    if a.side_stream:
        torch.cuda.set_stream(torch.cuda.Stream())
    dims = get_dims(a.model)
    opts = {k: int(v) for k, v in (o.split("=", 1) for o in a.opt)}
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0), dtype=a.dtype, options=opts or None)
    pcm = torch.from_numpy(synth_batch(a.batch)).cuda()
    mel = m.log_mel(pcm)
    phrases = synth_bias_list(a.phrases, eot=dims.eos_token_id) if a.phrases else None

    def run(n):
        ids = m.generate(mel, max_length=n, min_new_tokens=n, num_beams=a.beams, bias_list=phrases,
                         bias_boost=2.0 if phrases else 0.0)
        m.synchronize()
        torch.cuda.synchronize()
        return ids

    # same-length calls back to back: the decode graph of each context is captured by its first call
    # of a length and replayed afterwards (alternating lengths would re-capture every call)
    def timed(n):
        for _ in range(2):          # one warm call per decode context
            run(n)
        out = []
        for _ in range(a.reps):
            t0 = time.perf_counter(); run(n); out.append(time.perf_counter() - t0)
        return out
    ts = timed(a.short)
    tl = timed(a.long)
    per_tok = (min(tl) - min(ts)) / (a.long - a.short) * 1e3
    print(f"{a.model} B={a.batch} beams={a.beams} {a.dtype} {opts or ''}: call {a.short} tok {min(ts)*1e3:.2f} ms, "
          f"{a.long} tok {min(tl)*1e3:.2f} ms -> {per_tok:.3f} ms/token (decode alone), "
          f"encoder+setup ~{(min(ts) * 1e3 - a.short * per_tok):.2f} ms", flush=True)


    if a.concurrent:
        def many(c):
            keep = []
            t0 = time.perf_counter()
            for _ in range(c):
                keep.append(m.generate(mel, max_length=a.long, min_new_tokens=a.long, num_beams=a.beams,
                                       bias_list=phrases, bias_boost=2.0 if phrases else 0.0, block=False))
            m.synchronize()
            torch.cuda.synchronize()
            return time.perf_counter() - t0
        many(a.concurrent)
        t1 = min(many(1) for _ in range(2))
        tc = min(many(a.concurrent) for _ in range(2))
        print(f"async calls of {a.long} tokens: 1 call {t1*1e3:.1f} ms, {a.concurrent} calls {tc*1e3:.1f} ms "
              f"({tc / t1:.2f}x the time for {a.concurrent}x the work)", flush=True)


if __name__ == "__main__":
    main()
