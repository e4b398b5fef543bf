"""Where the C2 step goes when batches overlap: the bench's pipelined step (log-mel + encoder + 64-token
boosted greedy decode, batches in flight) with the full encoder, with the encoder cut to its conv stem
(wcb_debug_copy's layer limit: the decode chains alone), and the front end + encoder alone.
  python tools/overlap_probe.py [--steps 10] [--opt NAME=VALUE ...]"""
import argparse
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisper_context_biasing_amd.config import get_dims  # noqa: E402
from whisper_context_biasing_amd.model import WhisperCB  # noqa: E402
from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list, synth_word_start  # noqa: E402
from whisper_context_biasing_amd.weights import make_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="small")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("--views", action="store_true", help="weights as device views of the packed bf16 blob (bench.py)")
    ap.add_argument("--warm-forward", action="store_true", help="one teacher-forced forward() before timing")
    ap.add_argument("--warm-plain", action="store_true", help="one unboosted generate() before timing")
    ap.add_argument("--torch-first", action="store_true", help="a torch device allocation before the model")
    ap.add_argument("--only-full", action="store_true")
    ap.add_argument("--side-stream", action="store_true", help="issue from a non-default torch stream")
    a = ap.parse_args()
    if a.side_stream:
        torch.cuda.set_stream(torch.cuda.Stream())
    if a.torch_first:
        torch.zeros(1, device="cuda")
    dims = get_dims(a.model)
    opts = {k: int(v) for k, v in (o.split("=", 1) for o in a.opt)}
    if a.views:
        from whisper_context_biasing_amd.shard import broadcast_weights
        sd = broadcast_weights(dims, torch.device("cuda", 0), seed=0, views=True)
    else:
        sd = make_weights(dims, seed=0)
    m = WhisperCB.from_state_dict(dims, sd, dtype="bf16", options=opts or None)
    del sd
    m.set_word_start(synth_word_start(dims.eos_token_id, dims.vocab))
    phrases = synth_bias_list(1000, eot=dims.eos_token_id)
    pcm = torch.from_numpy(synth_batch(a.batch)).cuda()

    def layers(n):
        m._lib.wcb_debug_copy(m._h, b"x", None, C.c_int64(0), n)

    def pipelined(n):
        keep = []

        def step():
            mel = m.log_mel(pcm)
            keep.append(mel)   # inputs stay alive until the final synchronize (the library reads them asynchronously)
            keep.append(m.generate(mel, max_length=a.tokens, min_new_tokens=a.tokens, bias_list=phrases,
                                   bias_boost=2.0, block=False))
        for _ in range(3):
            step()
        m.synchronize(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        m.synchronize(); torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    def encoder_only(n):
        for _ in range(2):
            m.encode(m.log_mel(pcm))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            m.encode(m.log_mel(pcm))
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    if a.warm_plain or a.warm_forward:
        mel0 = m.log_mel(pcm)
        plain = m.generate(mel0, max_length=a.tokens, min_new_tokens=a.tokens)
        if a.warm_forward:
            m.forward(mel0, decoder_input_ids=plain)
        m.synchronize()
    layers(-1)
    full = pipelined(a.steps)
    if a.only_full:
        print(f"{a.model} B={a.batch} {opts or ''} views={a.views} torch_first={a.torch_first} warm_forward={a.warm_forward} warm_plain={a.warm_plain}: "
              f"pipelined step {full:.2f} ms", flush=True)
        return
    enc = encoder_only(a.steps)
    layers(0)
    dec = pipelined(a.steps)
    stem = encoder_only(a.steps)
    layers(-1)
    full2 = pipelined(a.steps)
    print(f"{a.model} B={a.batch} {opts or ''}: pipelined step {full:.2f} / {full2:.2f} ms (full encoder), "
          f"{dec:.2f} ms (encoder = conv stem only); front end + encoder alone {enc:.2f} ms, stem alone {stem:.2f} ms; "
          f"overlap = dec + enc - full = {dec + enc - stem - full:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
