"""Beam-row projection microbenchmark (decode rows > 64): the LDS-ring tiles (op kernel 6, the current
beam path) against the wide single-burst tiles (gemm_wide_kernel, op kernel 10·FM + FN) on C3's
(whisper-medium, 320 rows) and C5's (large-v3, 80 rows) K = d_model projections, weights rotated over
enough copies to miss the Infinity Cache (as in a decode step), graph-replayed; each config is checked
against a torch fp32 product first.
  python tools/beam_gemm_bench.py [--configs 6,12,22,42] [--shapes c3,c5]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisper_context_biasing_amd import _lib  # noqa: E402

lib = _lib.load()

SHAPES = {
    "c3": [("qkv", 320, 3072, 1024, 0, False), ("out", 320, 1024, 1024, 0, True), ("fc1", 320, 4096, 1024, 1, False),
           ("fc2", 320, 1024, 4096, 0, True)],
    "c5": [("qkv", 80, 3840, 1280, 0, False), ("out", 80, 1280, 1280, 0, True), ("fc1", 80, 5120, 1280, 1, False),
           ("fc2", 80, 1280, 5120, 0, True)],
}


def run(kernel, A, W, bias, act, out, resid):
    M, K = A.shape
    N = W.shape[0]
    rc = lib.wcb_op_gemm_kernel(0, A.data_ptr(), W.data_ptr(), M, N, K, bias.data_ptr(), act,
                                resid.data_ptr() if resid is not None else None, out.data_ptr(),
                                int(resid is not None), kernel, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, (kernel, rc)


def frag_major(W):
    N, K = W.shape
    return W.view(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().view(N, K)


def check(kernel, M, N, K, act, resid):
    g = torch.Generator(device="cuda").manual_seed(1)
    A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    W0 = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / K ** 0.5).bfloat16()
    W = frag_major(W0) if kernel >= 100 else W0
    bias = torch.randn(N, device="cuda", generator=g)
    ref = A.float() @ W0.float().t() + bias
    if act:
        ref = torch.nn.functional.gelu(ref)
    if resid:
        x = torch.randn(M, N, device="cuda", generator=g)
        ref = ref + x
        out = x.clone()
        run(kernel, A, W, bias, act, out, out)
    else:
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        run(kernel, A, W, bias, act, out, None)
    torch.cuda.synchronize()
    err = (out.float() - ref).abs().max().item()
    tol = 2e-2 * ref.abs().max().item() if not resid else 1e-3 * ref.abs().max().item()
    return err, tol


def timed(kernel, M, N, K, act, resid, copies):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    Ws = [((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).bfloat16() for _ in range(copies)]
    bias = torch.randn(N, device="cuda")
    out = torch.randn(M, N, device="cuda") if resid else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for W in Ws:
            run(kernel, A, W, bias, act, out, out if resid else None)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for W in Ws:
                run(kernel, A, W, bias, act, out, out if resid else None)
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 5
    e0.record()
    for _ in range(iters):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (iters * copies)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="7,6,107,106,112,122")
    ap.add_argument("--shapes", default="c3,c5")
    ap.add_argument("--only", default="", help="comma-separated projection names (default: all)")
    args = ap.parse_args()
    cfgs = [int(c) for c in args.configs.split(",")]
    for sh in args.shapes.split(","):
        for name, M, N, K, act, resid in SHAPES[sh]:
            if args.only and name not in args.only.split(","):
                continue
            copies = max(8, int(1.2e9 / (N * K * 2)))   # > 1 GB of weights per replay
            line = f"{sh} {name:4s} M={M:4d} N={N:5d} K={K:5d}:"
            for c in cfgs:
                if c % 100 > 10 and N % (16 * (c % 10)):
                    line += f"  {c}: --"
                    continue
                err, tol = check(c, M, N, K, act, resid)
                ok = "" if err <= tol else f"(ERR {err:.3g} > {tol:.3g})"
                us = timed(c, M, N, K, act, resid, copies)
                line += f"  {c}: {us:6.2f}{ok}"
            print(line, flush=True)


if __name__ == "__main__":
    main()
