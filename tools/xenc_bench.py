"""Encoder-space cross-attention microbenchmark (wcb_op_cross_attention_enc = q'-GEMM + attn_xenc_kernel +
xenc_combine_kernel), whisper-small shapes, replayed from a captured graph; one encoder output buffer
read by 12 'layers' like the decode step. Run under rocprofv3 --kernel-trace --stats for per-kernel
times. Prints µs per op call and the encoder-output stream rate."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisper_context_biasing_amd import _lib  # noqa: E402

lib = _lib.load()
d, H, S, L = 768, 12, 1500, 12


def run(rows, nsplit, reps=5):
    q = torch.randn(rows, d, device="cuda").bfloat16() * 0.1
    enc = torch.randn(rows, S, d, device="cuda").bfloat16()
    wkt = (torch.randn(H, d, 64, device="cuda") / 28).bfloat16()
    wv = (torch.randn(d, d, device="cuda") / 28).bfloat16()
    bv = torch.zeros(d, device="cuda")
    o = torch.empty(rows, d, device="cuda").bfloat16()
    s = torch.cuda.Stream()

    def step():
        for _ in range(L):
            rc = lib.wcb_op_cross_attention_enc(0, q.data_ptr(), enc.data_ptr(), wkt.data_ptr(), wv.data_ptr(),
                                                bv.data_ptr(), o.data_ptr(), rows, H, S, nsplit, 1, s.cuda_stream)
            assert rc == 0
    with torch.cuda.stream(s):
        step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(4):
                step()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * 4 * L)
    return us, rows * S * d * 2 / us / 1e3


if __name__ == "__main__":
    for rows in [int(x) for x in os.environ.get("ROWS", "32,16").split(",")]:
        for ns in [int(x) for x in os.environ.get("SPLITS", "4,8,12,16").split(",")]:
            us, gbs = run(rows, ns)
            print(f"rows={rows:3d} nsplit={ns:2d}: {us:8.2f} us/op  {gbs:8.1f} GB/s (enc stream)", flush=True)
