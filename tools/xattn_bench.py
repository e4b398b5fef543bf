"""Decoder cross-attention microbenchmark in the runtime's layout (head-major K/V), cycling through
L distinct K/V buffers like the real decode step (so the 256 MB Infinity Cache cannot hold them).
Prints µs per launch and the K/V stream rate for each (rows, nsplit, kernel variant)."""
import itertools
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisper_context_biasing_amd import _lib  # noqa: E402

lib = _lib.load()
H, S, L = 12, 1500, 12


def run(rows, nsplit, variant, reps=3):
    q = torch.randn(rows, H * 64, device="cuda").bfloat16()
    o = torch.empty_like(q)
    kv = [torch.randn(2, rows, H, S, 64, device="cuda").bfloat16() for _ in range(L)]
    s = torch.cuda.Stream()

    def step():
        for l in range(L):
            rc = lib.wcb_op_attention_decode(0, q.data_ptr(), kv[l][0].data_ptr(), kv[l][1].data_ptr(), o.data_ptr(),
                                             rows, H, S, nsplit, variant, s.cuda_stream)
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
    byts = 2 * rows * H * S * 64 * 2
    return us, byts / us / 1e3


if __name__ == "__main__":
    rows_list = [int(x) for x in os.environ.get("ROWS", "16,32").split(",")]
    splits = [int(x) for x in os.environ.get("SPLITS", "1,2,4,6,8").split(",")]
    variants = [int(x) for x in os.environ.get("VARIANTS_K", "0,1,2,3,4,5").split(",")]
    for rows, ns, v in itertools.product(rows_list, splits, variants):
        us, gbs = run(rows, ns, v)
        print(f"rows={rows:3d} nsplit={ns} variant={v}: {us:8.2f} us  {gbs:8.1f} GB/s", flush=True)
