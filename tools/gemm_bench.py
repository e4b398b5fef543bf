"""Encoder GEMM microbenchmark with the encoder's own epilogues (whisper-small, 32 clips: M = 48000),
random operands, graph-replayed; prints µs and TFLOP/s per shape and the 50-GEMM encoder total.
WCB_GEMM_TILE selects the 16-bit tile kernel (gemm_impl.h gemm_t)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisper_context_biasing_amd import _lib  # noqa: E402

lib = _lib.load()


def per_launch_us(fn, reps=10, iters=5):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * iters)


def case(name, M, N, K, act=0, resid=False):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    W = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda")
    R = torch.randn(M, N, device="cuda") if resid else None
    out = torch.empty(M, N, device="cuda", dtype=torch.float32 if resid else torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream

    def fn():
        rc = lib.wcb_op_gemm(0, A.data_ptr(), W.data_ptr(), M, N, K, bias.data_ptr(), act,
                             R.data_ptr() if resid else None, out.data_ptr(), int(resid), torch.cuda.current_stream().cuda_stream)
        assert rc == 0
    us = per_launch_us(fn)
    tf = 2.0 * M * N * K / us / 1e6
    print(f"{name:5s} M={M} N={N:5d} K={K:5d}: {us:8.1f} us  {tf:7.1f} TFLOP/s", flush=True)
    return us


if __name__ == "__main__":
    torch.manual_seed(0)
    if os.environ.get("SHAPES"):
        for sh in os.environ["SHAPES"].split(","):
            M_, N_, K_ = map(int, sh.split("x"))
            case("shape", M_, N_, K_)
        sys.exit(0)
    M = 48000
    t = {}
    t["qkv"] = case("qkv", M, 2304, 768)
    t["out"] = case("out", M, 768, 768, resid=True)
    t["fc1"] = case("fc1", M, 3072, 768, act=1)
    t["fc2"] = case("fc2", M, 768, 3072, resid=True)
    tot = 12 * sum(t.values())
    fl = 12 * 2.0 * M * 768 * (2304 + 768 + 3072 + 3072)
    print(f"encoder layers GEMM total {tot / 1e3:.2f} ms  {fl / tot / 1e6:.1f} TFLOP/s (variant {os.environ.get('WCB_GEMM_TILE', '1')})")
