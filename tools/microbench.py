"""Kernel microbenchmarks through the C ABI, replayed from a captured graph (no host overhead).
Prints per-launch device time (graph of `reps` back-to-back launches / reps)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisper_context_biasing_amd import _lib  # noqa: E402

lib = _lib.load()


def per_launch_us(fn, reps=50, iters=5):
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


def stream():
    return torch.cuda.current_stream().cuda_stream


def gemm_case(M, N, K, dt=torch.bfloat16, kernel=1, act=0, resid=False):
    """kernel 1: the runtime's encoder-GEMM choice (ping-pong kernel where it is the faster one), 2 / 5: the
    ping-pong kernel's 256- / 192-wide tiles wherever they cover the shape, 0: the LDS-ring / tile kernels; act 1 = bias + GELU, resid = bias + residual into f32 (the encoder epilogues)"""
    A = torch.randn(M, K, device="cuda").to(dt)
    W = torch.randn(N, K, device="cuda").to(dt)
    bias = torch.randn(N, device="cuda")
    out = torch.zeros(M, N, device="cuda", dtype=torch.float32 if resid else dt)
    code = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2}[dt]

    def fn():
        assert lib.wcb_op_gemm_kernel(code, A.data_ptr(), W.data_ptr(), M, N, K, bias.data_ptr(), act,
                                      out.data_ptr() if resid else None, out.data_ptr(), int(resid), kernel,
                                      stream()) == 0
    us = per_launch_us(fn, reps=20 if M > 64 else 50)
    flops = 2.0 * M * N * K
    byts = (M * K + N * K + M * N) * A.element_size()
    print(f"gemm M={M:6d} N={N:6d} K={K:5d} kernel={kernel} act={act} resid={int(resid)}: {us:9.2f} us  "
          f"{flops / us / 1e6:8.1f} TFLOP/s  {byts / us / 1e3:8.1f} GB/s", flush=True)
    return us


def gemm_ln_case(M, N, K):
    X = torch.randn(M, K, device="cuda")
    w = torch.randn(K, device="cuda")
    b = torch.randn(K, device="cuda")
    st = torch.stack([X.view(M, K // 16, 16).sum(-1), (X * X).view(M, K // 16, 16).sum(-1)], -1).contiguous()
    W = torch.randn(N, K, device="cuda").bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

    def fn():
        lib.wcb_op_gemm_ln(0, X.data_ptr(), w.data_ptr(), b.data_ptr(), st.data_ptr(), W.data_ptr(), M, N, K, None, 0,
                           out.data_ptr(), 0, stream())
    us = per_launch_us(fn)
    print(f"gemm_ln M={M:6d} N={N:6d} K={K:5d}: {us:9.2f} us  {N * K * 2 / us / 1e3:8.1f} GB/s (weights)")


def ln_case(M, d):
    x = torch.randn(M, d, device="cuda")
    w = torch.ones(d, device="cuda")
    b = torch.zeros(d, device="cuda")
    y = torch.empty(M, d, device="cuda", dtype=torch.bfloat16)

    def fn():
        lib.wcb_op_layernorm(0, x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), M, d, stream())
    us = per_launch_us(fn)
    print(f"layernorm M={M:6d} d={d}: {us:8.2f} us  {M * d * 6 / us / 1e3:8.1f} GB/s")


def attn_case(B, H, Sq, Sk, flash):
    q = torch.randn(B, Sq, H * 64, device="cuda").bfloat16()
    k = torch.randn(B, Sk, H * 64, device="cuda").bfloat16()
    v = torch.randn(B, Sk, H * 64, device="cuda").bfloat16()
    o = torch.empty_like(q)

    def fn():
        lib.wcb_op_attention(0, q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, Sq, Sk, flash, stream())
    us = per_launch_us(fn, reps=10 if flash == 1 or flash >= 100 else 50)
    byts = 2 * B * Sk * H * 64 * 2
    fl = 4.0 * B * H * Sq * Sk * 64
    print(f"attn B={B} H={H} Sq={Sq} Sk={Sk} flash={flash}: {us:9.2f} us  {byts / us / 1e3:8.1f} GB/s (KV)  "
          f"{fl / us / 1e6:8.1f} TFLOP/s")


if __name__ == "__main__":
    torch.manual_seed(0)
    ln_case(1, 768)
    ln_case(32, 768)
    ln_case(48000, 768)
    for (M, N, K) in [(32, 768, 768), (32, 2304, 768), (32, 3072, 768), (32, 768, 3072), (32, 51865 // 8 * 8, 768),
                      (48000, 2304, 768), (48000, 768, 768), (48000, 3072, 768), (48000, 768, 3072),
                      (48000, 18432, 768), (8192, 8192, 8192)]:
        gemm_case(M, N, K)
    for N in (768, 2304, 3072):
        gemm_ln_case(32, N, 768)
    attn_case(32, 12, 1, 1500, 0)
    attn_case(32, 12, 1, 1500, 4)
    attn_case(16, 12, 1, 1500, 0)
    attn_case(16, 12, 1, 1500, 4)
    attn_case(32, 12, 1, 64, 0)
    for code in (1, 100):   # encoder tilings (option enc_flash 2 / 4)
        attn_case(32, 12, 1500, 1500, code)
        attn_case(64, 16, 1500, 1500, code)
