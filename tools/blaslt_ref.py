"""Reference point for the encoder GEMM kernels: torch's bf16 linear (hipBLASLt on ROCm) at the C2
encoder shapes (M = 32 clips x 1500 frames), random operands, graph-replayed like tools/microbench.py.
Not part of the product path; prints TFLOP/s per shape next to wcb_op_gemm's."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import gemm_case, per_launch_us  # noqa: E402

if __name__ == "__main__":
    torch.manual_seed(0)
    for (M, N, K) in [(48000, 2304, 768), (48000, 768, 768), (48000, 3072, 768), (48000, 768, 3072)]:
        A = torch.randn(M, K, device="cuda").bfloat16()
        W = torch.randn(N, K, device="cuda").bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        out = torch.empty(M, N, device="cuda").bfloat16()

        def fn():
            torch.nn.functional.linear(A, W, b, out=out) if False else out.copy_(torch.nn.functional.linear(A, W, b))
        us = per_launch_us(fn, reps=10)
        print(f"torch linear M={M} N={N} K={K}: {us:9.2f} us  {2.0 * M * N * K / us / 1e6:8.1f} TFLOP/s "
              f"(includes a {M * N * 2 / 1e6:.0f} MB copy)", flush=True)

        def fn2():
            torch.matmul(A, W.t())
        us2 = per_launch_us(fn2, reps=10)
        print(f"torch matmul M={M} N={N} K={K}: {us2:9.2f} us  {2.0 * M * N * K / us2 / 1e6:8.1f} TFLOP/s", flush=True)
        gemm_case(M, N, K)
