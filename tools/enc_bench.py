"""Encoder-side kernel timings at the C2 shapes (whisper-small, 32 clips) through the C ABI, replayed
from captured graphs (tools/microbench.per_launch_us): the encoder flash attention (enc_flash 4 = the
runtime default), the four layer GEMMs, the LayerNorm, and the decode step's encoder-space
cross-attention op (xattn + merge/W_v)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import attn_case, gemm_case, ln_case, per_launch_us, lib, stream  # noqa: E402


def xenc_case(rows=32, nsplit=8, variant=1):
    d, H, S = 768, 12, 1500
    q = torch.randn(rows, d, device="cuda").bfloat16() * 0.1
    enc = torch.randn(rows, S, d, device="cuda").bfloat16()
    wkt = (torch.randn(H, d, 64, device="cuda") / 28).bfloat16()
    wv = (torch.randn(d, d, device="cuda") / 28).bfloat16()
    bv = torch.zeros(d, device="cuda")
    o = torch.empty(rows, d, device="cuda").bfloat16()

    def fn():
        assert lib.wcb_op_cross_attention_enc(0, q.data_ptr(), enc.data_ptr(), wkt.data_ptr(), wv.data_ptr(),
                                              bv.data_ptr(), o.data_ptr(), rows, H, S, nsplit, variant, stream()) == 0
    us = per_launch_us(fn, reps=24)
    print(f"xenc op (kq + xattn + merge_v) rows={rows} nsplit={nsplit} variant={variant}: {us:8.2f} us "
          f"({rows * S * d * 2 / us / 1e3:7.1f} GB/s of encoder output)", flush=True)


if __name__ == "__main__":
    torch.manual_seed(0)
    only = sys.argv[1] if len(sys.argv) > 1 else ""
    if only in ("", "attn"):
        attn_case(32, 12, 1500, 1500, 100)
        attn_case(32, 12, 1500, 1500, 1)
    shapes = [(48000, 2304, 768, 0, False), (48000, 768, 768, 0, True),
              (48000, 3072, 768, 1, False), (48000, 768, 3072, 0, True)]
    if only == "gemm-medium":   # C3: whisper-medium, 64 clips
        shapes = [(96000, 3072, 1024, 0, False), (96000, 1024, 1024, 0, True),
                  (96000, 4096, 1024, 1, False), (96000, 1024, 4096, 0, True)]
        only = "gemm"
    for (M, N, K, act, resid) in shapes:
        if only in ("", "gemm"):
            for kernel in (0, 2, 5):   # LDS ring, ping-pong 256- / 192-wide tiles
                if kernel != 5 or N % 192 == 0:
                    gemm_case(M, N, K, kernel=kernel, act=act, resid=resid)
    if only == "":
        ln_case(48000, 768)
        xenc_case()
