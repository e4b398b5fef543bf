"""Bias-weighted cross entropy of the reference forward (`models/whisper_medical.py:113-156`).

SURVEY.md §8(f) rank 3. Runs on the device through `wcb_op_weighted_ce` (csrc/k_loss.hip): span
coverage, one streaming log-sum-exp pass over each logits row, label gather, weighting and a
fixed-order mean, fused — the [B·T, V] log_softmax the reference materialises is never written.
This module only packs `bias_spans` into int32 device arrays. Semantics kept exactly, including
the quirk that a padded span tensor is compared with its padding: the list form
keeps each span's own length, the tensor form gives every span the padded length.
"""
from __future__ import annotations

import torch

from . import _lib


def _pack_spans(bias_spans, B: int):
    """→ (spans int32 [B][N][Lmax], lengths int32 [B][N]) on the CPU, reference span semantics
    (`models/whisper_medical.py:120-127`: an empty list / zero-element tensor is skipped)."""
    if isinstance(bias_spans, torch.Tensor):
        t = bias_spans.to(torch.int64)
        if t.dim() != 3 or t.shape[0] != B:
            raise ValueError(f"bias_spans tensor must be [B, N, L], got {tuple(t.shape)}")
        N, L = t.shape[1], t.shape[2]
        lens = torch.full((B, N), L, dtype=torch.int32)
        return t.to(torch.int32).contiguous(), lens
    if len(bias_spans) != B:
        raise ValueError(f"bias_spans has {len(bias_spans)} utterances, labels have {B}")
    rows = []
    for spans in bias_spans:
        rows.append([sp.reshape(-1).tolist() if isinstance(sp, torch.Tensor) else list(sp) for sp in spans])
    N = max(1, max(len(r) for r in rows))
    L = max([1] + [len(sp) for r in rows for sp in r])
    packed = torch.zeros((B, N, L), dtype=torch.int32)
    lens = torch.zeros((B, N), dtype=torch.int32)
    for i, r in enumerate(rows):
        for n, sp in enumerate(r):
            if sp:
                packed[i, n, :len(sp)] = torch.tensor(sp, dtype=torch.int32)
                lens[i, n] = len(sp)
    return packed, lens


def weighted_ce(logits: torch.Tensor, labels: torch.Tensor, bias_spans, bias_weight: float,
                return_per_token: bool = False):
    """logits f32 [B, T, V] on the GPU, labels [B, T] (−100 = ignore). Returns the scalar loss
    (device f32), and the per-token −logp·w·valid terms when `return_per_token`."""
    if not logits.is_cuda:
        raise _lib.WcbError("weighted_ce runs on the GPU only (no CPU fallback)")
    B, T, V = logits.shape
    if logits.dtype != torch.float32 or logits.stride(2) != 1 or logits.stride(0) != T * logits.stride(1):
        logits = logits.float().contiguous()
    dev = logits.device
    lab = labels.to(dev, torch.int32).contiguous()
    if lab.shape != (B, T):
        raise ValueError(f"labels {tuple(lab.shape)} do not match logits {tuple(logits.shape)}")
    bad = (lab != -100) & ((lab < 0) | (lab >= V))
    if bool(bad.any()):
        raise IndexError("label id out of range [0, V)")
    per = torch.empty(B * T, dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    lib = _lib.load()
    stream = torch.cuda.current_stream(dev).cuda_stream
    if bias_spans is None:
        rc = lib.wcb_op_weighted_ce(logits.data_ptr(), logits.stride(1), B, T, V, lab.data_ptr(),
                                    None, None, 0, 0, 1.0, per.data_ptr(), loss.data_ptr(), None, stream)
    else:
        sp, ln = _pack_spans(bias_spans, B)
        sp, ln = sp.to(dev), ln.to(dev)
        rc = lib.wcb_op_weighted_ce(logits.data_ptr(), logits.stride(1), B, T, V, lab.data_ptr(),
                                    sp.data_ptr(), ln.data_ptr(), sp.shape[1], sp.shape[2], float(bias_weight),
                                    per.data_ptr(), loss.data_ptr(), None, stream)
    _lib.check(rc, None, "wcb_op_weighted_ce")
    return (loss, per.view(B, T)) if return_per_token else loss
