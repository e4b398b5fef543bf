"""Bias-weighted cross entropy of the reference forward (`models/whisper_medical.py:113-156`).

Training-loss path (not the inference hot path): computed with torch ops on
the logits libwcb returns, so `WhisperCB.forward(labels=..., bias_spans=...)` reports the same
`.loss` as the reference. Semantics kept exactly, including the quirk that padded spans are
compared with their 50256 padding.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def weighted_ce(logits: torch.Tensor, labels: torch.Tensor, bias_spans, bias_weight: float) -> torch.Tensor:
    B, T, V = logits.shape
    labels = labels.to(logits.device)
    if bias_spans is None:
        return F.cross_entropy(logits.reshape(-1, V), labels.reshape(-1), ignore_index=-100)
    weights = torch.ones_like(labels, dtype=torch.float32)
    lab = labels.tolist()
    for i in range(B):
        for span in bias_spans[i]:
            span = span.tolist() if isinstance(span, torch.Tensor) else list(span)
            if not span:
                continue
            n = len(span)
            for j in range(T - n + 1):
                if lab[i][j:j + n] == span:
                    weights[i, j:j + n] = bias_weight
    logp = F.log_softmax(logits.float(), dim=-1).view(-1, V)
    flat = labels.view(-1)
    w = weights.view(-1)
    valid = flat != -100
    per_tok = -logp[torch.arange(logp.size(0), device=logp.device), flat.clamp(min=0)]
    per_tok = per_tok * valid.float()
    return (per_tok * w * valid.float()).sum() / (valid.sum() + 1e-8)
