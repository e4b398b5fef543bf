"""Bias-weighted cross entropy — numpy float64 restatement (TEST INFRASTRUCTURE ONLY).

Restates the loss block of `WhisperForConditionalGenerationWeightCE.forward`
(`models/whisper_medical.py:113-156`), the checker for `wcb_op_weighted_ce` (k_loss.hip):
* weights: 1 everywhere, `bias_weight` on every token of a contiguous window of the labels equal to
  one of the utterance's spans (`:118-133`; empty spans skipped `:122-127`; a padded tensor's spans
  are compared WITH their padding);
* per token −log_softmax(logits)[label], zeroed where label == −100 (`:136-148`);
* Σ(per_token·w) / (Σvalid + 1e-8) (`:150-151`); spans None → nn.CrossEntropyLoss mean (`:152-155`).
Pinned by `tests/golden/wce_micro_s0.npz` (the reference forward's loss on the micro model, every
span form) through `tests/test_oracle_golden.py::test_weighted_ce_matches_reference`.
"""
from __future__ import annotations

import numpy as np


def span_weights(labels: np.ndarray, spans, bias_weight: float) -> np.ndarray:
    """`models/whisper_medical.py:118-133`. spans: per utterance, a sequence of token lists."""
    B, T = labels.shape
    w = np.ones((B, T), dtype=np.float64)
    for i in range(B):
        for sp in spans[i]:
            sp = list(np.asarray(sp).reshape(-1))
            if not sp:
                continue
            n = len(sp)
            for j in range(T - n + 1):
                if list(labels[i, j:j + n]) == sp:
                    w[i, j:j + n] = bias_weight
    return w


def weighted_ce(logits: np.ndarray, labels: np.ndarray, spans=None, bias_weight: float = 1.0):
    """Returns (loss, per_token) with per_token = −logp[label]·w·valid (the kernel's output)."""
    B, T, V = logits.shape
    x = logits.astype(np.float64).reshape(B * T, V)
    m = x.max(-1, keepdims=True)
    lse = (np.log(np.exp(x - m).sum(-1, keepdims=True)) + m)[:, 0]
    flat = labels.reshape(-1)
    valid = flat != -100
    picked = x[np.arange(B * T), np.where(valid, flat, 0)]
    per = np.where(valid, lse - picked, 0.0)
    if spans is None:
        return per.sum() / valid.sum(), per
    w = span_weights(labels, spans, bias_weight).reshape(-1)
    per = per * w
    return per.sum() / (valid.sum() + 1e-8), per


def spans_from_padded(padded: np.ndarray):
    """The collator's padded tensor form: every span has the full padded length."""
    return [[list(row) for row in padded[i]] for i in range(padded.shape[0])]
