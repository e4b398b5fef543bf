"""Synthetic inputs of the benchmark shapes.

* Audio: 30 s × 16 kHz float32 clips. Clip i = 0.05·N(0,1) + Σ_{k=1..3} 0.1·sin(2π f_k t + φ_k)
  from `numpy.random.default_rng(1000 + i)`, f_k ~ U[100, 4000] Hz, φ_k ~ U[0, 2π), clipped to [−1, 1].
* Bias lists: phrases sampled with `random.Random(7)` from the 9,884 unique lowercased
  `bias_words` of the reference's `data/medical-united-syn-med-75-jsonl/{dev,test}.jsonl`
  (extracted once into `data/bias_phrases.json`; the reference itself never travels).
  The Whisper BPE is unavailable offline, so token ids are synthetic: each word of a phrase gets
  max(1, round(len(word)/3.5)) tokens (at most 16 per phrase) drawn from a seeded hash of the
  phrase; a word's first token is a word-start token, the rest are continuation tokens.
* Word starts: `synth_word_start(eot)` marks a seeded half of [0, eot) as word-start tokens (the
  role of the leading-space tokens of a BPE vocabulary; oracle/bias_ref.py's gate).
"""
from __future__ import annotations

import hashlib
import json
import os
import random
from functools import lru_cache
from typing import List

import numpy as np

from .config import N_SAMPLES, SAMPLE_RATE

_DATA = os.path.join(os.path.dirname(__file__), "data", "bias_phrases.json")


def synth_clip(i: int, n_samples: int = N_SAMPLES) -> np.ndarray:
    rng = np.random.default_rng(1000 + i)
    t = np.arange(n_samples, dtype=np.float64) / SAMPLE_RATE
    x = 0.05 * rng.standard_normal(n_samples)
    f = rng.uniform(100.0, 4000.0, size=3)
    ph = rng.uniform(0.0, 2 * np.pi, size=3)
    for k in range(3):
        x = x + 0.1 * np.sin(2 * np.pi * f[k] * t + ph[k])
    return np.clip(x, -1.0, 1.0).astype(np.float32)


def synth_batch(n: int, start: int = 0, n_samples: int = N_SAMPLES) -> np.ndarray:
    return np.stack([synth_clip(start + i, n_samples) for i in range(n)])


def bias_phrase_pool() -> List[str]:
    with open(_DATA) as f:
        return json.load(f)["phrases"]


def sample_bias_phrases(n: int, seed: int = 7) -> List[str]:
    pool = bias_phrase_pool()
    return random.Random(seed).sample(pool, n)


@lru_cache(maxsize=8)
def _word_start_ids(eot: int):
    ws = np.random.Generator(np.random.PCG64(20240611)).random(eot) < 0.5
    return np.flatnonzero(ws), np.flatnonzero(~ws), ws


def synth_word_start(eot: int, vocab: int = 0) -> np.ndarray:
    """[max(vocab, eot)] bool: the synthetic word-start tokens (a seeded half of [0, eot); the special
    tokens from eot on are not word starts)."""
    ws = _word_start_ids(eot)[2]
    out = np.zeros(max(vocab, eot), dtype=bool)
    out[:eot] = ws
    return out


def phrase_token_ids(phrase: str, eot: int) -> List[int]:
    h = hashlib.sha256(("phrase:" + phrase).encode()).digest()
    rng = np.random.Generator(np.random.PCG64(int.from_bytes(h[:8], "little")))
    starts, conts, _ = _word_start_ids(eot)
    out: List[int] = []
    for word in phrase.split() or [phrase]:
        n = max(1, int(round(len(word) / 3.5)))
        out.append(int(starts[rng.integers(0, len(starts))]))
        out.extend(int(conts[i]) for i in rng.integers(0, len(conts), size=n - 1))
    return out[:16]


def synth_bias_list(n: int, eot: int, seed: int = 7) -> List[List[int]]:
    """Token-id sequences of `n` sampled phrases (the bias list fed to the boost operator)."""
    return [phrase_token_ids(p, eot) for p in sample_bias_phrases(n, seed)]


def runner_up_phrases(model, mel, n_tokens: int, lam: float, word_start=None, band=(0.25, 0.75), pool=None):
    """Bias phrases the boost can actually place (the bench's biased-WER workload): for every clip, the
    EARLIEST step (first step excluded) of the lam = 0 greedy decode whose top-1/top-2 logit gap lies
    in the band [band[0]·lam, band[1]·lam) — below lam, so one boost unit lifts the runner-up r over
    the top-1; above the 16-bit noise between the prefill and decode paths, so r is not the decode
    path's own choice at lam = 0 — whose runner-up may start a match (`word_start`), where the
    teacher-forced top-1 is the decode's own token (the two paths agree on the step), and — given the
    rest of the bias list `pool` — before the step where the decode boosted with `pool` alone first
    leaves the lam = 0 decode (a target after that point would be scored on a different prefix). The
    phrase is [r, n] with n the greedy token after r (the decode teacher-forced through r).
    Returns (plain_ids [B, n_tokens] int64, phrases, targets, gaps) with targets[i] = (clip, step) of
    phrase i and gaps the [B, n_tokens] top-1/top-2 gaps (numpy). Untimed setup on the GPU through the
    model's own generate / forward."""
    import torch

    dims = model.dims
    plain = model.generate(mel, max_length=n_tokens, min_new_tokens=n_tokens)
    B = plain.shape[0]
    sot = torch.full((B, 1), dims.decoder_start_token_id, dtype=plain.dtype, device=plain.device)
    logits = model.forward(mel, decoder_input_ids=torch.cat([sot, plain[:, :-1]], 1)).logits
    top2, idx2 = logits.topk(2, dim=-1)                                   # [B, T, 2]
    gap = (top2[..., 0] - top2[..., 1]).float()
    ru = idx2[..., 1]
    ok = (gap >= band[0] * lam) & (gap < band[1] * lam) & (ru != dims.eos_token_id) & (idx2[..., 0] == plain)
    ok[:, 0] = False
    if word_start is not None:
        ok &= torch.as_tensor(np.asarray(word_start, dtype=bool), device=ru.device)[ru]
    T = gap.shape[1]
    steps = torch.arange(T, device=gap.device)[None, :].expand(B, T)
    if pool:
        boosted = model.generate(mel, max_length=n_tokens, min_new_tokens=n_tokens, bias_list=pool, bias_boost=lam)
        diff = boosted[:, :T] != plain[:, :T]
        derail = torch.where(diff, steps, torch.full_like(steps, T)).min(dim=1).values
        ok &= steps < derail[:, None]
    t = torch.where(ok, steps, torch.full_like(steps, T)).min(dim=1).values.clamp(max=T - 1)   # earliest
    keep = ok.gather(1, t[:, None])[:, 0]
    r = ru.gather(1, t[:, None])[:, 0]
    forced = torch.cat([sot, plain], 1).clone()                          # [SOT, ids[:t], r, ...]
    forced[torch.arange(B, device=forced.device), t + 1] = r
    nxt = model.forward(mel, decoder_input_ids=forced).logits            # causal: later tokens are ignored
    n1 = nxt[torch.arange(B, device=nxt.device), t + 1].argmax(-1)
    phrases, targets = [], []
    for b in range(B):
        if bool(keep[b]):
            phrases.append([int(r[b]), int(n1[b])])
            targets.append((b, int(t[b])))
    return plain.cpu().numpy().astype(np.int64), phrases, targets, gap.cpu().numpy()
