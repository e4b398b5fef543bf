"""Synthetic inputs of the benchmark shapes.

* Audio: 30 s × 16 kHz float32 clips. Clip i = 0.05·N(0,1) + Σ_{k=1..3} 0.1·sin(2π f_k t + φ_k)
  from `numpy.random.default_rng(1000 + i)`, f_k ~ U[100, 4000] Hz, φ_k ~ U[0, 2π), clipped to [−1, 1].
* Bias lists: phrases sampled with `random.Random(7)` from the 9,884 unique lowercased
  `bias_words` of the reference's `data/medical-united-syn-med-75-jsonl/{dev,test}.jsonl`
  (extracted once into `data/bias_phrases.json`; the reference itself never travels).
  The Whisper BPE is unavailable offline, so token ids are synthetic: phrase token length =
  clamp(round(len(chars)/3.5), 1, 16), ids from a seeded hash of the phrase in [0, eot).
"""
from __future__ import annotations

import hashlib
import json
import os
import random
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


def phrase_token_ids(phrase: str, eot: int) -> List[int]:
    n = int(min(max(round(len(phrase) / 3.5), 1), 16))
    h = hashlib.sha256(("phrase:" + phrase).encode()).digest()
    rng = np.random.Generator(np.random.PCG64(int.from_bytes(h[:8], "little")))
    return [int(v) for v in rng.integers(0, eot, size=n)]


def synth_bias_list(n: int, eot: int, seed: int = 7) -> List[List[int]]:
    """Token-id sequences of `n` sampled phrases (the bias list fed to the boost operator)."""
    return [phrase_token_ids(p, eot) for p in sample_bias_phrases(n, seed)]
