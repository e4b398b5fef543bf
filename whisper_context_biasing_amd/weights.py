"""Deterministic synthetic Whisper weights (SURVEY.md §8(c) golden-vector recipe, step 1).

No checkpoint exists offline, so every test, fixture and benchmark uses weights drawn from a
build-owned generator keyed by `(seed, parameter name)`: numpy's PCG64 seeded from a SHA-256 of
that key. The GPU box regenerates bit-identical tensors without the reference. Every value is
rounded to bf16 (`round_bf16`) BEFORE anything consumes it, so the fp32 oracle, the reference
model and the bf16 HIP path all see the same weight values.

Parameter names and shapes are the HF Whisper state-dict ones consumed by the reference class
`WhisperForConditionalGenerationWeightCE` (`models/whisper_medical.py:12-22`); the LM head
`proj_out.weight` is tied to `model.decoder.embed_tokens.weight` (`:14`).

Recipes: "diverse" — Linear std 1/sqrt(fan_in), token embedding std 0.02;
"margin" — token embedding std 0.5 (large top-1/top-2 logit gaps, repetitive tokens).
"""
from __future__ import annotations

import hashlib
import math
from typing import Dict, Iterator, Tuple

import numpy as np

from .config import WhisperDims


def round_bf16(x: np.ndarray) -> np.ndarray:
    """Round float32 values to the nearest bf16 (ties to even), returned as float32."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """float32 → uint16 bf16 bit patterns (round to nearest even)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    return (((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF).astype(np.uint16)


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """Encoder positional table ([tf] modeling_whisper.py:55-64), float32."""
    inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-inc * np.arange(channels // 2, dtype=np.float32)).astype(np.float32)
    t = np.arange(length, dtype=np.float32)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


def param_shapes(dims: WhisperDims) -> Iterator[Tuple[str, Tuple[int, ...]]]:
    """HF Whisper parameter names/shapes (proj_out tied, so not listed)."""
    d, f, L = dims.d_model, dims.ffn, dims.n_layers
    yield "model.encoder.conv1.weight", (d, dims.n_mel, 3)
    yield "model.encoder.conv1.bias", (d,)
    yield "model.encoder.conv2.weight", (d, d, 3)
    yield "model.encoder.conv2.bias", (d,)
    yield "model.encoder.embed_positions.weight", (dims.n_audio_ctx, d)
    for side in ("encoder", "decoder"):
        attns = ("self_attn",) if side == "encoder" else ("self_attn", "encoder_attn")
        for i in range(L):
            p = f"model.{side}.layers.{i}."
            for a in attns:
                for proj in ("q_proj", "k_proj", "v_proj", "out_proj"):
                    yield p + f"{a}.{proj}.weight", (d, d)
                    if proj != "k_proj":
                        yield p + f"{a}.{proj}.bias", (d,)
                yield p + f"{a}_layer_norm.weight", (d,)
                yield p + f"{a}_layer_norm.bias", (d,)
            yield p + "fc1.weight", (f, d)
            yield p + "fc1.bias", (f,)
            yield p + "fc2.weight", (d, f)
            yield p + "fc2.bias", (d,)
            yield p + "final_layer_norm.weight", (d,)
            yield p + "final_layer_norm.bias", (d,)
        yield f"model.{side}.layer_norm.weight", (d,)
        yield f"model.{side}.layer_norm.bias", (d,)
    yield "model.decoder.embed_tokens.weight", (dims.vocab, d)
    yield "model.decoder.embed_positions.weight", (dims.n_text_ctx, d)


def _rng(seed: int, name: str) -> np.random.Generator:
    h = hashlib.sha256(f"wcb:{seed}:{name}".encode()).digest()
    return np.random.Generator(np.random.PCG64(int.from_bytes(h[:8], "little")))


def _std(name: str, shape, recipe: str) -> float:
    if name.endswith("embed_tokens.weight"):
        return 0.5 if recipe == "margin" else 0.02
    if name.endswith("embed_positions.weight"):
        return 0.02
    if "layer_norm" in name:
        return 0.05
    if name.endswith(".bias"):
        return 0.02
    if "conv" in name:
        return 1.0 / math.sqrt(shape[1] * shape[2])
    return 1.0 / math.sqrt(shape[1])


def make_weights(dims: WhisperDims, seed: int = 0, recipe: str = "diverse") -> Dict[str, np.ndarray]:
    """Seeded, bf16-rounded float32 state dict (HF names; no proj_out — it is tied)."""
    if recipe not in ("diverse", "margin"):
        raise ValueError(f"unknown recipe {recipe!r}")
    out: Dict[str, np.ndarray] = {}
    for name, shape in param_shapes(dims):
        if name == "model.encoder.embed_positions.weight":
            w = sinusoids(shape[0], shape[1])
        else:
            g = _rng(seed, name)
            w = g.standard_normal(shape, dtype=np.float32) * np.float32(_std(name, shape, recipe))
            if "layer_norm.weight" in name:
                w = w + np.float32(1.0)
        out[name] = round_bf16(w)
    return out
