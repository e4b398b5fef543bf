"""fp32 PyTorch-CPU restatement of the reference inference path — CPU BASELINE / TEST ORACLE ONLY.

BASELINE.md §3 defines the CPU baseline timed beside the GPU as "the build's own fp32 PyTorch-CPU
restatement of the reference path: log-mel → encoder → greedy decode → bias boost", in the two
modes of the reference evaluation: (i) `use_cache=False` exactly as `scripts/evaluation.py:178,180`
configures generate() (every step re-runs the decoder over the whole prefix and re-projects the
cross-attention K/V of every layer, `[tf] modeling_whisper.py:322-335` without a cache), and
(ii) KV-cached (cross-K/V once per clip, self-attention K/V appended per step).

Written from scratch with torch ops (no `transformers`); semantics follow oracle/whisper_np.py,
which is itself pinned to the reference's own outputs (tests/test_oracle_golden.py). Used only by
bench.py's cpu_baseline leg and by tests/ — never by the product package.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .bias_ref import AhoCorasick
from .whisper_np import mel_filter_bank

N_SAMPLES, N_FFT, HOP, N_FRAMES = 480000, 400, 160, 3000


def log_mel(pcm: torch.Tensor, n_mels: int = 80) -> torch.Tensor:
    """[B, N] f32 → [B, n_mels, 3000]: `_torch_extract_fbank_features`
    ([tf] feature_extraction_whisper.py:135-168) restated: pad/trim to 30 s, stft(400, 160, periodic
    hann, center, reflect), |.|², drop the last frame, slaney mel (f32), log10(clamp 1e-10), per-clip
    max − 8 clamp, (x + 4) / 4. Caller in the reference: data_utils/data_loader.py:171-172."""
    x = torch.zeros(pcm.shape[0], N_SAMPLES, dtype=torch.float32)
    n = min(N_SAMPLES, pcm.shape[1])
    x[:, :n] = pcm[:, :n].float()
    win = torch.hann_window(N_FFT, periodic=True, dtype=torch.float32)
    spec = torch.stft(x, N_FFT, HOP, window=win, center=True, pad_mode="reflect", return_complex=True)
    power = spec[..., :-1].abs() ** 2                                     # [B, 201, 3000]
    filt = torch.from_numpy(mel_filter_bank(n_mels).astype(np.float32))   # [201, n_mels]
    mel = filt.T @ power
    lg = torch.clamp(mel, min=1e-10).log10()
    mx = lg.amax(dim=(1, 2), keepdim=True)
    lg = torch.maximum(lg, mx - 8.0)
    return (lg + 4.0) / 4.0


class TorchWhisper:
    """Weights under HF state-dict names (proj_out tied to embed_tokens, models/whisper_medical.py:14)."""

    def __init__(self, dims, sd: Dict[str, np.ndarray]):
        self.dims = dims
        self.w = {k: torch.from_numpy(np.asarray(v, dtype=np.float32)) for k, v in sd.items()}
        self.d, self.L, self.H = dims.d_model, dims.n_layers, dims.n_heads
        self.hd = self.d // self.H

    # ------------------------------------------------------------------------------ blocks
    def _ln(self, x, p):
        return F.layer_norm(x, (self.d,), self.w[p + ".weight"], self.w[p + ".bias"], eps=1e-5)

    def _lin(self, x, p, bias=True):
        return F.linear(x, self.w[p + ".weight"], self.w[p + ".bias"] if bias else None)

    def _heads(self, t):
        B, T, _ = t.shape
        return t.view(B, T, self.H, self.hd).transpose(1, 2)

    def _attn(self, q, k, v, mask=None):
        s = q @ k.transpose(-1, -2)
        if mask is not None:
            s = s + mask
        o = torch.softmax(s, dim=-1) @ v
        B, H, T, hd = o.shape
        return o.transpose(1, 2).reshape(B, T, H * hd)

    def encode(self, mel: torch.Tensor) -> torch.Tensor:
        """WhisperEncoder.forward ([tf] modeling_whisper.py:592-646)."""
        w = self.w
        x = F.gelu(F.conv1d(mel, w["model.encoder.conv1.weight"], w["model.encoder.conv1.bias"], padding=1))
        x = F.gelu(F.conv1d(x, w["model.encoder.conv2.weight"], w["model.encoder.conv2.bias"], stride=2, padding=1))
        x = x.transpose(1, 2) + w["model.encoder.embed_positions.weight"]
        for i in range(self.L):
            p = f"model.encoder.layers.{i}."
            h = self._ln(x, p + "self_attn_layer_norm")
            q = self._heads(self._lin(h, p + "self_attn.q_proj") * self.hd ** -0.5)
            k = self._heads(self._lin(h, p + "self_attn.k_proj", bias=False))
            v = self._heads(self._lin(h, p + "self_attn.v_proj"))
            x = x + self._lin(self._attn(q, k, v), p + "self_attn.out_proj")
            h = self._ln(x, p + "final_layer_norm")
            x = x + self._lin(F.gelu(self._lin(h, p + "fc1")), p + "fc2")
        return self._ln(x, "model.encoder.layer_norm")

    def cross_kv(self, enc):
        out = []
        for i in range(self.L):
            p = f"model.decoder.layers.{i}.encoder_attn."
            out.append((self._heads(self._lin(enc, p + "k_proj", bias=False)), self._heads(self._lin(enc, p + "v_proj"))))
        return out

    def decode(self, ids: torch.Tensor, pos0: int, cache: Optional[dict], xkv) -> torch.Tensor:
        """WhisperDecoder.forward over `ids` [B, T] at positions pos0.. ([tf] modeling_whisper.py:690-795);
        `cache` None = no KV cache (the whole prefix is passed in ids, pos0 = 0)."""
        w = self.w
        B, T = ids.shape
        x = w["model.decoder.embed_tokens.weight"][ids] + w["model.decoder.embed_positions.weight"][pos0:pos0 + T]
        tk = pos0 + T
        mask = torch.full((T, tk), float("-inf")).triu(pos0 + 1) if T > 1 else None
        for i in range(self.L):
            p = f"model.decoder.layers.{i}."
            h = self._ln(x, p + "self_attn_layer_norm")
            q = self._heads(self._lin(h, p + "self_attn.q_proj") * self.hd ** -0.5)
            k = self._heads(self._lin(h, p + "self_attn.k_proj", bias=False))
            v = self._heads(self._lin(h, p + "self_attn.v_proj"))
            if cache is not None:
                if i in cache:
                    k = torch.cat([cache[i][0], k], dim=2)
                    v = torch.cat([cache[i][1], v], dim=2)
                cache[i] = (k, v)
            x = x + self._lin(self._attn(q, k, v, mask), p + "self_attn.out_proj")
            h = self._ln(x, p + "encoder_attn_layer_norm")
            q = self._heads(self._lin(h, p + "encoder_attn.q_proj") * self.hd ** -0.5)
            ck, cv = xkv[i] if xkv is not None else (None, None)
            x = x + self._lin(self._attn(q, ck, cv), p + "encoder_attn.out_proj")
            h = self._ln(x, p + "final_layer_norm")
            x = x + self._lin(F.gelu(self._lin(h, p + "fc1")), p + "fc2")
        return self._ln(x, "model.decoder.layer_norm")

    def lm_head(self, h):
        return h @ self.w["model.decoder.embed_tokens.weight"].T

    # ------------------------------------------------------------------------------ generate
    @torch.no_grad()
    def generate(self, mel: torch.Tensor, max_length: int = 225, min_new_tokens: int = 0, use_cache: bool = True,
                 bias: Optional[Sequence[Sequence[int]]] = None, bias_boost: float = 0.0,
                 word_start=None) -> np.ndarray:
        """Greedy decode with the reference's eval semantics (oracle/whisper_np.py generate): start from
        [decoder_start], argmax of fp32 logits (lowest index on ties), finished rows emit pad, stop when
        every row finished or max_length new tokens. `use_cache=False` = scripts/evaluation.py:178: every
        step re-runs the decoder over the whole prefix and re-projects the cross K/V of every layer."""
        dims = self.dims
        enc = self.encode(mel)
        B = enc.shape[0]
        ac = AhoCorasick(bias or [], word_start)
        lam = float(bias_boost)
        seq = torch.full((B, 1), dims.decoder_start_token_id, dtype=torch.long)
        cache = {} if use_cache else None
        xkv = self.cross_kv(enc) if use_cache else None
        h = self.decode(seq, 0, cache, xkv if use_cache else self.cross_kv(enc))
        logits = self.lm_head(h[:, -1])
        states = [0] * B
        finished = torch.zeros(B, dtype=torch.bool)
        out = []
        while True:
            row = logits.clone()
            if lam != 0.0:   # bonus lam * n(state, v), oracle/bias_ref.py
                for b in range(B):
                    row[b] += torch.from_numpy(np.float32(lam) * ac.unit_vector(states[b], row.shape[1]).astype(np.float32))
            if len(out) < min_new_tokens:
                row[:, dims.eos_token_id] = float("-inf")
            tok = row.argmax(dim=-1)
            tok = torch.where(finished, torch.full_like(tok, dims.pad_token_id), tok)
            for b in range(B):
                states[b] = ac.delta(states[b], int(tok[b]))
            finished |= tok == dims.eos_token_id
            out.append(tok)
            if bool(finished.all()) or len(out) >= max_length:
                break
            seq = torch.cat([seq, tok[:, None]], dim=1)
            if use_cache:
                h = self.decode(tok[:, None], seq.shape[1] - 1, cache, xkv)
            else:   # the reference's use_cache=False: full prefix, cross K/V re-projected every step
                h = self.decode(seq, 0, None, self.cross_kv(enc))
            logits = self.lm_head(h[:, -1])
        return torch.stack(out, dim=1).numpy()
