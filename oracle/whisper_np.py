"""numpy float32 restatement of the Whisper inference hot path — TEST ORACLE ONLY.

Used by tests/ (parity checker), `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg.
Never imported by the product package.

Every function cites the code it restates. `[tf]` = HF transformers 5.15.0 installed in the
survey container (the reference pins 4.51.3, `requirements.txt:1`; semantics used here are
identical in both, SURVEY.md §8(c) "Version drift").
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
from scipy.special import erf

from .beam_np import whisper_trim
from .bias_ref import AhoCorasick

N_SAMPLES, N_FFT, HOP, N_FRAMES = 480000, 400, 160, 3000
F32 = np.float32


# ----------------------------------------------------------------------------------------- A1
def _hz_to_mel_slaney(f):
    """[tf] audio_utils.py:448-481 (slaney branch)."""
    f = np.asarray(f, dtype=np.float64)
    mels = 3.0 * f / 200.0
    logstep = 27.0 / np.log(6.4)
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-30) / 1000.0) * logstep, mels)


def _mel_to_hz_slaney(m):
    """[tf] audio_utils.py:484-518 (slaney branch)."""
    m = np.asarray(m, dtype=np.float64)
    freq = 200.0 * m / 3.0
    logstep = np.log(6.4) / 27.0
    return np.where(m >= 15.0, 1000.0 * np.exp(logstep * (m - 15.0)), freq)


def mel_filter_bank(n_mels: int, n_freqs: int = 201, sr: int = 16000,
                    fmin: float = 0.0, fmax: float = 8000.0) -> np.ndarray:
    """Slaney mel filters [n_freqs, n_mels] float64: [tf] audio_utils.py:638-729 with
    norm="slaney", mel_scale="slaney" as configured by [tf] feature_extraction_whisper.py:95-103."""
    mel_freqs = np.linspace(_hz_to_mel_slaney(fmin), _hz_to_mel_slaney(fmax), n_mels + 2)
    filter_freqs = _mel_to_hz_slaney(mel_freqs)
    fft_freqs = np.linspace(0, sr // 2, n_freqs)
    # _create_triangular_filter_bank, [tf] audio_utils.py:541-561
    fdiff = np.diff(filter_freqs)
    slopes = filter_freqs[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / fdiff[:-1]
    up = slopes[:, 2:] / fdiff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    enorm = 2.0 / (filter_freqs[2:n_mels + 2] - filter_freqs[:n_mels])
    return fb * enorm[None, :]


def pad_or_trim(pcm: np.ndarray, n: int = N_SAMPLES) -> np.ndarray:
    """Zero-pad / truncate every clip to 30 s ([tf] feature_extraction_whisper.py:300-307)."""
    pcm = np.asarray(pcm, dtype=F32)
    if pcm.ndim == 1:
        pcm = pcm[None]
    out = np.zeros((pcm.shape[0], n), dtype=F32)
    m = min(n, pcm.shape[1])
    out[:, :m] = pcm[:, :m]
    return out


def log_mel(pcm: np.ndarray, n_mels: int = 80) -> np.ndarray:
    """[B, 480000] f32 → [B, n_mels, 3000] f32.

    Restates `_torch_extract_fbank_features` ([tf] feature_extraction_whisper.py:135-168):
    torch.stft(n_fft=400, hop=160, hann(400, periodic), center=True, reflect) → |.|² → drop last
    frame → mel_filters.T (f32) @ power → clamp(1e-10).log10 → max(x, max−8) per clip → (x+4)/4.
    Caller: `data_utils/data_loader.py:171-172`.
    """
    x = pad_or_trim(pcm)
    B = x.shape[0]
    win = (0.5 - 0.5 * np.cos(2 * np.pi * np.arange(N_FFT) / N_FFT)).astype(F32)  # periodic hann
    xp = np.pad(x, ((0, 0), (N_FFT // 2, N_FFT // 2)), mode="reflect")
    idx = np.arange(N_FRAMES)[:, None] * HOP + np.arange(N_FFT)[None, :]
    filt = mel_filter_bank(n_mels).astype(F32)              # [201, n_mels]
    out = np.empty((B, n_mels, N_FRAMES), dtype=F32)
    for b in range(B):
        frames = xp[b][idx] * win[None, :]                    # [3000, 400] f32
        spec = np.fft.rfft(frames.astype(np.float64), axis=1)
        power = (spec.real ** 2 + spec.imag ** 2).astype(F32)  # [3000, 201]
        mel = (power @ filt).T.astype(F32)                    # [n_mels, 3000]
        lg = np.log10(np.maximum(mel, F32(1e-10))).astype(F32)
        lg = np.maximum(lg, lg.max() - F32(8.0))
        out[b] = ((lg + F32(4.0)) / F32(4.0)).astype(F32)
    return out


# ------------------------------------------------------------------------------------- layers
def gelu(x):
    """nn.functional.gelu (erf form), ACT2FN["gelu"] in [tf] activations."""
    return (F32(0.5) * x * (F32(1.0) + erf(x / F32(math.sqrt(2.0))).astype(F32))).astype(F32)


def layer_norm(x, w, b, eps=1e-5):
    """nn.LayerNorm(d), eps 1e-5 ([tf] modeling_whisper.py:379-413 self_attn_layer_norm etc.)."""
    x = x.astype(F32)
    mu = x.mean(-1, keepdims=True, dtype=np.float64).astype(F32)
    xc = x - mu
    var = (xc.astype(np.float64) ** 2).mean(-1, keepdims=True).astype(F32)
    return (xc / np.sqrt(var + F32(eps)) * w + b).astype(F32)


def linear(x, w, b=None):
    y = np.matmul(x, w.T).astype(F32)
    return y if b is None else (y + b).astype(F32)


def softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    e = np.exp((x - m).astype(F32))
    return (e / e.sum(axis=axis, keepdims=True)).astype(F32)


def conv1d(x, w, b, stride=1):
    """nn.Conv1d(k=3, padding=1) on [B, C, T] via im2col ([tf] modeling_whisper.py:566-567)."""
    B, C, T = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1)))
    To = (T + 2 - 3) // stride + 1
    cols = np.stack([xp[:, :, k: k + stride * (To - 1) + 1: stride] for k in range(3)], axis=-1)  # B,C,To,3
    cols = cols.transpose(0, 2, 1, 3).reshape(B, To, C * 3)
    y = np.matmul(cols, w.reshape(w.shape[0], C * 3).T).astype(F32) + b
    return y.transpose(0, 2, 1).astype(F32)                 # B, d, To


@dataclass
class OracleModel:
    """Weights (HF state-dict names) + dims; proj_out is tied to embed_tokens
    (`models/whisper_medical.py:14,19,111`)."""
    sd: Dict[str, np.ndarray]
    d: int
    L: int
    H: int
    eos: int
    pad: int
    start: int

    @classmethod
    def from_dims(cls, dims, sd):
        return cls({k: np.asarray(v, dtype=F32) for k, v in sd.items()}, dims.d_model,
                   dims.n_layers, dims.n_heads, dims.eos_token_id, dims.pad_token_id,
                   dims.decoder_start_token_id)

    def w(self, name):
        return self.sd[name]

    # ------------------------------------------------------------------------------ encoder
    def _attn(self, p, xq, xkv, mask=None):
        """WhisperAttention.forward ([tf] modeling_whisper.py:284-356): q = (xWq+bq)·hd^-0.5,
        k = xWk (no bias), v = xWv+bv, softmax(qkᵀ [+mask]) v, out_proj."""
        B, Tq, d = xq.shape
        hd = d // self.H
        q = (linear(xq, self.w(p + "q_proj.weight"), self.w(p + "q_proj.bias")) * F32(hd ** -0.5)).astype(F32)
        k = linear(xkv, self.w(p + "k_proj.weight"))
        v = linear(xkv, self.w(p + "v_proj.weight"), self.w(p + "v_proj.bias"))
        q = q.reshape(B, Tq, self.H, hd).transpose(0, 2, 1, 3)
        k = k.reshape(B, -1, self.H, hd).transpose(0, 2, 1, 3)
        v = v.reshape(B, -1, self.H, hd).transpose(0, 2, 1, 3)
        s = np.matmul(q, k.transpose(0, 1, 3, 2)).astype(F32)
        if mask is not None:
            s = s + mask
        o = np.matmul(softmax(s), v).astype(F32).transpose(0, 2, 1, 3).reshape(B, Tq, d)
        return linear(o, self.w(p + "out_proj.weight"), self.w(p + "out_proj.bias"))

    def encode(self, mel: np.ndarray) -> np.ndarray:
        """WhisperEncoder.forward ([tf] modeling_whisper.py:592-646): [B, n_mel, 3000] → [B, 1500, d]."""
        if mel.shape[-1] != N_FRAMES:
            raise ValueError(f"Whisper expects mel length {N_FRAMES}, got {mel.shape[-1]}")
        x = gelu(conv1d(mel.astype(F32), self.w("model.encoder.conv1.weight"), self.w("model.encoder.conv1.bias")))
        x = gelu(conv1d(x, self.w("model.encoder.conv2.weight"), self.w("model.encoder.conv2.bias"), stride=2))
        x = (x.transpose(0, 2, 1) + self.w("model.encoder.embed_positions.weight")[None]).astype(F32)
        for i in range(self.L):
            p = f"model.encoder.layers.{i}."
            h = layer_norm(x, self.w(p + "self_attn_layer_norm.weight"), self.w(p + "self_attn_layer_norm.bias"))
            x = (x + self._attn(p + "self_attn.", h, h)).astype(F32)
            h = layer_norm(x, self.w(p + "final_layer_norm.weight"), self.w(p + "final_layer_norm.bias"))
            h = gelu(linear(h, self.w(p + "fc1.weight"), self.w(p + "fc1.bias")))
            x = (x + linear(h, self.w(p + "fc2.weight"), self.w(p + "fc2.bias"))).astype(F32)
        return layer_norm(x, self.w("model.encoder.layer_norm.weight"), self.w("model.encoder.layer_norm.bias"))

    # ------------------------------------------------------------------------------ decoder
    def cross_kv(self, enc):
        """Cross-attention K/V per decoder layer, computed once per clip (A4;
        [tf] modeling_whisper.py:322-335 reuses them from the cache after step 0)."""
        B = enc.shape[0]
        hd = self.d // self.H
        out = []
        for i in range(self.L):
            p = f"model.decoder.layers.{i}.encoder_attn."
            k = linear(enc, self.w(p + "k_proj.weight")).reshape(B, -1, self.H, hd).transpose(0, 2, 1, 3)
            v = linear(enc, self.w(p + "v_proj.weight"), self.w(p + "v_proj.bias")).reshape(B, -1, self.H, hd).transpose(0, 2, 1, 3)
            out.append((k.astype(F32), v.astype(F32)))
        return out

    def decode_tokens(self, ids: np.ndarray, pos0: int, cache: dict, xkv) -> np.ndarray:
        """WhisperDecoder.forward over new tokens `ids` [B, T] at positions pos0.. with a KV
        cache (dict layer -> (K, V) [B, H, t, hd]) ([tf] modeling_whisper.py:690-795, layer
        :448-505, causal mask [tf] masking_utils.py:864). Returns final-LN hidden [B, T, d]."""
        B, T = ids.shape
        hd = self.d // self.H
        x = (self.w("model.decoder.embed_tokens.weight")[ids] +
             self.w("model.decoder.embed_positions.weight")[pos0:pos0 + T][None]).astype(F32)
        for i in range(self.L):
            p = f"model.decoder.layers.{i}."
            h = layer_norm(x, self.w(p + "self_attn_layer_norm.weight"), self.w(p + "self_attn_layer_norm.bias"))
            a = p + "self_attn."
            q = (linear(h, self.w(a + "q_proj.weight"), self.w(a + "q_proj.bias")) * F32(hd ** -0.5)).astype(F32)
            k = linear(h, self.w(a + "k_proj.weight"))
            v = linear(h, self.w(a + "v_proj.weight"), self.w(a + "v_proj.bias"))
            q = q.reshape(B, T, self.H, hd).transpose(0, 2, 1, 3)
            k = k.reshape(B, T, self.H, hd).transpose(0, 2, 1, 3)
            v = v.reshape(B, T, self.H, hd).transpose(0, 2, 1, 3)
            if i in cache:
                k = np.concatenate([cache[i][0], k], axis=2)
                v = np.concatenate([cache[i][1], v], axis=2)
            cache[i] = (k, v)
            tk = k.shape[2]
            s = np.matmul(q, k.transpose(0, 1, 3, 2)).astype(F32)
            qpos = pos0 + np.arange(T)[:, None]
            kpos = np.arange(tk)[None, :]
            s = np.where(kpos <= qpos, s, F32(-np.inf))
            o = np.matmul(softmax(s), v).astype(F32).transpose(0, 2, 1, 3).reshape(B, T, self.d)
            x = (x + linear(o, self.w(a + "out_proj.weight"), self.w(a + "out_proj.bias"))).astype(F32)
            # cross attention
            h = layer_norm(x, self.w(p + "encoder_attn_layer_norm.weight"), self.w(p + "encoder_attn_layer_norm.bias"))
            c = p + "encoder_attn."
            q = (linear(h, self.w(c + "q_proj.weight"), self.w(c + "q_proj.bias")) * F32(hd ** -0.5)).astype(F32)
            q = q.reshape(B, T, self.H, hd).transpose(0, 2, 1, 3)
            ck, cv = xkv[i]
            s = np.matmul(q, ck.transpose(0, 1, 3, 2)).astype(F32)
            o = np.matmul(softmax(s), cv).astype(F32).transpose(0, 2, 1, 3).reshape(B, T, self.d)
            x = (x + linear(o, self.w(c + "out_proj.weight"), self.w(c + "out_proj.bias"))).astype(F32)
            # MLP
            h = layer_norm(x, self.w(p + "final_layer_norm.weight"), self.w(p + "final_layer_norm.bias"))
            h = gelu(linear(h, self.w(p + "fc1.weight"), self.w(p + "fc1.bias")))
            x = (x + linear(h, self.w(p + "fc2.weight"), self.w(p + "fc2.bias"))).astype(F32)
        return layer_norm(x, self.w("model.decoder.layer_norm.weight"), self.w("model.decoder.layer_norm.bias"))

    def lm_head(self, h):
        """proj_out (tied embedding, no bias) `models/whisper_medical.py:111`."""
        return np.matmul(h, self.w("model.decoder.embed_tokens.weight").T).astype(F32)

    def forward_logits(self, mel, decoder_input_ids):
        """Teacher-forced `forward` (`models/whisper_medical.py:45-111`): logits f32 [B, T, V]."""
        enc = self.encode(mel)
        return self.lm_head(self.decode_tokens(np.asarray(decoder_input_ids), 0, {}, self.cross_kv(enc))), enc

    # ---------------------------------------------------------------------------- generation
    def generate(self, mel=None, max_length: int = 225, enc=None, min_new_tokens: int = 0,
                 bias: Optional[Sequence[Sequence[int]]] = None, bias_boost: float = 0.0,
                 prefix: Optional[Sequence[int]] = None, return_logits: bool = False,
                 use_cache: bool = True, trim: bool = True, return_margins: bool = False,
                 word_start=None):
        """Greedy decode with the reference's eval semantics:
        init = [decoder_start] ([tf] generation_whisper.py:1489,1591-1606); ≤ max_length new
        tokens (max_length+1 total incl. SOT, [tf] generation_whisper.py:1932-1940); fp32
        logits; argmax, lowest index on ties ([tf] generation/utils.py:2894,2925); finished rows
        emit pad; stop when all rows finished ([tf] :2928-2936); output excludes SOT and is right-
        padded with pad ([tf] generation_whisper.py:936-943,1141-1144); with `trim` the trailing EOS
        and pads are dropped per row as Whisper does ([tf] generation_whisper.py:1063-1086).
        `min_new_tokens` masks EOS (benchmark mode); `bias`/`bias_boost`/`word_start`
        apply the A8 boost (oracle/bias_ref.py). `use_cache=False` recomputes the whole prefix every
        step exactly like `scripts/evaluation.py:178`. `return_margins` adds the per-step gap between
        the best and the second-best selection score (after boost and mask) of every row [B, steps]
        (inf for finished rows): the margin gate of the reduced-precision parity tests.
        """
        if enc is None:
            enc = self.encode(mel)
        B = enc.shape[0]
        xkv = self.cross_kv(enc)
        ac = AhoCorasick(bias or [], word_start)
        lam = float(bias_boost)
        pre = list(prefix) if prefix else [self.start]
        seq = np.tile(np.asarray(pre, dtype=np.int64)[None], (B, 1))
        cache = {}
        h = self.decode_tokens(seq, 0, cache, xkv)
        logits_last = self.lm_head(h[:, -1])
        states = [0] * B
        finished = np.zeros(B, dtype=bool)
        out = []
        all_logits = []
        margins = []
        n_new = 0
        while True:
            if return_logits:
                all_logits.append(logits_last.copy())
            mask_eos = self.eos if n_new < min_new_tokens else -1
            toks = np.empty(B, dtype=np.int64)
            mg = np.full(B, np.inf, dtype=np.float64)
            for b in range(B):
                if finished[b]:
                    toks[b] = self.pad
                    continue
                if lam == 0.0 and mask_eos < 0:
                    row = logits_last[b]
                else:
                    row = ac.boost_row(logits_last[b], states[b], lam) if lam != 0.0 else logits_last[b].copy()
                    if mask_eos >= 0:
                        row[mask_eos] = -np.inf
                toks[b] = int(np.argmax(row))
                if return_margins:
                    top2 = np.partition(row, -2)[-2:]
                    mg[b] = float(top2[1]) - float(top2[0])
                states[b] = ac.delta(states[b], int(toks[b]))
            margins.append(mg)
            finished |= toks == self.eos
            out.append(toks)
            n_new += 1
            if finished.all() or n_new >= max_length:
                break
            seq = np.concatenate([seq, toks[:, None]], axis=1)
            if use_cache:
                h = self.decode_tokens(toks[:, None], seq.shape[1] - 1, cache, xkv)
            else:
                h = self.decode_tokens(seq, 0, {}, xkv)
            logits_last = self.lm_head(h[:, -1])
        ids = np.stack(out, axis=1)
        if trim:   # Whisper's post-processing of the generate() output (oracle/beam_np.py)
            ids = whisper_trim(ids, self.eos, self.pad)
        if return_margins:
            return ids, np.stack(margins, axis=1)
        return (ids, np.stack(all_logits, axis=1)) if return_logits else ids
