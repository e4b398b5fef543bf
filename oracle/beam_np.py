"""Beam-search restatement (A9) — TEST ORACLE ONLY.

Used by tests/ (parity checker) only; never imported by the product package.

Restates HF `GenerationMixin._beam_search` ([tf] generation/utils.py:3208-3524, helpers
:3008-3204) as WhisperForConditionalGeneration.generate drives it for short-form audio:
* GenerationConfig(num_beams=nb) with the library defaults length_penalty = 1.0,
  early_stopping = False; beams_to_keep K = 2·nb (one EOS id, [tf] utils.py:3286);
* the static sequence buffers hold min(prefix + max_length, max_target_positions) tokens
  ([tf] generation_whisper.py:1932-1940);
* Whisper strips the prefix, each row's trailing pads and final EOS, and right-pads with
  pad_token_id to the longest row ([tf] generation_whisper.py:1063-1086, 213-225) — `whisper_trim`.
The build-defined bias boost (A8, oracle/bias_ref.py) and the MinNewTokens EOS mask
([tf] logits_process.py:227-235) act as logits processors, i.e. on the log-probabilities
([tf] utils.py:3388-3389).

Pinned by `beam5_ids` in tests/golden/model_*_diverse_s0.npz (the reference model's generate with
num_beams = 5, max_length = 24, tests/golden/make_golden.py:117-121).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .bias_ref import AhoCorasick

F32 = np.float32
NEG = F32(-1.0e9)


def log_softmax_f32(x: np.ndarray) -> np.ndarray:
    """torch.nn.functional.log_softmax over the last axis in f32: (x - max) - log Σ exp(x - max)
    (the sum accumulated in f64 here; torch accumulates in f32 vector lanes — 1-ulp drift)."""
    m = x.max(-1, keepdims=True)
    s = (x - m).astype(F32)
    lse = np.log(np.exp(s.astype(np.float64)).sum(-1, keepdims=True)).astype(F32)
    return (s - lse).astype(F32)


def topk(vals: np.ndarray, k: int):
    """torch.topk(k) along the last axis: descending value, ties to the lower index."""
    idx = np.argsort(-vals, axis=-1, kind="stable")[..., :k]
    return np.take_along_axis(vals, idx, -1), idx


def whisper_trim(ids: np.ndarray, eos: int, pad: int) -> np.ndarray:
    """Per row: drop the pads (keeping one when pad == eos) and the final EOS, then right-pad every
    row with pad to the longest ([tf] generation_whisper.py:1063-1086, 213-225)."""
    rows = []
    for r in np.asarray(ids):
        r = np.asarray(r)
        if len(r) and r[-1] == pad:
            n = int((r == pad).sum())
            if pad == eos:
                n -= 1
            if n:
                r = r[:-n]
        if len(r) and r[-1] == eos:
            r = r[:-1]
        rows.append(r)
    W = max((len(r) for r in rows), default=0)
    out = np.full((len(rows), W), pad, dtype=np.int64)
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out


def generate_beam(om, mel=None, num_beams: int = 5, max_length: int = 225, enc=None,
                  min_new_tokens: int = 0, bias: Optional[Sequence[Sequence[int]]] = None,
                  bias_boost: float = 0.0, prefix: Optional[Sequence[int]] = None,
                  length_penalty: float = 1.0, trim: bool = True, return_scores: bool = False,
                  word_start=None):
    """Beam search over `om` (oracle/whisper_np.OracleModel). Returns the best finished sequence of
    every utterance (new tokens only), Whisper-trimmed unless `trim=False` (then [B, W] with
    W = longest best sequence incl. its EOS, pad-filled — the C-ABI output)."""
    if enc is None:
        enc = om.encode(mel)
    B, nb = enc.shape[0], int(num_beams)
    K = 2 * nb
    R = B * nb
    pre = list(prefix) if prefix else [om.start]
    P = len(pre)
    n_ctx = om.w("model.decoder.embed_positions.weight").shape[0]
    Lt = min(P + int(max_length), n_ctx)
    ac = AhoCorasick(bias or [], word_start)
    lam = F32(bias_boost)
    # beams of one clip share its encoder state: cross-K/V once per clip, repeated per beam row
    xkv = [(np.repeat(k, nb, axis=0), np.repeat(v, nb, axis=0)) for k, v in om.cross_kv(enc)]

    run_seq = np.full((B, nb, Lt), om.pad, dtype=np.int64)
    run_seq[:, :, :P] = np.asarray(pre, dtype=np.int64)
    fin_seq = run_seq.copy()
    run_sc = np.zeros((B, nb), F32)
    run_sc[:, 1:] = NEG
    fin_sc = np.full((B, nb), NEG, F32)
    fin_done = np.zeros((B, nb), bool)
    fin_len = np.zeros((B, nb), np.int64)                # generated tokens (beam_indices count)
    unsat = np.ones(B, bool)
    states = np.zeros((B, nb), np.int64)
    top_mask = np.arange(K) < nb

    cache: dict = {}
    h = om.decode_tokens(run_seq[:, :, :P].reshape(R, P), 0, cache, xkv)
    logits = om.lm_head(h[:, -1])
    V = logits.shape[-1]
    cur = P
    while True:
        logp = log_softmax_f32(logits)
        if lam != 0:
            for r in range(R):
                logp[r] = ac.boost_row(logp[r], int(states[r // nb, r % nb]), lam)
        if cur - P < min_new_tokens:
            logp[:, om.eos] = -np.inf
        acc = (logp.reshape(B, nb, V) + run_sc[:, :, None]).astype(F32).reshape(B, nb * V)
        top_lp, top_i = topk(acc, K)                     # _get_top_k_continuations
        parent_k, tok_k = top_i // V, top_i % V
        cand = np.take_along_axis(run_seq, parent_k[:, :, None], 1).copy()
        cand[:, :, cur] = tok_k
        hits = (tok_k == om.eos) | (cur + 1 >= Lt)       # EOS / MaxLength on cur + 1 tokens
        # _get_running_beams_for_next_iteration
        run_lp = (top_lp + hits.astype(F32) * NEG).astype(F32)
        _, sel = topk(run_lp, nb)
        new_seq = np.take_along_axis(cand, sel[:, :, None], 1)
        new_sc = np.take_along_axis(run_lp, sel, 1)
        parent = np.take_along_axis(parent_k, sel, 1)
        ntok = np.take_along_axis(tok_k, sel, 1)
        # _update_finished_beams (uses the heuristic flag of the previous iteration)
        did = hits & top_mask[None]
        fl = (top_lp / F32((cur + 1 - P) ** length_penalty)).astype(F32)
        fl = (fl + (~unsat)[:, None].astype(F32) * NEG).astype(F32)
        fl = (fl + (~did).astype(F32) * NEG).astype(F32)
        m_sc = np.concatenate([fin_sc, fl], 1)
        _, fsel = topk(m_sc, nb)
        fin_seq = np.take_along_axis(np.concatenate([fin_seq, cand], 1), fsel[:, :, None], 1)
        fin_sc = np.take_along_axis(m_sc, fsel, 1)
        fin_done = np.take_along_axis(np.concatenate([fin_done, did], 1), fsel, 1)
        fin_len = np.take_along_axis(np.concatenate([fin_len, np.full((B, K), cur + 1 - P)], 1), fsel, 1)
        # AC states of the new running beams
        states = np.array([[ac.delta(int(states[b, parent[b, i]]), int(ntok[b, i])) for i in range(nb)]
                           for b in range(B)], dtype=np.int64)
        run_seq, run_sc = new_seq, new_sc
        cur += 1
        # _check_early_stop_heuristic (early_stopping=False) + _beam_search_has_unfinished_sequences
        best = (run_sc[:, :1] / F32((cur - P) ** length_penalty)).astype(F32)
        worst = np.where(fin_done, fin_sc.min(1, keepdims=True), NEG)
        unsat = unsat & (best > worst).any(1)
        if not unsat.any() or hits.all():
            break
        # reorder the self-attention cache to the parents, feed the selected tokens
        rows = (np.arange(B)[:, None] * nb + parent).reshape(R)
        for l in list(cache):
            cache[l] = (cache[l][0][rows], cache[l][1][rows])
        h = om.decode_tokens(run_seq[:, :, cur - 1].reshape(R, 1), cur - 1, cache, xkv)
        logits = om.lm_head(h[:, -1])

    W = int(fin_len[:, 0].max())
    out = fin_seq[:, 0, P:P + W]
    if trim:
        out = whisper_trim(out, om.eos, om.pad)
    return (out, fin_sc[:, 0]) if return_scores else out
