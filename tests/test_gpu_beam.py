"""GPU: beam search (A9) through the C ABI (k_beam.hip, key-map self-attention, shared encoder rows).

* f32 mode: token-exact against the reference's own beam-5 goldens (HF generate, num_beams = 5).
* boost / MinNewTokens / prompt prefix / more than 64 rows (row groups): identical to the oracle
  (oracle/beam_np.py) in f32 mode — parity vs the reference unpinned for the boost (no reference code).
* bf16, both cross-attention formulations for beams (default: precomputed per-clip cross-K/V shared by
  the beams, b_div; option beam_xmode = 1: encoder space, rows_per_enc = beams): batch invariance (every utterance
  decoded alone gives the same beams as in the batch: the row maps and the shared encoder rows are
  exact) and identical to the oracle on the high-margin recipe.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import whisper_np as W  # noqa: E402
from oracle.beam_np import generate_beam  # noqa: E402
from whisper_context_biasing_amd.config import get_dims  # noqa: E402
from whisper_context_biasing_amd.model import WhisperCB  # noqa: E402
from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list, synth_word_start  # noqa: E402
from whisper_context_biasing_amd.weights import make_weights  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
_CASES, _MODELS = {}, {}


def case(size, seed, recipe, B):
    key = (size, seed, recipe, B)
    if key not in _CASES:
        dims = get_dims(size)
        sd = make_weights(dims, seed=seed, recipe=recipe)
        om = W.OracleModel.from_dims(dims, sd)
        mel = W.log_mel(synth_batch(B), dims.n_mel)
        _CASES[key] = (dims, om, mel, om.encode(mel))
    return _CASES[key]


def model(size, seed, recipe, dtype, beam_xmode="0"):
    key = (size, seed, recipe, dtype, beam_xmode)
    if key not in _MODELS:
        dims = get_dims(size)
        _MODELS[key] = WhisperCB.from_state_dict(dims, make_weights(dims, seed=seed, recipe=recipe), dtype=dtype,
                                                 options={"beam_xmode": int(beam_xmode)})
    return _MODELS[key]


@pytest.mark.parametrize("size", ["micro", "tiny.en"])
def test_beam5_f32_matches_reference_golden(size):
    g = np.load(os.path.join(GOLD, f"model_{size}_diverse_s0.npz"))
    ref = g["beam5_ids"]
    dims, om, mel, enc = case(size, 0, "diverse", ref.shape[0])
    m = model(size, 0, "diverse", "f32")
    for use_graph in (True, False):
        ids = m.generate(torch.from_numpy(mel), max_length=24, num_beams=5, use_graph=use_graph).cpu().numpy()
        assert ids.shape == ref.shape and np.array_equal(ids, ref), (use_graph, ids, ref)


@pytest.mark.parametrize("nb,lam,min_new,n_phr,gate", [(2, 0.0, 0, 0, False), (3, 2.0, 0, 200, False),
                                                       (5, 2.0, 12, 1000, False), (8, 8.0, 0, 50, False),
                                                       (5, 2.0, 12, 1000, True), (4, 4.0, 0, 200, True)])
def test_beam_boost_matches_oracle_f32(nb, lam, min_new, n_phr, gate):
    """Beam scores carry the per-step bonus including the retraction of abandoned matches (and, with
    `gate`, word-start gated starts): token-exact against the oracle's beam search."""
    dims, om, mel, enc = case("micro", 0, "diverse", 2)
    m = model("micro", 0, "diverse", "f32")
    ws = synth_word_start(dims.eos_token_id, dims.vocab) if gate else None
    m.set_word_start(ws)
    plain = om.generate(mel, enc=enc, max_length=24, min_new_tokens=24)
    phrases = synth_bias_list(n_phr, eot=dims.eos_token_id) if n_phr else []
    phrases = phrases + [list(map(int, plain[0, 2:5])), list(map(int, plain[1, 1:3])) + [7, 8]]
    ids = m.generate(torch.from_numpy(mel), max_length=24, num_beams=nb, bias_list=phrases, bias_boost=lam,
                     min_new_tokens=min_new).cpu().numpy()
    m.set_word_start(None)
    ref = generate_beam(om, enc=enc, num_beams=nb, max_length=24, bias=phrases, bias_boost=lam,
                        min_new_tokens=min_new, word_start=ws)
    assert ids.shape == ref.shape and np.array_equal(ids, ref), (ids, ref)


def test_beam_natural_eos_matches_oracle_f32():
    """Long decode (beams finish on EOS, early-stop heuristic, Whisper trim)."""
    dims, om, mel, enc = case("micro", 0, "diverse", 2)
    m = model("micro", 0, "diverse", "f32")
    ids = m.generate(torch.from_numpy(mel), max_length=120, num_beams=4).cpu().numpy()
    ref = generate_beam(om, enc=enc, num_beams=4, max_length=120)
    assert ids.shape == ref.shape and np.array_equal(ids, ref), (ids, ref)


@pytest.mark.parametrize("group_rows", ["512", "64"])
def test_beam_row_groups_match_oracle_f32(group_rows):
    """16 clips x 5 beams = 80 decoder rows: one 80-row chain (default), or two row groups on
    parallel streams (option group_rows = 64)."""
    dims, om, mel, enc = case("micro", 0, "diverse", 16)
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0, recipe="diverse"), dtype="f32",
                                  options={"group_rows": int(group_rows)})
    ids = m.generate(torch.from_numpy(mel), max_length=16, num_beams=5).cpu().numpy()
    ref = generate_beam(om, enc=enc, num_beams=5, max_length=16)
    assert ids.shape == ref.shape and np.array_equal(ids, ref), (ids, ref)


def test_beam_prompt_prefix_matches_oracle_f32():
    dims, om, mel, enc = case("micro", 0, "diverse", 2)
    m = model("micro", 0, "diverse", "f32")
    prompt = [50361, 100, 200, 300]
    ids = m.generate(torch.from_numpy(mel), max_length=10, num_beams=3, prompt_ids=prompt).cpu().numpy()
    ref = generate_beam(om, enc=enc, num_beams=3, max_length=10, prefix=prompt + [dims.decoder_start_token_id])
    assert ids.shape == ref.shape and np.array_equal(ids, ref), (ids, ref)


@pytest.mark.parametrize("beam_xmode", ["0", "1"])
def test_beam_bf16_batch_invariant_and_high_margin(beam_xmode):
    dims, om, mel, enc = case("tiny.en", 1, "margin", 4)
    m = model("tiny.en", 1, "margin", "bf16", beam_xmode)
    x = torch.from_numpy(mel)
    ids = m.generate(x, max_length=24, num_beams=5).cpu().numpy()
    for b in range(x.shape[0]):
        one = m.generate(x[b:b + 1], max_length=24, num_beams=5).cpu().numpy()
        assert np.array_equal(one[0], ids[b, :one.shape[1]]), (b, one, ids[b])
    ref = generate_beam(om, enc=enc, num_beams=5, max_length=24)
    assert ids.shape == ref.shape and np.array_equal(ids, ref), (ids, ref)


def _one_layer(size, seed, recipe, B, dtype, beam_xmode="0", group_rows=512):
    dims = get_dims(size, n_layers=1)
    sd = make_weights(dims, seed=seed, recipe=recipe)
    om = W.OracleModel.from_dims(dims, sd)
    mel = W.log_mel(synth_batch(B), dims.n_mel)
    return dims, om, mel, WhisperCB.from_state_dict(dims, sd, dtype=dtype,
                                                    options={"beam_xmode": int(beam_xmode), "group_rows": group_rows})


def _batch_invariant(m, x, **kw):
    ids = m.generate(x, **kw).cpu().numpy()
    for b in range(x.shape[0]):
        one = m.generate(x[b:b + 1], **kw).cpu().numpy()[0]
        assert np.array_equal(one, ids[b, :len(one)]), (b, one, ids[b])
        assert (ids[b, len(one):] == m.dims.pad_token_id).all()
    return ids


def test_beam_c5_shape_f16_kv_mode():
    """C5 shape (large-v3 layer: d = 1280, 20 heads, 128 mels, V = 51866) in fp16: the precomputed
    cross-K/V path shared by the beams of a clip (b_div), the f16 encoder clamp epilogue, a 5000-phrase
    boost. Batch-invariant; identical to the oracle without boost on the high-margin recipe."""
    dims, om, mel, m = _one_layer("large-v3", 1, "margin", 3, "f16")
    x = torch.from_numpy(mel)
    phrases = synth_bias_list(5000, eot=dims.eos_token_id)
    _batch_invariant(m, x, max_length=12, num_beams=5, bias_list=phrases, bias_boost=2.0)
    ids = m.generate(x, max_length=12, num_beams=5).cpu().numpy()
    ref = generate_beam(om, mel=mel, num_beams=5, max_length=12)
    assert ids.shape == ref.shape and np.array_equal(ids, ref), (ids, ref)


@pytest.mark.parametrize("beam_xmode,group_rows", [("0", "512"), ("1", "512"), ("0", "64"), ("1", "64")])
def test_beam_c3_shape_bf16_row_groups(beam_xmode, group_rows):
    """C3 shape (medium layer: d = 1024; per-clip cross-K/V or encoder-space cross-attention) with 13
    clips x 5 beams = 65 decoder rows (two row groups): batch-invariant, and identical to the oracle on
    the high-margin recipe."""
    # one 65-row chain, or two chains of row groups
    dims, om, mel, m = _one_layer("medium", 1, "margin", 13, "bf16", beam_xmode, int(group_rows))
    x = torch.from_numpy(mel)
    ids = _batch_invariant(m, x, max_length=8, num_beams=5)
    ref = generate_beam(om, mel=mel, num_beams=5, max_length=8)
    assert ids.shape == ref.shape and np.array_equal(ids, ref), (ids, ref)


def test_greedy_and_beam_calls_interleave_on_one_handle():
    """One bf16 handle alternates greedy (encoder-space cross-attention) and beam (per-clip cross-K/V)
    calls: the decode workspaces regrow / graphs are re-captured, and every call returns what a fresh
    sequence of the same call returns."""
    dims, om, mel, enc = case("tiny.en", 1, "margin", 4)
    m = model("tiny.en", 1, "margin", "bf16")
    x = torch.from_numpy(mel)
    g1 = m.generate(x, max_length=20).cpu().numpy()
    b1 = m.generate(x, max_length=20, num_beams=5).cpu().numpy()
    g2 = m.generate(x, max_length=20).cpu().numpy()
    b2 = m.generate(x, max_length=20, num_beams=3).cpu().numpy()
    b3 = m.generate(x, max_length=20, num_beams=5).cpu().numpy()
    assert np.array_equal(g1, g2) and np.array_equal(b1, b3)
    assert np.array_equal(b2, generate_beam(om, enc=enc, num_beams=3, max_length=20))


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_beam_async_output_equals_blocking(dtype):
    """block=False beam search (the serving / bench pipeline: no host read-back of the best length) writes
    every max_length column: the blocking call's generated columns, then pad_token_id."""
    dims, om, mel, _ = case("tiny.en", 0, "diverse", 3)
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0, recipe="diverse"), dtype=dtype)
    x = torch.from_numpy(mel)
    ref = m.generate(x, max_length=10, num_beams=5, return_dict_in_generate=True).sequences[:, 1:].cpu().numpy()
    out = m.generate(x, max_length=10, num_beams=5, block=False)
    m.synchronize()
    got = out.cpu().numpy()
    assert got.shape == (3, 10)
    L = ref.shape[1]
    assert np.array_equal(got[:, :L], ref), (got, ref)
    assert (got[:, L:] == dims.pad_token_id).all()
