"""CPU: the numpy oracle against the reference's own outputs at the benchmark model sizes
(tests/golden/make_golden.py big: whisper-small for C2/C4, full-depth medium for C3, full-depth
large-v3 for C5, and prompt-conditioned decoding). The GPU parity tests compare libwcb with this
oracle, so pinning it here pins them."""
import os

import numpy as np
import pytest

from oracle import whisper_np as W
from oracle.beam_np import generate_beam
from whisper_context_biasing_amd.config import get_dims
from whisper_context_biasing_amd.synth import synth_batch
from whisper_context_biasing_amd.weights import make_weights

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    g = np.load(os.path.join(GOLD, name))
    meta = eval(str(g["meta"][0]), {})   # our own fixture's dict literal
    return g, meta


@pytest.mark.parametrize("name", ["model_small_diverse_s0.npz", "model_small_margin_s1.npz",
                                  pytest.param("model_medium_margin_s1.npz", marks=pytest.mark.slow),
                                  pytest.param("model_medium_diverse_s0.npz", marks=pytest.mark.slow),
                                  pytest.param("model_large-v3_margin_s1.npz", marks=pytest.mark.slow)])
def test_oracle_matches_reference_at_benchmark_sizes(name):
    g, meta = _load(name)
    dims = get_dims(meta["size"])
    om = W.OracleModel.from_dims(dims, make_weights(dims, seed=meta["seed"], recipe=meta["recipe"]))
    mel = W.log_mel(synth_batch(meta["B"]), dims.n_mel)
    enc = om.encode(mel)
    ref_enc = g["enc_slices"]
    got = np.concatenate([enc[:, s] for s in (slice(0, 4), slice(748, 752), slice(1496, 1500))], axis=1)
    assert np.abs(got - ref_enc).max() < 2e-4 * max(1.0, np.abs(ref_enc).max())
    ids, margins = om.generate(enc=enc, max_length=meta["n_tokens"], return_margins=True)
    assert np.array_equal(ids, g["greedy_ids"]), (ids, g["greedy_ids"])
    # the reference's own top-1/top-2 gaps (fp32): same ordering evidence as the oracle's
    assert np.allclose(margins[:, :g["greedy_margin"].shape[1]], g["greedy_margin"], atol=2e-3)
    if "beam5_ids" in g.files:
        b = generate_beam(om, enc=enc, num_beams=5, max_length=meta["beam_len"])
        assert np.array_equal(b, g["beam5_ids"]), (b, g["beam5_ids"])


@pytest.mark.parametrize("name", ["prompt_micro_diverse_s0.npz", "prompt_small_margin_s1.npz"])
def test_oracle_prompt_conditioned_matches_reference(name):
    """Reference generate(prompt_ids=[<|startofprev|>, ...]): decoder input = prompt + [SOT], output
    strips both ([tf] generation_whisper.py:1909-1911, 1141)."""
    g, meta = _load(name)
    dims = get_dims(meta["size"])
    om = W.OracleModel.from_dims(dims, make_weights(dims, seed=meta["seed"], recipe=meta["recipe"]))
    mel = W.log_mel(synth_batch(meta["B"]), dims.n_mel)
    enc = om.encode(mel)
    prefix = [int(t) for t in g["prompt_ids"]] + [dims.decoder_start_token_id]
    ids = om.generate(enc=enc, max_length=meta["n_tokens"], prefix=prefix)
    assert np.array_equal(ids, g["greedy_ids"]), (ids, g["greedy_ids"])
    b = generate_beam(om, enc=enc, num_beams=5, max_length=meta["beam_len"], prefix=prefix)
    assert np.array_equal(b, g["beam5_ids"]), (b, g["beam5_ids"])
