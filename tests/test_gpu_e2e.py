"""GPU: end-to-end parity of the HIP path (through the C ABI) with the oracle, which is itself
pinned to the reference (tests/test_oracle_golden.py).

* f32 mode ("exact"): greedy token ids identical to the oracle / reference goldens.
* bf16 mode: encoder within bf16 tolerance; greedy ids identical on the high-margin recipe and
  margin-gated on the diverse recipe (steps whose oracle top-1/top-2 gap < tau may differ).
* bias boost: lam = 0 bit-identical to plain greedy; lam > 0 identical to the oracle's
  Aho-Corasick boost in f32 mode (parity vs the reference itself: unpinned, no reference code).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import whisper_np as W  # noqa: E402
from whisper_context_biasing_amd.config import get_dims  # noqa: E402
from whisper_context_biasing_amd.model import WhisperCB  # noqa: E402
from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list, synth_word_start  # noqa: E402
from whisper_context_biasing_amd.weights import make_weights  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
_CACHE = {}


def case(size, seed, recipe, B):
    key = (size, seed, recipe, B)
    if key not in _CACHE:
        dims = get_dims(size)
        sd = make_weights(dims, seed=seed, recipe=recipe)
        om = W.OracleModel.from_dims(dims, sd)
        mel = W.log_mel(synth_batch(B), dims.n_mel)
        enc = om.encode(mel)
        _CACHE[key] = (dims, sd, om, mel, enc)
    return _CACHE[key]


_MODELS = {}


def model(size, seed, recipe, dtype):
    key = (size, seed, recipe, dtype)
    if key not in _MODELS:
        dims = get_dims(size)
        _MODELS[key] = WhisperCB.from_state_dict(dims, make_weights(dims, seed=seed, recipe=recipe), dtype=dtype)
    return _MODELS[key]


@pytest.mark.parametrize("dtype,tol", [("f32", 2e-4), ("bf16", 6e-2), ("f16", 1.5e-2)])
@pytest.mark.parametrize("size", ["micro", "tiny.en"])
def test_encoder_matches_oracle(size, dtype, tol):
    dims, sd, om, mel, enc = case(size, 0, "diverse", 2)
    m = model(size, 0, "diverse", dtype)
    got = m.encode(torch.from_numpy(mel)).float().cpu().numpy()
    err = np.abs(got - enc)
    # bf16: activations rounded to 8 mantissa bits at every GEMM input; f32: exact-f32 MFMA
    assert err.max() < tol * max(1.0, np.abs(enc).max()), err.max()


@pytest.mark.parametrize("size,seed,recipe", [("micro", 0, "diverse"), ("tiny.en", 0, "diverse"),
                                              ("tiny.en", 1, "margin")])
def test_greedy_f32_matches_reference_golden(size, seed, recipe):
    g = np.load(os.path.join(GOLD, f"model_{size}_{recipe}_s{seed}.npz"))
    ref = g["greedy_ids"]
    dims, sd, om, mel, enc = case(size, seed, recipe, ref.shape[0])
    m = model(size, seed, recipe, "f32")
    for use_graph in (True, False):
        ids = m.generate(torch.from_numpy(mel), max_length=ref.shape[1], use_graph=use_graph).cpu().numpy()
        assert ids.shape == ref.shape and np.array_equal(ids, ref), (use_graph, ids, ref)


def test_greedy_bf16_high_margin_exact():
    g = np.load(os.path.join(GOLD, "model_tiny.en_margin_s1.npz"))
    ref = g["greedy_ids"]
    dims, sd, om, mel, enc = case("tiny.en", 1, "margin", ref.shape[0])
    ids = model("tiny.en", 1, "margin", "bf16").generate(torch.from_numpy(mel), max_length=ref.shape[1]).cpu().numpy()
    assert np.array_equal(ids, ref)


def test_greedy_bf16_margin_gated():
    """Diverse recipe: compare token-by-token until the first step whose oracle margin < tau."""
    tau = 0.05
    g = np.load(os.path.join(GOLD, "model_tiny.en_diverse_s0.npz"))
    ref, margin = g["greedy_ids"], g["greedy_margin"]
    dims, sd, om, mel, enc = case("tiny.en", 0, "diverse", ref.shape[0])
    ids = model("tiny.en", 0, "diverse", "bf16").generate(torch.from_numpy(mel), max_length=ref.shape[1]).cpu().numpy()
    for b in range(ref.shape[0]):
        for t in range(ref.shape[1]):
            if margin[b, t] < tau:
                break
            assert ids[b, t] == ref[b, t], (b, t, ids[b], ref[b])


def test_natural_eos_and_padding():
    """Reference mode: rows stop at EOS, finished rows emit pad, output trimmed when all finished."""
    dims, sd, om, mel, enc = case("micro", 0, "diverse", 2)
    m = model("micro", 0, "diverse", "f32")
    ids = m.generate(torch.from_numpy(mel), max_length=225).cpu().numpy()
    ref = om.generate(mel, max_length=225)
    assert np.array_equal(ids, ref)


@pytest.mark.parametrize("n_phr,lam,gate", [(50, 0.0, False), (50, 2.0, False), (1000, 2.0, False), (200, 8.0, False),
                                            (1000, 2.0, True), (200, 8.0, True)])
def test_bias_boost_matches_oracle_f32(n_phr, lam, gate):
    """The boost of oracle/bias_ref.py (retraction of unfinished matches; with `gate`, matches start only
    at the synthetic word-start tokens), token-exact in f32 mode."""
    dims, sd, om, mel, enc = case("micro", 0, "diverse", 2)
    m = model("micro", 0, "diverse", "f32")
    ws = synth_word_start(dims.eos_token_id, dims.vocab) if gate else None
    m.set_word_start(ws)
    phrases = synth_bias_list(n_phr, eot=dims.eos_token_id)
    # make phrases reachable: include prefixes of the plain greedy output as phrases
    plain = om.generate(mel, enc=enc, max_length=24)
    phrases = phrases + [list(map(int, plain[0, 2:5])), list(map(int, plain[1, 1:3])) + [7, 8]]
    ids = m.generate(torch.from_numpy(mel), max_length=24, bias_list=phrases, bias_boost=lam,
                     min_new_tokens=24).cpu().numpy()
    m.set_word_start(None)
    ref = om.generate(mel, enc=enc, max_length=24, bias=phrases, bias_boost=lam, min_new_tokens=24, word_start=ws)
    assert np.array_equal(ids, ref), (ids, ref)
    if lam == 0.0:
        plain24 = m.generate(torch.from_numpy(mel), max_length=24, min_new_tokens=24).cpu().numpy()
        assert np.array_equal(ids, plain24)


def test_forward_logits_match_reference_golden():
    g = np.load(os.path.join(GOLD, "model_micro_diverse_s0.npz"))
    dims, sd, om, mel, enc = case("micro", 0, "diverse", 2)
    m = model("micro", 0, "diverse", "f32")
    out = m.forward(torch.from_numpy(mel), decoder_input_ids=torch.from_numpy(g["tf_decoder_input_ids"]))
    logits = out.logits.cpu().numpy()
    probe = np.array([0, 1, 2, 13, 220, 1000, 5000, 12345, 25000, 40000, 50255, 50256, 50257,
                      50258, 50300, 50363, 51000, 51863])
    np.testing.assert_allclose(logits[:, :, probe], g["tf_logits_probe"], atol=5e-4, rtol=1e-4)


def test_prompt_prefix_matches_oracle():
    dims, sd, om, mel, enc = case("micro", 0, "diverse", 2)
    m = model("micro", 0, "diverse", "f32")
    prompt = [50361, 100, 200, 300]
    ids = m.generate(torch.from_numpy(mel), max_length=10, prompt_ids=prompt, min_new_tokens=10).cpu().numpy()
    ref = om.generate(mel, enc=enc, max_length=10, prefix=prompt + [dims.decoder_start_token_id], min_new_tokens=10)
    assert np.array_equal(ids, ref)


def test_greedy_bf16_kv_formulation_high_margin_exact():
    """The precomputed cross-K/V formulation (xmode 0: f32 mode and large-v3 use it) in bf16 gives the
    same greedy ids as the reference on the high-margin recipe; the default bf16 path is encoder space."""
    g = np.load(os.path.join(GOLD, "model_tiny.en_margin_s1.npz"))
    ref = g["greedy_ids"]
    dims, sd, om, mel, enc = case("tiny.en", 1, "margin", ref.shape[0])
    m = WhisperCB.from_state_dict(dims, sd, dtype="bf16", options={"xmode": 0})
    ids = m.generate(torch.from_numpy(mel), max_length=ref.shape[1]).cpu().numpy()
    assert np.array_equal(ids, ref)


def _collate_spans(samples, pad=50256):
    """bias_spans exactly as the reference collator pads them (data_utils/data_collator.py:107-125):
    every span right-padded with 50256 to the longest span, every sample to the most spans."""
    L = max(len(sp) for s in samples for sp in s)
    N = max(len(s) for s in samples)
    return torch.tensor([[list(sp) + [pad] * (L - len(sp)) for sp in s] + [[pad] * L] * (N - len(s))
                         for s in samples], dtype=torch.long)


def test_generate_with_collator_bias_spans():
    """The drop-in path: generate(input_features, labels, bias_spans=<collator tensor>, bias_boost>0) boosts
    the union of the batch's spans (padding stripped); the collator's all-zeros [B, 1, 1] form boosts
    nothing; bias_boost = 0 ignores the spans like the reference."""
    dims, sd, om, mel, enc = case("micro", 0, "diverse", 2)
    m = model("micro", 0, "diverse", "f32")
    plain = om.generate(mel, enc=enc, max_length=16, min_new_tokens=16)
    samples = [[list(map(int, plain[0, 2:5])), [11, 12]], [list(map(int, plain[1, 1:3])) + [7, 8]]]
    spans = _collate_spans(samples)
    union = [s for smp in samples for s in smp]
    x = torch.from_numpy(mel)
    kw = dict(max_length=16, min_new_tokens=16)
    got = m.generate(x, bias_spans=spans, bias_boost=2.0, **kw).cpu().numpy()
    via_list = m.generate(x, bias_list=union, bias_boost=2.0, **kw).cpu().numpy()
    ref = om.generate(mel, enc=enc, bias=union, bias_boost=2.0, **kw)
    assert np.array_equal(got, via_list) and np.array_equal(got, ref), (got, ref)
    zeros = m.generate(x, bias_spans=torch.zeros(2, 1, 1, dtype=torch.long), bias_boost=2.0, **kw).cpu().numpy()
    unboosted = m.generate(x, bias_spans=spans, bias_boost=0.0, **kw).cpu().numpy()
    assert np.array_equal(zeros, plain) and np.array_equal(unboosted, plain)


def test_generate_splits_batches_above_64_clips():
    """A reference eval batch larger than one library call (64 clips) is decoded in order in several
    calls and re-padded: the same rows as decoding the parts separately."""
    dims = get_dims("micro")
    m = model("micro", 0, "diverse", "f32")
    mel = torch.from_numpy(W.log_mel(synth_batch(70), dims.n_mel))
    ids = m.generate(mel, max_length=12).cpu().numpy()
    a = m.generate(mel[:64], max_length=12).cpu().numpy()
    b = m.generate(mel[64:], max_length=12).cpu().numpy()
    w = max(a.shape[1], b.shape[1])
    pad = lambda t: np.pad(t, ((0, 0), (0, w - t.shape[1])), constant_values=dims.pad_token_id)
    assert ids.shape == (70, w) and np.array_equal(ids, np.concatenate([pad(a), pad(b)]))
    beams = m.generate(mel[:70], max_length=6, num_beams=8).cpu().numpy()   # 512 / 8 = 64 clips per call
    assert beams.shape[0] == 70


def test_device_weight_views_match_host_upload():
    """wcb_load_weights: the state dict as borrowed device tensors (bf16 blob views, f32 and f16
    tensors, non-contiguous strides) stages on the device without a host round trip and yields the
    same model as the host f32 upload: identical greedy ids and bit-identical logits (f32 mode)."""
    dims, sd, om, mel, enc = case("micro", 0, "diverse", 2)
    host = WhisperCB.from_state_dict(dims, sd, dtype="f32")
    dev = {}
    for i, (n, a) in enumerate(sd.items()):
        t = torch.from_numpy(np.asarray(a, dtype=np.float32)).cuda()
        if i % 3 == 1 and t.dim() == 2:
            t = t.t().contiguous().t()                 # same values, column-major strides
        elif i % 3 == 2:
            t = t.to(torch.float16) if np.all(np.asarray(a, np.float32) == np.asarray(a, np.float16)) else t
        dev[n] = t
    viewed = WhisperCB.from_state_dict(dims, dev, dtype="f32")
    x = torch.from_numpy(mel)
    a = host.generate(x, max_length=12, min_new_tokens=12).cpu().numpy()
    b = viewed.generate(x, max_length=12, min_new_tokens=12).cpu().numpy()
    assert np.array_equal(a, b)
    ids = torch.from_numpy(np.concatenate([np.full((2, 1), dims.decoder_start_token_id), a[:, :5]], 1))
    la = host.forward(x, decoder_input_ids=ids).logits
    lb = viewed.forward(x, decoder_input_ids=ids).logits
    assert torch.equal(la, lb)


def test_broadcast_blob_views_load_without_host_copy():
    """The bench's path: the packed bf16 blob (what the RCCL broadcast delivers) unpacked as device
    views and loaded through wcb_load_weights equals loading the same bf16-rounded values from host."""
    from whisper_context_biasing_amd.shard import pack_state_dict, unpack_state_dict, unpack_state_dict_views
    dims = get_dims("micro")
    sd = make_weights(dims, seed=0, recipe="diverse")
    flat = pack_state_dict(dims, sd).cuda()
    views = unpack_state_dict_views(dims, flat)
    assert all(v.is_cuda and v.dtype == torch.bfloat16 for v in views.values())
    m1 = WhisperCB.from_state_dict(dims, views, dtype="bf16")
    m2 = WhisperCB.from_state_dict(dims, unpack_state_dict(dims, flat), dtype="bf16")
    x = torch.from_numpy(W.log_mel(synth_batch(2), dims.n_mel))
    assert np.array_equal(m1.generate(x, max_length=10, min_new_tokens=10).cpu().numpy(),
                          m2.generate(x, max_length=10, min_new_tokens=10).cpu().numpy())


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_fused_lean_launches_are_bit_identical(dtype):
    """The lean decode path's in-launch fusion (gemm_impl.h dec_lean_kernel FZ 2): option xq_kq — q'_h =
    W_k,hᵀ q_h inside the LN-fused q_proj launch (common.h group_arrive_wait hand-off) — against the
    separate launches it replaces: identical arithmetic, so identical ids even on the diverse recipe,
    whose near-ties (gaps ~1e-3) flip on any rounding difference. 32 rows (32-row QKV blocks), 13 and 40
    rows (16-row blocks, ragged), 1000-phrase boost. Then the fused model again with its 64-bit arrival
    counters seeded just below 2^31 and 2^32 (an int32 generation count wrapped there): the
    same ids, and no hand-off wait timed out (wcb_synchronize reports one as an error)."""
    dims = get_dims("small")
    sd = make_weights(dims, seed=0, recipe="diverse")
    phrases = synth_bias_list(1000, eot=dims.eos_token_id)
    models = [WhisperCB.from_state_dict(dims, sd, dtype=dtype, options=o)   # (the q_proj LayerNorm unfolded in both)
              for o in ({"xq_kq": 1, "lean_fold": 0}, {"xq_kq": 0, "lean_fold": 0})]
    kw = dict(max_length=24, min_new_tokens=24, bias_list=phrases, bias_boost=2.0)
    for B in (32, 13, 40):
        x = torch.from_numpy(W.log_mel(synth_batch(B, start=3), dims.n_mel))
        out = [m.generate(x, **kw).cpu().numpy() for m in models]
        for o in out[1:]:
            np.testing.assert_array_equal(out[0], o)
    fused = models[0]
    x = torch.from_numpy(W.log_mel(synth_batch(32, start=3), dims.n_mel))
    ref = fused.generate(x, **kw).cpu().numpy()
    for seed in ((1 << 31) - 8, (1 << 32) - 8):
        fused.set_option("kq_cnt_seed", seed // 4)
        for _ in range(2):   # both decode contexts
            np.testing.assert_array_equal(fused.generate(x, **kw).cpu().numpy(), ref)
        fused.synchronize()


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_fused_cross_query_is_bit_identical(dtype):
    """Option xqk (gemm_impl.h dec_xqk_kernel): each workgroup recomputes its head's q_h with the folded lean
    q_proj's K split, MFMA and sum order, then its chunk of q'_h = W_k,hᵀ q_h in the kq launch's order — the
    same arithmetic as the xq → kq launches, so identical ids even on the diverse recipe's near-ties: 32 rows,
    13 and 40 rows (ragged 16-row blocks), 1000-phrase boost."""
    dims = get_dims("small")
    sd = make_weights(dims, seed=0, recipe="diverse")
    phrases = synth_bias_list(1000, eot=dims.eos_token_id)
    models = [WhisperCB.from_state_dict(dims, sd, dtype=dtype, options=o)
              for o in ({"xqk": 1}, {"xqk": 0}, {"xqk": 1, "xqk_chunks": 2}, {"xqk": 1, "xqk_chunks": 16})]
    kw = dict(max_length=24, min_new_tokens=24, bias_list=phrases, bias_boost=2.0)
    for B in (32, 13, 40):
        x = torch.from_numpy(W.log_mel(synth_batch(B, start=3), dims.n_mel))
        out = [m.generate(x, **kw).cpu().numpy() for m in models]
        for o in out[1:]:
            np.testing.assert_array_equal(out[0], o)


def test_merge_output_split_is_bit_identical():
    """Option merge_os 2 (xenc_merge_v_kernel OS: a head's 64 W_v outputs over two workgroups of 4 rows) runs
    the same range merge and MFMA sequence per output as merge_os 1: identical ids on the diverse recipe,
    32 and 13 rows, 1000-phrase boost."""
    dims = get_dims("small")
    sd = make_weights(dims, seed=0, recipe="diverse")
    phrases = synth_bias_list(1000, eot=dims.eos_token_id)
    models = [WhisperCB.from_state_dict(dims, sd, dtype="bf16", options=o) for o in ({"merge_os": 2}, {"merge_os": 1})]
    kw = dict(max_length=24, min_new_tokens=24, bias_list=phrases, bias_boost=2.0)
    for B in (32, 13):
        x = torch.from_numpy(W.log_mel(synth_batch(B, start=5), dims.n_mel))
        out = [m.generate(x, **kw).cpu().numpy() for m in models]
        np.testing.assert_array_equal(out[0], out[1])


def test_lean_32_row_workgroups_are_bit_identical():
    """Option lean_mf2 (every lean projection on 32-row workgroups where the chain has > 16 rows) keeps each
    row's K split, MFMA and sum order: identical ids to the default 16-row residual writers, 32 and 40 rows."""
    dims = get_dims("small")
    sd = make_weights(dims, seed=0, recipe="diverse")
    phrases = synth_bias_list(1000, eot=dims.eos_token_id)
    models = [WhisperCB.from_state_dict(dims, sd, dtype="bf16", options=o) for o in ({"lean_mf2": 1}, {"lean_mf2": 0})]
    kw = dict(max_length=24, min_new_tokens=24, bias_list=phrases, bias_boost=2.0)
    for B in (32, 40):
        x = torch.from_numpy(W.log_mel(synth_batch(B, start=7), dims.n_mel))
        out = [m.generate(x, **kw).cpu().numpy() for m in models]
        np.testing.assert_array_equal(out[0], out[1])


def test_bias_from_another_handle_is_rejected():
    """A bias automaton belongs to the handle that built it (its decode graphs are keyed on it): passing
    it to another handle is an argument error, not a silently wrong boost."""
    from whisper_context_biasing_amd import _lib
    dims = get_dims("micro")
    sd = make_weights(dims, seed=0, recipe="margin")
    m1 = WhisperCB.from_state_dict(dims, sd, dtype="f32")
    m2 = WhisperCB.from_state_dict(dims, sd, dtype="f32")
    phrases = synth_bias_list(20, eot=dims.eos_token_id)
    b1 = m1.bias_list(phrases)
    x = torch.from_numpy(W.log_mel(synth_batch(2), dims.n_mel))
    m1.generate(x, max_length=4, bias_list=phrases, bias_boost=2.0)
    with pytest.raises(_lib.WcbError, match="another handle"):
        m2.generate(x, max_length=4, bias_list=b1, bias_boost=2.0)
    # its own handle takes the prebuilt automaton
    assert m1.generate(x, max_length=4, bias_list=b1, bias_boost=2.0).shape[0] == 2


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_folded_layernorm_beam_rows_match_layernorm_launch(dtype):
    """Decode rows > 64 (beam search: 16 clips x 5 beams = 80 rows): the ring-tile projections with the
    pre-block LayerNorm folded in (option ln_fold 1, default: W·diag(γ) weights, row statistics from the
    residual writers' 32-column partials, r·(acc − μ·u) + c in the epilogue) against a LayerNorm launch
    before each projection (ln_fold 0): the same beams on the high-margin recipe, and both equal to the
    numpy oracle's beam search on the first clip."""
    from oracle.beam_np import generate_beam
    dims = get_dims("small")
    sd = make_weights(dims, seed=1, recipe="margin")
    fold = WhisperCB.from_state_dict(dims, sd, dtype=dtype)
    launch = WhisperCB.from_state_dict(dims, sd, dtype=dtype, options={"ln_fold": 0})
    phrases = synth_bias_list(1000, eot=dims.eos_token_id)
    x = torch.from_numpy(W.log_mel(synth_batch(16), dims.n_mel))
    kw = dict(max_length=10, num_beams=5, bias_list=phrases, bias_boost=2.0)
    a = fold.generate(x, **kw).cpu().numpy()
    b = launch.generate(x, **kw).cpu().numpy()
    np.testing.assert_array_equal(a, b)
    om = W.OracleModel.from_dims(dims, sd)
    ref = generate_beam(om, mel=x[:1].numpy(), num_beams=5, max_length=10, bias=phrases, bias_boost=2.0)
    np.testing.assert_array_equal(a[:1, :ref.shape[1]], ref)


