"""GPU: step-wise decoding (wcb_decode_begin / wcb_decode_step) against generate() on the
same clips: the same decode step one token per call, so the ids must be identical (greedy on the f32 K/V
cross-attention and bf16 encoder-space paths, the bias boost, a prompt prefix; beam search with parents and
the best finished sequences, also against the reference beam goldens); and the
reference forward()'s encoder_outputs / past_key_values / use_cache arguments (wcb_forward_enc,
wcb_forward_cached)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import whisper_np as W  # noqa: E402
from whisper_context_biasing_amd.config import get_dims  # noqa: E402
from whisper_context_biasing_amd.model import WhisperCB  # noqa: E402
from whisper_context_biasing_amd.synth import synth_batch, synth_bias_list  # noqa: E402
from whisper_context_biasing_amd.weights import make_weights  # noqa: E402


@pytest.mark.parametrize("size,dtype,prompt", [("tiny.en", "f32", False), ("small", "bf16", False),
                                               ("small", "bf16", True)])
def test_stepwise_decode_equals_generate(size, dtype, prompt):
    dims = get_dims(size)
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0, recipe="diverse"), dtype=dtype)
    B, n = 4, 12
    x = torch.from_numpy(W.log_mel(synth_batch(B), dims.n_mel))
    phrases = synth_bias_list(200, eot=dims.eos_token_id)
    pr = [50360, 1000, 2000, 3000] if prompt else None   # <|startofprev|>-style prefix tokens
    ref = m.generate(x, max_length=n, min_new_tokens=n, bias_list=phrases, bias_boost=2.0, prompt_ids=pr,
                     return_dict_in_generate=True).sequences
    ref = ref[:, ref.shape[1] - n:].cpu().numpy()
    dec = m.decode_begin(m.encode(x), prompt_ids=pr, bias_list=phrases, bias_boost=2.0, min_new_tokens=n)
    ids, scores = zip(*[dec.step() for _ in range(n)])
    dec.close()
    got = torch.stack(ids, 1).cpu().numpy()
    assert np.array_equal(got, ref), (got, ref)
    assert torch.isfinite(torch.stack(scores)).all()
    # a second decode on the same handle (the state was released)
    dec = m.decode_begin(m.encode(x), min_new_tokens=2)
    dec.step()
    dec.close()


@pytest.mark.parametrize("size,dtype,B", [("small", "bf16", 32), ("medium", "f16", 5)])
def test_stepwise_scores_lm_head_layernorm_split_bit_identical(size, dtype, B):
    """The lean LM head with the final LayerNorm inside its column walk (default), in a launch of its own
    (option lm_ln_split: gemm_impl.h ln_rows_kernel, the same K split, sum order and normalisation), and
    the general decode kernel's fused form (option lean = 0): the chosen tokens' boosted logits returned
    per step must be equal bit for bit (the projections' LayerNorm unfolded: lean_fold 0 in all three)."""
    dims = get_dims(size)
    sd = make_weights(dims, seed=1, recipe="diverse")
    x = torch.from_numpy(W.log_mel(synth_batch(B), dims.n_mel))
    phrases = synth_bias_list(200, eot=dims.eos_token_id)
    out = []
    for opts in ({"lean": 1, "lean_fold": 0}, {"lean": 1, "lm_ln_split": 1, "lean_fold": 0}, {"lean": 0, "lean_fold": 0}):
        m = WhisperCB.from_state_dict(dims, sd, dtype=dtype, options=opts)
        dec = m.decode_begin(m.encode(x), bias_list=phrases, bias_boost=2.0, min_new_tokens=6)
        steps = [dec.step() for _ in range(6)]
        dec.close()
        out.append((torch.stack([i for i, _ in steps], 1).cpu(), torch.stack([s for _, s in steps], 1).float().cpu()))
        del m
    for o in out[1:]:
        assert torch.equal(out[0][0], o[0])
        assert torch.equal(out[0][1], o[1])


# ---------------------------------------------------------------- step-wise beam search
def _golden(size, recipe, seed):
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", f"model_{size}_{recipe}_s{seed}.npz"))
    return g, eval(str(g["meta"][0]), {})


@pytest.mark.parametrize("dtype,boost,prompt", [("f32", False, False), ("bf16", False, False), ("bf16", True, False),
                                                ("bf16", True, True)])
def test_stepwise_beam5_equals_generate(dtype, boost, prompt):
    """Step-wise beam search (wcb_decode_begin_beams / wcb_decode_step / wcb_decode_parents /
    wcb_decode_result) against generate(num_beams=5) ([tf] generation/utils.py:3208) on the
    same clips: one HF beam iteration per step, so after the steps generate() takes the best finished
    sequences are identical — on whisper-small's high-margin recipe also identical to the reference
    model's own beam-5 goldens; with the 1000-phrase boost (lambda 2, EOS masked) and with a prompt
    prefix against generate() with the same arguments. Every parent index lies in [0, 5)."""
    dims = get_dims("small")
    g, meta = _golden("small", "margin", 1)
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=1, recipe="margin"), dtype=dtype)
    B, L = meta["B"], meta["beam_len"]
    x = torch.from_numpy(W.log_mel(synth_batch(B), dims.n_mel))
    kw = dict(bias_list=synth_bias_list(1000, eot=dims.eos_token_id), bias_boost=2.0, min_new_tokens=L) if boost else {}
    pr = [50360, 1000, 2000, 3000] if prompt else None
    ref = m.generate(x, max_length=L, num_beams=5, prompt_ids=pr, **kw).cpu().numpy()
    if not boost and not prompt:
        assert np.array_equal(ref, g["beam5_ids"]), (ref, g["beam5_ids"])
    dec = m.decode_begin(m.encode(x), num_beams=5, max_length=L, prompt_ids=pr, **kw)
    for _ in range(L):
        toks, scores = dec.step()
        par = dec.parents().cpu().numpy()
        assert toks.shape == (B * 5,) and ((par >= 0) & (par < 5)).all()
        assert torch.isfinite(scores[::5]).all()
    got = dec.result(L).cpu().numpy()
    # the length cap finished every utterance: the search is frozen — a further step gives
    # identity parents and pad ids, and the result does not change
    assert dec.done and dec.info()[:2] == (L, L)
    toks, _ = dec.step()
    assert (dec.parents().cpu().numpy() == np.tile(np.arange(5), B)).all()
    assert (toks.cpu().numpy() == dims.pad_token_id).all()
    assert np.array_equal(dec.result().cpu().numpy(), got)
    dec.close()
    assert np.array_equal(got, ref), (got, ref)


def test_stepwise_greedy_result_equals_generate_and_guards():
    """StepDecoder.result() (wcb_decode_result) for greedy decoding against generate() with the same
    arguments; the output width comes from the library (wcb_decode_info), a caller width below the
    generated columns is refused, and every decode option that shapes the state carried between steps
    (lean_x, merge_v, xq_kq, ...) is refused while the decode is open."""
    from whisper_context_biasing_amd import _lib
    dims = get_dims("small")
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0, recipe="diverse"), dtype="bf16")
    B, n = 3, 9
    x = torch.from_numpy(W.log_mel(synth_batch(B), dims.n_mel))
    ref = m.generate(x, max_length=n, min_new_tokens=n).cpu().numpy()
    dec = m.decode_begin(m.encode(x), min_new_tokens=n)
    for opt, v in (("lean_x", 0), ("merge_v", 0), ("xq_kq", 1), ("lm_ln_split", 1), ("xvariant", 1)):
        with pytest.raises(_lib.WcbError, match=opt):
            m.set_option(opt, v)
    m.set_option("enc_raster", 8)                       # encoder-side options stay free
    for _ in range(n):
        dec.step()
    mx, steps, done = dec.info()
    assert mx == dims.n_text_ctx - 1 and steps == n and not done
    got = dec.result().cpu().numpy()
    assert np.array_equal(got, ref), (got, ref)
    with pytest.raises(ValueError):
        dec.result(n - 1)
    # the raw ABI refuses an out_ld below the generated columns instead of writing past the buffer
    out = torch.empty(B, n - 1, dtype=torch.int32, device=m.device)
    ns = _lib.C.c_int32(0)
    rc = m._lib.wcb_decode_result(m._h, dec._st, out.data_ptr(), n - 1, _lib.C.byref(ns), None)
    assert rc == -1
    dec.close()
    m.set_option("lean_x", 1)                            # allowed again once the state is closed


# ---------------------------------------------------------------- forward(encoder_outputs / past_key_values)
GOLD = os.path.join(os.path.dirname(__file__), "golden")
PROBE = np.array([0, 1, 2, 13, 220, 1000, 5000, 12345, 25000, 40000, 50255, 50256, 50257, 50258, 50300, 50363,
                  51000, 51863])


def test_forward_encoder_outputs_bit_identical_and_golden():
    """forward(encoder_outputs=..., decoder_input_ids=...) decodes from the given encoder state without
    re-encoding (models/whisper_medical.py:54-55, 93-111 → wcb_forward_enc): logits bit-identical to
    forward(input_features=...) for every form HF accepts (tensor, tuple, BaseModelOutput-like), and within
    5e-4 of the reference's teacher-forced logits (micro golden, f32); input_features=None works."""
    from types import SimpleNamespace
    g = np.load(os.path.join(GOLD, "model_micro_diverse_s0.npz"))
    dims = get_dims("micro")
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0, recipe="diverse"), dtype="f32")
    x = torch.from_numpy(W.log_mel(synth_batch(2), dims.n_mel))
    ids = torch.from_numpy(g["tf_decoder_input_ids"])
    full = m.forward(x, decoder_input_ids=ids)
    enc = m.encode(x)
    assert torch.equal(enc, full.encoder_last_hidden_state)
    for form in (enc, (enc,), SimpleNamespace(last_hidden_state=enc)):
        out = m.forward(encoder_outputs=form, decoder_input_ids=ids)
        assert torch.equal(out.logits, full.logits)
    np.testing.assert_allclose(full.logits.cpu().numpy()[:, :, PROBE], g["tf_logits_probe"], atol=5e-4, rtol=1e-4)
    with pytest.raises(ValueError):
        m.forward(decoder_input_ids=ids)                       # neither input_features nor encoder_outputs
    with pytest.raises(ValueError):
        m.forward(encoder_outputs=enc[:, :100], decoder_input_ids=ids)
    with pytest.raises(NotImplementedError):
        m.forward(x, decoder_input_ids=ids, decoder_inputs_embeds=torch.zeros(1))


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_forward_encoder_outputs_bit_identical_small(dtype):
    """The same at whisper-small (bf16: the encoder-space cross-attention reads the given encoder output)."""
    dims = get_dims("small")
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=1, recipe="margin"), dtype=dtype)
    B = 5
    x = torch.from_numpy(W.log_mel(synth_batch(B), dims.n_mel))
    rng = np.random.default_rng(5)
    ids = torch.from_numpy(np.concatenate([np.full((B, 1), dims.decoder_start_token_id),
                                           rng.integers(0, 50000, (B, 9))], 1))
    a = m.forward(x, decoder_input_ids=ids)
    b = m.forward(encoder_outputs=a.encoder_last_hidden_state, decoder_input_ids=ids)
    assert torch.equal(a.logits, b.logits)


@pytest.mark.parametrize("split", [1, 4, 7])
def test_forward_past_key_values_continues_the_cache(split):
    """forward(..., use_cache=True) returns the decoder KV cache as past_key_values; forward(next ids,
    past_key_values=cache) appends positions and returns only their logits (models/whisper_medical.py:
    54-55, 89-110 → wcb_forward_cached). The two halves equal the one-pass logits (f32, within 1e-4:
    the halves run as other row counts) and the reference golden within 5e-4."""
    g = np.load(os.path.join(GOLD, "model_micro_diverse_s0.npz"))
    dims = get_dims("micro")
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0, recipe="diverse"), dtype="f32")
    x = torch.from_numpy(W.log_mel(synth_batch(2), dims.n_mel))
    ids = torch.from_numpy(g["tf_decoder_input_ids"])
    full = m.forward(x, decoder_input_ids=ids).logits
    o1 = m.forward(x, decoder_input_ids=ids[:, :split], use_cache=True)
    cache = o1.past_key_values
    assert cache is not None and cache.get_seq_length() == split
    parts = [o1.logits]
    for t0 in range(split, ids.shape[1], 3):          # several continuation calls
        o = m.forward(decoder_input_ids=ids[:, t0:t0 + 3], past_key_values=cache)
        assert o.past_key_values is cache
        parts.append(o.logits)
    got = torch.cat(parts, 1)
    assert cache.get_seq_length() == ids.shape[1]
    torch.testing.assert_close(got, full, atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(got.cpu().numpy()[:, :, PROBE], g["tf_logits_probe"], atol=5e-4, rtol=1e-4)
    with pytest.raises(TypeError):
        m.forward(decoder_input_ids=ids[:, :1], past_key_values=((torch.zeros(1),),))
    cache.close()
    # the state slot is free again: a step-wise decode can start
    dec = m.decode_begin(m.encode(x), min_new_tokens=2)
    dec.step()
    dec.close()


def test_decode_contexts_guard_while_stepwise_decode_is_open():
    """The step-wise state owns decode context 3: raising decode_contexts to 4 while it is
    open is refused, and generate() calls interleaved with its steps at decode_contexts 3 leave both
    decodes unchanged (micro f32)."""
    from whisper_context_biasing_amd import _lib
    dims = get_dims("micro")
    m = WhisperCB.from_state_dict(dims, make_weights(dims, seed=0, recipe="diverse"), dtype="f32")
    x = torch.from_numpy(W.log_mel(synth_batch(3), dims.n_mel))
    n = 10
    ref_gen = m.generate(x, max_length=n, min_new_tokens=n).cpu().numpy()
    dec = m.decode_begin(m.encode(x), min_new_tokens=n)
    ref_steps = torch.stack([dec.step()[0] for _ in range(n)], 1).cpu().numpy()
    dec.close()
    m.set_option("decode_contexts", 3)
    dec = m.decode_begin(m.encode(x), min_new_tokens=n)
    with pytest.raises(_lib.WcbError, match="decode_contexts"):
        m.set_option("decode_contexts", 4)
    # the state's copy of the encoder output keeps the layout chosen at begin
    for opt, v in (("xenc_fm", 0), ("xenc_variant", 0)):
        with pytest.raises(_lib.WcbError, match=opt):
            m.set_option(opt, v)
    steps = []
    for i in range(n):
        steps.append(dec.step()[0])
        if i % 3 == 0:                                    # generate() cycles through contexts 0-2 meanwhile
            assert np.array_equal(m.generate(x, max_length=n, min_new_tokens=n).cpu().numpy(), ref_gen)
    dec.close()
    assert np.array_equal(torch.stack(steps, 1).cpu().numpy(), ref_steps)
    m.set_option("decode_contexts", 4)                   # allowed again once the state is closed
