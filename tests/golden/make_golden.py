"""Generate the golden parity fixtures by running the REFERENCE itself (survey container only).

Imports the reference model class `WhisperForConditionalGenerationWeightCE`
(`/root/reference/models/whisper_medical.py`) and HF's `WhisperFeatureExtractor` (the A1 code the
reference calls at `data_utils/data_loader.py:171`), feeds them the build's seeded bf16-rounded
synthetic weights and synthetic clips, and stores SMALL slices / summaries of their outputs as
`tests/golden/*.npz`. The fixtures are data (inputs are regenerated from seeds; expected outputs
are slices), never reference source. The reference does not travel to the GPU box; only these
fixtures do.

Harness-side shim (no reference file is edited): `_tied_weights_keys` is a list in the reference
(`models/whisper_medical.py:14`, 4.x convention) and transformers 5.x expects a dict
(SURVEY.md §8(c)).

Decode semantics follow `scripts/evaluation.py:173-180`: bare GenerationConfig(max_length, pad,
eos, decoder_start, use_cache=False), no suppression, fp32, greedy.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference"

from whisper_context_biasing_amd.config import get_dims  # noqa: E402
from whisper_context_biasing_amd.weights import make_weights  # noqa: E402
from whisper_context_biasing_amd.synth import synth_batch, synth_clip  # noqa: E402

MEL_COLS = [slice(0, 48), slice(1476, 1524), slice(2952, 3000)]
ENC_ROWS = [slice(0, 4), slice(748, 752), slice(1496, 1500)]
VOCAB_PROBE = np.array([0, 1, 2, 13, 220, 1000, 5000, 12345, 25000, 40000, 50255, 50256, 50257,
                        50258, 50300, 50363, 51000, 51863], dtype=np.int64)


def ref_model(dims, sd, attn="sdpa"):
    sys.path.insert(0, REF)
    from transformers import WhisperConfig
    from models.whisper_medical import WhisperForConditionalGenerationWeightCE as Ref
    Ref._tied_weights_keys = {"proj_out.weight": "model.decoder.embed_tokens.weight"}  # shim
    cfg = WhisperConfig(**dims.hf_config_kwargs())
    cfg._attn_implementation = attn
    torch.manual_seed(0)
    m = Ref(cfg, bias_weight=10.0)
    state = {k: torch.from_numpy(v) for k, v in sd.items()}
    state["proj_out.weight"] = state["model.decoder.embed_tokens.weight"]
    missing, unexpected = m.load_state_dict(state, strict=False)
    assert not unexpected, unexpected
    assert all(k == "proj_out.weight" for k in missing), missing
    m.eval()
    assert m.proj_out.weight.data_ptr() == m.model.decoder.embed_tokens.weight.data_ptr() or \
        torch.equal(m.proj_out.weight, m.model.decoder.embed_tokens.weight)
    return m


def mel_fixture():
    from transformers import WhisperFeatureExtractor
    clips = [synth_clip(0), synth_clip(1), synth_clip(2, n_samples=5 * 16000),
             (synth_clip(3) * 0.001).astype(np.float32)]
    out = {}
    for n_mel in (80, 128):
        fe = WhisperFeatureExtractor(feature_size=n_mel)
        out[f"filters_{n_mel}"] = fe.mel_filters.astype(np.float64)
        for i, c in enumerate(clips):
            # single-waveform call exactly like data_utils/data_loader.py:171-172
            m = fe(c, sampling_rate=16000).input_features[0]
            assert m.shape == (n_mel, 3000), m.shape
            out[f"mel{n_mel}_clip{i}_slices"] = np.concatenate([m[:, s] for s in MEL_COLS], axis=1)
            out[f"mel{n_mel}_clip{i}_stats"] = np.array(
                [m.sum(dtype=np.float64), np.abs(m).sum(dtype=np.float64), m.max(), m.min()])
    np.savez_compressed(os.path.join(HERE, "mel_golden.npz"), **out)
    print("mel fixture written")


def model_fixture(size, seed, recipe, B, n_tokens, tf_len, beams=True, eager=True, beam_len=24):
    """Reference outputs for one (size, seed, recipe): encoder slices, teacher-forced logits
    probes, greedy ids / margins (scripts/evaluation.py decode config) and HF beam-5 ids.
    The larger sizes (medium, large-v3: the C3 / C5 models at full depth) skip the eager-attention
    cross-check (eager=False) and may skip the teacher-forced forward (tf_len=0) to bound CPU time."""
    from transformers import GenerationConfig
    dims = get_dims(size)
    sd = make_weights(dims, seed=seed, recipe=recipe)
    from transformers import WhisperFeatureExtractor
    fe = WhisperFeatureExtractor(feature_size=dims.n_mel)
    pcm = synth_batch(B)
    mel = np.stack([fe(c, sampling_rate=16000).input_features[0] for c in pcm]).astype(np.float32)
    out = {"mel_sum": mel.sum(dtype=np.float64)}
    rng = np.random.default_rng(seed + 17)
    dec_ids = np.concatenate([np.full((B, 1), dims.decoder_start_token_id),
                              rng.integers(0, dims.eos_token_id, size=(B, max(tf_len, 1) - 1))], axis=1)
    if tf_len:
        out["tf_decoder_input_ids"] = dec_ids
    res = {}
    for attn in (("sdpa", "eager") if eager else ("sdpa",)):
        m = ref_model(dims, sd, attn)
        with torch.no_grad():
            x = torch.from_numpy(mel)
            enc = m.model.encoder(x).last_hidden_state.numpy()
            logits = None
            if tf_len:
                fw = m(input_features=x, decoder_input_ids=torch.from_numpy(dec_ids), return_dict=True)
                logits = fw.logits.float().numpy()
            gc = GenerationConfig(max_length=n_tokens, pad_token_id=dims.pad_token_id,
                                  eos_token_id=dims.eos_token_id,
                                  decoder_start_token_id=dims.decoder_start_token_id, use_cache=False)
            # scripts/evaluation.py:173-182: the bare config replaces model.generation_config;
            # Seq2SeqTrainer then calls generate(**inputs, max_length=...) ([tf] trainer_seq2seq.py:329)
            m.generation_config = gc
            m.config.use_cache = False
            m.config.suppress_tokens = []
            g = m.generate(input_features=x, max_length=n_tokens, return_dict_in_generate=True,
                           output_scores=True)
            ids = g.sequences.numpy()
            scores = torch.stack(g.scores, 1).float().numpy()       # [B, steps, V]
            plain = m.generate(input_features=x, max_length=n_tokens).numpy()
            res[attn] = (enc, logits, ids, scores, plain)
            if attn == "sdpa" and beams:
                gcb = GenerationConfig(max_length=min(n_tokens, beam_len), pad_token_id=dims.pad_token_id,
                                       eos_token_id=dims.eos_token_id, num_beams=5,
                                       decoder_start_token_id=dims.decoder_start_token_id, use_cache=True)
                out["beam5_ids"] = m.generate(input_features=x, generation_config=gcb).numpy()
    enc, logits, ids, scores, plain = res["sdpa"]
    out["enc_slices"] = np.concatenate([enc[:, s] for s in ENC_ROWS], axis=1)
    out["enc_stats"] = np.array([enc.sum(dtype=np.float64), np.abs(enc).sum(dtype=np.float64)])
    if logits is not None:
        out["tf_logits_probe"] = logits[:, :, VOCAB_PROBE]
        out["tf_logits_top5_idx"] = np.argsort(-logits, axis=-1, kind="stable")[:, :, :5]
        out["tf_logits_top5_val"] = np.take_along_axis(logits, out["tf_logits_top5_idx"], -1)
        lse = np.log(np.exp(logits - logits.max(-1, keepdims=True)).sum(-1)) + logits.max(-1)
        out["tf_logits_lse"] = lse
    out["greedy_sequences"] = ids                    # return_dict_in_generate: includes SOT
    out["greedy_ids"] = plain                        # plain generate(): SOT stripped, pad-right
    srt = np.sort(scores, axis=-1)
    out["greedy_margin"] = srt[..., -1] - srt[..., -2]
    out["greedy_top1"] = scores.argmax(-1)
    out["greedy_step_max"] = srt[..., -1]
    if "eager" in res:
        e_enc, e_logits, e_ids, _, _ = res["eager"]
        out["eager_vs_sdpa_enc_maxdiff"] = np.abs(e_enc - enc).max()
        if logits is not None:
            out["eager_vs_sdpa_logits_maxdiff"] = np.abs(e_logits - logits).max()
        out["eager_greedy_ids"] = e_ids
    meta = dict(size=size, seed=seed, recipe=recipe, B=B, n_tokens=n_tokens, beam_len=min(n_tokens, beam_len))
    out["meta"] = np.array([str(meta)])
    name = f"model_{size}_{recipe}_s{seed}.npz"
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(name, "greedy", plain.shape, "min margin", out["greedy_margin"].min(),
          "eager/sdpa enc diff", out.get("eager_vs_sdpa_enc_maxdiff"), flush=True)


def prompt_fixture(size, seed, recipe, B, n_tokens, prompt, beam_len=12):
    """Prompt-conditioned decoding: the reference's biasing prompt
    `<|startofprev|>` + bias / description tokens (data_utils/data_loader.py:182-366) fed to the
    reference's generate() as `prompt_ids` ([tf] generation_whisper.py:1909-1911: decoder input =
    prompt + [decoder_start]; output strips both, :1141; max_length counts new tokens, :1932-1940).
    Greedy and beam-5 ids."""
    from transformers import GenerationConfig, WhisperFeatureExtractor
    dims = get_dims(size)
    sd = make_weights(dims, seed=seed, recipe=recipe)
    fe = WhisperFeatureExtractor(feature_size=dims.n_mel)
    mel = np.stack([fe(c, sampling_rate=16000).input_features[0] for c in synth_batch(B)]).astype(np.float32)
    m = ref_model(dims, sd)
    x = torch.from_numpy(mel)
    pr = torch.tensor(prompt, dtype=torch.long)
    out = {"prompt_ids": np.asarray(prompt, dtype=np.int64)}
    with torch.no_grad():
        m.generation_config = GenerationConfig(max_length=n_tokens, pad_token_id=dims.pad_token_id,
                                               eos_token_id=dims.eos_token_id,
                                               decoder_start_token_id=dims.decoder_start_token_id, use_cache=False)
        m.config.use_cache = False
        m.config.suppress_tokens = []
        g = m.generate(input_features=x, max_length=n_tokens, prompt_ids=pr, return_dict_in_generate=True,
                       output_scores=True)
        scores = torch.stack(g.scores, 1).float().numpy()
        srt = np.sort(scores, axis=-1)
        out["greedy_sequences"] = g.sequences.numpy()
        out["greedy_margin"] = srt[..., -1] - srt[..., -2]
        out["greedy_ids"] = m.generate(input_features=x, max_length=n_tokens, prompt_ids=pr).numpy()
        gcb = GenerationConfig(max_length=beam_len, pad_token_id=dims.pad_token_id, eos_token_id=dims.eos_token_id,
                               num_beams=5, decoder_start_token_id=dims.decoder_start_token_id, use_cache=True)
        out["beam5_ids"] = m.generate(input_features=x, generation_config=gcb, prompt_ids=pr).numpy()
    out["meta"] = np.array([str(dict(size=size, seed=seed, recipe=recipe, B=B, n_tokens=n_tokens,
                                     beam_len=beam_len))])
    name = f"prompt_{size}_{recipe}_s{seed}.npz"
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(name, "greedy", out["greedy_ids"].shape, "beam", out["beam5_ids"].shape, flush=True)


def metric_fixture():
    """Reference-run transcript dumps (results/*.txt, `Ref :`/`Pred:` format of
    utils/compute_metric.py:150-153) + the matching JSONL bias_words: data for the metric goldens."""
    import gzip
    import json
    for split, res in (("dev", "refs_and_pred_desc_only.txt"), ("test", "refs_and_pred_baseline_ko_prompt.txt")):
        raw = open(os.path.join(REF, "results", res), encoding="utf-8").read()
        jl = os.path.join(REF, "data", "medical-united-syn-med-75-jsonl", f"{split}.jsonl")
        bw = [json.loads(line).get("bias_words") or [] for line in open(jl, encoding="utf-8")]
        with gzip.open(os.path.join(HERE, f"metric_{split}.json.gz"), "wt", encoding="utf-8") as f:
            json.dump({"source_results": f"results/{res}",
                       "source_bias_words": f"data/medical-united-syn-med-75-jsonl/{split}.jsonl",
                       "raw_lines": raw, "bias_words": bw}, f)
    print("metric fixtures written")


def wce_fixture(seed=0, T=10):
    """Weighted-CE loss of the reference forward (`models/whisper_medical.py:113-156`) on the micro
    model: labels with planted bias spans (list form with an empty span, the collator's padded
    tensor form, the zeros[B,1,1] "no spans" form) and bias_spans=None (plain CE). Stores the
    labels, spans and the reference's loss for each form (bias_weight = 10)."""
    dims = get_dims("micro")
    sd = make_weights(dims, seed=seed, recipe="diverse")
    from transformers import WhisperFeatureExtractor
    fe = WhisperFeatureExtractor(feature_size=dims.n_mel)
    B = 2
    pcm = synth_batch(B)
    mel = np.stack([fe(c, sampling_rate=16000).input_features[0] for c in pcm]).astype(np.float32)
    rng = np.random.default_rng(seed + 99)
    labels = rng.integers(0, dims.eos_token_id, size=(B, T)).astype(np.int64)
    eos = dims.eos_token_id
    # planted spans: row 0 holds [11, 22, 33] at 2 and [44] at 7; row 1 holds [55, 66] twice and
    # the padded-form match [77, 88, eos] at the end (span followed by EOS)
    labels[0, 2:5] = [11, 22, 33]; labels[0, 7] = 44; labels[0, 0] = -100
    labels[1, 1:3] = [55, 66]; labels[1, 4:6] = [55, 66]; labels[1, 7:10] = [77, 88, eos]
    labels[1, 3] = 0
    spans_list = [[[11, 22, 33], [44], []], [[55, 66], [77, 88], [99, 98, 97]]]
    Lmax = 3
    padded = np.full((B, 3, Lmax), eos, dtype=np.int64)
    for i, row in enumerate(spans_list):
        for n, sp in enumerate(row):
            padded[i, n, :len(sp)] = sp
    m = ref_model(dims, sd)
    x = torch.from_numpy(mel)
    lab = torch.from_numpy(labels)
    out = {"labels": labels, "spans_padded": padded, "bias_weight": np.float64(10.0)}
    out["spans_list_len"] = np.array([[len(sp) for sp in row] for row in spans_list], dtype=np.int64)
    with torch.no_grad():
        out["loss_list"] = np.float64(m(input_features=x, labels=lab, bias_spans=spans_list).loss)
        out["loss_padded"] = np.float64(m(input_features=x, labels=lab, bias_spans=torch.from_numpy(padded)).loss)
        out["loss_zeros"] = np.float64(m(input_features=x, labels=lab,
                                         bias_spans=torch.zeros(B, 1, 1, dtype=torch.long)).loss)
        out["loss_none"] = np.float64(m(input_features=x, labels=lab).loss)
    np.savez_compressed(os.path.join(HERE, "wce_micro_s0.npz"), **out)
    print("wce", {k: float(v) for k, v in out.items() if k.startswith("loss")})


def big_fixtures():
    """Round 2: the benchmark model sizes at full depth (C2 small, C3 medium, C5 large-v3) and the
    prompt-conditioned decode."""
    model_fixture("small", 0, "diverse", B=2, n_tokens=64, tf_len=6, beam_len=24)
    model_fixture("small", 1, "margin", B=2, n_tokens=64, tf_len=6, eager=False, beam_len=24)
    model_fixture("medium", 1, "margin", B=1, n_tokens=16, tf_len=0, eager=False, beam_len=16)
    model_fixture("medium", 0, "diverse", B=1, n_tokens=16, tf_len=0, eager=False, beams=False)
    model_fixture("large-v3", 1, "margin", B=1, n_tokens=12, tf_len=0, eager=False, beam_len=12)
    # <|startofprev|> (multilingual 50361 / .en 50360) + synthetic bias-word tokens
    prompt_fixture("micro", 0, "diverse", B=2, n_tokens=16, prompt=[50361, 100, 200, 300, 4000, 17])
    prompt_fixture("small", 1, "margin", B=2, n_tokens=16,
                   prompt=[50361] + [int(v) for v in np.random.default_rng(5).integers(0, 50257, 40)])


if __name__ == "__main__":
    if sys.argv[1:] == ["wce"]:
        wce_fixture()
        sys.exit(0)
    if sys.argv[1:] == ["big"]:
        torch.set_num_threads(8)
        big_fixtures()
        sys.exit(0)
    metric_fixture()
    torch.set_num_threads(8)
    mel_fixture()
    model_fixture("micro", 0, "diverse", B=2, n_tokens=32, tf_len=8)
    model_fixture("tiny.en", 0, "diverse", B=2, n_tokens=48, tf_len=6)
    model_fixture("tiny.en", 1, "margin", B=2, n_tokens=48, tf_len=6, beams=False)
