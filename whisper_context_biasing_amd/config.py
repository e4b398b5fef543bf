"""Model dimensions and special token ids for the Whisper sizes on the hot path.

The reference never defines dimensions itself: it loads them from the hub config of the
checkpoint it evaluates (`scripts/evaluation.py:164`, `models/whisper_medical.py:16-22`).
These tables restate the public OpenAI Whisper configs that `BASELINE.json` names
(tiny.en for C1, small for C2/C4, medium for C3, large-v3 for C5).
Special ids follow SURVEY.md §9.10: `.en` vocab uses eot 50256 / sot 50257, multilingual
uses eot 50257 / sot 50258 — never hard-code them elsewhere.
"""
from __future__ import annotations

from dataclasses import dataclass, asdict, replace

N_AUDIO_CTX = 1500          # encoder positions ([tf] modeling_whisper.py:612-616)
N_SAMPLES = 480000          # 30 s at 16 kHz ([tf] feature_extraction_whisper.py:91)
N_FRAMES = 3000             # mel frames = N_SAMPLES // HOP
N_FFT = 400
HOP = 160
SAMPLE_RATE = 16000
N_TEXT_CTX = 448            # decoder positions (max_target_positions)


@dataclass(frozen=True)
class WhisperDims:
    name: str
    d_model: int
    n_layers: int           # encoder layers == decoder layers for every released size
    n_heads: int
    ffn: int
    vocab: int
    n_mel: int
    eos_token_id: int
    pad_token_id: int
    decoder_start_token_id: int
    n_audio_ctx: int = N_AUDIO_CTX
    n_text_ctx: int = N_TEXT_CTX

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    def to_dict(self):
        return asdict(self)

    def hf_config_kwargs(self):
        """Keyword arguments for `transformers.WhisperConfig` describing the same model."""
        return dict(
            vocab_size=self.vocab, num_mel_bins=self.n_mel, d_model=self.d_model,
            encoder_layers=self.n_layers, decoder_layers=self.n_layers,
            encoder_attention_heads=self.n_heads, decoder_attention_heads=self.n_heads,
            encoder_ffn_dim=self.ffn, decoder_ffn_dim=self.ffn,
            max_source_positions=self.n_audio_ctx, max_target_positions=self.n_text_ctx,
            pad_token_id=self.pad_token_id, eos_token_id=self.eos_token_id,
            bos_token_id=self.eos_token_id, decoder_start_token_id=self.decoder_start_token_id,
            activation_function="gelu", scale_embedding=False, use_cache=True,
        )


_EN = dict(eos_token_id=50256, pad_token_id=50256, decoder_start_token_id=50257)
_ML = dict(eos_token_id=50257, pad_token_id=50257, decoder_start_token_id=50258)

MODELS = {
    # micro: the golden-fixture config of SURVEY.md §8(c) recipe (i)
    "micro": WhisperDims("micro", 64, 2, 1, 256, 51865, 80, **_ML),   # head_dim 64 like every release
    "tiny.en": WhisperDims("tiny.en", 384, 4, 6, 1536, 51864, 80, **_EN),
    "tiny": WhisperDims("tiny", 384, 4, 6, 1536, 51865, 80, **_ML),
    "base.en": WhisperDims("base.en", 512, 6, 8, 2048, 51864, 80, **_EN),
    "small": WhisperDims("small", 768, 12, 12, 3072, 51865, 80, **_ML),
    "medium": WhisperDims("medium", 1024, 24, 16, 4096, 51865, 80, **_ML),
    "large-v3": WhisperDims("large-v3", 1280, 32, 20, 5120, 51866, 128, **_ML),
}


def get_dims(name: str, **overrides) -> WhisperDims:
    if name not in MODELS:
        raise KeyError(f"unknown Whisper size {name!r}; known: {sorted(MODELS)}")
    d = MODELS[name]
    return replace(d, **overrides) if overrides else d


def dims_from_hf_config(cfg) -> WhisperDims:
    """Build dims from a `transformers.WhisperConfig`-like object (attribute access)."""
    if cfg.encoder_layers != cfg.decoder_layers:
        raise ValueError("encoder_layers != decoder_layers is not a released Whisper shape")
    return WhisperDims(
        name=getattr(cfg, "name_or_path", "") or "custom", d_model=cfg.d_model,
        n_layers=cfg.encoder_layers, n_heads=cfg.encoder_attention_heads,
        ffn=cfg.encoder_ffn_dim, vocab=cfg.vocab_size, n_mel=cfg.num_mel_bins,
        eos_token_id=cfg.eos_token_id, pad_token_id=cfg.pad_token_id,
        decoder_start_token_id=cfg.decoder_start_token_id,
        n_audio_ctx=cfg.max_source_positions, n_text_ctx=cfg.max_target_positions)
