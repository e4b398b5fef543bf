"""Drop-in inference surface of the reference model class, backed by libwcb.so.

`WhisperCB` mirrors the parts of `WhisperForConditionalGenerationWeightCE`
(`models/whisper_medical.py:12-172`) that the reference's evaluation path touches
(`scripts/evaluation.py:164-206` → `[tf] trainer_seq2seq.py:329`):

* `generate(input_features, labels=None, bias_spans=None, max_length=...)` → LongTensor [B, ≤max_length]
  without the start token, right-padded with pad_token_id (same return convention as HF);
  `return_dict_in_generate=True` returns `.sequences` that include the start token.
* `forward(input_features, decoder_input_ids, labels=None, bias_spans=None)` → output with
  `.logits` f32 [B, T, V], `.encoder_last_hidden_state`, and the reference's weighted-CE `.loss`
  (`models/whisper_medical.py:113-156`, computed host-side on the returned logits: a training-loss
  path, not the inference hot path).
* `generation_config`, `config.use_cache`, `config.suppress_tokens`, `freeze_encoder()` and `.to()` are
  accepted exactly as the reference mutates them (`scripts/evaluation.py:173-183`).

All arithmetic runs in hand-written HIP kernels through the C ABI; torch only holds device
memory and streams. There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from dataclasses import dataclass
from types import SimpleNamespace
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .config import N_SAMPLES, WhisperDims, dims_from_hf_config, get_dims

_TORCH_DT = {_lib.WCB_BF16: torch.bfloat16, _lib.WCB_F16: torch.float16, _lib.WCB_F32: torch.float32}


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


@dataclass
class GenerateOutput:
    sequences: torch.Tensor


@dataclass
class Seq2SeqLMOutput:
    loss: Optional[torch.Tensor]
    logits: torch.Tensor
    encoder_last_hidden_state: torch.Tensor
    past_key_values: Optional["DecoderCache"] = None

    def to_tuple(self):
        return tuple(v for v in (self.loss, self.logits, self.past_key_values, self.encoder_last_hidden_state)
                     if v is not None)

    def __getitem__(self, i):
        return self.to_tuple()[i]


class BiasList:
    """Device Aho-Corasick automaton of a bias list (list of token-id sequences)."""

    def __init__(self, model: "WhisperCB", phrases: Sequence[Sequence[int]]):
        lib = _lib.load()
        phrases = [list(map(int, p)) for p in phrases if len(p) > 0]
        toks = np.asarray([t for p in phrases for t in p] or [0], dtype=np.int32)
        offs = np.zeros(len(phrases) + 1, dtype=np.int32)
        offs[1:] = np.cumsum([len(p) for p in phrases]) if phrases else []
        ws = model.word_start
        h = C.c_void_p()
        _lib.check(lib.wcb_bias_create(model._h, toks.ctypes.data, offs.ctypes.data, len(phrases),
                                       ws.ctypes.data if ws is not None else None, C.byref(h)),
                   model._h, "wcb_bias_create")
        self._h = h
        self._lib = lib   # held so the destructor still works during interpreter shutdown
        self.n_phrases = len(phrases)
        self.n_states = lib.wcb_bias_num_states(h)

    def __del__(self):
        if getattr(self, "_h", None) and getattr(self, "_lib", None) is not None:
            self._lib.wcb_bias_destroy(self._h)
            self._h = None


class StepDecoder:
    """One step-wise decode (WhisperCB.decode_begin). Greedy: step() -> (next ids [B] int32, scores [B] f32:
    the chosen token's logit + bias boost). Beam search (num_beams = nb > 1): step() -> (the token each
    running beam appended [B·nb] int32, the running log-prob sums [B·nb] f32), parents() -> [B·nb] int32,
    the beam (0..nb-1 of the same clip) each running beam extends. result() -> generate()'s output for the
    steps taken (beams: the best finished sequence of every clip so far). All on the model's device;
    close() ends the decode."""

    def __init__(self, model, st, B, bias, num_beams=1):
        self.model, self._st, self.B, self._bias, self.num_beams = model, st, B, bias, num_beams

    def step(self):
        m = self.model
        R = self.B * self.num_beams
        ids = torch.empty(R, dtype=torch.int32, device=m.device)
        sc = torch.empty(R, dtype=torch.float32, device=m.device)
        _lib.check(m._lib.wcb_decode_step(m._h, self._st, self._bias._h if self._bias else None, _ptr(ids), _ptr(sc),
                                          _stream(m.device)), m._h, "wcb_decode_step")
        return ids, sc

    def parents(self):
        m = self.model
        par = torch.empty(self.B * self.num_beams, dtype=torch.int32, device=m.device)
        _lib.check(m._lib.wcb_decode_parents(m._h, self._st, _ptr(par), _stream(m.device)), m._h, "wcb_decode_parents")
        return par

    def info(self):
        """(max_new, steps, done): the state's column capacity, the steps taken, and whether every utterance
        has finished (beams: the search is frozen — further steps give identity parents and pad ids)."""
        m = self.model
        mx, st, dn = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        _lib.check(m._lib.wcb_decode_info(m._h, self._st, C.byref(mx), C.byref(st), C.byref(dn)), m._h,
                   "wcb_decode_info")
        return mx.value, st.value, bool(dn.value)

    @property
    def done(self) -> bool:
        return self.info()[2]

    def result(self, max_new: Optional[int] = None):
        """[B, n] int64 ids as generate() returns them (Whisper-trimmed), n = the generated columns. The
        output width is the library's (wcb_decode_info); `max_new` is accepted for compatibility and, when
        given, must be at least the number of generated columns."""
        m = self.model
        width = self.info()[0]
        out = torch.empty(self.B, width, dtype=torch.int32, device=m.device)
        n = C.c_int32(0)
        _lib.check(m._lib.wcb_decode_result(m._h, self._st, _ptr(out), width, C.byref(n), _stream(m.device)), m._h,
                   "wcb_decode_result")
        if max_new is not None and max_new < n.value:
            raise ValueError(f"result(max_new={max_new}): {n.value} columns were generated")
        return m._whisper_trim(out[:, :n.value].to(torch.int64))

    def close(self):
        if self._st:
            _lib.check(self.model._lib.wcb_decode_end(self.model._h, self._st), self.model._h, "wcb_decode_end")
            self._st = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DecoderCache:
    """`past_key_values` of `WhisperCB.forward(..., use_cache=True)` (models/whisper_medical.py:54-55, 89-110):
    the decoder's self-attention KV cache and the encoder state, held on the device by a prefix-free step-wise
    state (wcb_decode_begin); each forward(past_key_values=cache) appends its decoder_input_ids' positions
    (wcb_forward_cached). One open cache (or StepDecoder) per model: a new use_cache=True forward closes the
    previous cache, and close() frees it."""

    def __init__(self, model: "WhisperCB", enc: torch.Tensor):
        self.model, self.encoder_last_hidden_state, self.B = model, enc, enc.shape[0]
        st = C.c_void_p()
        _lib.check(model._lib.wcb_decode_begin(model._h, _ptr(enc), self.B, 1, None, 1, 0.0, 0, C.byref(st),
                                               _stream(model.device)), model._h, "wcb_decode_begin")
        self._st = st
        self._seen = 0

    def get_seq_length(self) -> int:   # the HF Cache accessor
        return self._seen

    def extend(self, ids: torch.Tensor) -> torch.Tensor:
        m = self.model
        if not self._st:
            raise _lib.WcbError("past_key_values was closed (one open cache per model)")
        if ids.shape[0] != self.B:
            raise ValueError(f"decoder_input_ids has {ids.shape[0]} rows, the cache {self.B}")
        T = ids.shape[1]
        logits = torch.empty(self.B, T, m.dims.vocab, dtype=torch.float32, device=m.device)
        _lib.check(m._lib.wcb_forward_cached(m._h, self._st, _ptr(ids), T, _ptr(logits), _stream(m.device)),
                   m._h, "wcb_forward_cached")
        self._seen += T
        return logits

    def close(self):
        if self._st:
            _lib.check(self.model._lib.wcb_decode_end(self.model._h, self._st), self.model._h, "wcb_decode_end")
            self._st = None
            if self.model._cache is self:
                self.model._cache = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class WhisperCB:
    main_input_name = "input_features"

    def __init__(self, dims: WhisperDims, dtype: str = "bf16", device: int = 0, bias_weight: float = 10.0,
                 options: Optional[Dict[str, int]] = None):
        if not torch.cuda.is_available():
            raise _lib.WcbError("WhisperCB needs a ROCm GPU (no CPU fallback by design)")
        lib = _lib.load()
        self.dims = dims
        self.dtype_code = _lib.DTYPES[dtype]
        self.device = torch.device("cuda", device)
        self.bias_weight = bias_weight
        desc = _lib.WcbModelDesc(dims.d_model, dims.n_layers, dims.n_heads, dims.ffn, dims.vocab,
                                 dims.n_mel, dims.n_audio_ctx, dims.n_text_ctx, dims.eos_token_id,
                                 dims.pad_token_id, dims.decoder_start_token_id, self.dtype_code)
        h = C.c_void_p()
        _lib.check(lib.wcb_create(C.byref(desc), device, C.byref(h)), None, "wcb_create")
        self._h = h
        self._lib = lib
        self.config = SimpleNamespace(use_cache=True, suppress_tokens=[], forced_decoder_ids=None,
                                      decoder_start_token_id=dims.decoder_start_token_id,
                                      pad_token_id=dims.pad_token_id, eos_token_id=dims.eos_token_id,
                                      vocab_size=dims.vocab, d_model=dims.d_model,
                                      max_target_positions=dims.n_text_ctx, num_mel_bins=dims.n_mel)
        self.generation_config = SimpleNamespace(max_length=448, pad_token_id=dims.pad_token_id,
                                                 eos_token_id=dims.eos_token_id,
                                                 decoder_start_token_id=dims.decoder_start_token_id,
                                                 use_cache=True, num_beams=1, forced_decoder_ids=None)
        # device automatons of recently used bias lists (LRU: per-batch bias_spans lists would otherwise
        # accumulate one V-sized automaton per distinct batch)
        self._bias_cache: "OrderedDict[tuple, BiasList]" = OrderedDict()
        self.bias_cache_size = 8
        # automatons evicted from the LRU: destroying one waits for this handle's queued work
        # (wcb_bias_destroy drops the decode graphs that captured it), so they are kept until the next
        # synchronize() — where the streams are idle and the wait is free — instead of stalling an
        # asynchronous (block=False) generate call. Past kRetiredMax they are released anyway (one stall).
        self._bias_retired: List[BiasList] = []
        self._word_start: Optional[np.ndarray] = None
        self._loaded = False
        self._cache: Optional["DecoderCache"] = None   # the open forward(use_cache=True) state, if any
        # options last: a rejected option raises with every attribute __del__ reads already set
        for k, v in (options or {}).items():   # wcb_set_option: alternative formulations (tests)
            _lib.check(lib.wcb_set_option(h, k.encode(), int(v)), h, f"wcb_set_option({k})")

    # ------------------------------------------------------------------ construction / weights
    @classmethod
    def from_state_dict(cls, dims_or_config, state_dict, dtype: str = "bf16", device: int = 0,
                        bias_weight: float = 10.0, options: Optional[Dict[str, int]] = None) -> "WhisperCB":
        dims = dims_or_config if isinstance(dims_or_config, WhisperDims) else (
            get_dims(dims_or_config) if isinstance(dims_or_config, str) else dims_from_hf_config(dims_or_config))
        m = cls(dims, dtype=dtype, device=device, bias_weight=bias_weight, options=options)
        m.load_state_dict(state_dict)
        return m

    @classmethod
    def from_seed(cls, size: str, seed: int = 0, recipe: str = "diverse", dtype: str = "bf16",
                  device: int = 0) -> "WhisperCB":
        from .weights import make_weights
        dims = get_dims(size)
        return cls.from_state_dict(dims, make_weights(dims, seed=seed, recipe=recipe), dtype, device)

    _VIEW_DTYPES = {torch.float32: _lib.WCB_F32, torch.bfloat16: _lib.WCB_BF16, torch.float16: _lib.WCB_F16}

    def load_state_dict(self, state_dict):
        """Device tensors (this GPU; f32 / bf16 / f16, any strides) are handed over as borrowed views
        (wcb_load_weights: gathered on the device, no host round trip); host arrays go through
        wcb_set_weight. Then wcb_finalize_weights builds the device layouts."""
        views, keep = [], []
        for name, t in state_dict.items():
            if (isinstance(t, torch.Tensor) and t.is_cuda and t.device.index == self.device.index
                    and t.dtype in self._VIEW_DTYPES and 1 <= t.dim() <= 4):
                nm = name.encode()
                keep.append(nm)
                v = _lib.WcbTensorView(nm, t.data_ptr(), self._VIEW_DTYPES[t.dtype], t.dim(),
                                       (C.c_int64 * 4)(*t.shape), (C.c_int64 * 4)(*t.stride()))
                views.append((v, t))
                continue
            if isinstance(t, torch.Tensor):
                a = t.detach().to("cpu", torch.float32).contiguous().numpy()
            else:
                a = np.ascontiguousarray(t, dtype=np.float32)
            shape = (C.c_int64 * a.ndim)(*a.shape)
            _lib.check(self._lib.wcb_set_weight(self._h, name.encode(), a.ctypes.data, shape, a.ndim),
                       self._h, f"wcb_set_weight({name})")
        if views:
            arr = (_lib.WcbTensorView * len(views))(*[v for v, _ in views])
            _lib.check(self._lib.wcb_load_weights(self._h, arr, len(views), _stream(self.device)), self._h,
                       "wcb_load_weights")
        _lib.check(self._lib.wcb_finalize_weights(self._h), self._h, "wcb_finalize_weights")
        self._loaded = True
        return self

    def __del__(self):
        if getattr(self, "_h", None):
            getattr(self, "_bias_cache", {}).clear()
            self._lib.wcb_destroy(self._h)
            self._h = None

    def set_option(self, name: str, value: int) -> None:
        """wcb_set_option on this handle (alternative formulations; include/wcb.h lists them)."""
        _lib.check(self._lib.wcb_set_option(self._h, name.encode(), int(value)), self._h, f"wcb_set_option({name})")

    # reference-compatible no-ops (scripts/evaluation.py:181-183)
    def freeze_encoder(self):
        return self

    def to(self, device=None, *a, **k):
        return self

    def eval(self):
        return self

    # --------------------------------------------------------------------------- front end
    @property
    def torch_dtype(self):
        return _TORCH_DT[self.dtype_code]

    def log_mel(self, pcm) -> torch.Tensor:
        """WhisperFeatureExtractor equivalent: f32 PCM [B, N] (or [N]) → f32 mel [B, n_mel, 3000]."""
        x = torch.as_tensor(pcm, dtype=torch.float32)
        if x.dim() == 1:
            x = x[None]
        x = x.to(self.device).contiguous()
        B, N = x.shape
        out = torch.empty(B, self.dims.n_mel, 3000, dtype=torch.float32, device=self.device)
        _lib.check(self._lib.wcb_log_mel(self._h, _ptr(x), B, min(N, N_SAMPLES), N, _ptr(out),
                                         _stream(self.device)), self._h, "wcb_log_mel")
        return out

    def _features(self, input_features) -> torch.Tensor:
        x = torch.as_tensor(input_features)
        if x.dim() == 2:
            x = x[None]
        if x.shape[-1] != 3000:
            # same check as [tf] modeling_whisper.py:612-616
            raise ValueError(f"Whisper expects the mel input features to be of length 3000, but found {x.shape[-1]}")
        if x.shape[-2] != self.dims.n_mel:
            raise ValueError(f"expected {self.dims.n_mel} mel bins, got {x.shape[-2]}")
        return x.to(self.device, torch.float32).contiguous()

    def encode(self, input_features) -> torch.Tensor:
        x = self._features(input_features)
        B = x.shape[0]
        enc = torch.empty(B, self.dims.n_audio_ctx, self.dims.d_model, dtype=self.torch_dtype, device=self.device)
        _lib.check(self._lib.wcb_encode(self._h, _ptr(x), B, _ptr(enc), _stream(self.device)), self._h, "wcb_encode")
        return enc

    # ------------------------------------------------------------------------------ biasing
    @property
    def word_start(self) -> Optional[np.ndarray]:
        """[vocab] uint8 mask of the tokens a bias match may start at (None = every token)."""
        return self._word_start

    def set_word_start(self, mask) -> None:
        """Word-start gate of the bias boost: for a BPE vocabulary, True on the tokens that begin a word
        (a leading space), e.g. `[t.startswith("\u0120") for t in tokenizer.convert_ids_to_tokens(range(V))]`.
        None disables the gate. Cached automata are rebuilt."""
        if mask is not None:
            mask = np.ascontiguousarray(np.asarray(mask, dtype=bool).astype(np.uint8))
            if mask.shape != (self.dims.vocab,):
                raise ValueError(f"word_start must have shape ({self.dims.vocab},), got {mask.shape}")
        self._word_start = mask
        self._bias_cache.clear()

    def bias_list(self, phrases: Sequence[Sequence[int]]) -> BiasList:
        key = tuple(tuple(int(t) for t in p) for p in phrases)
        b = self._bias_cache.get(key)
        if b is None:
            b = BiasList(self, phrases)
            self._bias_cache[key] = b
            while len(self._bias_cache) > self.bias_cache_size:
                self._bias_retired.append(self._bias_cache.popitem(last=False)[1])
            if len(self._bias_retired) > self.kRetiredMax:
                self.synchronize()
        else:
            self._bias_cache.move_to_end(key)
        return b

    # the reference collator pads bias_spans with the literal 50256 whatever the model
    # (data_utils/data_collator.py:119-121)
    collator_span_pad = 50256

    def _spans_to_phrases(self, bias_spans) -> List[List[int]]:
        """Union of the collator's padded per-sample spans ([B, N, L], pad 50256 —
        data_utils/data_collator.py:107-125; the all-zeros [B, 1, 1] "no spans" form gives none) with
        the padding stripped."""
        pad = self.collator_span_pad
        arr = torch.as_tensor(bias_spans).cpu().numpy()
        out, seen = [], set()
        for sample in arr:
            for span in sample:
                toks = tuple(int(t) for t in span if int(t) != pad)
                if toks and any(toks) and toks not in seen:
                    seen.add(toks)
                    out.append(list(toks))
        return out

    # ---------------------------------------------------------------------------- generation
    def generate(self, input_features=None, labels=None, bias_spans=None, max_length: Optional[int] = None,
                 num_beams: Optional[int] = None, bias_list=None, bias_boost: float = 0.0,
                 min_new_tokens: int = 0, prompt_ids=None, return_dict_in_generate: bool = False,
                 generation_config=None, use_graph: bool = True, block: bool = True, **kwargs):
        """Greedy (num_beams = 1, the reference's eval setting) or HF beam
        search (num_beams = 2..8, [tf] generation/utils.py:3208) on the device.

        Returns Whisper's post-processed ids ([tf] generation_whisper.py:1063-1086, 213-225): per row
        the trailing pads and the final EOS dropped, right-padded with pad to the longest row.

        `labels` / `bias_spans` are accepted and ignored for token selection exactly like the
        reference (`[tf] trainer_seq2seq.py:310-329`), unless `bias_boost > 0` and no explicit
        `bias_list` is given — then the batch's spans form the boosted bias list.

        `block=False` (serving pipelines): the caller's stream is not made to wait for the decode, so
        the next call's front end + encoder overlap this decode; the returned ids (and the inputs)
        must be kept alive and are valid only after `synchronize()`. Only meaningful with
        `min_new_tokens >= max_length` (no early-exit polling). Beam search returns all `max_length`
        columns then (pad past each clip's best sequence: its length is not read back).
        """
        if not self._loaded:
            raise _lib.WcbError("weights not loaded")
        x_all = self._features(input_features)
        nb_req = int(num_beams if num_beams is not None else getattr(generation_config or self.generation_config,
                                                                      "num_beams", 1) or 1)
        per_call = self.max_clips_per_call(nb_req)
        if x_all.shape[0] > per_call:
            # the library takes at most 64 clips (512 decoder rows) per call: split, decode in order,
            # re-pad to the longest row (Whisper's padding of the joined output)
            kw = dict(labels=labels, bias_spans=bias_spans, max_length=max_length, num_beams=num_beams,
                      bias_list=bias_list, bias_boost=bias_boost, min_new_tokens=min_new_tokens,
                      prompt_ids=prompt_ids, return_dict_in_generate=return_dict_in_generate,
                      generation_config=generation_config, use_graph=use_graph, block=True)
            if bias_list is None and bias_boost > 0 and bias_spans is not None:
                kw["bias_list"], kw["bias_spans"] = self._spans_to_phrases(bias_spans), None
            parts = [self.generate(x_all[i:i + per_call], **kw) for i in range(0, x_all.shape[0], per_call)]
            seqs = [p.sequences if return_dict_in_generate else p for p in parts]
            Wd = max(t.shape[1] for t in seqs)
            fill = self.dims.pad_token_id
            out = torch.cat([torch.nn.functional.pad(t, (0, Wd - t.shape[1]), value=fill) for t in seqs])
            return GenerateOutput(sequences=out) if return_dict_in_generate else out
        gc = generation_config or self.generation_config
        max_length = int(max_length if max_length is not None else getattr(gc, "max_length", 448))
        num_beams = int(num_beams if num_beams is not None else getattr(gc, "num_beams", 1) or 1)
        if not 1 <= num_beams <= 8:
            raise ValueError("num_beams must be in [1, 8]")
        x = x_all
        B = x.shape[0]
        prefix = [self.dims.decoder_start_token_id]
        if prompt_ids is not None:
            prefix = [int(t) for t in prompt_ids] + prefix
        # HF: max_length + prompt tokens, capped at max_target_positions ([tf] generation_whisper.py:1932-1940)
        max_new = min(max_length, self.dims.n_text_ctx - len(prefix))
        if max_new < 1:
            raise ValueError("prompt leaves no room for new tokens")
        phrases = bias_list
        if phrases is None and bias_boost > 0 and bias_spans is not None:
            phrases = self._spans_to_phrases(bias_spans)
        if isinstance(phrases, BiasList):          # a prebuilt automaton (it must belong to this model)
            bl = phrases if bias_boost > 0 else None
        else:
            bl = self.bias_list(phrases) if (phrases and bias_boost > 0) else None
        cfg = _lib.WcbGenCfg(max_new, int(min_new_tokens), num_beams, float(bias_boost), int(use_graph), int(not block))
        out = torch.empty(B, max_new, dtype=torch.int32, device=self.device)
        steps = C.c_int32(0)
        pre = np.asarray(prefix, dtype=np.int32)
        _lib.check(self._lib.wcb_generate(self._h, _ptr(x), B, C.byref(cfg), bl._h if bl else None,
                                          pre.ctypes.data if len(prefix) > 1 else None, len(prefix),
                                          _ptr(out), C.byref(steps), _stream(self.device)),
                   self._h, "wcb_generate")
        if not block:
            return out[:, :steps.value]            # int32, valid after synchronize()
        ids = out[:, :steps.value].to(torch.int64)
        if return_dict_in_generate:
            sot = torch.tensor(prefix, dtype=torch.int64, device=self.device)[None].expand(B, -1)
            return GenerateOutput(sequences=torch.cat([sot, ids], dim=1))
        return self._whisper_trim(ids)

    def decode_begin(self, encoder_outputs, prompt_ids=None, bias_list=None, bias_boost: float = 0.0,
                     min_new_tokens: int = 0, num_beams: int = 1, max_length: Optional[int] = None) -> "StepDecoder":
        """Step-wise decoding from an encoder output [B, 1500, d] (this model's dtype, on its device): the
        streaming form of generate() (wcb_decode_begin / wcb_decode_begin_beams). Greedy (num_beams = 1) or
        beam search (num_beams 2..8; `max_length` = generate()'s, the beams' length cap: None = the
        max_target_positions cap). `prompt_ids` = one prompt for every clip or a [B, P] array of per-clip
        prompts (decoder_start_token_id is appended as generate() does)."""
        enc = self._encoder_state(encoder_outputs)   # [B, 1500, d] checked: the library copies B·1500·d
        B = enc.shape[0]
        if B > 64:
            raise ValueError("decode_begin takes at most 64 clips")
        start = self.dims.decoder_start_token_id
        if prompt_ids is None:
            pre = None
        else:
            p = np.asarray(prompt_ids, dtype=np.int32)
            if p.ndim == 1:
                p = np.broadcast_to(p, (B, p.shape[-1]))
            elif p.ndim != 2 or p.shape[0] != B:
                raise ValueError(f"prompt_ids must be one prompt or a [{B}, P] array, got shape {p.shape}")
            pre = np.ascontiguousarray(np.concatenate([p, np.full((B, 1), start, np.int32)], axis=1))
        if isinstance(bias_list, BiasList):   # a prebuilt automaton, as generate() accepts
            bl = bias_list if bias_boost > 0 else None
        else:
            bl = self.bias_list(bias_list) if (bias_list and bias_boost > 0) else None
        st = C.c_void_p()
        nb = int(num_beams)
        if nb > 1 and max_length is not None:
            _lib.check(self._lib.wcb_decode_begin_beams(self._h, _ptr(enc), B, nb, pre.ctypes.data if pre is not None else None,
                                                        pre.shape[1] if pre is not None else 1, int(max_length),
                                                        float(bias_boost), int(min_new_tokens), C.byref(st),
                                                        _stream(self.device)), self._h, "wcb_decode_begin_beams")
        else:
            _lib.check(self._lib.wcb_decode_begin(self._h, _ptr(enc), B, nb, pre.ctypes.data if pre is not None else None,
                                                  pre.shape[1] if pre is not None else 1, float(bias_boost),
                                                  int(min_new_tokens), C.byref(st), _stream(self.device)), self._h,
                       "wcb_decode_begin")
        return StepDecoder(self, st, B, bl, nb)

    @staticmethod
    def max_clips_per_call(num_beams: int = 1) -> int:
        """Clips one wcb_generate call takes (64, and at most 512 decoder rows = clips x beams)."""
        return max(1, min(64, 512 // max(1, int(num_beams))))

    def _whisper_trim(self, ids: torch.Tensor) -> torch.Tensor:
        """Whisper's short-form post-processing ([tf] generation_whisper.py:1063-1086, then
        _pad_to_max_length :213-225): per row drop the pads (all but one when pad == eos) and the
        final EOS, then right-pad every row with pad to the longest one."""
        eos, pad = self.dims.eos_token_id, self.dims.pad_token_id
        rows = ids.cpu().numpy()
        lens = []
        for r in rows:
            n = len(r)
            if n and r[-1] == pad:
                n -= int((r == pad).sum()) - (1 if pad == eos else 0)
            if n and r[n - 1] == eos:
                n -= 1
            lens.append(n)
        W = max(lens, default=0)
        out = ids[:, :W].clone()
        for i, n in enumerate(lens):
            if n < W:
                out[i, n:] = pad
        return out

    kRetiredMax = 32

    def synchronize(self):
        """Wait for every queued front-end / encoder / decode operation of this model (and release the
        bias automatons evicted since the last call, now that no queued work reads them)."""
        _lib.check(self._lib.wcb_synchronize(self._h), self._h, "wcb_synchronize")
        self._bias_retired.clear()

    # ------------------------------------------------------------------------------- forward
    # forward() arguments of the reference signature (models/whisper_medical.py:45-65) that change nothing here:
    # Whisper's encoder ignores attention_mask, and return_dict / output flags left at their defaults
    _FORWARD_NOOP = {"attention_mask": None, "output_attentions": (None, False), "output_hidden_states": (None, False),
                     "cache_position": None, "decoder_attention_mask": None}

    def _encoder_state(self, encoder_outputs) -> torch.Tensor:
        """encoder_outputs as HF accepts it: a BaseModelOutput, a tuple whose [0] is the last hidden state
        ([tf] modeling_whisper.py WhisperModel.forward), or that tensor; [B, 1500, d], cast to the model dtype."""
        e = getattr(encoder_outputs, "last_hidden_state", None)
        if e is None:
            e = encoder_outputs[0] if isinstance(encoder_outputs, (tuple, list)) else encoder_outputs
        e = torch.as_tensor(e)
        if e.dim() == 2:
            e = e[None]
        if tuple(e.shape[1:]) != (self.dims.n_audio_ctx, self.dims.d_model):
            raise ValueError(f"encoder_outputs must be [B, {self.dims.n_audio_ctx}, {self.dims.d_model}], "
                             f"got {tuple(e.shape)}")
        return e.to(self.device, self.torch_dtype).contiguous()

    def forward(self, input_features=None, decoder_input_ids=None, labels=None, bias_spans=None,
                encoder_outputs=None, past_key_values=None, use_cache=None, return_dict: bool = True,
                **kwargs) -> Seq2SeqLMOutput:
        """Teacher-forced decoder logits (models/whisper_medical.py:45-172): from `input_features` (encoded
        here), from a given `encoder_outputs` (not re-encoded: bit-identical logits), or continuing a
        `past_key_values` cache. `use_cache=True` returns the cache as `.past_key_values` (a DecoderCache:
        one open per model); the default keeps none. The reference's weighted-CE `.loss` with `labels`."""
        for k, v in kwargs.items():
            ok = self._FORWARD_NOOP.get(k, "missing")
            if ok == "missing" or (v is not None and not (isinstance(ok, tuple) and v in ok)):
                raise NotImplementedError(f"forward(): argument {k}={v!r} is not supported by this path")
        if labels is not None:
            labels = torch.as_tensor(labels)
            if labels.shape[1] > self.dims.n_text_ctx:
                raise ValueError(f"Labels' sequence length {labels.shape[1]} cannot exceed the maximum allowed "
                                 f"length of {self.dims.n_text_ctx} tokens.")
            if decoder_input_ids is None:
                # shift_tokens_right ([tf] modeling_whisper.py:67-80)
                dec = torch.full_like(labels, self.dims.pad_token_id)
                dec[:, 1:] = labels[:, :-1].clone()
                dec[:, 0] = self.dims.decoder_start_token_id
                dec[dec == -100] = self.dims.pad_token_id
                decoder_input_ids = dec
        if decoder_input_ids is None:
            raise ValueError("forward() needs decoder_input_ids (or labels)")
        ids = torch.as_tensor(decoder_input_ids).to(self.device, torch.int32).contiguous()

        def out(logits, enc, cache=None):
            loss = None
            if labels is not None:
                from .loss import weighted_ce
                loss = weighted_ce(logits, labels.to(self.device), bias_spans, self.bias_weight)
            return Seq2SeqLMOutput(loss=loss, logits=logits, encoder_last_hidden_state=enc, past_key_values=cache)

        if past_key_values is not None:   # continue a cache: logits of the new positions only
            if not isinstance(past_key_values, DecoderCache) or past_key_values.model is not self:
                raise TypeError("past_key_values must be the DecoderCache this model returned (use_cache=True)")
            return out(past_key_values.extend(ids), past_key_values.encoder_last_hidden_state, past_key_values)
        if input_features is None and encoder_outputs is None:
            raise ValueError("You have to specify either input_features or encoder_outputs")
        if use_cache:
            enc = self._encoder_state(encoder_outputs) if encoder_outputs is not None else self.encode(input_features)
            if enc.shape[0] > 64:
                raise ValueError("use_cache=True takes at most 64 clips per cache")
            if self._cache is not None:
                self._cache.close()
            self._cache = DecoderCache(self, enc)
            return out(self._cache.extend(ids), enc, self._cache)
        if encoder_outputs is not None:
            enc = self._encoder_state(encoder_outputs)
            B, T = ids.shape
            if enc.shape[0] != B:
                raise ValueError(f"encoder_outputs has {enc.shape[0]} clips, decoder_input_ids {B} rows")
            logits = torch.empty(B, T, self.dims.vocab, dtype=torch.float32, device=self.device)
            for i in range(0, B, 64):   # 64 clips per library call
                n = min(64, B - i)
                _lib.check(self._lib.wcb_forward_enc(self._h, _ptr(enc[i:i + n]), n, _ptr(ids[i:i + n]), T,
                                                     _ptr(logits[i:i + n]), _stream(self.device)),
                           self._h, "wcb_forward_enc")
            return out(logits, enc)
        x = self._features(input_features)
        if x.shape[0] > 64:   # 64 clips per library call: split, concatenate
            outs = [self.forward(x[i:i + 64], decoder_input_ids=ids[i:i + 64]) for i in range(0, x.shape[0], 64)]
            return out(torch.cat([o.logits for o in outs]), torch.cat([o.encoder_last_hidden_state for o in outs]))
        B, T = ids.shape
        logits = torch.empty(B, T, self.dims.vocab, dtype=torch.float32, device=self.device)
        enc = torch.empty(B, self.dims.n_audio_ctx, self.dims.d_model, dtype=self.torch_dtype, device=self.device)
        _lib.check(self._lib.wcb_forward(self._h, _ptr(x), B, _ptr(ids), T, _ptr(logits), _ptr(enc),
                                         _stream(self.device)), self._h, "wcb_forward")
        return out(logits, enc)

    __call__ = forward

    # ---------------------------------------------------------------------------- profiling
    def profile_enable(self, on: bool = True, events: bool = True, stamps: bool = True):
        """HIP-event timing of front-end/encoder launches (`events`) and device-stamped timing of the
        decode cross-attention graph nodes (`stamps`); counters reset."""
        mode = (int(events) | (int(stamps) << 1)) if on else 0
        _lib.check(self._lib.wcb_profile_enable(self._h, mode), self._h, "wcb_profile_enable")

    def profile_read(self) -> Dict[str, dict]:
        n = 64
        names = (C.c_char * 32 * n)()
        launches = (C.c_int64 * n)()
        ms = (C.c_double * n)()
        flops = (C.c_double * n)()
        byts = (C.c_double * n)()
        cnt = _lib.check(self._lib.wcb_profile_read(self._h, n, names, launches, ms, flops, byts), self._h,
                         "wcb_profile_read")
        out = {}
        for i in range(min(cnt, n)):
            nm = bytes(names[i]).split(b"\0", 1)[0].decode()
            kname = C.create_string_buffer(512)
            grid = C.c_int64(0)
            _lib.check(self._lib.wcb_profile_kernel(self._h, i, kname, 512, C.byref(grid)), self._h,
                       "wcb_profile_kernel")
            out[nm] = dict(launches=launches[i], ms=ms[i], flops=flops[i], bytes=byts[i],
                           kernel=kname.value.decode(errors="replace"), grid=grid.value)
        return out
