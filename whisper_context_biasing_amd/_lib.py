"""ctypes binding of libwcb.so (C ABI: include/wcb.h).

The library is the ONLY compute path: if it is missing or fails to load, every product entry point
raises — there is no CPU fallback (the numpy oracle lives under /oracle and is test-only).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libwcb.so")
CSRC = os.path.join(_HERE, "csrc")

WCB_BF16, WCB_F16, WCB_F32 = 0, 1, 2
DTYPES = {"bf16": WCB_BF16, "f16": WCB_F16, "fp16": WCB_F16, "f32": WCB_F32, "fp32": WCB_F32}


class WcbModelDesc(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "d_model", "n_layers", "n_heads", "ffn", "vocab", "n_mel", "n_audio_ctx", "n_text_ctx",
        "eos_token_id", "pad_token_id", "decoder_start_token_id", "dtype")]


class WcbGenCfg(C.Structure):
    _fields_ = [("max_new_tokens", C.c_int), ("min_new_tokens", C.c_int), ("num_beams", C.c_int),
                ("bias_boost", C.c_float), ("use_graph", C.c_int), ("async_out", C.c_int)]


class WcbTensorView(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data", C.c_void_p), ("dtype", C.c_int), ("ndim", C.c_int),
                ("shape", C.c_int64 * 4), ("stride", C.c_int64 * 4)]


# name -> (restype, argtypes)
_P = C.c_void_p
SIGNATURES = {
    "wcb_create": (C.c_int, [C.POINTER(WcbModelDesc), C.c_int, C.POINTER(_P)]),
    "wcb_destroy": (None, [_P]),
    "wcb_last_error": (C.c_char_p, [_P]),
    "wcb_set_weight": (C.c_int, [_P, C.c_char_p, _P, C.POINTER(C.c_int64), C.c_int]),
    "wcb_load_weights": (C.c_int, [_P, C.POINTER(WcbTensorView), C.c_int, _P]),
    "wcb_finalize_weights": (C.c_int, [_P]),
    "wcb_log_mel": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int64, _P, _P]),
    "wcb_encode": (C.c_int, [_P, _P, C.c_int, _P, _P]),
    "wcb_generate": (C.c_int, [_P, _P, C.c_int, C.POINTER(WcbGenCfg), _P, _P, C.c_int, _P,
                               C.POINTER(C.c_int32), _P]),
    "wcb_synchronize": (C.c_int, [_P]),
    "wcb_decode_begin": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_float, C.c_int, C.POINTER(_P), _P]),
    "wcb_decode_step": (C.c_int, [_P, _P, _P, _P, _P, _P]),
    "wcb_decode_end": (C.c_int, [_P, _P]),
    "wcb_decode_begin_beams": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.c_float, C.c_int,
                                         C.POINTER(_P), _P]),
    "wcb_decode_parents": (C.c_int, [_P, _P, _P, _P]),
    "wcb_decode_info": (C.c_int, [_P, _P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "wcb_decode_result": (C.c_int, [_P, _P, _P, C.c_int, C.POINTER(C.c_int32), _P]),
    "wcb_forward": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, _P, _P, _P]),
    "wcb_forward_enc": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, _P, _P]),
    "wcb_forward_cached": (C.c_int, [_P, _P, _P, C.c_int, _P, _P]),
    "wcb_bias_create": (C.c_int, [_P, _P, _P, C.c_int, _P, C.POINTER(_P)]),
    "wcb_bias_destroy": (None, [_P]),
    "wcb_bias_num_states": (C.c_int, [_P]),
    "wcb_debug_copy": (C.c_int, [_P, C.c_char_p, _P, C.c_int64, C.c_int]),
    "wcb_profile_enable": (C.c_int, [_P, C.c_int]),
    "wcb_profile_read": (C.c_int, [_P, C.c_int, _P, _P, _P, _P, _P]),
    "wcb_profile_kernel": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int64)]),
    "wcb_op_gemm": (C.c_int, [C.c_int, _P, _P, C.c_int, C.c_int, C.c_int, _P, C.c_int, _P, _P,
                              C.c_int, _P]),
    "wcb_op_gemm_kernel": (C.c_int, [C.c_int, _P, _P, C.c_int, C.c_int, C.c_int, _P, C.c_int, _P, _P,
                                     C.c_int, C.c_int, _P]),
    "wcb_op_gemm_ln": (C.c_int, [C.c_int, _P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int, _P, C.c_int, _P,
                                 C.c_int, _P]),
    "wcb_op_weighted_ce": (C.c_int, [_P, C.c_long, C.c_int, C.c_int, C.c_int, _P, _P, _P, C.c_int, C.c_int,
                                     C.c_float, _P, _P, _P, _P]),
    "wcb_wer_counts": (C.c_int, [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_int,
                                 C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_int]),
    "wcb_bias_counts": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(C.c_char_p), C.c_int,
                                  C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "wcb_op_layernorm": (C.c_int, [C.c_int, _P, _P, _P, _P, C.c_int, C.c_int, _P]),
    "wcb_op_attention_decode": (C.c_int, [C.c_int, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                          _P]),
    "wcb_op_attention": (C.c_int, [C.c_int, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, _P]),
    "wcb_op_cross_attention_enc": (C.c_int, [C.c_int, _P, _P, _P, _P, _P, _P, C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.c_int, _P]),
    "wcb_set_option": (C.c_int, [_P, C.c_char_p, C.c_int]),
}


class WcbError(RuntimeError):
    pass


class WcbArgError(WcbError, ValueError):
    """WCB_ERR_ARG: the reference raises ValueError for these (e.g. whisper_medical.py:87-90)."""


_lib = None


def build(force: bool = False, jobs: int = 8) -> str:
    """Compile libwcb.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", CSRC, f"-j{jobs}"], check=True)
    return LIB_PATH


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise WcbError(f"libwcb.so not found at {LIB_PATH}; build it with "
                       f"`make -C {CSRC}` (no CPU fallback exists)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, handle=None, what: str = ""):
    if rc < 0:
        lib = load()
        msg = lib.wcb_last_error(handle)
        cls = WcbArgError if rc == -1 else WcbError
        raise cls(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc
