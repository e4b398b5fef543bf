"""MI355X-native Whisper contextual-biasing inference path (hot path of thanh-nt25/Whisper-context-biasing).

Hand-written HIP kernels for gfx950 in `csrc/`, built into `libwcb.so` (C ABI: include/wcb.h).
`WhisperCB` (model.py) is the drop-in for the reference model's generate()/forward() surface.
"""
from .config import MODELS, WhisperDims, get_dims  # noqa: F401

__all__ = ["MODELS", "WhisperDims", "get_dims", "WhisperCB"]


def __getattr__(name):
    if name == "WhisperCB":
        from .model import WhisperCB
        return WhisperCB
    raise AttributeError(name)
