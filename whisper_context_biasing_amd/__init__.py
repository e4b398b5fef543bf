"""MI355X-native Whisper contextual-biasing inference path (hot path of thanh-nt25/Whisper-context-biasing).

Hand-written HIP kernels for gfx950 in `csrc/`, built into `libwcb.so` (C ABI: include/wcb.h).
`WhisperCB` (model.py) is the drop-in for the reference model's generate()/forward() surface.
"""
# The library runs one encoder stream and two decode streams beside the caller's stream. Round 2
# measured the C2 benchmark at GPU_MAX_HW_QUEUES = 4 (the HIP default), 5, 6, 8 and 16: 14,818-14,966
# audio-s/s, i.e. no dependence on the hardware-queue count, so nothing is set here (round 1 set 16
# before HIP initialised, which silently did nothing when torch initialised HIP first).

from .config import MODELS, WhisperDims, get_dims  # noqa: E402,F401

__all__ = ["MODELS", "WhisperDims", "get_dims", "WhisperCB"]


def __getattr__(name):
    if name == "WhisperCB":
        from .model import WhisperCB
        return WhisperCB
    raise AttributeError(name)
