"""MI355X-native Whisper contextual-biasing inference path (hot path of thanh-nt25/Whisper-context-biasing).

Hand-written HIP kernels for gfx950 in `csrc/`, built into `libwcb.so` (C ABI: include/wcb.h).
`WhisperCB` (model.py) is the drop-in for the reference model's generate()/forward() surface.
"""
import os

# The library runs the encoder stream and two decode streams concurrently (plus the caller's stream);
# HIP multiplexes streams onto GPU_MAX_HW_QUEUES hardware queues (default 4), and streams sharing a
# queue serialise against each other. Measured on MI355X: 4 or 8 queues cost 35-55 % of throughput.
# The variable is read when the HIP runtime initialises, so it is set here, before any GPU call,
# unless the user chose a value.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

from .config import MODELS, WhisperDims, get_dims  # noqa: E402,F401

__all__ = ["MODELS", "WhisperDims", "get_dims", "WhisperCB"]


def __getattr__(name):
    if name == "WhisperCB":
        from .model import WhisperCB
        return WhisperCB
    raise AttributeError(name)
