"""Stage-by-stage comparison of the HIP encoder with the numpy oracle (GPU debugging aid)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import whisper_np as W  # noqa: E402
from whisper_context_biasing_amd import _lib  # noqa: E402
from whisper_context_biasing_amd.config import get_dims  # noqa: E402
from whisper_context_biasing_amd.model import WhisperCB  # noqa: E402
from whisper_context_biasing_amd.synth import synth_batch  # noqa: E402
from whisper_context_biasing_amd.weights import make_weights  # noqa: E402


def dbg(m, name, shape, dtype, layers=-1):
    t = torch.empty(*shape, dtype=dtype, device="cuda")
    _lib.check(m._lib.wcb_debug_copy(m._h, name.encode(), t.data_ptr(), t.numel() * t.element_size(), layers), m._h)
    return t.float().cpu().numpy()


def main(size="micro", dtype="f32"):
    dims = get_dims(size)
    sd = make_weights(dims, seed=0)
    om = W.OracleModel.from_dims(dims, sd)
    m = WhisperCB.from_state_dict(dims, sd, dtype=dtype)
    B, d, nm = 2, dims.d_model, dims.n_mel
    mel = W.log_mel(synth_batch(B), nm)
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dtype]
    # conv stem only
    m._lib.wcb_debug_copy(m._h, b"x", None, 0, 0)
    m.encode(torch.from_numpy(mel))
    torch.cuda.synchronize()
    xt = dbg(m, "xt", (B, 3002, nm), tdt, 0)
    ref_xt = np.zeros((B, 3002, nm), np.float32)
    ref_xt[:, 1:3001] = mel.transpose(0, 2, 1)
    print("xt maxdiff", np.abs(xt - ref_xt).max())
    c1 = W.gelu(W.conv1d(mel, sd["model.encoder.conv1.weight"], sd["model.encoder.conv1.bias"]))   # B,d,3000
    hb = dbg(m, "hbuf", (B, 3001, d), tdt, 0)
    print("hbuf row0 max", np.abs(hb[:, 0]).max(), "conv1 maxdiff", np.abs(hb[:, 1:] - c1.transpose(0, 2, 1)).max(),
          "ref max", np.abs(c1).max())
    c2 = W.gelu(W.conv1d(c1, sd["model.encoder.conv2.weight"], sd["model.encoder.conv2.bias"], stride=2))
    x0 = c2.transpose(0, 2, 1) + sd["model.encoder.embed_positions.weight"][None]
    x = dbg(m, "x", (B, 1500, d), torch.float32, 0)
    print("x (conv2+pos) maxdiff", np.abs(x - x0).max(), "ref max", np.abs(x0).max())
    # first layer pieces
    p = "model.encoder.layers.0."
    h = W.layer_norm(x0, sd[p + "self_attn_layer_norm.weight"], sd[p + "self_attn_layer_norm.bias"])
    m._lib.wcb_debug_copy(m._h, b"x", None, 0, 1)
    m.encode(torch.from_numpy(mel))
    torch.cuda.synchronize()
    q = (W.linear(h, sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.q_proj.bias"]) * 0.125)
    k = W.linear(h, sd[p + "self_attn.k_proj.weight"])
    v = W.linear(h, sd[p + "self_attn.v_proj.weight"], sd[p + "self_attn.v_proj.bias"])
    qkv = dbg(m, "qkv", (B, 1500, 3 * d), tdt, 1)
    print("q maxdiff", np.abs(qkv[..., :d] - q).max(), "k", np.abs(qkv[..., d:2 * d] - k).max(),
          "v", np.abs(qkv[..., 2 * d:] - v).max())
    a = om._attn(p + "self_attn.", h, h)
    x1 = x0 + a
    h2 = W.layer_norm(x1, sd[p + "final_layer_norm.weight"], sd[p + "final_layer_norm.bias"])
    f = W.gelu(W.linear(h2, sd[p + "fc1.weight"], sd[p + "fc1.bias"]))
    ffn = dbg(m, "ffn", (B, 1500, dims.ffn), tdt, 1)
    print("ffn maxdiff", np.abs(ffn - f).max(), "ref max", np.abs(f).max())
    x2 = x1 + W.linear(f, sd[p + "fc2.weight"], sd[p + "fc2.bias"])
    xg = dbg(m, "x", (B, 1500, d), torch.float32, 1)
    print("x after layer0 maxdiff", np.abs(xg - x2).max(), "ref max", np.abs(x2).max())
    m._lib.wcb_debug_copy(m._h, b"x", None, 0, -1)
    enc = m.encode(torch.from_numpy(mel)).float().cpu().numpy()
    print("enc maxdiff", np.abs(enc - om.encode(mel)).max())


if __name__ == "__main__":
    main(*sys.argv[1:])
