"""GPU: kernel-level parity of libwcb entry points (wcb_op_*, wcb_log_mel) against fp32/fp64
references of the same op. Tolerances are written per test."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from whisper_context_biasing_amd import _lib  # noqa: E402

DT = {"bf16": (torch.bfloat16, _lib.WCB_BF16), "f16": (torch.float16, _lib.WCB_F16), "f32": (torch.float32, _lib.WCB_F32)}


def _s():
    return torch.cuda.current_stream().cuda_stream


def _gemm(dt, A, W, bias=None, act=0, resid=None, out_f32=True):
    lib = _lib.load()
    M, K = A.shape
    N = W.shape[0]
    out = torch.empty(M, N, device="cuda", dtype=torch.float32 if out_f32 else A.dtype)
    _lib.check(lib.wcb_op_gemm(DT[dt][1], A.data_ptr(), W.data_ptr(), M, N, K,
                               bias.data_ptr() if bias is not None else None, act,
                               resid.data_ptr() if resid is not None else None, out.data_ptr(),
                               int(out_f32), _s()), None, "gemm")
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("dt", ["bf16", "f16", "f32"])
@pytest.mark.parametrize("shape", [(256, 256, 256), (300, 192, 512), (16, 2304, 768), (40, 1000, 384),
                                   (1500, 768, 768), (3, 51864, 384)])
def test_gemm_matches_fp64(dt, shape):
    M, N, K = shape
    if dt == "f32" and K % 32:
        pytest.skip()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g).to(DT[dt][0]).cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(DT[dt][0]).cuda()
    bias = torch.randn(N, generator=g).float().cuda()
    out = _gemm(dt, A, W, bias=bias)
    ref = A.double() @ W.double().T + bias.double()
    scale = (A.double().abs() @ W.double().abs().T) + 1.0
    # exact products, f32 accumulation: error bounded by ~K·2^-24 relative to Σ|a·b|
    err = ((out.double() - ref).abs() / scale).max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("dt", ["bf16", "f32"])
def test_gemm_epilogues(dt):
    M, N, K = 384, 256, 256
    g = torch.Generator(device="cpu").manual_seed(3)
    A = torch.randn(M, K, generator=g).to(DT[dt][0]).cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(DT[dt][0]).cuda()
    bias = torch.randn(N, generator=g).float().cuda()
    resid = torch.randn(M, N, generator=g).float().cuda()
    ref = A.double() @ W.double().T + bias.double()
    gel = torch.nn.functional.gelu(ref)
    out = _gemm(dt, A, W, bias=bias, act=1)
    assert (out.double() - gel).abs().max().item() < 1e-4
    out = _gemm(dt, A, W, bias=bias, resid=resid.clone())
    assert (out.double() - (ref + resid.double())).abs().max().item() < 1e-4
    out = _gemm(dt, A, W, bias=bias, act=1, out_f32=False)
    # f32: erff vs fp64 erf; bf16: one output rounding (2^-8 relative)
    tol = 1e-5 if dt == "f32" else 8e-3
    assert ((out.double() - gel).abs() - tol * gel.abs()).max().item() < 2e-5


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("d", [64, 384, 768, 1280])
def test_layernorm(dt, d):
    lib = _lib.load()
    M = 77
    x = (torch.randn(M, d) * 3 + 1).float().cuda()
    w = torch.randn(d).float().cuda()
    b = torch.randn(d).float().cuda()
    y = torch.empty(M, d, dtype=DT[dt][0], device="cuda")
    _lib.check(lib.wcb_op_layernorm(DT[dt][1], x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), M, d, _s()))
    torch.cuda.synchronize()
    ref = torch.nn.functional.layer_norm(x.double(), (d,), w.double(), b.double(), eps=1e-5)
    tol = 1e-5 if dt == "f32" else 1e-2
    assert ((y.double() - ref).abs() / (ref.abs() + 1)).max().item() < tol


def _attn(dt, q, k, v, flash):
    lib = _lib.load()
    B, Sq, D = q.shape
    Sk = k.shape[1]
    H = D // 64
    o = torch.empty_like(q)
    _lib.check(lib.wcb_op_attention(DT[dt][1], q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, Sq,
                                    Sk, int(flash), _s()), None, "attention")
    torch.cuda.synchronize()
    return o


def _attn_ref(q, k, v):
    B, Sq, D = q.shape
    H = D // 64
    qh = q.double().view(B, Sq, H, 64).transpose(1, 2)
    kh = k.double().view(B, -1, H, 64).transpose(1, 2)
    vh = v.double().view(B, -1, H, 64).transpose(1, 2)
    p = torch.softmax(qh @ kh.transpose(-1, -2), -1)
    return (p @ vh).transpose(1, 2).reshape(B, Sq, D)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("S", [1500, 200, 64])
def test_flash_attention(dt, S):
    g = torch.Generator(device="cpu").manual_seed(S)
    B, H = 2, 3
    q = (torch.randn(B, S, H * 64, generator=g) * 0.3).to(DT[dt][0]).cuda()
    k = torch.randn(B, S, H * 64, generator=g).to(DT[dt][0]).cuda()
    v = torch.randn(B, S, H * 64, generator=g).to(DT[dt][0]).cuda()
    o = _attn(dt, q, k, v, True)
    ref = _attn_ref(q, k, v)
    # P is rounded to the 16-bit type before P·V: |err| ≲ 2^-8 relative for bf16
    tol = 1e-2 if dt == "bf16" else 2e-3
    assert (o.double() - ref).abs().max().item() < tol
    o4 = _attn(dt, q, k, v, 100)   # 64 queries per wave (encoder option enc_flash = 4)
    assert (o4.double() - ref).abs().max().item() < tol


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("qscale", [0.3, 1.0])
def test_flash_attention_moving_max(dt, qscale):
    """Key norms growing along the sequence: the row maxima keep rising tile after tile, so the online
    softmax rescales the accumulators often and late; both encoder tilings (64 / 32 queries per wave)
    against fp64."""
    g = torch.Generator(device="cpu").manual_seed(int(qscale * 10))
    B, H, S = 2, 2, 1500
    ramp = (0.2 + 3.0 * torch.arange(S, dtype=torch.float32) / S).view(1, S, 1)
    q = (torch.randn(B, S, H * 64, generator=g) * qscale).to(DT[dt][0]).cuda()
    k = (torch.randn(B, S, H * 64, generator=g) * ramp).to(DT[dt][0]).cuda()
    v = torch.randn(B, S, H * 64, generator=g).to(DT[dt][0]).cuda()
    ref = _attn_ref(q, k, v)
    # peaked rows: outputs reach |v| ~ 4, so the bound is relative — the 16-bit P (2^-9 per term) and
    # the 16-bit output (2^-9) with 4x headroom; a wrong rescale is off by O(1)
    c = 2.0 ** -6 if dt == "bf16" else 2.0 ** -9
    for code in (100, 1):
        o = _attn(dt, q, k, v, code)
        assert torch.isfinite(o.float()).all()
        err = (o.double() - ref).abs() / (ref.abs() + 0.25)
        assert err.max().item() < c, (code, err.max().item())


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("B,H,Sq,Sk", [(3, 16, 5, 1500), (2, 20, 5, 1500), (4, 6, 2, 1500), (2, 4, 8, 777),
                                       (1, 2, 16, 64), (2, 3, 17, 1500)])
@pytest.mark.parametrize("split", [1, 4, 7, "beam", "beam8", "beam9"])
def test_flash_attention_query_groups(dt, B, H, Sq, Sk, split):
    """A few query rows per K/V set (beam search: the nb beams of a clip against its cross K/V, one
    K/V pass per (clip, head); Sq <= 16 takes the 16-queries-per-wave instance, optionally over
    `split` key ranges merged in a fixed order, or — "beam", the runtime default — the beam kernel whose
    4 waves split the keys and merge in the workgroup) vs fp64."""
    if isinstance(split, int) and split > 1 and Sq > 16:
        pytest.skip("key split is the few-query form")
    g = torch.Generator(device="cpu").manual_seed(B * 1000 + Sq * 10 + H)
    q = (torch.randn(B, Sq, H * 64, generator=g) * 0.3).to(DT[dt][0]).cuda()
    k = torch.randn(B, Sk, H * 64, generator=g).to(DT[dt][0]).cuda()
    v = torch.randn(B, Sk, H * 64, generator=g).to(DT[dt][0]).cuda()
    code = {"beam": 200, "beam8": 201, "beam9": 202}[split] if isinstance(split, str) else (1 if split == 1 else -split)
    if str(split).startswith("beam") and Sq > 16:
        pytest.skip("the beam kernel takes <= 16 queries")
    o = _attn(dt, q, k, v, code)
    tol = 1e-2 if dt == "bf16" else 2e-3
    assert (o.double() - _attn_ref(q, k, v)).abs().max().item() < tol
    assert torch.equal(_attn(dt, q, k, v, code), o)   # deterministic


@pytest.mark.parametrize("code", [1, 100])
def test_flash_attention_xcd_grouped(code):
    """B·H % 8 == 0 (the C2 / C3 / C5 encoder batches): the query blocks of one
    (clip, head) are mapped to one XCD (1-D grid). Same results as the fp64 reference, deterministic."""
    g = torch.Generator(device="cpu").manual_seed(11 + code)
    B, H, S = 4, 6, 1500
    q = (torch.randn(B, S, H * 64, generator=g) * 0.3).bfloat16().cuda()
    k = torch.randn(B, S, H * 64, generator=g).bfloat16().cuda()
    v = torch.randn(B, S, H * 64, generator=g).bfloat16().cuda()
    o = _attn("bf16", q, k, v, code)
    assert (o.double() - _attn_ref(q, k, v)).abs().max().item() < 1e-2
    assert torch.equal(_attn("bf16", q, k, v, code), o)


def test_flash_attention_spike():
    """Force the online-softmax rescale: one key dominates late in the sequence."""
    B, H, S = 1, 1, 1500
    g = torch.Generator(device="cpu").manual_seed(5)
    q = torch.randn(B, S, 64, generator=g).bfloat16().cuda() * 0.2
    k = torch.randn(B, S, 64, generator=g).bfloat16().cuda()
    k[0, 1400] = q[0, 0] * 40
    v = torch.randn(B, S, 64, generator=g).bfloat16().cuda()
    o = _attn("bf16", q, k, v, True)
    assert (o.double() - _attn_ref(q, k, v)).abs().max().item() < 1e-2


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("Sq,Sk,split", [(1, 1500, 0), (3, 700, 0), (1, 1, 0), (5, 33, 0), (1, 1500, 4), (2, 1500, 3),
                                         (1, 5, 4), (1, 2, 4)])
def test_decode_attention(dt, Sq, Sk, split):
    g = torch.Generator(device="cpu").manual_seed(Sq * 1000 + Sk)
    B, H = 3, 2
    q = (torch.randn(B, Sq, H * 64, generator=g) * 0.3).to(DT[dt][0]).cuda()
    k = torch.randn(B, Sk, H * 64, generator=g).to(DT[dt][0]).cuda()
    v = torch.randn(B, Sk, H * 64, generator=g).to(DT[dt][0]).cuda()
    o = _attn(dt, q, k, v, split)
    tol = 1e-5 if dt == "f32" else 1e-2
    assert (o.double() - _attn_ref(q, k, v)).abs().max().item() < tol
    if split:   # tickets were reset: a second call combines again, bit-identically
        assert torch.equal(_attn(dt, q, k, v, split), o)


@pytest.mark.parametrize("n_mel", [80, 128])
def test_log_mel_matches_oracle(n_mel):
    from oracle.whisper_np import log_mel
    from whisper_context_biasing_amd.config import get_dims
    from whisper_context_biasing_amd.model import WhisperCB
    from whisper_context_biasing_amd.synth import synth_batch, synth_clip
    dims = get_dims("large-v3" if n_mel == 128 else "micro")
    m = WhisperCB(dims, dtype="f32")
    pcm = synth_batch(3)
    pcm[2] *= 0.001                                  # quiet clip: exercises the max − 8 clamp
    short = synth_clip(7, n_samples=5 * 16000)       # 5 s clip: zero-padded to 30 s
    got = m.log_mel(torch.from_numpy(pcm)).cpu().numpy()
    ref = log_mel(pcm, n_mel)
    # exact-f32 DFT vs float64 FFT: HF quotes 1e-5 between its own CPU/GPU paths; near-silent
    # bins carry f32 roundoff — tolerance 2e-4 max, 2e-6 mean
    assert np.abs(got - ref).max() < 2e-4
    assert np.abs(got - ref).mean() < 2e-6
    got_s = m.log_mel(torch.from_numpy(short)[None]).cpu().numpy()
    ref_s = log_mel(short[None], n_mel)
    assert np.abs(got_s - ref_s).max() < 2e-4


def _xattn_enc(dt, q, enc, wk, wv, bv, nsplit, variant=1):
    lib = _lib.load()
    B, S, d = enc.shape
    H = d // 64
    wkt = wk.view(H, 64, d).transpose(1, 2).contiguous()     # [H][d][64]: (h, c, i) = W_k[h*64+i][c]
    o = torch.empty(B, d, dtype=enc.dtype, device="cuda")
    _lib.check(lib.wcb_op_cross_attention_enc(DT[dt][1], q.data_ptr(), enc.data_ptr(), wkt.data_ptr(), wv.data_ptr(),
                                              bv.data_ptr(), o.data_ptr(), B, H, S, nsplit, variant, _s()), None,
               "xattn_enc")
    torch.cuda.synchronize()
    return o


@pytest.mark.parametrize("variant", ["1", "2", "0", "3", "101", "1001"])
@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("d,B,S,nsplit", [(768, 32, 1500, 8), (768, 5, 1500, 1), (384, 3, 1500, 16), (64, 2, 1500, 3),
                                          (1024, 2, 1500, 8), (512, 4, 100, 4), (768, 3, 37, 2), (384, 1, 1, 1)])
def test_cross_attention_encoder_space(dt, d, B, S, nsplit, variant):
    """Encoder-space cross-attention (k_xenc.hip, both chunk-ring variants) vs the K/V formulation of the
    reference ([tf] modeling_whisper.py:284-356): K = enc W_kᵀ (no bias), V = enc W_vᵀ + b_v, softmax(q Kᵀ) V
    in fp64."""
    g = torch.Generator(device="cpu").manual_seed(d + B * 7 + S)
    H = d // 64
    tdt = DT[dt][0]
    q = (torch.randn(B, d, generator=g) * 0.125).to(tdt).cuda()
    enc = torch.randn(B, S, d, generator=g).to(tdt).cuda()
    wk = (torch.randn(d, d, generator=g) / d ** 0.5 * 2).to(tdt).cuda()
    wv = (torch.randn(d, d, generator=g) / d ** 0.5).to(tdt).cuda()
    bv = torch.randn(d, generator=g).float().cuda()
    o = _xattn_enc(dt, q, enc, wk, wv, bv, nsplit, int(variant))
    K = enc.double() @ wk.double().T
    V = enc.double() @ wv.double().T + bv.double()
    qh = q.double().view(B, 1, H, 64).transpose(1, 2)
    Kh = K.view(B, S, H, 64).transpose(1, 2)
    Vh = V.view(B, S, H, 64).transpose(1, 2)
    p = torch.softmax(qh @ Kh.transpose(-1, -2), -1)
    ref = (p @ Vh).transpose(1, 2).reshape(B, d)
    # q' and P are rounded to the 16-bit type before their MFMAs, the output once: bf16 2^-8 relative
    tol = 3e-2 if dt == "bf16" else 5e-3
    err = (o.double() - ref).abs().max().item()
    assert err < tol * max(1.0, ref.abs().max().item()), err
    assert torch.equal(_xattn_enc(dt, q, enc, wk, wv, bv, nsplit, int(variant)), o)   # deterministic


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,N,K,act,resid", [(4096, 768, 768, 0, False), (6000, 2304, 768, 0, False),
                                             (5000, 768, 3072, 0, True), (4100, 3072, 768, 1, False),
                                             (4097, 256, 2304, 1, True)])
def test_gemm_ring_encoder_shapes(dt, M, N, K, act, resid):
    """The LDS-ring tile kernel (16-bit, M >= 4096, N % 128 == 0: the encoder GEMMs) with the encoder's
    epilogues, ragged M, vs fp64."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(DT[dt][0]).cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(DT[dt][0]).cuda()
    bias = torch.randn(N, generator=g).float().cuda()
    R = torch.randn(M, N, generator=g).float().cuda() if resid else None
    out = _gemm(dt, A, W, bias=bias, act=act, resid=R.clone() if resid else None, out_f32=resid)
    ref = A.double() @ W.double().T + bias.double()
    if act:
        ref = torch.nn.functional.gelu(ref)
    if resid:
        ref = ref + R.double()
    # f32 accumulation; 16-bit output rounding (2^-8 bf16, 2^-11 f16 relative) when not f32
    tol = 1e-4 if resid else (8e-3 if dt == "bf16" else 1e-3)
    err = ((out.double() - ref).abs() - tol * ref.abs()).max().item()
    assert err < 2e-4, err


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,N,K,act,resid,bias,f32", [
    (4096, 768, 768, 0, False, True, False), (6000, 2304, 768, 0, False, True, False),
    (5000, 768, 3072, 0, True, True, True), (4100, 3072, 768, 1, False, True, False),
    (300, 256, 64, 0, False, True, False),      # one K tile (the LDS-ring kernel takes it)
    (511, 512, 128, 1, False, False, False),    # two K tiles, no bias
    (257, 256, 192, 0, True, True, True),       # three K tiles, one row past a tile
    (1000, 1024, 320, 0, False, False, True),   # f32 out without a residual
    # more tiles than workgroups (256): each workgroup streams several tiles' K tiles back to back
    (8200, 2304, 128, 0, False, True, False), (16500, 1024, 192, 1, False, True, False),
    (48000, 768, 768, 0, True, True, True), (33000, 2304, 768, 0, False, True, False),
    # 192-wide tiles (kernel 5): two / three K tiles, ragged M, the d-wide shapes of the encoder
    (700, 192, 128, 1, False, True, False), (257, 576, 192, 0, True, True, True), (20000, 768, 3072, 0, True, True, True)])
@pytest.mark.parametrize("kernel", [2, 5])
def test_gemm_pingpong_kernel(dt, M, N, K, act, resid, bias, f32, kernel):
    """The ping-pong encoder GEMM (gemm_pp_kernel: 256x256 (kernel 2) or 256x192 (kernel 5: where N % 192 ==
    0, else the LDS-ring kernel takes the launch) tiles, staggered wave halves, counted LDS-DMA waits,
    persistent K-tile stream) through wcb_op_gemm_kernel, every K-tile count of its piece schedule's tail
    (1, 2, 3, many), ragged M, each epilogue, vs fp64 and against the LDS-ring kernel (kernel=0)."""
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + 1)
    A = torch.randn(M, K, generator=g).to(DT[dt][0]).cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(DT[dt][0]).cuda()
    b = torch.randn(N, generator=g).float().cuda() if bias else None
    R = torch.randn(M, N, generator=g).float().cuda() if resid else None

    def run(kernel):
        out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.float32 if f32 else A.dtype)
        if resid:
            out.copy_(R)   # in place, as the encoder's residual stream
        _lib.check(lib.wcb_op_gemm_kernel(DT[dt][1], A.data_ptr(), W.data_ptr(), M, N, K,
                                          b.data_ptr() if bias else None, act,
                                          out.data_ptr() if resid else None, out.data_ptr(), int(f32), kernel,
                                          _s()), None, "gemm")
        torch.cuda.synchronize()
        return out
    out = run(kernel)
    ref = A.double() @ W.double().T
    if bias:
        ref = ref + b.double()
    if act:
        ref = torch.nn.functional.gelu(ref)
    if resid:
        ref = ref + R.double()
    tol = 1e-4 if f32 else (8e-3 if dt == "bf16" else 1e-3)
    err = ((out.double() - ref).abs() - tol * ref.abs()).max().item()
    assert err < 2e-4, err
    assert torch.equal(run(kernel), out)   # deterministic
    other = run(0)
    err0 = ((other.double() - ref).abs() - tol * ref.abs()).max().item()
    assert err0 < 2e-4, err0


def _frag_major(W):
    """[N][K] → [N / 16][K / 32][64 lanes][8]: element (n, k) at lane 16·((k % 32) / 8) + n % 16, slot k % 8."""
    N, K = W.shape
    return W.view(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().view(N, K)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("M,N,K,act,resid", [
    (80, 1280, 1280, 0, True), (80, 5120, 1280, 1, False), (80, 3840, 1280, 0, False),   # C5's beam rows
    (320, 1024, 1024, 0, True), (320, 4096, 1024, 1, False), (70, 768, 768, 0, False),   # C3's, ragged rows
    (97, 512, 1024, 1, False)])
@pytest.mark.parametrize("kernel", [6, 7, 106, 107, 12, 22, 42, 51, 112, 122, 152])
def test_gemm_decode_row_tiles(dt, M, N, K, act, resid, kernel):
    """Beam-row projections (decode rows > 64) through wcb_op_gemm_kernel: the LDS-ring tiles (kernel 6) and
    the wide single-burst tiles (gemm_wide_kernel, 10·FM + FN; + 100: fragment-major W) vs fp64, bias, GELU
    and the in-place residual epilogue, ragged row tiles, deterministic."""
    lib = _lib.load()
    if kernel % 100 > 10 and N % (16 * (kernel % 10)):
        pytest.skip("N not a multiple of the tile width")
    g = torch.Generator(device="cpu").manual_seed(M + N + K + kernel)
    A = torch.randn(M, K, generator=g).to(DT[dt][0]).cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(DT[dt][0]).cuda()
    Wk = _frag_major(W) if kernel >= 100 else W
    b = torch.randn(N, generator=g).float().cuda()
    R = torch.randn(M, N, generator=g).float().cuda() if resid else None

    def run():
        out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.float32 if resid else A.dtype)
        if resid:
            out.copy_(R)
        _lib.check(lib.wcb_op_gemm_kernel(DT[dt][1], A.data_ptr(), Wk.data_ptr(), M, N, K, b.data_ptr(), act,
                                          out.data_ptr() if resid else None, out.data_ptr(), int(resid), kernel,
                                          _s()), None, "gemm")
        torch.cuda.synchronize()
        return out
    out = run()
    ref = A.double() @ W.double().T + b.double()
    if act:
        ref = torch.nn.functional.gelu(ref)
    if resid:
        ref = ref + R.double()
    tol = 1e-4 if resid else (8e-3 if dt == "bf16" else 1e-3)
    err = ((out.double() - ref).abs() - tol * ref.abs()).max().item()
    assert err < 2e-4, err
    assert torch.equal(run(), out)


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("Sk,split", [(1500, 1), (1500, 4), (37, 1), (1, 3), (64, 1), (65, 1), (200, 1)])
def test_decode_attention_variants(dt, variant, Sk, split):
    """Every cross-attention kernel variant in the runtime's head-major K/V layout, with and without
    split-KV (variant 0 = the two-pass kernel beam search over precomputed K/V runs), vs fp64."""
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(variant * 100 + Sk + split)
    B, H = 5, 3
    q = (torch.randn(B, H * 64, generator=g) * 0.3).to(DT[dt][0]).cuda()
    k = torch.randn(B, H, Sk, 64, generator=g).to(DT[dt][0]).cuda()
    v = torch.randn(B, H, Sk, 64, generator=g).to(DT[dt][0]).cuda()
    o = torch.empty_like(q)
    _lib.check(lib.wcb_op_attention_decode(DT[dt][1], q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, Sk,
                                           split, variant, _s()), None, "attention_decode")
    torch.cuda.synchronize()
    p = torch.softmax(q.double().view(B, H, 1, 64) @ k.double().transpose(-1, -2), -1)
    ref = (p @ v.double()).view(B, H * 64)
    tol = 1e-5 if dt == "f32" else 1e-2
    assert (o.double() - ref).abs().max().item() < tol
    if variant == 7 and split == 1 and dt == "bf16":   # the lean one-token kernel: bit-identical to variant 6
        o6 = torch.empty_like(q)
        _lib.check(lib.wcb_op_attention_decode(DT[dt][1], q.data_ptr(), k.data_ptr(), v.data_ptr(), o6.data_ptr(), B, H,
                                               Sk, split, 6, _s()), None, "attention_decode")
        torch.cuda.synchronize()
        assert torch.equal(o, o6)


@pytest.mark.parametrize("mel_split", [0, 1])
@pytest.mark.parametrize("n_mel", [80, 128])
def test_log_mel_matches_reference_golden(n_mel, mel_split):
    """The GPU front end against the reference's own feature extractor outputs (tests/golden/mel_golden.npz,
    WhisperFeatureExtractor run by make_golden.py): the same bar the numpy oracle meets (2e-5 on the
    golden slices; HF quotes 1e-5 between its CPU and GPU paths), plus the global statistics — for the f32
    MFMA DFT and the split-bf16 one (option mel_split)."""
    import os
    MEL_COLS = [slice(0, 48), slice(1476, 1524), slice(2952, 3000)]   # as tests/test_oracle_golden.py
    from whisper_context_biasing_amd.config import get_dims
    from whisper_context_biasing_amd.model import WhisperCB
    from whisper_context_biasing_amd.synth import synth_clip
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "mel_golden.npz"))
    m = WhisperCB(get_dims("large-v3" if n_mel == 128 else "micro"), dtype="f32", options={"mel_split": mel_split})
    for clip in range(4):
        pcm = synth_clip(clip, n_samples=5 * 16000) if clip == 2 else synth_clip(clip)
        if clip == 3:
            pcm = (pcm * 0.001).astype(np.float32)
        mel = m.log_mel(torch.from_numpy(pcm)[None]).cpu().numpy()[0]
        got = np.concatenate([mel[:, s] for s in MEL_COLS], axis=1)
        err = np.abs(got - gold[f"mel{n_mel}_clip{clip}_slices"]).max()
        assert err < 2e-5, (clip, err)
        st = gold[f"mel{n_mel}_clip{clip}_stats"]
        assert abs(mel.max() - st[2]) < 1e-5 and abs(mel.min() - st[3]) < 1e-4, (clip, mel.max(), mel.min(), st)
        assert abs(mel.sum(dtype=np.float64) - st[0]) < 1e-5 * mel.size
