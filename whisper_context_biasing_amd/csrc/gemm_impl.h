// MFMA GEMMs for the encoder stack, the conv stem (implicit im2col), the cross-KV precompute and
// the decode-step projections / LM head.
//
// Replaces the nn.Linear / nn.Conv1d calls of WhisperEncoderLayer / WhisperDecoderLayer /
// WhisperAttention ([tf] modeling_whisper.py:284-356, 379-413, 448-505, 566-567, 618-624) and the
// reference LM head `proj_out` (models/whisper_medical.py:19,111).
//
// gemm_tile_kernel: BMxBN tile per workgroup, 128-byte K rows (BK = 64 bf16/f16 or 32 f32)
//   staged HBM → LDS with global_load_lds (16 B per lane, 2 LDS stages), XOR-swizzled on the
//   SOURCE address so ds_read_b128 fragment reads are conflict-free (chunk ^= (row>>1)&7),
//   16x16x32 MFMA per wave, epilogue staged through LDS as f32 and written 16 B per lane.
// gemm_skinny_kernel: M <= 64 rows (decode), 16 output columns per workgroup, K split over the
//   workgroup's waves, fragments straight from global memory (weights are streamed once), wave
//   partials reduced through LDS.
#pragma once
#include <stdexcept>
#include <string>
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace wcb {

WCB_DEV void glds16(const void* gptr, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(gptr, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// 32-bit row arithmetic (M < 2^31); the batched form only for the conv stem
WCB_DEV long a_row(const GemmArgs& g, int m) {
  return g.a_Mb ? (long)(m / g.a_Mb) * g.a_strideB + (long)(m % g.a_Mb) * g.lda : (long)m * g.lda;
}
WCB_DEV long c_row(const GemmArgs& g, int m) {
  return g.c_Mb ? (long)(m / g.c_Mb) * g.c_strideB + (long)(m % g.c_Mb) * g.ldc : (long)m * g.ldc;
}

// Epilogue selection. EPI is a compile-time set of E_* bits for the encoder's fixed shapes
// (no per-element branches); E_RUNTIME reads the same options from GemmArgs at run time.
enum : int { E_BIAS = 1, E_GELU = 2, E_RESID = 4, E_F32 = 8, E_ADDROW = 16, E_HEAD = 32, E_RUNTIME = 1 << 30 };

template <int EPI> WCB_DEV bool has(const GemmArgs& g, int bit) {
  if constexpr (EPI == E_RUNTIME) {
    switch (bit) {
      case E_BIAS: return g.bias != nullptr;
      case E_GELU: return g.act == 1;
      case E_RESID: return g.resid != nullptr;
      case E_F32: return g.out_f32 != 0;
      case E_ADDROW: return g.addrow != nullptr;
      case E_HEAD: return g.mode == 1;
      default: return false;
    }
  } else {
    return (EPI & bit) != 0;
  }
}

// GELU(erf). f32 ("exact" parity mode) keeps ocml erff; 16-bit modes use a branch-free
// Abramowitz-Stegun 7.1.26 erfc (|err| <= 1.5e-7 absolute, far below bf16/f16 resolution).
template <typename T> WCB_DEV float gelu_t(float x) {
  if constexpr (sizeof(T) == 4) {
    return gelu_erf(x);
  } else {
    const float z = fabsf(x) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    const float q = p * t * __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);   // erfc(|x|/√2)
    return 0.5f * x * (x >= 0.f ? 2.0f - q : q);
  }
}

// Store 8 consecutive output columns n..n+7 of row m (n % 8 == 0, all in one head for E_HEAD).
template <typename T, int EPI>
WCB_DEV void epi_store8(const GemmArgs& g, int m, int n, float* v) {
  if (EPI == E_RUNTIME && g.mode == 2 && n >= g.n_split) {   // k / v of decoder rows → self-attention KV cache
    const int n2 = n - g.n_split;
    const int hh = n2 >> 6, dd = n2 & 63;
    const int kv = hh / g.hs_H, h = hh % g.hs_H;
    const int rps = g.kv_rps > 1 ? g.kv_rps : 1;
    const long off = ((((long)kv * g.hs_B + m / rps) * g.hs_H + h) * g.kv_T + *g.pos + m % rps) * 64 + dd;
    store8<T>(reinterpret_cast<T*>(g.kv_out) + off, v);
    return;
  }
  if (has<EPI>(g, E_HEAD)) {
    const int hh = n >> 6, dd = n & 63;
    const int grp = hh / g.hs_H, h = hh % g.hs_H;
    const int b = m / g.hs_S, t = m % g.hs_S;
    const long off = ((((long)grp * g.hs_B + b) * g.hs_H + h) * g.hs_S + t) * 64 + dd;
    store8<T>(reinterpret_cast<T*>(g.out) + off, v);
    return;
  }
  const long off = c_row(g, m) + n;
  if (has<EPI>(g, E_RESID)) {
    const f32x4 r0 = *reinterpret_cast<const f32x4*>(g.resid + off);
    const f32x4 r1 = *reinterpret_cast<const f32x4*>(g.resid + off + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += r0[j]; v[j + 4] += r1[j]; }
    if (g.clamp != 0.f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fminf(fmaxf(v[j], -g.clamp), g.clamp);
    }
  }
  if (has<EPI>(g, E_F32)) store8<float>(reinterpret_cast<float*>(g.out) + off, v);
  else store8<T>(reinterpret_cast<T*>(g.out) + off, v);
  if (EPI == E_RUNTIME && g.out16) store8<T>(reinterpret_cast<T*>(g.out16) + off, v);   // decode: 16-bit residual copy
}

template <typename T>
WCB_DEV float epi_store1(const GemmArgs& g, int m, int n, float v) {
  if (g.mode == 2 && n >= g.n_split) {
    const int n2 = n - g.n_split;
    const int hh = n2 >> 6, dd = n2 & 63;
    const int kv = hh / g.hs_H, h = hh % g.hs_H;
    const int rps = g.kv_rps > 1 ? g.kv_rps : 1;   // prefill: rows (cache row, position) row-major
    const long off = ((((long)kv * g.hs_B + m / rps) * g.hs_H + h) * g.kv_T + *g.pos + m % rps) * 64 + dd;
    reinterpret_cast<T*>(g.kv_out)[off] = DT<T>::fromf(v);
    return v;
  }
  if (g.mode == 1) {
    const int hh = n >> 6, dd = n & 63;
    const int grp = hh / g.hs_H, h = hh % g.hs_H;
    const int b = m / g.hs_S, t = m % g.hs_S;
    const long off = ((((long)grp * g.hs_B + b) * g.hs_H + h) * g.hs_S + t) * 64 + dd;
    reinterpret_cast<T*>(g.out)[off] = DT<T>::fromf(v);
    return v;
  }
  const long off = c_row(g, m) + n;
  if (g.resid) v += g.resid[off];
  if (g.out_f32) reinterpret_cast<float*>(g.out)[off] = v;
  else reinterpret_cast<T*>(g.out)[off] = DT<T>::fromf(v);
  return v;
}

template <typename T, int EPI = E_RUNTIME>
WCB_DEV float epi_pointwise(const GemmArgs& g, int m, int n, float v) {
  if (has<EPI>(g, E_BIAS)) v += g.bias[n];
  if (has<EPI>(g, E_GELU)) v = gelu_t<T>(v);
  if (has<EPI>(g, E_ADDROW)) v += g.addrow[(long)(g.c_Mb ? m % g.c_Mb : m) * g.N + n];
  return v;
}

template <typename T, int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(WM * WN * 64) void gemm_tile_kernel(GemmArgs g) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int EB = sizeof(T);
  constexpr int BK = 128 / EB;           // elements per 128-byte LDS row
  constexpr int CE = 16 / EB;            // elements per 16-byte chunk
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int KSUB = BK / 32;
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int IA = BM / 8 / NW, IB = BN / 8 / NW;
  static_assert(IA * NW * 8 == BM && IB * NW * 8 == BN, "tile rows must split over waves");
  using Frag = typename DT<T>::frag;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int m0 = (wg / tiles_n) * BM, n0 = (wg % tiles_n) * BN;

  const T* A = reinterpret_cast<const T*>(g.A);
  const T* W = reinterpret_cast<const T*>(g.W);
  const T* a_src[IA];
  const T* b_src[IB];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int r = (wave + i * NW) * 8 + (lane >> 3);
    const int m = min(m0 + r, g.M - 1);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    a_src[i] = A + a_row(g, m) + c * CE;
  }
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int r = (wave + i * NW) * 8 + (lane >> 3);
    const long n = min(n0 + r, g.N - 1);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    b_src[i] = W + n * g.ldw + c * CE;
  }
  auto stage = [&](int s, int k0) {
    char* base = smem + s * STAGE;
#pragma unroll
    for (int i = 0; i < IA; ++i) glds16(a_src[i] + k0, base + (wave + i * NW) * 1024);
#pragma unroll
    for (int i = 0; i < IB; ++i) glds16(b_src[i] + k0, base + BM * 128 + (wave + i * NW) * 1024);
  };
  auto lds_frag = [&](const char* base, int r, int ks) -> Frag {
    if constexpr (EB == 2) {
      const int c = ks * 4 + (lane >> 4);
      return *reinterpret_cast<const Frag*>(base + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
    } else {
      const int c = 2 * (lane >> 4);
      const f32x4 lo = *reinterpret_cast<const f32x4*>(base + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
      const f32x4 hi = *reinterpret_cast<const f32x4*>(base + r * 128 + (((c + 1) ^ ((r >> 1) & 7)) << 4));
      return Frag{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nk) stage(s ^ 1, (kt + 1) * BK);
    const char* base = smem + s * STAGE;
#pragma unroll
    for (int ks = 0; ks < KSUB; ++ks) {
      Frag a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = lds_frag(base, wm * TM + i * 16 + (lane & 15), ks);
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = lds_frag(base + BM * 128, wn * TN + j * 16 + (lane & 15), ks);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mma16(a[i], b[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: f32 tile through LDS, then 8 columns (16-32 B) per lane per store
  constexpr int LDC = BN + 4;
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = wn * TN + j * 16 + (lane & 15);
    const int n = min(n0 + col, g.N - 1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * TM + i * 16 + (lane >> 4) * 4 + e;
        const int m = min(m0 + row, g.M - 1);
        ct[row * LDC + col] = epi_pointwise<T, EPI>(g, m, n, acc[i][j][e]);
      }
  }
  __syncthreads();
  constexpr int C8 = BN / 8;
#pragma unroll 2
  for (int idx = tid; idx < BM * C8; idx += NT) {
    const int row = idx / C8, c8 = idx % C8;
    const int m = m0 + row;
    const int n = n0 + c8 * 8;
    if (m >= g.M || n >= g.N) continue;
    float v[8];
    const f32x4 lo = *reinterpret_cast<const f32x4*>(ct + row * LDC + c8 * 8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(ct + row * LDC + c8 * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = lo[e]; v[e + 4] = hi[e]; }
    epi_store8<T, EPI>(g, m, n, v);
  }
}

// gemm_ring_kernel (16-bit types, the encoder / conv-stem GEMMs): BMxBN tile per workgroup of
// WMxWN waves, K tiles of 64 staged HBM/L2 → LDS by global_load_lds into a ring of NS stages, so
// NS-1 tiles stay in flight while one is multiplied. One barrier per K tile: each wave retires its own
// loads of tile k with a COUNTED s_waitcnt vmcnt (the younger tiles stay in flight across the
// barrier), the raw s_barrier makes every wave's tile-k bytes visible and tells the issuers that the
// stage of tile k-1 is free, then tile k+NS-1 is issued into it. No plain global loads inside the
// loop (hipcc would drain the DMA ring at their use); __syncthreads only after it.
// LNF (decode rows > 64, 16-bit): the consumer's pre-block LayerNorm folded into the weights and the
// epilogue, no per-element work in the K loop. LN(x)·Wᵀ + b = r·(Σ_k x_k W'[n][k] − μ·u[n]) + c[n] with
// W' = W·diag(γ) (rounded to T at finalize, GemmArgs::W), u[n] = Σ_k W'[n][k], c[n] = Σ_k β_k W[n][k] +
// b[n] (GemmArgs::bias); A = the 16-bit copy of the residual rows. The row statistics (μ, r) come from
// the per-32-column partial sums (Σx, Σx²) the residual writer published (GemmArgs::rst_in, fixed-order
// sums: deterministic); they are fetched into LDS by the same LDS-DMA as the first ring stage.
// KT: 64-deep sub-tiles per ring stage (2 for the small decode-row tiles: half the K-loop
// iterations, and with them half the barriers, of a loop that is latency-bound at 2-8 MFMAs per wave
// per sub-tile).
// BKB: bytes of K per LDS row of a sub-tile: 128 (64-deep) or 64 (32-deep: half the stage bytes, so
// twice the stages in the same LDS — the encoder's 256x256 tiles keep 3 stages in flight across the
// barrier instead of 1). The MFMA sequence over K is the same: bit-identical outputs.
// WFM (decode rows, BKB 128): W given fragment-major (g.W_fm: [N / 16][K / 32][64 lanes][8]); each lane's
// 16-byte piece is gathered from there into the same swizzled LDS row layout (a wave-instruction's 8 rows
// x 64 k then read 2 KiB of contiguous weights instead of 8 rows at the K-row stride).
template <typename T, int BM, int BN, int WM, int WN, int NS, int EPI, bool LNF = false, int KT = 1, int BKB = 128,
          int PRIO = 0, bool WFM = false>
__global__ __launch_bounds__(WM * WN * 64) void gemm_ring_kernel(GemmArgs g) {
  constexpr int NW = WM * WN, NT = NW * 64;
  static_assert(BKB == 128 || BKB == 64, "LDS row: 128 or 64 bytes");
  constexpr int BK = BKB / 2, CE = 8;
  constexpr int CPR = BKB / 16, RPI = 64 / CPR, KS = BKB / 64;   // chunks per row, rows per glds, k-steps per sub-tile
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int SUB = (BM + BN) * BKB, STAGE = SUB * KT;
  constexpr int IA = BM / RPI / NW, IB = BN / RPI / NW, GL = (IA + IB) * KT;   // glds per wave per stage
  static_assert(IA * NW * RPI == BM && IB * NW * RPI == BN, "tile rows must split over waves");
  // 16-byte chunk c of LDS row r sits in slot c ^ swz(r): the 16 rows of a fragment read hit 16
  // distinct 16-byte bank groups
  auto swz = [](int r) { return BKB == 128 ? (r >> 1) & 7 : (r >> 2) & 3; };
  using Frag = typename DT<T>::frag;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  int m0, n0;
  if (g.raster > 0) {   // bands of `raster` row panels, column tiles outer within a band (the
                        // concurrently resident tiles of one XCD share A and W panels in its L2)
    const int tiles_m = (g.M + BM - 1) / BM, band = g.raster * tiles_n;
    const int fm = (wg / band) * g.raster, gm = min(tiles_m - fm, g.raster), r = wg % band;
    m0 = (fm + r % gm) * BM;
    n0 = (r / gm) * BN;
  } else {
    m0 = (wg / tiles_n) * BM;
    n0 = (wg % tiles_n) * BN;
  }

  const T* A = reinterpret_cast<const T*>(g.A);
  const T* W = reinterpret_cast<const T*>(g.W);
  const T* a_src[IA];
  const T* b_src[IB];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int r = (wave + i * NW) * RPI + lane / CPR;
    const int m = min(m0 + r, g.M - 1);
    a_src[i] = A + a_row(g, m) + ((lane % CPR) ^ swz(r)) * CE;
  }
  static_assert(!WFM || BKB == 128, "fragment-major W: 64-deep sub-tiles");
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int r = (wave + i * NW) * RPI + lane / CPR;
    const long n = min(n0 + r, g.N - 1);
    const int c = (lane % CPR) ^ swz(r);   // chunk (8 k) of the 64-deep sub-tile
    if constexpr (WFM)   // k-step c / 4 of the sub-tile, lane 16·(c % 4) + n % 16 of that k-step's fragment
      b_src[i] = reinterpret_cast<const T*>(g.W_fm) + ((n / 16) * (g.K / 32) + c / 4) * 512 + (16 * (c % 4) + n % 16) * 8;
    else
      b_src[i] = W + n * g.ldw + c * CE;
  }
  // (fragment-major W: k advances 512 elements per 32-deep k-step, i.e. 16 per element of k)
  constexpr int WKS = WFM ? 16 : 1;
  auto stage = [&](int st, int k0) {
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      char* base = smem + st * STAGE + t * SUB;
#pragma unroll
      for (int i = 0; i < IA; ++i) glds16(a_src[i] + k0 + t * BK, base + (wave + i * NW) * 1024);
#pragma unroll
      for (int i = 0; i < IB; ++i) glds16(b_src[i] + (long)(k0 + t * BK) * WKS, base + BM * BKB + (wave + i * NW) * 1024);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LNF: the tile rows' statistics partials [BM][rst_nb] float2 (LDS-DMA, older than ring stage 0:
  // the first stage wait retires them), then (μ, r) per tile row
  constexpr int LNF_OFF = NS * STAGE > BM * (BN + 4) * 4 ? NS * STAGE : BM * (BN + 4) * 4;
  float* lnraw = reinterpret_cast<float*>(smem + LNF_OFF);
  float* lnst = lnraw + BM * (kLnfMaxK / 32) * 2;
  const int nk = g.K / (BK * KT);
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) stage(p, p * BK * KT);
  if constexpr (LNF) {   // after the prologue stages (younger: the first waits over-wait by a few
                         // pieces of stage 1 at most; the loop's last vmcnt(0) retires them)
    const int per_row = g.rst_nb * 8 / 16;                  // 16-byte chunks per row (rst_nb float2)
    const int chunks = BM * per_row;
    for (int q0 = wave * 64; q0 < chunks; q0 += NT) {
      const int q = min(q0 + lane, chunks - 1), r = q / per_row, j = q % per_row;
      const int m = min(m0 + r, g.M - 1);
      glds16(g.rst_in + ((long)m * g.rst_nb) * 2 + j * 4, reinterpret_cast<char*>(lnraw) + (long)q0 * 16);
    }
  }
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // tiles issued so far: kt .. min(nk, kt + NS - 1) - 1; keep the ones after kt in flight
    const int ahead = min(nk - 1 - kt, NS - 2);
    if constexpr (NS >= 4) {   // up to min(NS - 2, 4) younger tiles stay in flight (vmcnt <= 63)
      static_assert(4 * GL <= 63, "vmcnt range");
      if (NS >= 6 && ahead >= 4) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 * GL) : "memory");
      else if (NS >= 5 && ahead == 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * GL) : "memory");
      else if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * GL) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(GL) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (NS == 3) {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(GL) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    {
      const int nxt = kt + NS - 1;
      int sn = st + NS - 1;
      if (sn >= NS) sn -= NS;
      if (nxt < nk) stage(sn, nxt * BK * KT);
    }
#pragma unroll
    for (int kq = 0; kq < KS * KT; ++kq) {
      const char* base = smem + st * STAGE + (kq / KS) * SUB;
      const int ks = kq % KS;
      Frag a[FM], b[FN];
      const int c = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * TM + i * 16 + (lane & 15);
        a[i] = *reinterpret_cast<const Frag*>(base + r * BKB + ((c ^ swz(r)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * TN + j * 16 + (lane & 15);
        b[j] = *reinterpret_cast<const Frag*>(base + BM * BKB + r * BKB + ((c ^ swz(r)) << 4));
      }
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mma16(a[i], b[j], acc[i][j]);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
    }
    st = st + 1 == NS ? 0 : st + 1;
  }
  if constexpr (LNF) {   // (μ, r) per tile row from the producer's partials: LPR lanes per row, each a
                         // strided subset in column order, then a fixed butterfly (deterministic)
    __syncthreads();     // every wave's statistics pieces have landed (each waited vmcnt(0) above)
    constexpr int LPR = NT / BM;
    static_assert(LPR >= 1 && (LPR & (LPR - 1)) == 0 && LPR <= 64, "lanes per row");
    const int r = tid / LPR, sub = tid % LPR;
    float a1 = 0.f, a2 = 0.f;
    for (int j = sub; j < g.rst_nb; j += LPR) {
      const float2 t = *reinterpret_cast<const float2*>(lnraw + ((long)r * g.rst_nb + j) * 2);
      a1 += t.x;
      a2 += t.y;
    }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) { a1 += __shfl_xor(a1, o, 64); a2 += __shfl_xor(a2, o, 64); }
    if (sub == 0) {
      const float mean = a1 / g.K;
      lnst[2 * r] = mean;
      lnst[2 * r + 1] = rsqrtf(fmaxf(a2 / g.K - mean * mean, 0.f) + 1e-5f);
    }
  }
  __syncthreads();   // every wave is done with the ring: the epilogue reuses its LDS

  // epilogue: f32 accumulators through LDS (in WM passes of TM rows when the whole tile does not
  // fit), then 8 columns per lane: bias / GELU / row table applied there, by all the waves (in the
  // LDS-write phase only the waves of one pass would), then the store
  constexpr int LDC = BN + 4;
  constexpr int PASSES = (BM * LDC * 4 <= 160 * 1024) ? 1 : WM;
  constexpr int PR = BM / PASSES;
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int ps = 0; ps < PASSES; ++ps) {
    if (PASSES == 1 || wm == ps) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * TN + j * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = wm * TM + i * 16 + (lane >> 4) * 4 + e;
            float v = acc[i][j][e];
            if constexpr (LNF) v = lnst[2 * row + 1] * (v - lnst[2 * row] * g.ln_u[min(n0 + col, g.N - 1)]);
            ct[(row - ps * PR) * LDC + col] = v;
          }
      }
    }
    __syncthreads();
    constexpr int C8 = BN / 8, RPIT = NT / C8;   // rows per iteration (threads past RPIT·C8 idle)
    // a thread keeps its 8 columns over the store loop: their bias once, before it
    const int c8 = tid % C8;
    float b8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (has<EPI>(g, E_BIAS)) {
      const int nb = min(n0 + c8 * 8, g.N - 8);
      const f32x4 lo = *reinterpret_cast<const f32x4*>(g.bias + nb);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(g.bias + nb + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { b8[e] = lo[e]; b8[e + 4] = hi[e]; }
    }
    const int row0 = tid < RPIT * C8 ? tid / C8 : PR;
    constexpr int UNR = PR >= 2 * RPIT && EPI != E_RUNTIME ? 2 : 1;   // (E_RUNTIME: convergent shuffles)
#pragma unroll UNR
    for (int row = row0; row < PR; row += RPIT) {
      const int m = m0 + ps * PR + row;
      const int n = n0 + c8 * 8;
      const bool ok = m < g.M && n < g.N;
      float v[8];
      const f32x4 lo = *reinterpret_cast<const f32x4*>(ct + row * LDC + c8 * 8);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(ct + row * LDC + c8 * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = lo[e]; v[e + 4] = hi[e]; }
#pragma unroll
      for (int e = 0; e < 8; ++e) {   // epi_pointwise's order: + bias, GELU, + row table
        if (has<EPI>(g, E_BIAS)) v[e] += b8[e];
        if (has<EPI>(g, E_GELU)) v[e] = gelu_t<T>(v[e]);
        if (has<EPI>(g, E_ADDROW))
          v[e] += g.addrow[(long)(g.c_Mb ? min(m, g.M - 1) % g.c_Mb : min(m, g.M - 1)) * g.N + min(n + e, g.N - 1)];
      }
      if (ok) epi_store8<T, EPI>(g, m, n, v);
      if (EPI == E_RUNTIME && g.rst_out) {   // residual writer: (Σx, Σx²) of the new row per 32 columns
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) { a1 += v[e]; a2 = fmaf(v[e], v[e], a2); }
        a1 += __shfl_xor(a1, 1, 64); a2 += __shfl_xor(a2, 1, 64);   // the 4 lanes of a 32-column block
        a1 += __shfl_xor(a1, 2, 64); a2 += __shfl_xor(a2, 2, 64);
        if (ok && (c8 & 3) == 0) *reinterpret_cast<float2*>(g.rst_out + ((long)m * (g.N / 32) + n / 32) * 2) = float2{a1, a2};
      }
    }
    if (PASSES > 1) __syncthreads();
  }
}

template <typename T, int BM, int BN, int WM, int WN, int NS, int EPI, bool LNF = false, int KT = 1, int BKB = 128,
          int PRIO = 0, bool WFM = false>
static void launch_ring_e(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  constexpr int ring_bytes = NS * (BM + BN) * BKB * KT;
  constexpr int epi_full = BM * (BN + 4) * 4;
  constexpr int epi_bytes = epi_full <= 160 * 1024 ? epi_full : epi_full / WM;
  constexpr int base = ring_bytes > epi_bytes ? ring_bytes : epi_bytes;
  constexpr int lds = base + (LNF ? BM * (kLnfMaxK / 32) * 2 * 4 + 2 * BM * 4 : 0);
  static_assert(lds <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_ring_kernel<T, BM, BN, WM, WN, NS, EPI, LNF, KT, BKB, PRIO, WFM>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  WCB_LAUNCH((gemm_ring_kernel<T, BM, BN, WM, WN, NS, EPI, LNF, KT, BKB, PRIO, WFM>), dim3(tiles), dim3(WM * WN * 64), lds, s, g);
}

// decode-row ring tiles: the weights fragment-major where the runtime hands a copy over (g.W_fm)
template <typename T, int BM, int BN, int NS, bool LNF, int KT = 1>
static void launch_ring_dec(const GemmArgs& g, hipStream_t s) {
  if (g.W_fm && g.K % 32 == 0) launch_ring_e<T, BM, BN, 2, 2, NS, E_RUNTIME, LNF, KT, 128, 0, true>(g, s);
  else launch_ring_e<T, BM, BN, 2, 2, NS, E_RUNTIME, LNF, KT>(g, s);
}

// PRIO 1: s_setprio(1) around each MFMA cluster (keeps hipcc from moving the MFMAs across the
// barriers, cdna_hip_programming.md T5): the encoder shapes 1-4 % faster (tools/enc_gemm_bench.hip)
template <typename T, int BM, int BN, int WM, int WN, int NS, int BKB = 128, int PRIO = 1>
static void launch_ring(const GemmArgs& g, hipStream_t s) {
  const int bits = (g.bias ? E_BIAS : 0) | (g.act == 1 ? E_GELU : 0) | (g.resid ? E_RESID : 0) |
                   (g.out_f32 ? E_F32 : 0) | (g.addrow ? E_ADDROW : 0) | (g.mode == 1 ? E_HEAD : 0);
  switch (bits) {
    case E_BIAS: launch_ring_e<T, BM, BN, WM, WN, NS, E_BIAS, false, 1, BKB, PRIO>(g, s); break;
    case E_BIAS | E_GELU: launch_ring_e<T, BM, BN, WM, WN, NS, E_BIAS | E_GELU, false, 1, BKB, PRIO>(g, s); break;
    case E_BIAS | E_RESID | E_F32: launch_ring_e<T, BM, BN, WM, WN, NS, E_BIAS | E_RESID | E_F32, false, 1, BKB, PRIO>(g, s); break;
    case E_BIAS | E_GELU | E_F32 | E_ADDROW:
      launch_ring_e<T, BM, BN, WM, WN, NS, E_BIAS | E_GELU | E_F32 | E_ADDROW, false, 1, BKB, PRIO>(g, s); break;
    case E_BIAS | E_HEAD: launch_ring_e<T, BM, BN, WM, WN, NS, E_BIAS | E_HEAD, false, 1, BKB, PRIO>(g, s); break;
    default: launch_ring_e<T, BM, BN, WM, WN, NS, E_RUNTIME, false, 1, BKB, PRIO>(g, s); break;
  }
}

// ---- Encoder GEMM, ping-pong form (gemm_pp_kernel): 256 x 256 output tiles, 64-deep K tiles, 8 waves
// as 2 (row halves) x 4 (64-column quarters), one persistent workgroup per CU (128 KiB of LDS: two
// K-tile buffers, each A [256][64] + W [256][64] in 128-byte rows, 16-byte chunk c of row r at slot
// c ^ ((r >> 1) & 7), the swizzle applied to the DMA source address) walking tiles blockIdx.x,
// blockIdx.x + gridDim.x, ... as ONE stream of K tiles: the LDS-DMA for the next tile's first K tiles is
// issued during the current tile's last ones, and its epilogue stores drain behind the next tile's
// multiplies (measured before: a 12-K-tile tile spent 9k of its 54k cycles filling the pipe and 10k
// draining its stores, tools/gemm_probe).
// Waves 4-7 run one barrier behind waves 0-3, and each SIMD holds one wave of each half, so in every
// barrier interval one wave of a SIMD multiplies while its partner reads its next fragments from LDS
// and issues LDS-DMA for later K tiles (MI355X_MICROARCH.md "Two waves per SIMD";
// cdna_hip_programming.md "The 256² 8-phase template").
// A K tile is 4 phases; phase p multiplies the wave's rows [32p, 32p + 32) (2 row fragments) with its
// 64 columns (4 weight fragments, read in phase 0 and kept) over 2 k-steps: 16 MFMAs.
// LDS-DMA pieces (one 16-byte load per thread each): "A quarter" q = the 64 tile rows phase q reads
// (rows 32q.. of both halves), one piece; the weight halves (128 rows), two pieces each. K tile t of the
// stream: W left + A q0 in phase 2 and W right + A q1 in phase 3 of K tile t - 2, A q2 / A q3 in phases
// 0 / 1 of K tile t - 1: every piece is issued >= 3 phases before its first read and restaged >= 2
// phases after its last read (the distance the one-barrier stagger needs for WAR). Waits are counted
// s_waitcnt vmcnt; a tile's epilogue issues exactly S vector-memory operations (rows past M are
// stored to a scratch slot, not skipped), counted into the waits they sit behind.
// The weight fragment is the MFMA's A operand, so a lane's accumulator holds 4 consecutive columns
// of one output row: the epilogue (bias, GELU, residual, store) runs from registers, no LDS pass.
// tools/gemm_probe.hip builds this header with WCB_GEMM_PROBE: wave 0 of every workgroup then stamps
// s_memtime at its phases into wcb_gemm_probe[workgroup][8] (its first tile)
#ifdef WCB_GEMM_PROBE
__device__ unsigned long long* wcb_gemm_probe;
#define GPROBE(k)                                                                              \
  do {                                                                                         \
    if (threadIdx.x == 0) wcb_gemm_probe[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define GPROBE(k) do {} while (0)
#endif
__device__ float wcb_pp_zeros[8192];            // the bias of a launch without one
__device__ __attribute__((aligned(16))) char wcb_pp_scratch[64 * 16];   // stores of rows past M

template <int N> WCB_DEV void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N < 63 ? N : 63) : "memory"); }

template <typename T, int EPI, int BN = 256>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmArgs g) {
  using Frag = typename DT<T>::frag;
  constexpr int BUF = 65536, WOFF = 32768;
  // BN = 256 or 192 output columns per tile: each wave's 16·FW columns are FW fragments, the weight
  // tile FW DMA pieces of 64 rows (192: the d-wide N = 768 shapes tile the chip in whole rounds)
  static_assert(BN == 256 || BN == 192, "tile width");
  constexpr int FW = BN / 64;
  // vector-memory operations per wave per K tile (A quarters 2, 3 of the next tile, W pieces + A quarters
  // 0, 1 of the one after), and a tile's epilogue: 8·FW stores (+ 8·FW residual loads). (Wave 0 also
  // moves the tile's bias values into LDS by one more DMA in phase 0 of its first K tile: every count
  // below then over-waits by one for that wave, which is safe.)
  constexpr int OPK = FW + 4;
  constexpr int S = 8 * FW + ((EPI & E_RESID) ? 8 * FW : 0);
  constexpr int BIAS_LDS = 2 * BUF;   // [tile parity][256] f32
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  GPROBE(0);
  const int tiles_n = g.N / BN, tiles_m = (g.M + 255) >> 8, ntiles = tiles_m * tiles_n;
  const int nk = g.K >> 6;
  const int my = (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;   // tiles of this workgroup
  const int total = my * nk;                                             // K tiles of its stream
  auto origin = [&](int it, int& m0, int& n0) {
    const int wg = xcd_remap((int)blockIdx.x + it * (int)gridDim.x, ntiles);
    if (g.raster > 0) {   // bands of `raster` row panels, column tiles outer within a band
      const int band = g.raster * tiles_n;
      const int fm = (wg / band) * g.raster, gm = min(tiles_m - fm, g.raster), r = wg % band;
      m0 = (fm + r % gm) * 256;
      n0 = (r / gm) * BN;
    } else {
      m0 = (wg / tiles_n) * 256;
      n0 = (wg % tiles_n) * BN;
    }
  };
  auto swzr = [](int r) { return (r >> 1) & 7; };
  const T* A = reinterpret_cast<const T*>(g.A);
  const T* W = reinterpret_cast<const T*>(g.W);
  // DMA geometry of this lane: A piece p → tile row ar[p] (element offset aoff[p] from the tile's first
  // row), W piece t → tile row 64t + i8 (boff[t])
  const int i8 = 8 * wave + (lane >> 3), ch = lane & 7;
  // the last row panel (m0 = m_last) re-reads row M - 1 for the rows past M: aoff_last
  const int m_last = (tiles_m - 1) * 256;
  int aoff[4], aoff_last[4], boff[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int ar = i8 < 32 ? 32 * p + i8 : 96 + 32 * p + i8;
    const int cs = (ch ^ swzr(ar)) << 3;
    aoff[p] = ar * (int)g.lda + cs;
    aoff_last[p] = (min(m_last + ar, g.M - 1) - m_last) * (int)g.lda + cs;
    boff[p] = (64 * min(p, FW - 1) + i8) * (int)g.ldw + ((ch ^ swzr(64 * p + i8)) << 3);
  }
  // stream cursors: tile iteration, K tile, tile origin, and the tile's A / W panel pointers advanced to
  // the K tile (scalar: a DMA adds only the lane's offset)
  struct Cur { int it, kt, m0, n0; const T* a; const T* b; bool last; };
  auto set_tile = [&](Cur& c) {
    origin(c.it, c.m0, c.n0);
    c.a = A + (long)c.m0 * g.lda;
    c.b = W + (long)c.n0 * g.ldw;
    c.last = c.m0 == m_last;
  };
  auto advance = [&](Cur& c) {
    c.a += 64;
    c.b += 64;
    if (++c.kt == nk) {
      c.kt = 0;
      if (++c.it < my) set_tile(c);
    }
  };
  auto dma_a = [&](int p, const Cur& c, int gk) {
    glds16(c.a + (c.last ? aoff_last[p] : aoff[p]),
           smem + (gk & 1) * BUF + (wave < 4 ? 32 * p + 8 * wave : 96 + 32 * p + 8 * wave) * 128);
  };
  auto dma_b = [&](int t, const Cur& c, int gk) {
    glds16(c.b + boff[t], smem + (gk & 1) * BUF + WOFF + (64 * t + 8 * wave) * 128);
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 acc[8][FW];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Cur cc;   // the K tile being multiplied
  cc.it = 0; cc.kt = 0;
  set_tile(cc);
  Cur c1 = cc, c2 = cc;   // the K tiles one and two ahead (their DMA)
  advance(c1);
  advance(c2);
  advance(c2);
  // K tiles 0 and 1 in the steady-state piece order
  dma_b(0, cc, 0); dma_b(1, cc, 0); dma_a(0, cc, 0); dma_b(2, cc, 0);
  if constexpr (FW == 4) dma_b(3, cc, 0);
  dma_a(1, cc, 0); dma_a(2, cc, 0); dma_a(3, cc, 0);
  if (total > 1) {
    dma_b(0, c1, 1); dma_b(1, c1, 1); dma_a(0, c1, 1); dma_b(2, c1, 1);
    if constexpr (FW == 4) dma_b(3, c1, 1);
    dma_a(1, c1, 1);
  }
  GPROBE(1);
  if (total > 1) vm_wait<3 + FW + 2>();   // W(0) and A q0(0) landed
  else vm_wait<3>();
  GPROBE(2);
  barrier();
  if (wr == 1) barrier();   // the stagger: waves 4-7 one barrier behind

  const int c0 = lane >> 4;
  const float* bias = g.bias ? g.bias : wcb_pp_zeros;
  // one K tile of the stream. ST (steady): K tile >= 2 of its tile with two more after it in the stream —
  // the waits are the plain counts and every DMA is issued, no run-time branch in its phases (the
  // general form's branches cost ≈ 600 cycles per K tile, tools/gemm_probe)
  // fragment reads: the swizzle term of row base + (lane & 15) is ((lane >> 1) & 7) for every 16-aligned
  // base, so a read address is a per-lane constant (one per k-step) plus a compile-time offset
  const int sl = (lane >> 1) & 7;
  const int lo0 = (lane & 15) * 128 + ((c0 ^ sl) << 4), lo1 = (lane & 15) * 128 + (((4 + c0) ^ sl) << 4);
  const int wb0 = WOFF + 16 * FW * wc * 128 + lo0, wb1 = WOFF + 16 * FW * wc * 128 + lo1;   // this wave's W rows
  const int ab0 = 128 * wr * 128 + lo0, ab1 = 128 * wr * 128 + lo1;                 // this wave's A rows
  auto ktile = [&](int gk, auto steady_tag) {
    constexpr bool ST = decltype(steady_tag)::value;
    const char* buf = smem + (gk & 1) * BUF;
    const bool n1 = ST || gk + 1 < total, n2 = ST || gk + 2 < total;
    // the previous tile's epilogue operations sit between this phase's piece and the younger ones
    const bool e0 = !ST && cc.kt == 0 && cc.it > 0, e1 = !ST && cc.kt == 1 && cc.it > 0;
    // the plain counts (one scalar branch per phase; the general cases below run on <= 3 K tiles a tile)
    const bool plain = ST || (n2 && !e0 && !e1);
    Frag bw[FW][2];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // retire the piece the NEXT phase reads (this phase's own pieces were retired one phase ago)
      if (plain) {
        if (p < 3) vm_wait<OPK>();
        else vm_wait<6>();
      } else if (p == 0) {
        if (n1) { if (e0 || e1) vm_wait<OPK + S>(); else vm_wait<OPK>(); }
        else { if (e0 || e1) vm_wait<2 + S>(); else vm_wait<2>(); }
      } else if (p == 1) {
        if (n1) { if (e0) vm_wait<OPK + S>(); else vm_wait<OPK>(); }
        else { if (e0) vm_wait<1 + S>(); else vm_wait<1>(); }
      } else if (p == 2) {
        if (n1) { if (e0) vm_wait<OPK + S>(); else vm_wait<OPK>(); }
        else { if (e0) vm_wait<S>(); else vm_wait<0>(); }
      } else if (n1) {
        if (n2) { if (e0) vm_wait<6 + S>(); else vm_wait<6>(); }
        else { if (e0) vm_wait<3 + S>(); else vm_wait<3>(); }
      }
      if (p == 0) {
#pragma unroll
        for (int j = 0; j < FW; ++j) {
          bw[j][0] = *reinterpret_cast<const Frag*>(buf + wb0 + j * 16 * 128);
          bw[j][1] = *reinterpret_cast<const Frag*>(buf + wb1 + j * 16 * 128);
        }
      }
      if (!ST && p == 0 && cc.kt == 0 && wave == 0)   // this tile's bias into LDS (a global load in the
                                                      // epilogue would make hipcc wait for every DMA piece)
        glds16(bias + (BN == 256 ? cc.n0 + 4 * lane : min(cc.n0 + 4 * lane, g.N - 4)), smem + BIAS_LDS + (cc.it & 1) * 1024);
      Frag af[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i][0] = *reinterpret_cast<const Frag*>(buf + ab0 + (32 * p + 16 * i) * 128);
        af[i][1] = *reinterpret_cast<const Frag*>(buf + ab1 + (32 * p + 16 * i) * 128);
      }
      if (p == 0 && n1) dma_a(2, c1, gk + 1);
      if (p == 1 && n1) dma_a(3, c1, gk + 1);
      if (p == 2 && n2) { dma_b(0, c2, gk + 2); dma_b(1, c2, gk + 2); dma_a(0, c2, gk + 2); }
      if (p == 3 && n2) {
        dma_b(2, c2, gk + 2);
        if constexpr (FW == 4) dma_b(3, c2, gk + 2);
        dma_a(1, c2, gk + 2);
      }
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < FW; ++j) acc[2 * p + i][j] = mma16(bw[j][ks], af[i][ks], acc[2 * p + i][j]);
      __builtin_amdgcn_s_setprio(0);
      barrier();
    }
  };
  for (int gk = 0; gk < total; ++gk) {
    ktile(gk, std::false_type{});
    if (gk == 0) GPROBE(3);
    if (gk == nk / 2) GPROBE(4);
    if (gk == 2 * nk - 1) GPROBE(7);   // the second tile's last K tile done
    if (cc.kt == nk - 1) {
      // epilogue of tile cc.it: lane → row m0 + 128·wr + 16·mi + (lane & 15), columns
      // n0 + 64·wc + 16·j + 4·(lane >> 4) + e; exactly S vector-memory operations per wave
      if (cc.it == 0) GPROBE(5);
      const int rb = cc.m0 + 128 * wr + (lane & 15);
      const int cb = cc.n0 + 16 * FW * wc + 4 * c0;
      f32x4 b4[FW];
#pragma unroll
      for (int j = 0; j < FW; ++j)
        b4[j] = *reinterpret_cast<const f32x4*>(smem + BIAS_LDS + (cc.it & 1) * 1024 + (16 * FW * wc + 4 * c0 + 16 * j) * 4);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const int m = rb + 16 * mi;
        const long off = (long)min(m, g.M - 1) * g.ldc + cb;
        f32x4 r4[FW];
        if constexpr ((EPI & E_RESID) != 0) {
#pragma unroll
          for (int j = 0; j < FW; ++j) r4[j] = *reinterpret_cast<const f32x4*>(g.resid + off + 16 * j);
        }
#pragma unroll
        for (int j = 0; j < FW; ++j) {
          f32x4 v = acc[mi][j] + b4[j];
          acc[mi][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          if constexpr ((EPI & E_GELU) != 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gelu_t<T>(v[e]);
          }
          if constexpr ((EPI & E_RESID) != 0) v += r4[j];
          if constexpr ((EPI & E_F32) != 0) {
            float* dst = m < g.M ? reinterpret_cast<float*>(g.out) + off + 16 * j
                                 : reinterpret_cast<float*>(wcb_pp_scratch + lane * 16);
            *reinterpret_cast<f32x4*>(dst) = v;
          } else {
            typedef short s4 __attribute__((ext_vector_type(4)));
            s4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = __builtin_bit_cast(short, DT<T>::fromf(v[e]));
            T* dst = m < g.M ? reinterpret_cast<T*>(g.out) + off + 16 * j : reinterpret_cast<T*>(wcb_pp_scratch + lane * 16);
            *reinterpret_cast<s4*>(dst) = o;
          }
        }
      }
      if (cc.it == 0) GPROBE(6);   // (issued, not drained)
    }
    cc = c1;
    c1 = c2;
    advance(c2);
  }
  if (wr == 0) barrier();   // balance the stagger
}

template <typename T, int EPI, int BN = 256>
static void launch_pp_e(const GemmArgs& g, hipStream_t s) {
  constexpr int kLds = 2 * 65536 + 2048;   // two K-tile buffers + two tiles' bias
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<T, EPI, BN>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    attr_set = true;
  }
  const int tiles = ((g.M + 255) / 256) * (g.N / BN);
  // one persistent workgroup per CU (LDS-bound); pp 3 (tools/gemm_probe): one tile per workgroup
  const dim3 grid((unsigned)(g.pp == 3 ? tiles : std::min(tiles, 256)));
  WCB_LAUNCH((gemm_pp_kernel<T, EPI, BN>), grid, dim3(512), kLds, s, g);
}

// the ping-pong kernel where it covers the launch: 16-bit, N % 256 == 0, K % 64 == 0 (>= 128), plain
// rows, epilogue (bias) / (bias) + GELU / (bias) + residual, f32 or T out, no clamp. g.pp 1 (runtime
// default): where it measured at least as fast as the LDS-ring kernel; 2: every covered shape (tests,
// microbenchmarks). tools/enc_bench.py: C2 (small) QKV 875 vs 868 TFLOP/s, fc1 880 vs 797; C3 (medium)
// QKV 1007 vs 1008, out 697 vs 614, fc1 949 vs 888, fc2 1064 vs 1002
template <typename T>
static bool launch_pp(const GemmArgs& g, hipStream_t s) {
  if constexpr (sizeof(T) != 2) {
    return false;
  } else {
    const bool n256 = g.N % 256 == 0, n192 = g.N % 192 == 0;
    if ((!n256 && !n192) || g.N > 8192 || g.K % 64 != 0 || g.K < 128 || g.a_Mb || g.c_Mb || g.addrow || g.mode != 0 ||
        g.clamp != 0.f || g.rst_out || g.out16 || g.M < 256 || (g.resid && !g.out_f32) || (g.resid && g.act))
      return false;
    // 192-wide tiles where they leave fewer tile rounds on 256 CUs (d-wide N = 768). pp 1: those shapes go
    // to the LDS-ring kernel's 256x192 tiles instead (measured faster than 256-wide ping-pong tiles: C2 out
    // 99 vs 104 µs, fc2 271 vs 277 µs); pp 4: the ping-pong kernel's own 192-wide tiles; pp 2 / 5 (tests,
    // microbenchmarks): 256- / 192-wide ping-pong tiles wherever N allows
    bool w192;
    if (g.pp == 2 || g.pp == 5) {
      w192 = g.pp == 5;
    } else {
      const long tm = (g.M + 255) / 256;
      const long r256 = n256 ? (tm * (g.N / 256) + 255) / 256 : 0, r192 = n192 ? (tm * (g.N / 192) + 255) / 256 : 0;
      w192 = !n256 || (n192 && r192 * 192 * 10 < r256 * 256 * 9);
      if (w192 && g.pp == 1) return false;
    }
    if ((w192 && !n192) || (!w192 && !n256)) return false;
    const int bits = (g.act == 1 ? E_GELU : 0) | (g.resid ? E_RESID : 0) | (g.out_f32 ? E_F32 : 0);
    if (w192) {
      switch (bits) {
        case 0: launch_pp_e<T, 0, 192>(g, s); return true;
        case E_GELU: launch_pp_e<T, E_GELU, 192>(g, s); return true;
        case E_F32: launch_pp_e<T, E_F32, 192>(g, s); return true;
        case E_RESID | E_F32: launch_pp_e<T, E_RESID | E_F32, 192>(g, s); return true;
        default: return false;
      }
    }
    switch (bits) {
      case 0: launch_pp_e<T, 0>(g, s); return true;
      case E_GELU: launch_pp_e<T, E_GELU>(g, s); return true;
      case E_F32: launch_pp_e<T, E_F32>(g, s); return true;
      case E_RESID | E_F32: launch_pp_e<T, E_RESID | E_F32>(g, s); return true;
      default: return false;
    }
  }
}

// Skinny GEMM for the decode step (M = batch <= 64 rows): one workgroup = NF·16 output columns,
// its NW waves split K into NW contiguous ranges of KS 32-deep MFMA steps, every load of a wave is
// issued up front (weights are streamed once from HBM, activations come from L2), partial tiles
// are summed through LDS.
//  * LN: the A operand is the f32 residual stream, normalised on the fly (the decoder's pre-block
//    LayerNorm fused into the projection that consumes it). Row statistics come from the
//    deterministic per-16-column partial sums (Σx, Σx²) the producer of x wrote (st_in).
//  * st_out: a residual-writing GEMM (NF = 1) publishes those partial sums of the new x rows.
//  * sel_val: the LM head reduces its logits tile to a per-row (max, argmax) partial with the
//    bias-list root boost and the EOS mask applied (k_select.hip finishes the reduction).
template <typename T, int MF, int NF, int NW, int KS, bool LN>
__global__ __launch_bounds__(NW * 64) void gemm_skinny_kernel(GemmArgs g) {
  using Frag = typename DT<T>::frag;
  constexpr int NT = NW * 64, BNC = NF * 16;
  // LDS slabs for the cross-wave K reduction: as many as fit in 48 KB, extra waves accumulate in rounds
  constexpr int SLAB = MF * 16 * (BNC + 1) * 4;
  constexpr int SL = (NW * SLAB <= 49152) ? NW : (NW / 2 * SLAB <= 49152) ? NW / 2 : (NW / 4 * SLAB <= 49152) ? NW / 4 : 1;
  __shared__ __attribute__((aligned(16))) float red[SL][MF * 16][BNC + 1];
  __shared__ float st_mean[MF * 16], st_rstd[MF * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mb = blockIdx.y * MF * 16;   // row block (M split over grid.y: more workgroups, less A per CU)
  // LN statistics partials first: the oldest loads retire first (in-order vmcnt), so the row
  // statistics are ready while the weight stream is still in flight
  constexpr int NB = NW * KS * 2;                          // 16-column blocks per row (K / 16)
  constexpr int TPR = NB % 16 == 0 ? 16 : NB % 8 == 0 ? 8 : NB % 4 == 0 ? 4 : NB % 2 == 0 ? 2 : 1;
  constexpr int RPP = NT / TPR;                            // rows per pass
  constexpr int PASSES = (MF * 16 + RPP - 1) / RPP;
  float s1[PASSES], s2[PASSES];
  if constexpr (LN) {
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int m = min(mb + ps * RPP + tid / TPR, g.M - 1);
      s1[ps] = 0.f;
      s2[ps] = 0.f;
      float2 pv[NB / TPR];
#pragma unroll
      for (int j = 0; j < NB / TPR; ++j)
        pv[j] = *reinterpret_cast<const float2*>(g.st_in + ((long)m * NB + j * TPR + tid % TPR) * 2);
#pragma unroll
      for (int j = 0; j < NB / TPR; ++j) { s1[ps] += pv[j].x; s2[ps] += pv[j].y; }
    }
  }
  const int n0 = blockIdx.x * BNC;
  const int kb = wave * (KS * 32) + 8 * (lane >> 4);
  Frag b[NF][KS];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const long n = min(n0 + j * 16 + (lane & 15), g.N - 1);
    const T* W = reinterpret_cast<const T*>(g.W) + n * g.ldw + kb;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) b[j][ks] = load_frag<T>(W + ks * 32);
  }
  // Epilogue operands (bias, residual, decode position) are fetched now, behind the weight
  // stream, instead of after the K reduction: one memory round trip less on the critical path.
  constexpr int EP = (MF * 16 * BNC + NT - 1) / NT;
  float pf_bias[EP], pf_res[EP];
#pragma unroll
  for (int ep = 0; ep < EP; ++ep) {
    const int t = ep * NT + tid, row = mb + t / BNC, nn = n0 + t % BNC;
    const bool ok = t < MF * 16 * BNC && row < g.M && nn < g.N;
    pf_bias[ep] = (ok && g.bias) ? g.bias[nn] : 0.f;
    pf_res[ep] = (ok && g.resid && g.mode == 0) ? g.resid[c_row(g, row) + nn] : 0.f;
  }
  const int pos_v = g.mode == 2 ? *g.pos : 0;
  f32x4 acc[MF][NF];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (LN) {
    const float* X = reinterpret_cast<const float*>(g.A);
    float xv[MF][KS][8];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int m = min(mb + i * 16 + (lane & 15), g.M - 1);
      const float* xr = X + a_row(g, m) + kb;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(xr + ks * 32);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(xr + ks * 32 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { xv[i][ks][e] = x0[e]; xv[i][ks][e + 4] = x1[e]; }
      }
    }
    float gw[KS][8], gb[KS][8];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(g.ln_w + kb + ks * 32);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(g.ln_w + kb + ks * 32 + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.ln_b + kb + ks * 32);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.ln_b + kb + ks * 32 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { gw[ks][e] = w0[e]; gw[ks][e + 4] = w1[e]; gb[ks][e] = b0[e]; gb[ks][e + 4] = b1[e]; }
    }
    // row statistics: TPR threads per row, fixed-order sums of the producer's partials
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      float a1 = s1[ps], a2 = s2[ps];
#pragma unroll
      for (int o = 1; o < TPR; o <<= 1) { a1 += __shfl_xor(a1, o, 64); a2 += __shfl_xor(a2, o, 64); }
      const int r = ps * RPP + tid / TPR;
      if (tid % TPR == 0 && r < MF * 16) {
        const float mean = a1 / g.K;
        st_mean[r] = mean;
        st_rstd[r] = rsqrtf(fmaxf(a2 / g.K - mean * mean, 0.f) + 1e-5f);
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const float mean = st_mean[i * 16 + (lane & 15)], rstd = st_rstd[i * 16 + (lane & 15)];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        Frag a;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = (xv[i][ks][e] - mean) * rstd * gw[ks][e] + gb[ks][e];
          if constexpr (sizeof(T) == 4) a[e] = v;
          else a[e] = __builtin_bit_cast(typename std::remove_reference<decltype(a[0])>::type, DT<T>::fromf(v));
        }
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = mma16(a, b[j][ks], acc[i][j]);
      }
    }
  } else {
    const T* A = reinterpret_cast<const T*>(g.A) + (g.a_grp_n ? (long)(n0 / g.a_grp_n) * g.a_grp_off : 0L);
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int m = min(mb + i * 16 + (lane & 15), g.M - 1);
      const T* ap = A + a_row(g, m) + kb;
      Frag a[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) a[ks] = load_frag<T>(ap + ks * 32);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = mma16(a[ks], b[j][ks], acc[i][j]);
    }
  }
#pragma unroll
  for (int round = 0; round < NW / SL; ++round) {
    if (wave / SL == round) {
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float& r = red[wave % SL][i * 16 + (lane >> 4) * 4 + e][j * 16 + (lane & 15)];
            r = round == 0 ? acc[i][j][e] : r + acc[i][j][e];
          }
    }
    __syncthreads();
  }
  const bool mask_eos = g.sel_val && *g.sel_step < g.sel_min_new;
  // epilogue: thread → (row, col) with the columns of a row contiguous in the wave, so row-wise
  // reductions (stats partials: 16 lanes; argmax partial: BNC lanes) are shuffles
#pragma unroll
  for (int ep = 0; ep < EP; ++ep) {
    const int t = ep * NT + tid;
    const int lrow = t / BNC, col = t % BNC, row = mb + lrow;
    const int nn = n0 + col;
    const bool valid = t < MF * 16 * BNC && row < g.M && nn < g.N;
    float v = 0.f;
    if (valid) {
#pragma unroll
      for (int w = 0; w < SL; ++w) v += red[w][lrow][col];
      v += pf_bias[ep];
      if (g.act == 1) v = gelu_t<T>(v);
      if (g.addrow) v += g.addrow[(long)(g.c_Mb ? row % g.c_Mb : row) * g.N + nn];
      if (g.mode == 2 && nn >= g.n_split) {   // k / v of the new token → self-attention KV cache
        const int n2 = nn - g.n_split;
        const int hh = n2 >> 6, dd = n2 & 63;
        const int kv = hh / g.hs_H, h = hh % g.hs_H;
        const int rps = g.kv_rps > 1 ? g.kv_rps : 1;
        const long off = ((((long)kv * g.hs_B + row / rps) * g.hs_H + h) * g.kv_T + pos_v + row % rps) * 64 + dd;
        reinterpret_cast<T*>(g.kv_out)[off] = DT<T>::fromf(v);
      } else if (g.mode == 1) {
        v = epi_store1<T>(g, row, nn, v);
      } else {
        const long off = c_row(g, row) + nn;
        v += pf_res[ep];
        if (g.out_f32) reinterpret_cast<float*>(g.out)[off] = v;
        else reinterpret_cast<T*>(g.out)[off] = DT<T>::fromf(v);
      }
    }
    if (g.st_out) {   // NF == 1: 16 contiguous lanes hold one row of the block
      float s1 = valid ? v : 0.f, s2 = valid ? v * v : 0.f;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
      if (valid && (t & 15) == 0) {
        float* p = g.st_out + ((long)row * g.st_nb + blockIdx.x) * 2;
        p[0] = s1;
        p[1] = s2;
      }
    }
    if (g.sel_val) {  // BNC == 64: one wave per row
      float x = -INFINITY;
      int xi = 0x7fffffff;
      if (valid) {
        x = v;
        if (g.sel_lam != 0.f)
          x = bias_bonus(x, g.sel_lam, g.sel_rowbase[row] + (int)((g.sel_root_bits[nn >> 5] >> (nn & 31)) & 1u));
        if (mask_eos && nn == g.sel_eos) x = -INFINITY;
        xi = nn;
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float ov = __shfl_xor(x, o, 64);
        const int oi = __shfl_xor(xi, o, 64);
        if (ov > x || (ov == x && oi < xi)) { x = ov; xi = oi; }
      }
      if (lane == 0 && row < g.M) {
        g.sel_val[(long)row * gridDim.x + blockIdx.x] = x;
        g.sel_idx[(long)row * gridDim.x + blockIdx.x] = xi;
      }
    }
  }
}

// Decode GEMM (gemm_dec_kernel): the decode-step projections at up to 32 rows per workgroup.
// Built from the chain-latency floor measured on MI355X (tools/chain_bench.hip): an empty kernel in a
// replayed chain costs 1.6 µs, one HBM round trip of 16 KB per workgroup +1.0 µs, 96 KB of the
// previous kernel's output per workgroup +2.2 µs — so a projection must (a) spread its weights over
// every CU (16 columns per tile), (b) issue every load of the launch in one burst before anything
// consumes one (hipcc otherwise sinks loads next to their uses and pays a round trip per group),
// (c) read as few activation bytes and issue as few load instructions per workgroup as possible.
//  * workgroup = NW waves (64·NW threads); rows [mb, mb + 16·MF); the K range is split over the waves
//    (KPW 32-deep k-steps each, K = 32·KPW·NW at compile time).
//  * AM 0: A = T rows; 3: grouped A (block-diagonal weights, A re-read per tile); 1 / 2: the decoder's
//    pre-block LayerNorm fused: A = LN(x) of the f32 residual rows g.A (1) or of their T-typed copy
//    g.ln_a16 (2, half the bytes). The row statistics are computed here from the very values the
//    workgroup loads (each wave sums its K slice of its lanes' rows, one LDS exchange), and the
//    LayerNorm weight / bias are staged once per workgroup through LDS: no per-lane parameter loads.
//  * the A fragments (MF×KPW per lane) are built once and stay in registers while the workgroup walks
//    its column tiles (P: blockIdx.x, blockIdx.x + gridDim.x, ...): the LM head streams its 79.7 MB
//    of weights through 256 column walkers without re-reading the activations per tile; the next
//    tile's weight fragments are loaded (nontemporal: read once) while the current tile reduces.
//  * one LDS exchange per tile (double-buffered: one barrier per tile), then every thread finishes
//    one (row, column) output: bias, GELU, residual, f32 / T / x16 stores, KV-cache append (mode 2),
//    per-16-column LN partial sums (st_out, the older skinny consumers) and the LM head's argmax
//    partial (sel_val: per workgroup and row, the running best over the tiles it walks).
template <typename T, int MF, int NW, int KPW, int AM, bool P, bool WFM = false>
__global__ __launch_bounds__(NW * 64) void gemm_dec_kernel(GemmArgs g) {
  using Frag = typename DT<T>::frag;
  constexpr int NT = NW * 64, K = NW * KPW * 32, R = MF * 16;
  constexpr bool LN = AM == 1 || AM == 2;
  constexpr int EP = (R * 16 + NT - 1) / NT;         // epilogue outputs per thread (per tile)
  __shared__ __attribute__((aligned(16))) float red[2][NW][R][17];
  __shared__ __attribute__((aligned(16))) float lnp[LN ? 2 * K : 4];        // LayerNorm weight, bias
  __shared__ float2 rst[LN ? NW : 1][LN ? R : 1];                          // per-wave (Σx, Σx²)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mb = blockIdx.y * R;
  const int ntile = (g.N + 15) >> 4;
  const int kb = wave * (KPW * 32) + 8 * (lane >> 4);
  const int pos_v = g.mode == 2 ? *g.pos : 0;
  const bool mask_eos = g.sel_val && *g.sel_step < g.sel_min_new;

  auto load_w = [&](Frag (&w)[KPW], int ct) {
    if constexpr (WFM) {   // fragment-major copy (kernels.h frag_major, this NW / KPW): 1 KiB per wave-instruction
      const T* W = reinterpret_cast<const T*>(g.W_fm) + (((long)ct * NW + wave) * KPW * 64 + lane) * 8;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) w[ks] = __builtin_nontemporal_load(reinterpret_cast<const Frag*>(W + ks * 512));
    } else {
      const long n = min(ct * 16 + (lane & 15), g.N - 1);
      const T* W = reinterpret_cast<const T*>(g.W) + n * g.ldw + kb;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) w[ks] = __builtin_nontemporal_load(reinterpret_cast<const Frag*>(W + ks * 32));
    }
  };
  // ---------------- every load of the launch is issued here
  // P (column walk): PD - 1 tiles of weights in flight ahead of the one being multiplied (PD 3 measured
  // slower than 2: LM head 27.0 vs 23.9 µs, rocprofv3 C2 decode)
  constexpr int PD = P ? 2 : 1;
  Frag wc[KPW], wn[PD][KPW];
  int ct = blockIdx.x;
  load_w(wc, ct);
  if constexpr (P) {
#pragma unroll
    for (int d = 0; d < PD - 1; ++d) load_w(wn[d], min(ct + (d + 1) * (int)gridDim.x, ntile - 1));
  }
  Frag a[MF][KPW];
  f32x4 xf[AM == 1 ? MF : 1][AM == 1 ? KPW : 1][2];
  if constexpr (AM == 0 || AM == 2) {
    const T* A0 = reinterpret_cast<const T*>(AM == 0 ? g.A : g.ln_a16);
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int m = min(mb + i * 16 + (lane & 15), g.M - 1);
      const T* ap = A0 + a_row(g, m) + kb;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) a[i][ks] = load_frag<T>(ap + ks * 32);
    }
  }
  if constexpr (AM == 1) {
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int m = min(mb + i * 16 + (lane & 15), g.M - 1);
      const float* xr = reinterpret_cast<const float*>(g.A) + a_row(g, m) + kb;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) {
        xf[i][ks][0] = *reinterpret_cast<const f32x4*>(xr + ks * 32);
        xf[i][ks][1] = *reinterpret_cast<const f32x4*>(xr + ks * 32 + 4);
      }
    }
  }
  constexpr int LQ = LN ? (2 * K / 4 + NT - 1) / NT : 1;   // LayerNorm parameter chunks per thread
  f32x4 lq[LQ];
  if constexpr (LN) {
#pragma unroll
    for (int j = 0; j < LQ; ++j) {
      const int c = (j * NT + tid) * 4;                      // [0, K): weight, [K, 2K): bias
      lq[j] = c < 2 * K ? *reinterpret_cast<const f32x4*>((c < K ? g.ln_w : g.ln_b) + (c < K ? c : c - K))
                        : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float pf_bias[EP], pf_res[EP];   // epilogue operands of this thread's outputs (single-tile launches)
  int pf_rb[EP];                   // bias-boost base units of this thread's rows (LM head)
#pragma unroll
  for (int it = 0; it < EP; ++it) {
    const int o = it * NT + tid;
    const int row = mb + (o >> 4), nn = ct * 16 + (o & 15);
    const bool ok = !P && o < R * 16 && row < g.M && nn < g.N;
    pf_bias[it] = (ok && g.bias) ? g.bias[nn] : 0.f;
    pf_res[it] = (ok && g.resid && !(g.mode == 2 && nn >= g.n_split)) ? g.resid[c_row(g, row) + nn] : 0.f;
    pf_rb[it] = (g.sel_val && g.sel_lam != 0.f && o < R * 16 && row < g.M) ? g.sel_rowbase[row] : 0;
  }
  __builtin_amdgcn_sched_barrier(0);
  // ---------------- LayerNorm of the A rows: statistics from the loaded values, parameters via LDS
  if constexpr (LN) {
    // the f32 value of an element is re-derived where needed (from the f32 rows, or exactly from the
    // loaded 16-bit bits): no f32 copy of the A fragments held across the statistics barrier (it put the
    // LN-fused LM-head walker at 256 VGPRs)
    auto xv = [&](int i, int ks, int e) -> float {
      if constexpr (AM == 1) return xf[i][ks][e >> 2][e & 3];
      else if constexpr (sizeof(T) == 4) return a[i][ks][e];
      else if constexpr (__is_same(T, bf16_t)) return bf16_to_f((bf16_t)a[i][ks][e]);
      else return float(a[i][ks][e]);
    };
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = xv(i, ks, e);
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
      }
      s1 = xor16_add(s1); s2 = xor16_add(s2);
      s1 = xor32_add(s1); s2 = xor32_add(s2);
      if (lane < 16) rst[wave][i * 16 + lane] = float2{s1, s2};
    }
#pragma unroll
    for (int j = 0; j < LQ; ++j) {
      const int c = (j * NT + tid) * 4;
      if (c < 2 * K) *reinterpret_cast<f32x4*>(lnp + c) = lq[j];
    }
    __syncthreads();
    if constexpr (AM == 2) {   // opaque to hipcc: the f32 values are converted again, not kept across the barrier
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int ks = 0; ks < KPW; ++ks) asm volatile("" : "+v"(a[i][ks]));
    }
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) { const float2 t = rst[w][i * 16 + (lane & 15)]; s1 += t.x; s2 += t.y; }
      const float mean = s1 / K;
      const float rstd = rsqrtf(fmaxf(s2 / K - mean * mean, 0.f) + 1e-5f);
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) {
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(lnp + kb + ks * 32);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(lnp + kb + ks * 32 + 4);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(lnp + K + kb + ks * 32);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(lnp + K + kb + ks * 32 + 4);
        Frag o;   // the fragment rebuilt whole (element-wise writes into a[i][ks] kept every f32 alive)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gw = e < 4 ? w0[e] : w1[e - 4], gb = e < 4 ? b0[e] : b1[e - 4];
          const float v = (xv(i, ks, e) - mean) * rstd * gw + gb;
          if constexpr (sizeof(T) == 4) o[e] = v;
          else o[e] = __builtin_bit_cast(typename std::remove_reference<decltype(o[0])>::type, DT<T>::fromf(v));
        }
        a[i][ks] = o;
      }
    }
  }

  float sel_best[EP];
  int sel_bi[EP];
#pragma unroll
  for (int it = 0; it < EP; ++it) { sel_best[it] = -INFINITY; sel_bi[it] = 0x7fffffff; }
  // bias-boost root bits of the tile's 16 columns (one 32-bit word: tiles are 16-aligned), fetched one
  // tile ahead with the weights (read in the epilogue they cost a dependent round trip per tile)
  const bool boost = g.sel_val && g.sel_lam != 0.f;
  uint32_t rbw = boost ? g.sel_root_bits[(ct * 16) >> 5] : 0u, rbn = 0u;
  int buf = 0;
  for (; ct < ntile; ct += gridDim.x) {
    const int n0 = ct * 16;
    // P (persistent column walk): the tile PD - 1 walker steps ahead goes in flight behind this one
    // (clamped: an unconditional load keeps hipcc from draining the queue at the loop head); the next
    // tile's boost bits one step ahead
    if constexpr (P) {
      load_w(wn[PD - 1], min(ct + PD * (int)gridDim.x, ntile - 1));
      if (boost) rbn = g.sel_root_bits[(min(ct + (int)gridDim.x, ntile - 1) * 16) >> 5];
    }
    if constexpr (AM == 3) {
      const T* A = reinterpret_cast<const T*>(g.A) + (long)(n0 / g.a_grp_n) * g.a_grp_off;
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int m = min(mb + i * 16 + (lane & 15), g.M - 1);
#pragma unroll
        for (int ks = 0; ks < KPW; ++ks) a[i][ks] = load_frag<T>(A + a_row(g, m) + kb + ks * 32);
      }
    }
    f32x4 acc[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) acc[i] = mma16(a[i][ks], wc[ks], acc[i]);
    }
    // partial tile of this wave → LDS: lane holds rows 4(lane>>4)+e of tile i, column lane&15
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[buf][wave][i * 16 + (lane >> 4) * 4 + e][lane & 15] = acc[i][e];
    __syncthreads();
    // epilogue: output o = tid + NT·it → (row o/16, column o%16): a row's 16 columns are 16
    // consecutive lanes, so the per-row reductions (LN partials, argmax partial) are shuffles
#pragma unroll
    for (int it = 0; it < EP; ++it) {
      const int o = it * NT + tid;
      const int lrow = o >> 4, col = o & 15, row = mb + lrow, nn = n0 + col;
      const bool valid = o < R * 16 && row < g.M && nn < g.N;
      float v = 0.f;
      if (o < R * 16) {
#pragma unroll
        for (int w = 0; w < NW; ++w) v += red[buf][w][lrow][col];
      }
      if (valid) {
        if (g.bias) v += P ? g.bias[nn] : pf_bias[it];
        if (g.act == 1) v = gelu_t<T>(v);
        if (g.mode == 2 && nn >= g.n_split) {   // k / v of the new token → self-attention KV cache
          const int n2 = nn - g.n_split;
          const int hh = n2 >> 6, dd = n2 & 63;
          const int kv = hh / g.hs_H, h = hh % g.hs_H;
          const int rps = g.kv_rps > 1 ? g.kv_rps : 1;
          const long off = ((((long)kv * g.hs_B + row / rps) * g.hs_H + h) * g.kv_T + pos_v + row % rps) * 64 + dd;
          reinterpret_cast<T*>(g.kv_out)[off] = DT<T>::fromf(v);
        } else if (!g.sel_val || g.out) {
          const long off = c_row(g, row) + nn;
          if (g.resid) v += P ? g.resid[off] : pf_res[it];
          if (g.out_f32) reinterpret_cast<float*>(g.out)[off] = v;
          else reinterpret_cast<T*>(g.out)[off] = DT<T>::fromf(v);
          if (g.out16) reinterpret_cast<T*>(g.out16)[off] = DT<T>::fromf(v);
        }
      }
      if (g.st_out) {
        float a1 = valid ? v : 0.f, a2 = valid ? v * v : 0.f;
#pragma unroll
        for (int x = 1; x < 16; x <<= 1) { a1 += __shfl_xor(a1, x, 64); a2 += __shfl_xor(a2, x, 64); }
        if (valid && col == 0) {
          float* p = g.st_out + ((long)row * g.st_nb + ct) * 2;
          p[0] = a1;
          p[1] = a2;
        }
      }
      if (g.sel_val) {
        float x = -INFINITY;
        int xi = 0x7fffffff;
        if (valid) {
          x = v;
          if (g.sel_lam != 0.f)
            x = bias_bonus(x, g.sel_lam, pf_rb[it] + (int)((rbw >> (nn & 31)) & 1u));
          if (mask_eos && nn == g.sel_eos) x = -INFINITY;
          xi = nn;
        }
#pragma unroll
        for (int x2 = 1; x2 < 16; x2 <<= 1) {
          const float ov = __shfl_xor(x, x2, 64);
          const int oi = __shfl_xor(xi, x2, 64);
          if (ov > x || (ov == x && oi < xi)) { x = ov; xi = oi; }
        }
        // tiles are walked in increasing column order: a later tile wins only when strictly better
        if (x > sel_best[it]) { sel_best[it] = x; sel_bi[it] = xi; }
      }
    }
    buf ^= 1;
    if constexpr (P) {
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) wc[ks] = wn[0][ks];
#pragma unroll
      for (int d = 0; d < PD - 1; ++d)
#pragma unroll
        for (int ks = 0; ks < KPW; ++ks) wn[d][ks] = wn[d + 1][ks];
      rbw = rbn;
    } else {
      break;
    }
  }
  if (g.sel_val) {   // one argmax partial per (row, workgroup): sel_val[row][blockIdx.x]
#pragma unroll
    for (int it = 0; it < EP; ++it) {
      const int o = it * NT + tid, row = mb + (o >> 4);
      if ((o & 15) == 0 && o < R * 16 && row < g.M) {
        g.sel_val[(long)row * gridDim.x + blockIdx.x] = sel_best[it];
        g.sel_idx[(long)row * gridDim.x + blockIdx.x] = sel_bi[it];
      }
    }
  }
}

// Lean decode projection (dec_lean_kernel): the single-tile launches of gemm_dec_kernel (every decode
// projection of <= 64 rows except the LM head) with the same arithmetic — the same K split over the
// waves, LayerNorm statistics and normalisation, MFMA order and wave-partial sum order, so the
// outputs are bit-identical — restructured for the launch-latency floor measured in
// tools/dec_kernel_bench.hip (a byte-matched stream kernel 2.0 µs per chained launch against 3.8-8.4
// µs for gemm_dec_kernel): (a) a compact argument block (DecLean, one scalar load batch, where
// GemmArgs took three dependent kernel-argument round trips before the activation loads were
// issued); (b) every vector load of the launch — weights, activations, LayerNorm γ/β (per lane,
// straight from global memory: no LDS staging), bias, residual, the device-side cache position — in
// one unconditional burst (clamped indices; a conditional load made hipcc drain the queue with
// vmcnt(0) before the LayerNorm parameters, i.e. a second memory round trip); (c) an epilogue of 4
// consecutive columns per thread (16-byte f32 and 8-byte 16-bit stores).
//   EPI 0: out (T) = act(acc + bias);  1: x (f32) += acc + bias, x16 = T(x);  2: QKV — columns below
//   n_split → out (T), the rest → the self-attention KV cache at the device-side position.
//   GRP: block-diagonal A (q'_h = W_k,hᵀ q_h: K = 64, the A row of column block n0 starts
//   (n0 / grp_n)·grp_off further), no bias.
template <typename T> struct DecLean {
  const T* W; const T* A; const float* bias; const float* gam; const float* bet;
  float* x; T* out; T* kv; const int* pos;
  int M, N, lda, ldo;
  int n_split, kvB, kvH, kvT;
  int grp_n, grp_off;
  unsigned long long* stamp = nullptr;   // tools/dec_kernel_bench: per-workgroup phase stamps (null: off)
  int cfm_nw = 0, cfm_kpw = 0;           // EPI 0: out written fragment-major for a consumer with this split (0: rows)
  T* out2 = nullptr;                     // EPI 1: the 16-bit copy again, fragment-major with (cfm_nw, cfm_kpw)
  // FZ 2 (EPI 0, the cross-attention query): q'_h = W_k,hᵀ q_h in the same launch — kq_w = W_kt's
  // fragment-major copy ([H·D/16 tiles][2 waves][lane][8]), qp → att [M][ld_att] (T). cnt: the 64-bit
  // arrival counters of the (row block, head) groups ([gridDim.y][kvH], monotonic); err: set when a wait
  // ran out its bound
  T* att = nullptr; int ld_att = 0; unsigned long long* cnt = nullptr; int* err = nullptr;
  const T* kq_w = nullptr;
  Stamp lst;                             // stamps pass: launch start / end inside the decode graph
  const float* ln_u = nullptr;           // FOLD: u[n] = Σ_k W'[n][k] (bias = c[n])
};

//   FZ 2 (EPI 0, LN: the cross-attention query q_h = LN(x) W_q,hᵀ + b_q): the 4 column tiles of a head store
//   q_h write-through, meet at the head's counter, and each then computes a quarter of q'_h = W_k,hᵀ q_h
//   (the grouped K = 64 product of the kq launch it replaces: the same two 32-deep MFMA halves summed in
//   the same order, weights prefetched with the launch's first loads) — bit-identical to the two launches.
//   FOLD (LN): the LayerNorm folded into the weights (the beam ring tiles' LNF algebra): W = W·diag(γ)
//   (fragment-major), bias = c[n] = Σ_k β_k W[n][k] + b[n], ln_u = u[n] = Σ_k W'[n][k]; the MFMAs start on the
//   raw 16-bit rows as soon as they land, the row statistics ride the partial-tile barrier, and the epilogue
//   applies r·(acc − μ·u[n]) + c[n] — no γ / β loads, no statistics barrier, no per-element normalisation.
template <typename T, int MF, int NW, int KPW, bool LN, int EPI, bool GELU, bool GRP, bool WFM = false, bool AFM = false,
          int FZ = 0, bool FOLD = false>
__global__ __launch_bounds__(NW * 64) void dec_lean_kernel(DecLean<T> p) {
  constexpr bool KQ = FZ == 2 && EPI == 0 && LN && !GELU && !GRP;
  static_assert(!FOLD || (LN && !KQ), "folded LayerNorm: LN-fused launches without the cross-query hand-off");
  constexpr bool LNN = LN && !FOLD;   // normalise the A rows in the kernel
  using Frag = typename DT<T>::frag;
  constexpr int NT = NW * 64, K = NW * KPW * 32, R = MF * 16;
  static_assert(R * 4 <= NT, "epilogue: 4 columns per thread");
  __shared__ __attribute__((aligned(16))) float red[NW][R][17];
  __shared__ float2 rst[LN ? NW : 1][LN ? R : 1];
  __shared__ __attribute__((aligned(16))) float lnp[LNN ? 2 * K : 4];   // γ [K], β [K]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = blockIdx.x, mb = blockIdx.y * R, n0 = ct * 16;
  const int kb = wave * (KPW * 32) + 8 * (lane >> 4);
  const unsigned long long t0 = (p.stamp || p.lst.base) ? stamp_now() : 0ull;
  // ---------------- the launch's loads, one burst
  Frag w[KPW];
  if constexpr (WFM) {   // fragment-major weights: [tile][wave][k-step][lane][8], 1 KiB per wave-instruction
    const T* Wr = p.W + (((long)ct * NW + wave) * KPW * 64 + lane) * 8;
#pragma unroll
    for (int ks = 0; ks < KPW; ++ks) w[ks] = __builtin_nontemporal_load(reinterpret_cast<const Frag*>(Wr + ks * 512));
  } else {
    const T* Wr = p.W + (long)min(n0 + (lane & 15), p.N - 1) * K + kb;
#pragma unroll
    for (int ks = 0; ks < KPW; ++ks) w[ks] = __builtin_nontemporal_load(reinterpret_cast<const Frag*>(Wr + ks * 32));
  }
  Frag a[MF][KPW];
  if constexpr (AFM) {   // fragment-major activations [row block][wave][k-step][lane][8] (the producer's layout)
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const T* ar = p.A + ((((long)(mb / 16 + i) * NW + wave) * KPW * 64) + lane) * 8;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) a[i][ks] = load_frag<T>(ar + ks * 512);
    }
  } else {
    const T* A0 = p.A + (GRP ? (long)(n0 / p.grp_n) * p.grp_off : 0L) + kb;
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const T* ar = A0 + (long)min(mb + i * 16 + (lane & 15), p.M - 1) * p.lda;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) a[i][ks] = load_frag<T>(ar + ks * 32);
    }
  }
  // LayerNorm γ / β: into LDS by LDS-DMA with the burst (one 16-byte piece per lane, K / 4 lanes each), read
  // per k-step after the statistics barrier (held in registers they took 2·KPW·8 floats per lane and kept
  // the LN-fused instances at one workgroup per CU)
  if constexpr (LNN) {
    for (int c = wave * 64; c < K / 4; c += NT) {   // (K / 4 is a multiple of 64: wave-uniform)
      glds16(p.gam + 4 * (c + lane), lnp + 4 * c);
      glds16(p.bet + 4 * (c + lane), lnp + K + 4 * c);
    }
  }
  // epilogue operands: thread → row er (local), columns ec .. ec + 3
  const int er = tid >> 2, ec = n0 + (tid & 3) * 4;
  const int erow = min(mb + min(er, R - 1), p.M - 1);
  const int ecc = min(ec, p.N - 4);
  f32x4 bias4 = f32x4{0.f, 0.f, 0.f, 0.f}, res4 = bias4, u4 = bias4;
  if constexpr (!GRP) bias4 = *reinterpret_cast<const f32x4*>(p.bias + ecc);
  if constexpr (FOLD) u4 = *reinterpret_cast<const f32x4*>(p.ln_u + ecc);
  if constexpr (EPI == 1) res4 = *reinterpret_cast<const f32x4*>(p.x + (long)erow * p.ldo + ecc);
  int pos = 0;
  if constexpr (EPI == 2) pos = __builtin_nontemporal_load(p.pos);
  // KQ: this workgroup's share of q'_h = W_k,hᵀ q_h — K / 64 of the head's K / 16 column tiles, tile t of
  // the share on wave t % NW — and their W_kt fragments (two 32-deep halves each), loaded with the burst
  constexpr int KQT = KQ ? (K / 64 + NW - 1) / NW : 1;
  Frag kqw[KQT][2];
  if constexpr (KQ) {
    const int hq = n0 >> 6, jq = (n0 >> 4) & 3;
#pragma unroll
    for (int t = 0; t < KQT; ++t) {
      const int tt = min(wave + t * NW, K / 64 - 1);
      const long ct = (long)hq * (K / 16) + jq * (K / 64) + tt;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
        kqw[t][kh] = __builtin_nontemporal_load(reinterpret_cast<const Frag*>(p.kq_w + ((ct * 2 + kh) * 64 + lane) * 8));
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = 0, t2 = 0;
  if (p.stamp) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); t1 = stamp_now(); }
  // ---------------- LayerNorm of the A rows (gemm_dec_kernel AM = 2 arithmetic)
  // (the f32 value of an element is re-derived from its 16-bit bits where needed: exact, no copy kept)
  auto xf = [&](int i, int ks, int e) -> float {
    if constexpr (__is_same(T, bf16_t)) return bf16_to_f((bf16_t)a[i][ks][e]);
    else return float(a[i][ks][e]);
  };
  if constexpr (LN) {   // row statistics partials of this wave's K slice (FOLD: read after the tile barrier)
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = xf(i, ks, e);
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
      }
      s1 = xor16_add(s1); s2 = xor16_add(s2);
      s1 = xor32_add(s1); s2 = xor32_add(s2);
      if (lane < 16) rst[wave][i * 16 + lane] = float2{s1, s2};
    }
  }
  if constexpr (LNN) {
    float mean[MF], rstd[MF];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's γ / β pieces landed (LDS-DMA)
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) { const float2 t = rst[q][i * 16 + (lane & 15)]; s1 += t.x; s2 += t.y; }
      mean[i] = s1 / K;
      rstd[i] = rsqrtf(fmaxf(s2 / K - mean[i] * mean[i], 0.f) + 1e-5f);
    }
#pragma unroll
    for (int ks = 0; ks < KPW; ++ks) {
      const f32x4 g0 = *reinterpret_cast<const f32x4*>(lnp + kb + ks * 32);
      const f32x4 g1 = *reinterpret_cast<const f32x4*>(lnp + kb + ks * 32 + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(lnp + K + kb + ks * 32);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(lnp + K + kb + ks * 32 + 4);
#pragma unroll
      for (int i = 0; i < MF; ++i) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gw = e < 4 ? g0[e] : g1[e - 4], gb = e < 4 ? b0[e] : b1[e - 4];
          const float v = (xf(i, ks, e) - mean[i]) * rstd[i] * gw + gb;
          a[i][ks][e] = __builtin_bit_cast(typename std::remove_reference<decltype(a[0][0][0])>::type, DT<T>::fromf(v));
        }
      }
    }
  }
  // ---------------- MFMA over this wave's K slice, partial tiles through LDS
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KPW; ++ks) acc = mma16(a[i][ks], w[ks], acc);
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wave][i * 16 + (lane >> 4) * 4 + e][lane & 15] = acc[e];
  }
  __syncthreads();
  if (p.stamp) t2 = stamp_now();
  // ---------------- epilogue: 4 consecutive columns of one row per thread
  const int row = mb + er;
  const bool live = er < R && row < p.M && ec < p.N;
  if (!KQ && !live) return;   // (KQ: every thread reaches the hand-off below)
  if (live) {
  float fm_mean = 0.f, fm_rstd = 1.f;
  if constexpr (FOLD) {   // the row's (μ, r) from the waves' partials, the LN path's order and formula
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) { const float2 t = rst[q][er]; s1 += t.x; s2 += t.y; }
    fm_mean = s1 / K;
    fm_rstd = rsqrtf(fmaxf(s2 / K - fm_mean * fm_mean, 0.f) + 1e-5f);
  }
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += red[q][er][(tid & 3) * 4 + e];
    if constexpr (FOLD) s = fm_rstd * (s - fm_mean * u4[e]);
    v[e] = s + bias4[e];
    if constexpr (GELU) v[e] = gelu_t<T>(v[e]);
  }
  typedef short s4 __attribute__((ext_vector_type(4)));
  if constexpr (EPI == 1) {
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = v[e] + res4[e];
    const long off = (long)row * p.ldo + ec;
    *reinterpret_cast<f32x4*>(p.x + off) = o;
    s4 h;
#pragma unroll
    for (int e = 0; e < 4; ++e) h[e] = __builtin_bit_cast(short, DT<T>::fromf(o[e]));
    *reinterpret_cast<s4*>(p.out + off) = h;
    if (p.out2) {   // fragment-major copy for the LN-fused consumers (4 elements of one fragment)
      const int kw = p.cfm_kpw * 32, w2 = ec / kw, ks2 = (ec % kw) >> 5, lg = (ec & 31) >> 3;
      *reinterpret_cast<s4*>(p.out2 + ((((long)(row >> 4) * p.cfm_nw + w2) * p.cfm_kpw + ks2) * 64 + lg * 16 + (row & 15)) * 8 +
                             (ec & 7)) = h;
    }
  } else {
    s4 hv;
#pragma unroll
    for (int e = 0; e < 4; ++e) hv[e] = __builtin_bit_cast(short, DT<T>::fromf(v[e]));
    if (EPI == 2 && ec >= p.n_split) {   // k / v of the new token → self-attention KV cache
      const int n2 = ec - p.n_split, hh = n2 >> 6, dd = n2 & 63;
      const int kvs = hh / p.kvH, hd = hh % p.kvH;
      const long off = ((((long)kvs * p.kvB + row) * p.kvH + hd) * p.kvT + pos) * 64 + dd;
      *reinterpret_cast<s4*>(p.kv + off) = hv;
    } else if (EPI == 0 && p.cfm_nw) {   // fragment-major for the consumer's (waves, k-steps): 4 elements of one fragment
      const int kw = p.cfm_kpw * 32, w2 = ec / kw, ks2 = (ec % kw) >> 5, lg = (ec & 31) >> 3;
      const long off = ((((long)(row >> 4) * p.cfm_nw + w2) * p.cfm_kpw + ks2) * 64 + lg * 16 + (row & 15)) * 8 + (ec & 7);
      *reinterpret_cast<s4*>(p.out + off) = hv;
    } else if constexpr (KQ) {           // q_h, handed to the head's W_k,hᵀ products
      st_sc1(p.out + (long)row * p.ldo + ec, __builtin_bit_cast(uint64_t, hv));
    } else {
      *reinterpret_cast<s4*>(p.out + (long)row * p.ldo + ec) = hv;
    }
  }
  }   // live
  if constexpr (KQ) {
    const int hq = n0 >> 6, jq = (n0 >> 4) & 3;
    group_arrive_wait(p.cnt + blockIdx.y * p.kvH + hq, 4, p.err);
    // A = q_h rows of this block (lane: row lane & 15, k = 32·kh + 8·(lane >> 4)), sc1 loads
    Frag qa[2];
    {
      const T* qr = p.out + (long)min(mb + (lane & 15), p.M - 1) * p.ldo + hq * 64 + 8 * (lane >> 4);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const uint64_t w0 = ld_sc1(qr + kh * 32), w1 = ld_sc1(qr + kh * 32 + 4);
        typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
        qa[kh] = __builtin_bit_cast(Frag, u2{w0, w1});
      }
    }
#pragma unroll
    for (int t = 0; t < KQT; ++t) {
      const int tt = wave + t * NW;
      if (tt < K / 64) {
        const int c0 = jq * (K / 4) + tt * 16;   // first q'_h column of the tile
        const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 a0 = mma16(qa[0], kqw[t][0], z), a1 = mma16(qa[1], kqw[t][1], z);
        // C layout: lane holds rows 4·(lane >> 4) + e of column lane & 15; the kq launch's sum order
        // ((0 + wave 0 half) + wave 1 half) + bias 0
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rr = mb + 4 * (lane >> 4) + e;
          float sum = 0.f;
          sum += a0[e];
          sum += a1[e];
          const float v = sum + 0.f;
          if (rr < p.M) p.att[(long)rr * p.ld_att + hq * K + c0 + (lane & 15)] = DT<T>::fromf(v);
        }
      }
    }
  }
  if (p.stamp && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long* st = p.stamp + (long)(blockIdx.y * gridDim.x + blockIdx.x) * 4;
    st[0] = t0; st[1] = t1; st[2] = t2; st[3] = stamp_now();
  }
  if (p.lst.base && tid == 0) stamp_commit(p.lst, t0);   // (thread 0 stores in every workgroup)
}

inline thread_local unsigned long long* g_lean_stamp = nullptr;   // tools/dec_kernel_bench only

template <typename T, int MF, int NW, int KPW, bool LN, int EPI, bool GELU, bool GRP, bool FOLD = false>
static void launch_lean_k(const GemmArgs& g, hipStream_t s) {
  DecLean<T> p;
  if constexpr (FOLD) {   // folded LayerNorm: W' fragment-major, c[n] as the bias, u[n]; A = the raw 16-bit rows
    if (!g.ln_wg_fm || !g.ln_u || !g.ln_c) throw std::runtime_error("internal error: folded lean launch without its folded weights");
    p.stamp = g_lean_stamp;
    if (g.lstamp) p.lst = *g.lstamp;
    p.W = reinterpret_cast<const T*>(g.ln_wg_fm);
    p.A = reinterpret_cast<const T*>(g.ln_a16);
    p.bias = g.ln_c; p.ln_u = g.ln_u;
    p.out = reinterpret_cast<T*>(g.out);
    p.kv = reinterpret_cast<T*>(g.kv_out); p.pos = g.pos;
    p.M = g.M; p.N = g.N; p.lda = (int)g.lda; p.ldo = (int)g.ldc;
    p.n_split = g.n_split; p.kvB = g.hs_B; p.kvH = g.hs_H; p.kvT = g.kv_T;
    if (g.c_fm) lean_cfg(g.N, p.cfm_nw, p.cfm_kpw);
    const dim3 grid((g.N + 15) / 16, (g.M + MF * 16 - 1) / (MF * 16));
    if (g.a_fm) WCB_LAUNCH((dec_lean_kernel<T, MF, NW, KPW, LN, EPI, GELU, GRP, true, true, 0, true>), grid, dim3(NW * 64), 0, s, p);
    else WCB_LAUNCH((dec_lean_kernel<T, MF, NW, KPW, LN, EPI, GELU, GRP, true, false, 0, true>), grid, dim3(NW * 64), 0, s, p);
    return;
  }
  p.stamp = g_lean_stamp;
  if (g.lstamp) p.lst = *g.lstamp;
  p.W = reinterpret_cast<const T*>(g.W_fm ? g.W_fm : g.W);
  p.A = reinterpret_cast<const T*>(LN ? g.ln_a16 : g.A);
  p.bias = g.bias; p.gam = g.ln_w; p.bet = g.ln_b;
  p.x = EPI == 1 ? reinterpret_cast<float*>(g.out) : nullptr;
  p.out = reinterpret_cast<T*>(EPI == 1 ? g.out16 : g.out);
  p.kv = reinterpret_cast<T*>(g.kv_out); p.pos = g.pos;
  p.M = g.M; p.N = g.N; p.lda = (int)g.lda; p.ldo = (int)g.ldc;
  p.n_split = g.n_split; p.kvB = g.hs_B; p.kvH = g.hs_H; p.kvT = g.kv_T;
  p.grp_n = g.a_grp_n; p.grp_off = (int)g.a_grp_off;
  if (g.c_fm || g.out16_fm) lean_cfg(g.N, p.cfm_nw, p.cfm_kpw);   // the consumer's split of K = this N
  p.out2 = reinterpret_cast<T*>(g.out16_fm);
  const dim3 grid((g.N + 15) / 16, (g.M + MF * 16 - 1) / (MF * 16));
  if constexpr (EPI == 0 && LN && !GELU && !GRP) {
    if (g.kq_w) {   // the cross-attention query and q'_h = W_k,hᵀ q_h in one launch (fragment-major weights)
      if (!g.W_fm) throw std::runtime_error("internal error: fused cross-query needs the fragment-major weights");
      if (!g.kq_cnt || !g.kq_err) throw std::runtime_error("internal error: fused cross-query without its arrival counters");
      p.att = reinterpret_cast<T*>(g.kq_out); p.ld_att = (int)g.kq_ld; p.cnt = g.kq_cnt; p.err = g.kq_err;
      p.kq_w = reinterpret_cast<const T*>(g.kq_w); p.kvH = g.hs_H;
      if (g.a_fm) WCB_LAUNCH((dec_lean_kernel<T, MF, NW, KPW, LN, EPI, GELU, GRP, true, true, 2>), grid, dim3(NW * 64), 0, s, p);
      else WCB_LAUNCH((dec_lean_kernel<T, MF, NW, KPW, LN, EPI, GELU, GRP, true, false, 2>), grid, dim3(NW * 64), 0, s, p);
      return;
    }
  }
  if (g.a_fm) {
    if constexpr (!GRP) WCB_LAUNCH((dec_lean_kernel<T, MF, NW, KPW, LN, EPI, GELU, GRP, true, true>), grid, dim3(NW * 64), 0, s, p);
  } else if (g.W_fm) {
    WCB_LAUNCH((dec_lean_kernel<T, MF, NW, KPW, LN, EPI, GELU, GRP, true>), grid, dim3(NW * 64), 0, s, p);
  } else {
    WCB_LAUNCH((dec_lean_kernel<T, MF, NW, KPW, LN, EPI, GELU, GRP>), grid, dim3(NW * 64), 0, s, p);
  }
}

// Greedy cross-attention query and its encoder-space form in ONE launch without a hand-off
// (dec_xqk_kernel): workgroup (head h, q' column chunk c, 16·MF-row block) computes the head's whole
// q_h = LN(x) W_q,hᵀ + b_q,h for its rows (the folded LayerNorm, the lean q_proj launch's K split, MFMA and
// wave-sum order and epilogue: bit-identical q_h), keeps it in LDS, and multiplies it by its chunk of
// W_k,hᵀ (the kq launch's two 32-deep halves summed in that launch's order: bit-identical q'_h). Each of a
// head's NCH chunk workgroups recomputes q_h (W_q,h re-read from L2 NCH times): no cross-workgroup
// dependency, one launch boundary less per layer than xq → kq.
template <typename T> struct XqkArgs {
  const T* A; const T* Wq; const float* u; const float* c; const T* Wk; T* qp;
  int M, H, D;   // rows, heads, d_model (K of the q projection; q'_h has D columns)
};
template <typename T, int MF, int NW, int KPW, int NCH, bool AFM>
__global__ __launch_bounds__(NW * 64) void dec_xqk_kernel(XqkArgs<T> p) {
  using Frag = typename DT<T>::frag;
  constexpr int NT = NW * 64, K = NW * KPW * 32, R = MF * 16;
  constexpr int CW = K / NCH, NT16 = CW / 16, TPW = (NT16 + NW - 1) / NW;   // q' columns per chunk, tiles
  static_assert(CW % 16 == 0 && R * 16 <= NT, "chunk of whole tiles; one 4-column item per thread");
  __shared__ __attribute__((aligned(16))) float red[NW][R][65];
  __shared__ float2 rst[NW][R];
  __shared__ __attribute__((aligned(16))) T qa[R][72];     // q_h (16-bit), rows padded against bank conflicts
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);          // a head's chunks run on one XCD (W_q,h in its L2)
  const int h = wg / NCH, ch = wg % NCH, mb = blockIdx.y * R;
  const int kb = wave * (KPW * 32) + 8 * (lane >> 4);
  // ---------------- the launch's loads, one burst: W_q,h's 4 column tiles, the A rows, this chunk's W_k,hᵀ
  Frag w[4][KPW], a[MF][KPW], wk[TPW][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const T* wr = p.Wq + ((((long)(h * 4 + j) * NW + wave) * KPW * 64) + lane) * 8;
#pragma unroll
    for (int ks = 0; ks < KPW; ++ks) w[j][ks] = __builtin_nontemporal_load(reinterpret_cast<const Frag*>(wr + ks * 512));
  }
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    if constexpr (AFM) {
      const T* ar = p.A + ((((long)(mb / 16 + i) * NW + wave) * KPW * 64) + lane) * 8;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) a[i][ks] = load_frag<T>(ar + ks * 512);
    } else {
      const T* ar = p.A + (long)min(mb + i * 16 + (lane & 15), p.M - 1) * K + kb;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) a[i][ks] = load_frag<T>(ar + ks * 32);
    }
  }
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tt = min(wave + t * NW, NT16 - 1);
    const long ct = (long)h * (K / 16) + ch * NT16 + tt;   // W_kt fragment-major tile (K = 64: two k-steps)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) wk[t][kh] = __builtin_nontemporal_load(reinterpret_cast<const Frag*>(p.Wk + ((ct * 2 + kh) * 64 + lane) * 8));
  }
  // epilogue item of the q_h phase: row er, columns cq .. cq + 3 of the head
  const int er = tid >> 4, cq = (tid & 15) * 4;
  const bool item = er < R;
  const f32x4 u4 = *reinterpret_cast<const f32x4*>(p.u + h * 64 + cq);
  const f32x4 c4 = *reinterpret_cast<const f32x4*>(p.c + h * 64 + cq);
  __builtin_amdgcn_sched_barrier(0);
  // ---------------- row statistics partials (the lean LN arithmetic) and the q_h MFMAs
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int ks = 0; ks < KPW; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v;
        if constexpr (__is_same(T, bf16_t)) v = bf16_to_f((bf16_t)a[i][ks][e]);
        else v = float(a[i][ks][e]);
        s1 += v;
        s2 = fmaf(v, v, s2);
      }
    s1 = xor16_add(s1); s2 = xor16_add(s2);
    s1 = xor32_add(s1); s2 = xor32_add(s2);
    if (lane < 16) rst[wave][i * 16 + lane] = float2{s1, s2};
  }
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) acc = mma16(a[i][ks], w[j][ks], acc);
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][i * 16 + (lane >> 4) * 4 + e][j * 16 + (lane & 15)] = acc[e];
    }
  __syncthreads();
  // ---------------- q_h = r·(acc − μ·u) + c (the folded lean epilogue), 16-bit, into LDS
  if (item) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) { const float2 t = rst[q][er]; s1 += t.x; s2 += t.y; }
    const float mean = s1 / K, rstd = rsqrtf(fmaxf(s2 / K - mean * mean, 0.f) + 1e-5f);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float sum = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) sum += red[q][er][cq + e];
      sum = rstd * (sum - mean * u4[e]);
      qa[er][cq + e] = DT<T>::fromf(sum + c4[e]);
    }
  }
  __syncthreads();
  // ---------------- q'_h = W_k,hᵀ q_h for this chunk's columns: the kq launch's two halves, its sum order
  Frag qf[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) qf[kh] = *reinterpret_cast<const Frag*>(&qa[lane & 15][kh * 32 + 8 * (lane >> 4)]);
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tt = wave + t * NW;
    if (tt < NT16) {
      const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 a0 = mma16(qf[0], wk[t][0], z), a1 = mma16(qf[1], wk[t][1], z);
      const int col = h * K + ch * CW + tt * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rr = mb + 4 * (lane >> 4) + e;
        float sum = 0.f;
        sum += a0[e];
        sum += a1[e];
        const float v = sum + 0.f;
        if (rr < p.M) p.qp[(long)rr * ((long)p.H * K) + col] = DT<T>::fromf(v);
      }
    }
  }
}

// the fused cross query where it applies (16-bit, <= 64 rows, 64-wide heads, the lean LN table's widths,
// the folded q_proj weights and W_kt fragment-major); false: the caller keeps xq → kq
template <typename T>
static bool launch_xqk(const void* A, bool a_fm, const void* Wq_fm, const float* u, const float* c, const void* Wk_fm,
                       void* qp, int M, int H, int D, hipStream_t s, int nch = 8) {
  if constexpr (sizeof(T) != 2) {
    return false;
  } else {
    if (M > 64 || H * 64 != D || !A || !Wq_fm || !u || !c || !Wk_fm || !qp) return false;
    if (nch != 2 && nch != 4 && nch != 8 && nch != 16) return false;
    XqkArgs<T> p{reinterpret_cast<const T*>(A), reinterpret_cast<const T*>(Wq_fm), u, c,
                 reinterpret_cast<const T*>(Wk_fm), reinterpret_cast<T*>(qp), M, H, D};
    const dim3 grid(H * nch, (M + 15) / 16);
    // NCH: q' column chunks per head (each chunk's workgroup recomputes q_h): 4 / 8 (default) / 16
#define WCB_XQKN(nw, kpw, NC)                                                                              \
  if (nch == NC) {                                                                                         \
    if (a_fm) WCB_LAUNCH((dec_xqk_kernel<T, 1, nw, kpw, NC, true>), grid, dim3(nw * 64), 0, s, p);         \
    else WCB_LAUNCH((dec_xqk_kernel<T, 1, nw, kpw, NC, false>), grid, dim3(nw * 64), 0, s, p);             \
    return true;                                                                                           \
  }
#define WCB_XQK(k, nw, kpw)                                                                                \
  if (D == k) {                                                                                            \
    WCB_XQKN(nw, kpw, 8) WCB_XQKN(nw, kpw, 4) WCB_XQKN(nw, kpw, 2) WCB_XQKN(nw, kpw, 16)                    \
    return false;                                                                                          \
  }
    WCB_XQK(512, 4, 4) WCB_XQK(768, 4, 6) WCB_XQK(1024, 4, 8) WCB_XQK(1280, 8, 5)
#undef WCB_XQK
#undef WCB_XQKN
    return false;
  }
}

// the lean form where it applies (16-bit, <= 64 rows, single-tile decode projections); false: the
// caller takes gemm_dec_kernel. Same (waves, k-steps) table as launch_dec_mf: bit-identical outputs.
template <typename T>
static bool launch_lean(const GemmArgs& g, hipStream_t s) {
  if constexpr (sizeof(T) != 2) {
    return false;
  } else {
    if (g.M > 64 || g.sel_val || g.st_out || g.addrow || g.tile || g.a_Mb || g.c_Mb || g.N % 16 || g.ldc % 4) return false;
    // fragment-major operands (the runtime pairs fc1 → fc2 only where both take this path): a_fm needs
    // the weights' fragment-major copy too (the residual writer table), c_fm the LN + GELU table
    if (g.a_fm && (!g.W_fm || g.a_grp_n)) return false;
    if (g.c_fm && (!g.ln_w || !g.act)) return false;
    if (g.out16_fm && (g.ln_w || !g.resid || !g.out16)) return false;
    if (g.mode != 0 && g.mode != 2) return false;
    if (g.mode == 2 && (g.kv_rps > 1 || !g.kv_out || !g.pos || g.n_split % 64 || g.out_f32 || g.resid)) return false;
    if (g.a_grp_n) {   // q'_h = W_k,hᵀ q_h
      if (g.K != 64 || g.bias || g.ln_w || g.resid || g.act || g.mode || g.out_f32 || g.a_grp_n % 16) return false;
      launch_lean_k<T, 1, 2, 1, false, 0, false, true>(g, s);
      return true;
    }
    if (!g.bias || g.clamp != 0.f) return false;
    if (g.ln_w) {
      if (!g.ln_a16 || !g.ln_b || g.resid || g.out_f32 || (g.act && g.mode)) return false;
// wide LN-fused projections (QKV, fc1: N >= 2048) take 32-row workgroups (each weight tile read once,
// half the workgroups; tools/dec_kernel_bench: QKV 6.86 -> 6.52, fc1 6.78 -> 6.37 µs); same per-row
// arithmetic
#define WCB_LN(k, nw, kpw)                                                                          \
  if (g.K == k) {                                                                                   \
    const bool mf2 = (g.N >= 2048 || g.lean_mf2) && g.M > 16;                                       \
    if (fold) {                                                                                     \
      if (g.mode == 2 && mf2) launch_lean_k<T, 2, nw, kpw, true, 2, false, false, true>(g, s);      \
      else if (g.mode == 2) launch_lean_k<T, 1, nw, kpw, true, 2, false, false, true>(g, s);        \
      else if (g.act && mf2) launch_lean_k<T, 2, nw, kpw, true, 0, true, false, true>(g, s);        \
      else if (g.act) launch_lean_k<T, 1, nw, kpw, true, 0, true, false, true>(g, s);               \
      else launch_lean_k<T, 1, nw, kpw, true, 0, false, false, true>(g, s);                         \
      return true;                                                                                  \
    }                                                                                               \
    if (g.mode == 2 && mf2) launch_lean_k<T, 2, nw, kpw, true, 2, false, false>(g, s);              \
    else if (g.mode == 2) launch_lean_k<T, 1, nw, kpw, true, 2, false, false>(g, s);                \
    else if (g.act && mf2) launch_lean_k<T, 2, nw, kpw, true, 0, true, false>(g, s);                \
    else if (g.act) launch_lean_k<T, 1, nw, kpw, true, 0, true, false>(g, s);                       \
    else launch_lean_k<T, 1, nw, kpw, true, 0, false, false>(g, s);                                 \
    return true;                                                                                    \
  }
      // folded LayerNorm (runtime option lean_fold): the folded weights' fragment-major copy at hand, and not
      // the cross-query hand-off launch
      const bool fold = g.lean_fold && g.ln_wg_fm && g.ln_u && g.ln_c && !g.kq_w;
      WCB_LN(512, 4, 4) WCB_LN(768, 4, 6) WCB_LN(1024, 4, 8) WCB_LN(1280, 8, 5)
#undef WCB_LN
      return false;
    }
    // residual writers: x (f32, in place) += A·Wᵀ + b, and its 16-bit copy
    if (g.mode || g.act || !g.resid || g.resid != g.out || !g.out_f32 || !g.out16) return false;
#define WCB_RS(k, nw, kpw) if (g.K == k) { launch_lean_k<T, 1, nw, kpw, false, 1, false, false>(g, s); return true; }
    // option lean_mf2: 32-row workgroups (each weight tile read once for 32 rows; same per-row arithmetic)
#define WCB_RS2(k, nw, kpw)                                                                               \
  if (g.K == k) {                                                                                         \
    if (g.lean_mf2 && g.M > 16) launch_lean_k<T, 2, nw, kpw, false, 1, false, false>(g, s);               \
    else launch_lean_k<T, 1, nw, kpw, false, 1, false, false>(g, s);                                      \
    return true;                                                                                          \
  }
    WCB_RS2(512, 4, 4) WCB_RS2(768, 4, 6) WCB_RS2(1024, 4, 8) WCB_RS2(1280, 8, 5) WCB_RS2(2048, 8, 8) WCB_RS2(3072, 8, 12)
    WCB_RS(4096, 16, 8) WCB_RS(5120, 16, 10)
#undef WCB_RS
#undef WCB_RS2
    return false;
  }
}

// Beam-row projections (decode rows > 64: C3's 320 / C5's 80 beam rows), K = d_model: gemm_wide_kernel.
// One BM x BN tile per workgroup (BM = 16·FM rows, BN = 16·FN columns), K split over the NW waves; each
// wave issues every operand load of the launch in one burst straight into registers (FM + FN fragments
// per 32-deep k-step, KPW k-steps; the folded-LayerNorm statistics, bias, u, residual and cache position
// with them), multiplies, and the wave partials meet in LDS in wave order. The LDS-ring tiles
// (gemm_ring_kernel, tile 2) keep NS - 1 K tiles in flight and pay a memory round trip per ring turn at
// 2-8 MFMAs per wave per tile; here the workgroup's whole K extent is in flight at once.
// Epilogue (the ring kernel's run-time forms): folded LayerNorm r·(acc − μ·u[n]) (LNF), + bias, GELU;
// the QKV launch's k / v columns → the self-attention cache at the device-side position; residual
// writers x += …, the 16-bit copy and the per-32-column (Σx, Σx²) partials for the next fold.
template <typename T> struct WideArgs {
  const T* A; const T* W; const float* bias; const float* ln_u; const float* rst_in;
  const float* resid; void* out; T* out16; T* kv; const int* pos; float* rst_out;
  int M, N, lda, ldw, ldc;
  int act, out_f32, mode, n_split, kvB, kvH, kvT;
};

template <typename T, int FM, int FN, int NW, int KPW, bool LNF, bool WFM = false>
__global__ __launch_bounds__(NW * 64) void gemm_wide_kernel(WideArgs<T> p) {
  using Frag = typename DT<T>::frag;
  constexpr int NT = NW * 64, BM = FM * 16, BN = FN * 16, K = NW * KPW * 32, C8 = BN / 8, LDC = BN + 4;
  static_assert(BM * C8 <= NT, "epilogue: one 8-column item per thread");
  constexpr int RNB = K / 32;                                   // LN statistics partials per row
  constexpr int LPR = NT / BM >= 8 ? 8 : NT / BM >= 4 ? 4 : NT / BM >= 2 ? 2 : 1;   // lanes per row
  constexpr int RPL = (RNB + LPR - 1) / LPR;
  __shared__ __attribute__((aligned(16))) float red[NW][BM][LDC];
  __shared__ float2 lnst[LNF ? BM : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // column tile outer, row tile inner over consecutive workgroups of an XCD (the row tiles of a column
  // tile share its weights in that XCD's L2)
  const int tiles_m = (p.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg % tiles_m) * BM, n0 = (wg / tiles_m) * BN;
  const int kb = wave * (KPW * 32) + 8 * (lane >> 4);
  // ---------------- the launch's loads, one burst
  Frag w[FN][KPW], a[FM][KPW];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    if constexpr (WFM) {   // fragment-major weights [N / 16][K / 32][lane][8]: 1 KiB per wave-instruction
      const T* wr = p.W + (((long)min(n0 / 16 + j, p.N / 16 - 1) * (K / 32) + wave * KPW) * 64 + lane) * 8;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) w[j][ks] = load_frag<T>(wr + ks * 512);
    } else {
      const T* wr = p.W + (long)min(n0 + j * 16 + (lane & 15), p.N - 1) * p.ldw + kb;
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) w[j][ks] = load_frag<T>(wr + ks * 32);
    }
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const T* ar = p.A + (long)min(m0 + i * 16 + (lane & 15), p.M - 1) * p.lda + kb;
#pragma unroll
    for (int ks = 0; ks < KPW; ++ks) a[i][ks] = load_frag<T>(ar + ks * 32);
  }
  // epilogue operands: thread → row er, columns ec .. ec + 7
  const int er = tid / C8, ec = n0 + (tid % C8) * 8;
  const bool item = er < BM;
  const int erow = min(m0 + min(er, BM - 1), p.M - 1);
  const int ecc = min(ec, p.N - 8);
  float b8[8], u8[8], r8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { b8[e] = 0.f; u8[e] = 0.f; r8[e] = 0.f; }
  if (p.bias) {
    const f32x4 lo = *reinterpret_cast<const f32x4*>(p.bias + ecc), hi = *reinterpret_cast<const f32x4*>(p.bias + ecc + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { b8[e] = lo[e]; b8[e + 4] = hi[e]; }
  }
  if constexpr (LNF) {
    const f32x4 lo = *reinterpret_cast<const f32x4*>(p.ln_u + ecc), hi = *reinterpret_cast<const f32x4*>(p.ln_u + ecc + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { u8[e] = lo[e]; u8[e + 4] = hi[e]; }
  }
  if (p.resid) {
    const float* rr = p.resid + (long)erow * p.ldc + ecc;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(rr), hi = *reinterpret_cast<const f32x4*>(rr + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { r8[e] = lo[e]; r8[e + 4] = hi[e]; }
  }
  int pos = 0;
  if (p.mode == 2) pos = *p.pos;
  // LNF: row sr's statistics partials, lane ss of its LPR takes partials ss, ss + LPR, ...
  const int sr = tid / LPR, ss = tid % LPR;
  float2 st[LNF ? RPL : 1];
  if constexpr (LNF) {
    const float* sp = p.rst_in + (long)min(m0 + min(sr, BM - 1), p.M - 1) * RNB * 2;
#pragma unroll
    for (int t = 0; t < RPL; ++t) {
      const int j = min(ss + t * LPR, RNB - 1);
      st[t] = *reinterpret_cast<const float2*>(sp + 2 * j);
    }
  }
  // ---------------- MFMA over this wave's K slice, partial tiles into LDS
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KPW; ++ks) acc = mma16(a[i][ks], w[j][ks], acc);
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][i * 16 + (lane >> 4) * 4 + e][j * 16 + (lane & 15)] = acc[e];
    }
  if constexpr (LNF) {   // (μ, r) per tile row: strided partial sums in column order, then a fixed butterfly
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < RPL; ++t)
      if (ss + t * LPR < RNB) { s1 += st[t].x; s2 += st[t].y; }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
    if (ss == 0 && sr < BM) {
      const float mean = s1 / K;
      lnst[sr] = float2{mean, rsqrtf(fmaxf(s2 / K - mean * mean, 0.f) + 1e-5f)};
    }
  }
  __syncthreads();
  // ---------------- epilogue: one row × 8 columns per thread, wave partials summed in wave order
  const int m = m0 + er;
  const bool ok = item && m < p.M && ec < p.N;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
  if (item) {
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(&red[q][er][(tid % C8) * 8]);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(&red[q][er][(tid % C8) * 8 + 4]);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] += lo[e]; v[e + 4] += hi[e]; }
    }
    float2 ls = float2{0.f, 1.f};
    if constexpr (LNF) ls = lnst[er];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if constexpr (LNF) v[e] = ls.y * (v[e] - ls.x * u8[e]);
      v[e] += b8[e];
      if (p.act == 1) v[e] = gelu_t<T>(v[e]);
    }
  }
  if (p.mode == 2 && ec >= p.n_split) {   // k / v of the new token → the self-attention cache
    if (ok) {
      const int n2 = ec - p.n_split, hh = n2 >> 6, dd = n2 & 63;
      const int kvs = hh / p.kvH, hd = hh % p.kvH;
      store8<T>(p.kv + ((((long)kvs * p.kvB + m) * p.kvH + hd) * p.kvT + pos) * 64 + dd, v);
    }
    return;
  }
  const long off = (long)m * p.ldc + ec;
  if (p.resid) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r8[e];
  }
  if (ok) {
    if (p.out_f32) store8<float>(reinterpret_cast<float*>(p.out) + off, v);
    else store8<T>(reinterpret_cast<T*>(p.out) + off, v);
    if (p.out16) store8<T>(p.out16 + off, v);
  }
  if constexpr (C8 % 4 == 0) {
    if (p.rst_out) {   // residual writer: (Σx, Σx²) of the new row per 32 columns (4 adjacent lanes)
      float a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) { a1 += v[e]; a2 = fmaf(v[e], v[e], a2); }
      a1 += __shfl_xor(a1, 1, 64); a2 += __shfl_xor(a2, 1, 64);
      a1 += __shfl_xor(a1, 2, 64); a2 += __shfl_xor(a2, 2, 64);
      if (ok && (tid & 3) == 0) *reinterpret_cast<float2*>(p.rst_out + ((long)m * (p.N / 32) + ec / 32) * 2) = float2{a1, a2};
    }
  }
}

template <typename T, int FM, int FN, int NW, int KPW>
static void launch_wide_k(const GemmArgs& g, hipStream_t s) {
  WideArgs<T> p;
  p.A = reinterpret_cast<const T*>(g.A); p.W = reinterpret_cast<const T*>(g.W);
  p.bias = g.bias; p.ln_u = g.ln_u; p.rst_in = g.rst_in;
  p.resid = g.resid; p.out = g.out; p.out16 = reinterpret_cast<T*>(g.out16);
  p.kv = reinterpret_cast<T*>(g.kv_out); p.pos = g.pos; p.rst_out = g.rst_out;
  p.M = g.M; p.N = g.N; p.lda = (int)g.lda; p.ldw = (int)g.ldw; p.ldc = (int)g.ldc;
  p.act = g.act; p.out_f32 = g.out_f32; p.mode = g.mode; p.n_split = g.n_split;
  p.kvB = g.hs_B; p.kvH = g.hs_H; p.kvT = g.kv_T;
  const int tiles = ((g.M + FM * 16 - 1) / (FM * 16)) * (g.N / (FN * 16));
  if (g.W_fm) {
    p.W = reinterpret_cast<const T*>(g.W_fm);
    if (g.ln_u) WCB_LAUNCH((gemm_wide_kernel<T, FM, FN, NW, KPW, true, true>), dim3(tiles), dim3(NW * 64), 0, s, p);
    else WCB_LAUNCH((gemm_wide_kernel<T, FM, FN, NW, KPW, false, true>), dim3(tiles), dim3(NW * 64), 0, s, p);
    return;
  }
  if (g.ln_u) WCB_LAUNCH((gemm_wide_kernel<T, FM, FN, NW, KPW, true>), dim3(tiles), dim3(NW * 64), 0, s, p);
  else WCB_LAUNCH((gemm_wide_kernel<T, FM, FN, NW, KPW, false>), dim3(tiles), dim3(NW * 64), 0, s, p);
}

// cfg = 10·FM + FN (FM 1..5, FN 1..2); false: the shape / epilogue is not covered (the caller keeps the
// ring tiles). K = d_model (NW waves × KPW 32-deep k-steps).
template <typename T>
static bool launch_wide(const GemmArgs& g, int cfg, hipStream_t s) {
  if constexpr (sizeof(T) != 2) {
    return false;
  } else {
    const int FMr = cfg / 10, FNr = cfg % 10;
    if (FMr < 1 || FMr > 5 || FNr < 1 || FNr > 2) return false;
    if (g.a_Mb || g.c_Mb || g.addrow || g.st_out || g.mode == 1 || g.clamp != 0.f || g.a_grp_n) return false;
    if (g.N % (16 * FNr) || g.ldc % 8 || g.lda % 8 || g.ldw % 8) return false;
    if (g.ln_u && (!g.rst_in || g.rst_nb * 32 != g.K)) return false;
    if (g.rst_out && (FNr < 2 || g.N % 32)) return false;
    if (g.mode == 2 && (g.kv_rps > 1 || !g.kv_out || !g.pos || g.n_split % 64 || g.out_f32 || g.resid)) return false;
    if (g.resid && g.resid != g.out) return false;
#define WCB_WD(k, nw, kpw)                                                              \
  if (g.K == k) {                                                                       \
    switch (cfg) {                                                                      \
      case 11: launch_wide_k<T, 1, 1, nw, kpw>(g, s); return true;                      \
      case 12: launch_wide_k<T, 1, 2, nw, kpw>(g, s); return true;                      \
      case 21: launch_wide_k<T, 2, 1, nw, kpw>(g, s); return true;                      \
      case 22: launch_wide_k<T, 2, 2, nw, kpw>(g, s); return true;                      \
      case 41: launch_wide_k<T, 4, 1, nw, kpw>(g, s); return true;                      \
      case 42: launch_wide_k<T, 4, 2, nw, kpw>(g, s); return true;                      \
      case 51: launch_wide_k<T, 5, 1, nw, kpw>(g, s); return true;                      \
      case 52: launch_wide_k<T, 5, 2, nw, kpw>(g, s); return true;                      \
      default: return false;                                                            \
    }                                                                                   \
  }
    WCB_WD(768, 8, 3) WCB_WD(1024, 8, 4) WCB_WD(1280, 8, 5)
#undef WCB_WD
    return false;
  }
}

// The LayerNorm of gemm_dec_kernel AM = 2 (the same K split over NW waves × KPW k-steps, sum order
// and normalisation) for 16-row blocks, written as 16-bit rows: the LM head's A operand.
template <typename T, int NW, int KPW>
__global__ __launch_bounds__(NW * 64) void ln_rows_kernel(const T* __restrict__ x16, long lda, const float* __restrict__ gw,
                                                          const float* __restrict__ gb, T* __restrict__ out, int M) {
  using Frag = typename DT<T>::frag;
  constexpr int K = NW * KPW * 32;
  __shared__ float2 rst[NW][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kb = wave * (KPW * 32) + 8 * (lane >> 4);
  const int r = blockIdx.x * 16 + (lane & 15), row = min(r, M - 1);
  Frag a[KPW];
  f32x4 w[KPW][2], b[KPW][2];
#pragma unroll
  for (int ks = 0; ks < KPW; ++ks) {
    a[ks] = load_frag<T>(x16 + (long)row * lda + kb + ks * 32);
    w[ks][0] = *reinterpret_cast<const f32x4*>(gw + kb + ks * 32);
    w[ks][1] = *reinterpret_cast<const f32x4*>(gw + kb + ks * 32 + 4);
    b[ks][0] = *reinterpret_cast<const f32x4*>(gb + kb + ks * 32);
    b[ks][1] = *reinterpret_cast<const f32x4*>(gb + kb + ks * 32 + 4);
  }
  float xv[KPW][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int ks = 0; ks < KPW; ++ks) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v;
      if constexpr (__is_same(T, bf16_t)) v = bf16_to_f((bf16_t)a[ks][e]);
      else v = float(a[ks][e]);
      xv[ks][e] = v;
      s1 += v;
      s2 = fmaf(v, v, s2);
    }
  }
  s1 = xor16_add(s1); s2 = xor16_add(s2);
  s1 = xor32_add(s1); s2 = xor32_add(s2);
  if (lane < 16) rst[wave][lane] = float2{s1, s2};
  __syncthreads();
  s1 = 0.f; s2 = 0.f;
#pragma unroll
  for (int q = 0; q < NW; ++q) { const float2 t = rst[q][lane & 15]; s1 += t.x; s2 += t.y; }
  const float mean = s1 / K;
  const float rstd = rsqrtf(fmaxf(s2 / K - mean * mean, 0.f) + 1e-5f);
  if (r >= M) return;
#pragma unroll
  for (int ks = 0; ks < KPW; ++ks) {
    Frag o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gwe = e < 4 ? w[ks][0][e] : w[ks][1][e - 4], gbe = e < 4 ? b[ks][0][e] : b[ks][1][e - 4];
      const float v = (xv[ks][e] - mean) * rstd * gwe + gbe;
      o[e] = __builtin_bit_cast(typename std::remove_reference<decltype(o[0])>::type, DT<T>::fromf(v));
    }
    *reinterpret_cast<Frag*>(out + (long)r * K + kb + ks * 32) = o;
  }
}

template <typename T, int MF, int NW, int KPW, int AM>
static void launch_dec_k(const GemmArgs& g, hipStream_t s) {
  const int ntile = (g.N + 15) / 16, gy = (g.M + MF * 16 - 1) / (MF * 16);
  // one tile per workgroup up to ~4 workgroups per CU; beyond (the LM head) a persistent column walk
  if (!g.sel_val && (AM == 3 || ntile * gy <= 1024)) {
    WCB_LAUNCH((gemm_dec_kernel<T, MF, NW, KPW, AM, false>), dim3(ntile, gy), dim3(NW * 64), 0, s, g);
  } else {   // the LM head: kDecWalkers column walkers per row block (= argmax partials per row)
    const int gx = std::min(ntile, g.walkers > 0 ? g.walkers : kDecWalkers);
    int nw = 0, kpw = 0;
    if constexpr (sizeof(T) == 2 && AM != 3) {
      // the copy's split matches; it covers whole 16-column tiles (the LM head's rows are padded with zeros)
      if (g.W_fm && lean_cfg(g.K, nw, kpw) && nw == NW && kpw == KPW) {
        if (AM == 2 && g.ln_scratch && g.sel_val && g.a_Mb == 0) {   // LayerNorm once, then the walk on LN(x)
          WCB_LAUNCH((ln_rows_kernel<T, NW, KPW>), dim3((g.M + 15) / 16), dim3(NW * 64), 0, s,
                     reinterpret_cast<const T*>(g.ln_a16), g.lda, g.ln_w, g.ln_b, reinterpret_cast<T*>(g.ln_scratch), g.M);
          GemmArgs h = g;
          h.A = g.ln_scratch; h.lda = g.K;
          h.ln_w = h.ln_b = nullptr; h.ln_a16 = nullptr; h.st_in = nullptr;
          WCB_LAUNCH((gemm_dec_kernel<T, MF, NW, KPW, 0, true, true>), dim3(gx, gy), dim3(NW * 64), 0, s, h);
          return;
        }
        WCB_LAUNCH((gemm_dec_kernel<T, MF, NW, KPW, AM, true, true>), dim3(gx, gy), dim3(NW * 64), 0, s, g);
        return;
      }
    }
    WCB_LAUNCH((gemm_dec_kernel<T, MF, NW, KPW, AM == 3 ? 0 : AM, true>), dim3(gx, gy), dim3(NW * 64), 0, s, g);
  }
}

template <typename T, int MF, int NW, int KPW>
static bool launch_dec_am(const GemmArgs& g, hipStream_t s) {
  constexpr int K = NW * KPW * 32;
  if (g.ln_w) {   // the decoder LayerNorms: K = d_model <= 1280
    if constexpr (K <= 1280) {
      if (g.ln_a16) launch_dec_k<T, MF, NW, KPW, 2>(g, s);
      else launch_dec_k<T, MF, NW, KPW, 1>(g, s);
      return true;
    }
    return false;
  }
  if (g.a_grp_n) {   // block-diagonal cross-attention products: K = 64 or d_model
    if constexpr (K <= 1280) {
      launch_dec_k<T, MF, NW, KPW, 3>(g, s);
      return true;
    }
    return false;
  }
  launch_dec_k<T, MF, NW, KPW, 0>(g, s);
  return true;
}

// K → (waves, k-steps per wave); f32 ("exact" mode, 2x the fragment registers) takes half the k-steps
// per wave on twice the waves where the workgroup allows it. Returns false for an unsupported K.
template <typename T, int MF>
static bool launch_dec_mf(const GemmArgs& g, hipStream_t s) {
  constexpr bool F32 = sizeof(T) == 4;
#define WCB_DEC(k, nw, kpw) if (g.K == k) return launch_dec_am<T, MF, nw, kpw>(g, s);
  WCB_DEC(64, 2, 1) WCB_DEC(128, 4, 1) WCB_DEC(256, 4, 2)
  if constexpr (F32) {
    WCB_DEC(384, 4, 3) WCB_DEC(512, 8, 2) WCB_DEC(768, 8, 3) WCB_DEC(1024, 8, 4) WCB_DEC(1280, 8, 5)
    WCB_DEC(1536, 16, 3) WCB_DEC(2048, 16, 4) WCB_DEC(3072, 16, 6) WCB_DEC(4096, 16, 8) WCB_DEC(5120, 16, 10)
  } else {
    WCB_DEC(384, 4, 3) WCB_DEC(512, 4, 4) WCB_DEC(768, 4, 6) WCB_DEC(1024, 4, 8) WCB_DEC(1280, 8, 5)
    WCB_DEC(1536, 8, 6) WCB_DEC(2048, 8, 8) WCB_DEC(3072, 8, 12) WCB_DEC(4096, 16, 8) WCB_DEC(5120, 16, 10)
  }
#undef WCB_DEC
  return false;
}

template <typename T, int BM, int BN, int WM, int WN, int EPI>
static void launch_tile_e(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  constexpr int stage_bytes = 2 * (BM + BN) * 128;
  constexpr int epi_bytes = BM * (BN + 4) * 4;
  constexpr int lds = stage_bytes > epi_bytes ? stage_bytes : epi_bytes;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_tile_kernel<T, BM, BN, WM, WN, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  WCB_LAUNCH((gemm_tile_kernel<T, BM, BN, WM, WN, EPI>), dim3(tiles), dim3(WM * WN * 64), lds, s, g);
}

template <typename T, int BM, int BN, int WM, int WN>
static void launch_tile(const GemmArgs& g, hipStream_t s) {
  const int bits = (g.bias ? E_BIAS : 0) | (g.act == 1 ? E_GELU : 0) | (g.resid ? E_RESID : 0) |
                   (g.out_f32 ? E_F32 : 0) | (g.addrow ? E_ADDROW : 0) | (g.mode == 1 ? E_HEAD : 0) |
                   (g.mode == 2 ? E_RUNTIME : 0);   // KV-cache append: run-time form
  switch (bits) {   // the encoder's epilogues, specialised; anything else takes the run-time form
    case E_BIAS: launch_tile_e<T, BM, BN, WM, WN, E_BIAS>(g, s); break;                                   // QKV
    case E_BIAS | E_GELU: launch_tile_e<T, BM, BN, WM, WN, E_BIAS | E_GELU>(g, s); break;                 // fc1, conv1
    case E_BIAS | E_RESID | E_F32: launch_tile_e<T, BM, BN, WM, WN, E_BIAS | E_RESID | E_F32>(g, s); break;  // out, fc2
    case E_BIAS | E_GELU | E_F32 | E_ADDROW:
      launch_tile_e<T, BM, BN, WM, WN, E_BIAS | E_GELU | E_F32 | E_ADDROW>(g, s); break;                  // conv2
    case E_BIAS | E_HEAD: launch_tile_e<T, BM, BN, WM, WN, E_BIAS | E_HEAD>(g, s); break;                 // cross K/V
    default: launch_tile_e<T, BM, BN, WM, WN, E_RUNTIME>(g, s); break;
  }
}

template <typename T, int MF, int NF, int NW, int KS>
static void launch_skinny_k(const GemmArgs& g, hipStream_t s) {
  const dim3 grid((g.N + NF * 16 - 1) / (NF * 16), (g.M + MF * 16 - 1) / (MF * 16));
  if (g.ln_w) WCB_LAUNCH((gemm_skinny_kernel<T, MF, NF, NW, KS, true>), grid, dim3(NW * 64), 0, s, g);
  else WCB_LAUNCH((gemm_skinny_kernel<T, MF, NF, NW, KS, false>), grid, dim3(NW * 64), 0, s, g);
}

// K = NW waves x KS steps x 32: pick the wave count first, then the (compile-time) steps per wave.
template <typename T, int MF, int NF>
static bool launch_skinny_mf(const GemmArgs& g, hipStream_t s) {
  const int K = g.K;
#define WCB_SK(nw, ks) if (K == nw * ks * 32) { launch_skinny_k<T, MF, NF, nw, ks>(g, s); return true; }
  WCB_SK(1, 1) WCB_SK(1, 2) WCB_SK(2, 2) WCB_SK(4, 2) WCB_SK(4, 3) WCB_SK(4, 4) WCB_SK(8, 2)
  WCB_SK(8, 3) WCB_SK(8, 4) WCB_SK(8, 5) WCB_SK(8, 6) WCB_SK(16, 4) WCB_SK(16, 5) WCB_SK(16, 6)
  WCB_SK(16, 8) WCB_SK(16, 10) WCB_SK(16, 12)
#undef WCB_SK
  return false;
}

template <typename T>
static void gemm_t(const GemmArgs& g, hipStream_t s) {
  if (g.tile) {   // decoder rows > 64 (beams, prefill): MFMA tiles, each weight tile read once per 64-128 rows
    if constexpr (sizeof(T) == 2) {
      // tile 2 (192+ rows, the d-wide and wide projections): 64-row tiles over a deep LDS-DMA ring, so
      // that even N = d_model spreads over 80-320 workgroups (C3: 320 rows = 5 row tiles); 64 columns
      // where that still fills the chip, else 32. Run-time epilogue (KV append, 16-bit residual copy).
      if (g.tile == 2 && g.wide && launch_wide<T>(g, g.wide, s)) return;
      if (g.tile == 2 && g.K % 64 == 0 && !g.st_out && g.mode != 1 && !g.addrow &&
          (!g.ln_u || (g.K <= kLnfMaxK && g.rst_in && g.rst_nb * 32 == g.K))) {
        const int mt = (g.M + 63) / 64;
        const bool lnf = g.ln_u != nullptr;
        const bool kt2 = g.ring_kt == 2 && g.K % 128 == 0;           // 128-deep stages
        if (g.N % 64 == 0 && mt * (g.N / 64) >= 240) {
          // (128-deep stages measured slower here: C3 4,871 vs 4,946 audio-s/s with all three tiles)
          if (lnf) launch_ring_dec<T, 64, 64, 4, true>(g, s);
          else launch_ring_dec<T, 64, 64, 4, false>(g, s);
        } else if (mt * ((g.N + 31) / 32) >= 240) {
          if (lnf && kt2) launch_ring_dec<T, 64, 32, 4, true, 2>(g, s);
          else if (lnf) launch_ring_dec<T, 64, 32, 6, true>(g, s);
          else if (kt2) launch_ring_dec<T, 64, 32, 4, false, 2>(g, s);
          else launch_ring_dec<T, 64, 32, 6, false>(g, s);
        } else {
          if (lnf && kt2) launch_ring_dec<T, 32, 32, 4, true, 2>(g, s);
          else if (lnf) launch_ring_dec<T, 32, 32, 6, true>(g, s);
          else if (kt2) launch_ring_dec<T, 32, 32, 4, false, 2>(g, s);
          else launch_ring_dec<T, 32, 32, 6, false>(g, s);
        }
        return;
      }
    }
    if (g.N % 128 == 0) launch_tile<T, 128, 128, 2, 2>(g, s);
    else launch_tile<T, 128, 64, 2, 2>(g, s);
    return;
  }
  if ((g.M <= 64 || g.mode == 2 || g.ln_w || g.skinny) && g.mode != 1 && !g.addrow) {
    // decode GEMM (K in its table; else the older skinny kernel below): 16-row workgroups up to 64
    // rows (measured C2: 1.074 vs 1.147 ms/token with 32-row workgroups); the LM head walks the
    // vocabulary persistently with 32-row workgroups, reading every weight tile once
    if (g.xqk_wk) {   // the fused cross query: the runtime sets it only where dec_xqk_kernel covers the launch
      if (launch_xqk<T>(g.ln_a16, g.a_fm != 0, g.ln_wg_fm, g.ln_u, g.ln_c, g.xqk_wk, g.xqk_out, g.M, g.hs_H, g.K, s,
                        g.xqk_nch > 0 ? g.xqk_nch : 8)) return;
      throw std::runtime_error("internal error: fused cross query on a launch dec_xqk_kernel does not cover (M " +
                               std::to_string(g.M) + ", H " + std::to_string(g.hs_H) + ", K " + std::to_string(g.K) +
                               ", operands " + std::to_string(!!g.ln_a16) + std::to_string(!!g.ln_wg_fm) +
                               std::to_string(!!g.ln_u) + std::to_string(!!g.ln_c) + std::to_string(!!g.xqk_out) + ")");
    }
    if (g.lean && launch_lean<T>(g, s)) return;
    if (g.kq_w) throw std::runtime_error("internal error: fused cross-query on a launch the lean kernel does not cover");
    if (g.a_fm || g.c_fm || g.out16_fm)   // the runtime pairs fragment-major operands only where the lean path takes both
      throw std::runtime_error("internal error: fragment-major operand on a launch the lean kernel does not cover");
    const bool mf1 = (g.M <= 64 && !(g.sel_val && g.M > 16)) || g.K >= 4096;
    const bool ok = mf1 ? launch_dec_mf<T, 1>(g, s) : launch_dec_mf<T, 2>(g, s);
    if (ok) return;
  }
  if (g.M <= 64 || g.mode == 2 || g.ln_w || g.skinny) {
    // rows per workgroup: up to 16·sk_mf; larger M is split over grid.y (more workgroups, less A
    // traffic per CU)
    // Default (auto): 16 rows per workgroup up to 32 rows (C2 greedy: measured best), 32 up to 160
    // (C5 80 beam rows: 983 -> 1075 audio-s/s), 64 beyond (C3 320 beam rows: 2217 -> 2437): with many
    // rows the A re-read per column block, not the weight stream, dominates
    const int mf = g.M <= 32 ? 1 : g.M <= 160 ? 2 : 4;
    bool ok;
    if (g.sel_val) {   // LM head: 64 columns per workgroup (A re-read 4x less), fused argmax partial
      if (mf == 1) ok = launch_skinny_mf<T, 1, 4>(g, s);
      else if (mf == 2) ok = launch_skinny_mf<T, 2, 4>(g, s);
      else ok = launch_skinny_mf<T, 4, 4>(g, s);
    } else if (mf == 1) ok = launch_skinny_mf<T, 1, 1>(g, s);
    else if (mf == 2) ok = launch_skinny_mf<T, 2, 1>(g, s);
    else ok = launch_skinny_mf<T, 4, 1>(g, s);
    if (!ok) fprintf(stderr, "wcb: no skinny GEMM instance for K=%d\n", g.K);
    return;
  }
  // 16-bit encoder-size GEMMs: the LDS-ring kernel, 256x256 (2 stages) when N allows it (measured
  // 1128 vs 990 TFLOP/s at 48000x2304x768 class shapes), else 256x128 (3 stages); f32 ("exact"
  // mode) and small shapes: the two-stage tile kernel, 128x128 (4 waves 2x2) when N fills it, else 128x64.
  // 256x192 where the 256-column grid leaves a short last round of tiles on the 256 CUs and the
  // 192-column one does not, at its measured per-tile efficiency (0.9 of 256x256): whisper-small's
  // d-wide out / fc2 (M = 48000, N = 768: 564 tiles = 2.2 rounds against 752 = 2.9), 12 % / 10 %
  // faster (tools/enc_gemm_bench.hip); QKV / fc1 keep 256x256 (192 measured 9 / 15 % slower)
  if constexpr (sizeof(T) == 2) {
    if (g.pp && launch_pp<T>(g, s)) return;
    if (g.N % 128 == 0 && g.M >= 4096) {
      const long tm = (g.M + 255) / 256;
      const long r256 = (tm * ((g.N + 255) / 256) + 255) / 256, r192 = (tm * ((g.N + 191) / 192) + 255) / 256;
      if (g.N % 192 == 0 && r192 * 192 * 10 < r256 * 256 * 9) launch_ring<T, 256, 192, 2, 4, 2>(g, s);
      else if (g.N % 256 == 0) launch_ring<T, 256, 256, 2, 4, 2>(g, s);
      else launch_ring<T, 256, 128, 4, 2, 3>(g, s);
      return;
    }
  }
  if (g.N % 128 == 0) launch_tile<T, 128, 128, 2, 2>(g, s);
  else launch_tile<T, 128, 64, 2, 2>(g, s);
}

}  // namespace wcb
