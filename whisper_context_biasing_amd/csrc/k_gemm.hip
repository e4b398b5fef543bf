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
#include "common.h"
#include "kernels.h"

#include <cstdio>
#include <type_traits>

namespace wcb {

WCB_DEV void glds16(const void* gptr, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(gptr, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

WCB_DEV long a_row(const GemmArgs& g, long m) { return (m / g.a_Mb) * g.a_strideB + (m % g.a_Mb) * g.lda; }
WCB_DEV long c_row(const GemmArgs& g, long m) { return (m / g.c_Mb) * g.c_strideB + (m % g.c_Mb) * g.ldc; }

// Store 8 consecutive output columns n..n+7 of row m (n % 8 == 0, all in one head for mode 1).
template <typename T>
WCB_DEV void epi_store8(const GemmArgs& g, long m, int n, float* v) {
  if (g.mode == 1) {
    const int hh = n >> 6, dd = n & 63;
    const int grp = hh / g.hs_H, h = hh % g.hs_H;
    const long b = m / g.hs_S, t = m % g.hs_S;
    const long off = ((((long)grp * g.hs_B + b) * g.hs_H + h) * g.hs_S + t) * 64 + dd;
    store8<T>(reinterpret_cast<T*>(g.out) + off, v);
    return;
  }
  const long off = c_row(g, m) + n;
  if (g.resid) {
    const f32x4 r0 = *reinterpret_cast<const f32x4*>(g.resid + off);
    const f32x4 r1 = *reinterpret_cast<const f32x4*>(g.resid + off + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += r0[j]; v[j + 4] += r1[j]; }
  }
  if (g.out_f32) store8<float>(reinterpret_cast<float*>(g.out) + off, v);
  else store8<T>(reinterpret_cast<T*>(g.out) + off, v);
}

template <typename T>
WCB_DEV void epi_store1(const GemmArgs& g, long m, int n, float v) {
  if (g.mode == 2 && n >= g.n_split) {
    const int n2 = n - g.n_split;
    const int hh = n2 >> 6, dd = n2 & 63;
    const int kv = hh / g.hs_H, h = hh % g.hs_H;
    const long off = ((((long)kv * g.hs_B + m) * g.hs_H + h) * g.kv_T + *g.pos) * 64 + dd;
    reinterpret_cast<T*>(g.kv_out)[off] = DT<T>::fromf(v);
    return;
  }
  if (g.mode == 1) {
    const int hh = n >> 6, dd = n & 63;
    const int grp = hh / g.hs_H, h = hh % g.hs_H;
    const long b = m / g.hs_S, t = m % g.hs_S;
    const long off = ((((long)grp * g.hs_B + b) * g.hs_H + h) * g.hs_S + t) * 64 + dd;
    reinterpret_cast<T*>(g.out)[off] = DT<T>::fromf(v);
    return;
  }
  const long off = c_row(g, m) + n;
  if (g.resid) v += g.resid[off];
  if (g.out_f32) reinterpret_cast<float*>(g.out)[off] = v;
  else reinterpret_cast<T*>(g.out)[off] = DT<T>::fromf(v);
}

WCB_DEV float epi_pointwise(const GemmArgs& g, long m, int n, float v) {
  if (g.bias) v += g.bias[n];
  if (g.act == 1) v = gelu_erf(v);
  if (g.addrow) v += g.addrow[(m % g.c_Mb) * g.N + n];
  return v;
}

template <typename T, int BM, int BN, int WM, int WN>
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
    const long m = min(m0 + r, g.M - 1);
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
        const long m = min((long)m0 + row, (long)g.M - 1);
        ct[row * LDC + col] = epi_pointwise(g, m, n, acc[i][j][e]);
      }
  }
  __syncthreads();
  constexpr int C8 = BN / 8;
#pragma unroll 2
  for (int idx = tid; idx < BM * C8; idx += NT) {
    const int row = idx / C8, c8 = idx % C8;
    const long m = m0 + row;
    const int n = n0 + c8 * 8;
    if (m >= g.M || n >= g.N) continue;
    float v[8];
    const f32x4 lo = *reinterpret_cast<const f32x4*>(ct + row * LDC + c8 * 8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(ct + row * LDC + c8 * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = lo[e]; v[e + 4] = hi[e]; }
    epi_store8<T>(g, m, n, v);
  }
}

// Skinny GEMM for the decode step (M = batch <= 64 rows): one workgroup = 16 output columns, its
// NW waves split K into NW contiguous ranges of KS 32-deep MFMA steps, every load of the wave is
// issued up front (weights are streamed once from HBM, activations come from L2), partial tiles
// are summed through LDS. With LN the A operand is the f32 residual stream normalised on the fly
// (the decoder's pre-attention / pre-MLP LayerNorm fused into the projection that consumes it).
template <typename T, int MF, int NW, int KS, bool LN>
__global__ __launch_bounds__(NW * 64) void gemm_skinny_kernel(GemmArgs g) {
  using Frag = typename DT<T>::frag;
  __shared__ __attribute__((aligned(16))) float red[NW][MF * 16][17];
  __shared__ float lnred[NW][MF * 16][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const long n = min(n0 + (lane & 15), g.N - 1);
  const int kb = wave * (KS * 32) + 8 * (lane >> 4);
  const T* W = reinterpret_cast<const T*>(g.W) + n * g.ldw + kb;
  Frag b[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) b[ks] = load_frag<T>(W + ks * 32);
  f32x4 acc[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (LN) {
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
    // one pass over this wave's K range: keep the x fragments, reduce Σx and Σx² per row over the
    // four lane groups and then over the waves (LDS) — no second read of the residual stream
    const float* X = reinterpret_cast<const float*>(g.A);
    float xv[MF][KS][8];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int m = min(i * 16 + (lane & 15), g.M - 1);
      const float* xr = X + a_row(g, m) + kb;
      float ps = 0.f, pq = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(xr + ks * 32);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(xr + ks * 32 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { xv[i][ks][e] = x0[e]; xv[i][ks][e + 4] = x1[e]; }
#pragma unroll
        for (int e = 0; e < 8; ++e) { ps += xv[i][ks][e]; pq += xv[i][ks][e] * xv[i][ks][e]; }
      }
      ps += __shfl_xor(ps, 16, 64); ps += __shfl_xor(ps, 32, 64);
      pq += __shfl_xor(pq, 16, 64); pq += __shfl_xor(pq, 32, 64);
      if (lane < 16) { lnred[wave][i * 16 + lane][0] = ps; lnred[wave][i * 16 + lane][1] = pq; }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) { s1 += lnred[w][i * 16 + (lane & 15)][0]; s2 += lnred[w][i * 16 + (lane & 15)][1]; }
      const float mean = s1 / g.K;
      const float rstd = rsqrtf(fmaxf(s2 / g.K - mean * mean, 0.f) + 1e-5f);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        Frag a;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = (xv[i][ks][e] - mean) * rstd * gw[ks][e] + gb[ks][e];
          if constexpr (sizeof(T) == 4) a[e] = v;
          else a[e] = __builtin_bit_cast(typename std::remove_reference<decltype(a[0])>::type, DT<T>::fromf(v));
        }
        acc[i] = mma16(a, b[ks], acc[i]);
      }
    }
  } else {
    const T* A = reinterpret_cast<const T*>(g.A);
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int m = min(i * 16 + (lane & 15), g.M - 1);
      const T* ap = A + a_row(g, m) + kb;
      Frag a[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) a[ks] = load_frag<T>(ap + ks * 32);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc[i] = mma16(a[ks], b[ks], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wave][i * 16 + (lane >> 4) * 4 + e][lane & 15] = acc[i][e];
  __syncthreads();
  for (int t = threadIdx.x; t < MF * 16 * 16; t += NW * 64) {
    const int row = t >> 4, col = t & 15;
    const int nn = n0 + col;
    if (row >= g.M || nn >= g.N) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][row][col];
    epi_store1<T>(g, row, nn, epi_pointwise(g, row, nn, v));
  }
}

template <typename T, int BM, int BN, int WM, int WN>
static void launch_tile(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  constexpr int stage_bytes = 2 * (BM + BN) * 128;
  constexpr int epi_bytes = BM * (BN + 4) * 4;
  constexpr int lds = stage_bytes > epi_bytes ? stage_bytes : epi_bytes;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_tile_kernel<T, BM, BN, WM, WN>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_tile_kernel<T, BM, BN, WM, WN>), dim3(tiles), dim3(WM * WN * 64), lds, s, g);
}

template <typename T, int MF, int NW, int KS>
static void launch_skinny_k(const GemmArgs& g, hipStream_t s) {
  const int grid = (g.N + 15) / 16;
  if (g.ln_w) hipLaunchKernelGGL((gemm_skinny_kernel<T, MF, NW, KS, true>), dim3(grid), dim3(NW * 64), 0, s, g);
  else hipLaunchKernelGGL((gemm_skinny_kernel<T, MF, NW, KS, false>), dim3(grid), dim3(NW * 64), 0, s, g);
}

// K = NW waves x KS steps x 32: pick the wave count first, then the (compile-time) steps per wave.
template <typename T, int MF>
static bool launch_skinny_mf(const GemmArgs& g, hipStream_t s) {
  const int K = g.K;
#define WCB_SK(nw, ks) if (K == nw * ks * 32) { launch_skinny_k<T, MF, nw, ks>(g, s); return true; }
  WCB_SK(1, 1) WCB_SK(1, 2) WCB_SK(2, 2) WCB_SK(4, 2) WCB_SK(4, 3) WCB_SK(4, 4) WCB_SK(8, 2)
  WCB_SK(8, 3) WCB_SK(8, 4) WCB_SK(8, 5) WCB_SK(8, 6) WCB_SK(16, 4) WCB_SK(16, 5) WCB_SK(16, 6)
  WCB_SK(16, 8) WCB_SK(16, 10) WCB_SK(16, 12)
#undef WCB_SK
  return false;
}

template <typename T>
static void gemm_t(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 64 || g.mode == 2 || g.ln_w) {
    bool ok;
    if (g.M <= 16) ok = launch_skinny_mf<T, 1>(g, s);
    else if (g.M <= 32) ok = launch_skinny_mf<T, 2>(g, s);
    else ok = launch_skinny_mf<T, 4>(g, s);
    if (!ok) fprintf(stderr, "wcb: no skinny GEMM instance for K=%d\n", g.K);
    return;
  }
  // Tile choice: 128x128 (4 waves 2x2) when N fills it, else 128x64.
  if (g.N % 128 == 0) launch_tile<T, 128, 128, 2, 2>(g, s);
  else launch_tile<T, 128, 64, 2, 2>(g, s);
}

void gemm(DType t, const GemmArgs& g, hipStream_t s) {
  switch (t) {
    case kBF16: gemm_t<bf16_t>(g, s); break;
    case kF16: gemm_t<f16_t>(g, s); break;
    case kF32: gemm_t<float>(g, s); break;
  }
}

}  // namespace wcb
