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

template <typename T, int MF, int NW>
__global__ __launch_bounds__(NW * 64) void gemm_skinny_kernel(GemmArgs g) {
  using Frag = typename DT<T>::frag;
  __shared__ __attribute__((aligned(16))) float red[NW][MF * 16][17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const long n = min(n0 + (lane & 15), g.N - 1);
  const T* W = reinterpret_cast<const T*>(g.W) + n * g.ldw + 8 * (lane >> 4);
  const T* A = reinterpret_cast<const T*>(g.A);
  const T* ap[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const long m = min(i * 16 + (lane & 15), g.M - 1);
    ap[i] = A + a_row(g, m) + 8 * (lane >> 4);
  }
  f32x4 acc[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int KW = g.K / NW;
  const int kb = wave * KW, ke = kb + KW;
  int k = kb;
  for (; k + 64 <= ke; k += 64) {
    const Frag b0 = load_frag<T>(W + k), b1 = load_frag<T>(W + k + 32);
    Frag a0[MF], a1[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) { a0[i] = load_frag<T>(ap[i] + k); a1[i] = load_frag<T>(ap[i] + k + 32); }
#pragma unroll
    for (int i = 0; i < MF; ++i) { acc[i] = mma16(a0[i], b0, acc[i]); acc[i] = mma16(a1[i], b1, acc[i]); }
  }
  for (; k < ke; k += 32) {
    const Frag b0 = load_frag<T>(W + k);
#pragma unroll
    for (int i = 0; i < MF; ++i) acc[i] = mma16(load_frag<T>(ap[i] + k), b0, acc[i]);
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

template <typename T, int MF>
static void launch_skinny_mf(const GemmArgs& g, hipStream_t s) {
  const int grid = (g.N + 15) / 16;
  if (g.K % (32 * 8) == 0 && g.K >= 512)
    hipLaunchKernelGGL((gemm_skinny_kernel<T, MF, 8>), dim3(grid), dim3(512), 0, s, g);
  else if (g.K % (32 * 4) == 0)
    hipLaunchKernelGGL((gemm_skinny_kernel<T, MF, 4>), dim3(grid), dim3(256), 0, s, g);
  else if (g.K % (32 * 2) == 0)
    hipLaunchKernelGGL((gemm_skinny_kernel<T, MF, 2>), dim3(grid), dim3(128), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_skinny_kernel<T, MF, 1>), dim3(grid), dim3(64), 0, s, g);
}

template <typename T>
static void gemm_t(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 64 || g.mode == 2) {
    if (g.M <= 16) launch_skinny_mf<T, 1>(g, s);
    else if (g.M <= 32) launch_skinny_mf<T, 2>(g, s);
    else launch_skinny_mf<T, 4>(g, s);
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
