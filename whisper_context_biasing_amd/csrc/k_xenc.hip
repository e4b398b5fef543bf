// Decoder cross-attention in encoder space (16-bit model dtypes).
//
// Replaces the cross-attention branch of WhisperAttention.forward
// ([tf] modeling_whisper.py:284-356, is_cross_attention: keys/values from the encoder output, k_proj
// without bias :279) as the decoder calls it once per layer and generated token
// (WhisperDecoderLayer.forward :448-505).
//
// Algebra (exact in real arithmetic; every Whisper size has k_proj bias = None):
//   score_j,h = q_h · (W_k,h e_j)        = (W_k,hᵀ q_h) · e_j  =: q'_h · e_j
//   out_h     = Σ_j p_j,h (W_v,h e_j + b_v,h) = W_v,h (Σ_j p_j,h e_j) + b_v,h      (Σ_j p_j,h = 1)
// so a decode step streams the encoder output e [1500][d] once per layer for ALL heads, instead of
// that layer's K and V (2·1500·d per clip): half the bytes of the K/V formulation, and no per-clip
// cross-K/V precompute (1.36 TFLOP and 1.77 GB of writes per 32-clip whisper-small batch).
// q'_h = W_k,hᵀ q_h and W_v,h u_h are block-diagonal skinny GEMMs (gemm_impl.h, grouped A).
//
// attn_xenc_kernel: workgroup = (key range s, row b), 8 waves. The row's key range streams through a
//   ring of NS LDS stages, 32 keys × D columns each (global_load_lds, 16 B per lane, source-address
//   swizzle of common.h), NS-1 chunks in flight. Per chunk each wave computes the 32 × 16 score tile
//   S = E·q'ᵀ over its share of the D contraction (A = E rows by ds_read_b128, B = q' fragments held
//   in registers; heads ≥ H are zero); the partials are summed through LDS in a fixed order, so every
//   wave holds the same S, runs the online softmax per head lane-locally (max over its 4 lane groups
//   by two shuffles) and accumulates its eighth of Uᵀ = Eᵀ·P (A = Eᵀ by ds_read_b64_tr_b16, B = P
//   straight from the score accumulators: the k order {4g..4g+3, 16+4g..16+4g+3} of lane group g
//   matches both).
//   Output: per (row, range) the range-local (max, Σp) per head and Σ p·e [H][D] in f32.
// xenc_merge_kernel: workgroup = (head, row): merges the ranges (fixed order: deterministic) and
//   normalises: u[row][h] = Σ_j p_j,h e_j in the model dtype. W_v,h and b_v are then one block-diagonal
//   skinny GEMM (gemm_impl.h, grouped A), whose output feeds the out-projection GEMM.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace wcb {

constexpr int kXencCK = 32;   // keys per chunk

// tools/xattn_probe.hip builds this file with WCB_XENC_PROBE: the register-ring kernel then writes
// s_memtime stamps of its phases (wave 0) to a.stamp.base[workgroup][16] instead of the launch stamps
#ifdef WCB_XENC_PROBE
#define XPROBE(k)                                                                                        \
  do {                                                                                                   \
    if (threadIdx.x == 0)                                                                                \
      a.stamp.base[(blockIdx.y * gridDim.x + blockIdx.x) * 16 + (k)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
// ... and xenc_merge_v_kernel stamps (wave 0) into wcb_merge_probe[workgroup][8]: start (0), loads issued
// (1), partials landed (2), range merge done (3), outputs stored (4)
__device__ unsigned long long* wcb_merge_probe;
#define MPROBE(k)                                                                                        \
  do {                                                                                                   \
    if (threadIdx.x == 0)                                                                                \
      wcb_merge_probe[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (k)] = __builtin_amdgcn_s_memtime();   \
  } while (0)
#else
#define XPROBE(k) do {} while (0)
#define MPROBE(k) do {} while (0)
#endif
constexpr int kXencNW = 8;    // waves per workgroup

template <int D> struct XencCfg {
  static constexpr int NP = D / 64;                       // 64-column panels of a chunk
  static constexpr int STAGE = kXencCK * D * 2;           // bytes per LDS stage
  static constexpr int RED = kXencNW * 2 * 64 * 16;       // score partials [wave][tile][lane] f32x4
  static constexpr int NS = (3 * STAGE + RED <= 160 * 1024) ? 3 : 2;
  static constexpr int LDS = NS * STAGE + RED;
  static constexpr int KST = D / 32;                      // k-steps of the score contraction
  static constexpr int KSW = (KST + kXencNW - 1) / kXencNW;   // k-steps per wave
  static constexpr int CTW = (D / 16 + kXencNW - 1) / kXencNW;  // 16-column Uᵀ tiles per wave
  static constexpr int GLW = (4 * NP + kXencNW - 1) / kXencNW;  // glds instructions per wave per chunk
};

typedef short s16x4_t __attribute__((ext_vector_type(4)));
// ds_read_b64_tr_b16 as inline asm: the builtin form makes hipcc drain every in-flight LDS-DMA
// (s_waitcnt vmcnt(0)) before it, which serialises the chunk ring. The caller waits lgkmcnt itself.
WCB_DEV s16x4_t tr_read_asm(const char* p) {
  s16x4_t r;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
template <typename T>
WCB_DEV typename DT<T>::frag tr_pair(const s16x4_t& x, const s16x4_t& y) {
  const s16x8 t8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  if constexpr (__is_same(T, bf16_t)) return t8;
  else return __builtin_bit_cast(h16x8, t8);
}

template <typename T, int D>
__global__ __launch_bounds__(512) void attn_xenc_kernel(XencArgs a) {
  using Frag = typename DT<T>::frag;
  using C = XencCfg<D>;
  constexpr int CK = kXencCK, NW = kXencNW, NP = C::NP, NS = C::NS, KST = C::KST, KSW = C::KSW, CTW = C::CTW;
  constexpr int GLW = C::GLW;
  constexpr int PANEL = CK * 128;                         // bytes of one panel in a stage
  extern __shared__ __attribute__((aligned(16))) char lds[];
  f32x4* red = reinterpret_cast<f32x4*>(lds + NS * C::STAGE);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x, b = blockIdx.y;
  const unsigned long long t_start = a.stamp.base ? stamp_now() : 0;
  const int per = ((a.S + a.nsplit - 1) / a.nsplit + CK - 1) / CK * CK;
  const int k_lo = split * per, k_hi = min(a.S, k_lo + per);
  const int nch = k_hi > k_lo ? (k_hi - k_lo + CK - 1) / CK : 0;
  const T* E = reinterpret_cast<const T*>(a.enc) + (long)((a.row0 + b) / a.rows_per_enc) * a.enc_sb;

  // q' fragments of this wave's k-steps: lane → head lane&15 (zero for heads >= H)
  const int hq = lane & 15;
  Frag qf[KSW];
  {
    const T* qrow = reinterpret_cast<const T*>(a.qp) + ((long)b * a.H + min(hq, a.H - 1)) * D + 8 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = wave * KSW + i;
      qf[i] = Frag{};
      if (ks < KST && hq < a.H) qf[i] = load_frag<T>(qrow + ks * 32);
    }
    // retire these plain loads before the LDS-DMA ring starts: a plain load still pending inside the
    // loop makes hipcc wait vmcnt(0) at its use, i.e. drain the whole ring every chunk
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
  }
  // staging: 4·NP wave-instructions of 1 KiB (8 rows × 128 B of one panel) per chunk; wave w issues
  // instructions w, w+NW, ...: panel q >> 2, row group q & 3
  int src_off[GLW], src_row[GLW];
#pragma unroll
  for (int i = 0; i < GLW; ++i) {
    const int q = wave + NW * i, p = q >> 2, r = (q & 3) * 8 + (lane >> 3);
    src_row[i] = r;
    src_off[i] = p * 64 + ((lane & 7) ^ ((r >> 1) & 7)) * 8;
  }
  auto stage = [&](int st, int c) {
    char* base = lds + st * C::STAGE;
    const int key0 = k_lo + c * CK;
#pragma unroll
    for (int i = 0; i < GLW; ++i) {
      const int q = wave + NW * i;
      if (GLW * NW == 4 * NP || q < 4 * NP) {
        const int key = min(key0 + src_row[i], a.S - 1);
        glds16a(E + (long)key * D + src_off[i], base + (q >> 2) * PANEL + (q & 3) * 1024);
      }
    }
  };

  f32x4 acc[CTW];
#pragma unroll
  for (int t = 0; t < CTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  const float L2E = 1.4426950408889634f;

  if (nch > 0) stage(0, 0);
  if (NS > 2 && nch > 1) stage(1, 1);
  for (int c = 0; c < nch; ++c) {
    // retire chunk c (this wave's loads; the barrier covers the other waves'), keep c+1 in flight
    if (NS > 2 && c + 1 < nch) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(GLW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // the stage read in iteration c-1 is free once every wave has passed the barrier above
    if (c + NS - 1 < nch) stage((c + NS - 1) % NS, c + NS - 1);
    const char* st = lds + (c % NS) * C::STAGE;

    // partial S = E·q'ᵀ over this wave's k-steps, keys [0,16) and [16,32) of the chunk
    f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0;
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = wave * KSW + i;
      if (KSW * NW == KST || ks < KST) {
        const char* pb = st + (ks >> 1) * PANEL;
        const int cc = (ks & 1) * 4 + (lane >> 4);
        const Frag a0 = *reinterpret_cast<const Frag*>(pb + swz(lane & 15, cc));
        const Frag a1 = *reinterpret_cast<const Frag*>(pb + swz(16 + (lane & 15), cc));
        s0 = mma16(a0, qf[i], s0);
        s1 = mma16(a1, qf[i], s1);
      }
    }
    red[(wave * 2 + 0) * 64 + lane] = s0;
    red[(wave * 2 + 1) * 64 + lane] = s1;
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's partials written
    __builtin_amdgcn_s_barrier();
    // every wave sums the partials in the same order: identical S (and P) in all waves
    s0 = red[lane];
    s1 = red[64 + lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      s0 += red[(w * 2 + 0) * 64 + lane];
      s1 += red[(w * 2 + 1) * 64 + lane];
    }
    // issue this wave's Eᵀ fragment reads (transposed) now; they overlap the softmax
    s16x4_t tx[CTW], ty[CTW];
#pragma unroll
    for (int t = 0; t < CTW; ++t) {
      const int c0 = (wave * CTW + t) * 16;
      if (CTW * NW * 16 == D || c0 < D) {
        const char* vt = st + (c0 >> 6) * PANEL;
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const int r1 = 4 * g + q, cch = ((c0 & 63) >> 4) * 2 + (p >> 1), byte = (p & 1) * 8;
        tx[t] = tr_read_asm(vt + swz(r1, cch) + byte);
        ty[t] = tr_read_asm(vt + swz(r1 + 16, cch) + byte);
      }
    }
    const int kb = k_lo + c * CK + 4 * (lane >> 4);
    if (k_lo + (c + 1) * CK > k_hi) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (kb + e >= k_hi) s0[e] = -INFINITY;
        if (kb + 16 + e >= k_hi) s1[e] = -INFINITY;
      }
    }
    float cm = fmaxf(fmaxf(fmaxf(s0[0], s0[1]), fmaxf(s0[2], s0[3])), fmaxf(fmaxf(s1[0], s1[1]), fmaxf(s1[2], s1[3])));
    cm = xor16_max(cm);
    cm = xor32_max(cm);
    const float mnew = fmaxf(m_run, cm);            // finite: every chunk holds >= 1 key of the range
    const float alpha = __builtin_amdgcn_exp2f((m_run - mnew) * L2E);
    m_run = mnew;
    const float mb = mnew * L2E;
    float ls = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s0[e] = __builtin_amdgcn_exp2f(fmaf(s0[e], L2E, -mb));
      s1[e] = __builtin_amdgcn_exp2f(fmaf(s1[e], L2E, -mb));
      ls += s0[e] + s1[e];
    }
    l_run = l_run * alpha + ls;
    const Frag pf = pack_p<T>(s0, s1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // Uᵀ[c][h] += Σ_k E[k][c] P[k][h] over this wave's column tiles
#pragma unroll
    for (int t = 0; t < CTW; ++t) {
      const int c0 = (wave * CTW + t) * 16;
      if (CTW * NW * 16 == D || c0 < D) acc[t] = mma16(tr_pair<T>(tx[t], ty[t]), pf, acc[t] * alpha);
    }
  }
  // ---- range partials: lane holds Uᵀ[c0 + 4(lane>>4) + e][head lane&15]
  l_run = xor16_add(l_run);
  l_run = xor32_add(l_run);
  if (hq < a.H) {
    const long slot = ((long)b * a.nsplit + split) * a.H + hq;
    float* pp = a.part + slot * D + 4 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < CTW; ++t) {
      const int c0 = (wave * CTW + t) * 16;
      if (CTW * NW * 16 == D || c0 < D) *reinterpret_cast<f32x4*>(pp + c0) = acc[t];
    }
    if (wave == 0 && lane < 16) *reinterpret_cast<float2*>(a.ml + slot * 2) = float2{m_run, l_run};
  }
  if (a.stamp.base) {
    __syncthreads();
    if (tid == 0) stamp_commit(a.stamp, t_start);
  }
}

// ---- register-ring variant (default): the chunk ring lives in VGPRs (512 KiB per CU, against 160 KiB
// of LDS), so a workgroup needs only its per-wave transpose tiles and the score exchange in LDS
// (64 KiB at D = 768): two of its workgroups, or one beside a GEMM tile, fit on a CU.
// Wave w owns columns [w·CW, (w+1)·CW): it loads its 32 × CW slice of each chunk straight into the
// MFMA A-operand registers (lane → key lane&15 (+16), 8 columns), two chunks ahead; computes its partial
// scores; writes the slice into its private LDS tile (128-byte-row panels, common.h swizzle) for the
// transposed Eᵀ reads; the 4 partial score tiles are summed through LDS (double-buffered, one barrier
// per chunk) in a fixed order.
// WNW: waves per workgroup for D >= 256 (4 default; 8 = variant 3: half the columns per wave, one
// workgroup per CU by LDS)
template <int D, int WNW = 4> struct XregCfg {
  static constexpr int NW = D >= 256 ? WNW : D >= 128 ? 4 : D / 32;   // waves = column slices
  static constexpr int CW = D / NW;                       // columns per wave
  static constexpr int KSW = CW / 32;                     // k-steps per wave
  static constexpr int CTW = CW / 16;                     // 16-column Uᵀ tiles per wave
  static constexpr int NPW = (CW + 63) / 64;              // 128-byte-row panels per wave tile
  static constexpr int PANEL = kXencCK * 128;
  static constexpr int TILE = NPW * PANEL;
  static constexpr int RED = 2 * NW * 2 * 64 * 16;
  static constexpr int LDS = NW * TILE + RED;
};

// NR = chunks in flight per wave (register ring depth): 2 (two workgroups per CU) or 3 (one).
// FM: the encoder output in the fragment-major chunk layout of xenc_fm_kernel (below): every load
// wave-instruction reads 1 KiB contiguous, where the row layout touches 16 key rows x 64 B.
// P16: the range partials stored in T, normalised by the range's own Σ p (XencArgs::part16)
template <typename T, int D, int NR, int WNW = 4, bool FM = false, bool P16 = false>
__global__ __launch_bounds__((XregCfg<D, WNW>::NW * 64), ((NR == 2 && WNW == 4) ? 2 : 1)) void attn_xenc_reg_kernel(XencArgs a) {
  using Frag = typename DT<T>::frag;
  using C = XregCfg<D, WNW>;
  constexpr int CK = kXencCK, NW = C::NW, CW = C::CW, KSW = C::KSW, CTW = C::CTW, PANEL = C::PANEL;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  char* tile = lds + wave * C::TILE;
  f32x4* red = reinterpret_cast<f32x4*>(lds + NW * C::TILE);
  const int split = blockIdx.x, b = blockIdx.y;
  const unsigned long long t_start = a.stamp.base ? stamp_now() : 0;
  XPROBE(0);
  const int per = ((a.S + a.nsplit - 1) / a.nsplit + CK - 1) / CK * CK;
  const int k_lo = split * per, k_hi = min(a.S, k_lo + per);
  const int nch = k_hi > k_lo ? (k_hi - k_lo + CK - 1) / CK : 0;
  const int cw0 = wave * CW;
  const T* E = reinterpret_cast<const T*>(a.enc) + (long)((a.row0 + b) / a.rows_per_enc) * a.enc_sb + cw0 + 8 * (lane >> 4);

  const int hq = lane & 15;
  Frag qf[KSW];
  {
    const T* qrow = reinterpret_cast<const T*>(a.qp) + ((long)b * a.H + min(hq, a.H - 1)) * D + cw0 + 8 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < KSW; ++i) qf[i] = hq < a.H ? load_frag<T>(qrow + i * 32) : Frag{};
  }
  auto load_chunk = [&](Frag (&f)[2][KSW], int c) {
    if constexpr (FM) {   // chunk g of the clip: [g][wave][half][ks][lane][8] (past the range: its last chunk)
      const int g = min((k_lo + c * CK) / CK, (k_hi - 1) / CK);
      const T* cb = reinterpret_cast<const T*>(a.enc) + (long)((a.row0 + b) / a.rows_per_enc) * a.enc_sb +
                    (((long)g * NW + wave) * 2 * KSW * 64 + lane) * 8;
#pragma unroll
      for (int ks = 0; ks < KSW; ++ks) {
        f[0][ks] = load_frag<T>(cb + ks * 512);
        f[1][ks] = load_frag<T>(cb + (KSW + ks) * 512);
      }
    } else {
      const int key0 = k_lo + c * CK + (lane & 15);   // past the range: re-read its last key (L2)
      const T* r0 = E + (long)min(key0, k_hi - 1) * D;
      const T* r1 = E + (long)min(key0 + 16, k_hi - 1) * D;
#pragma unroll
      for (int ks = 0; ks < KSW; ++ks) {
        f[0][ks] = load_frag<T>(r0 + ks * 32);
        f[1][ks] = load_frag<T>(r1 + ks * 32);
      }
    }
  };

  f32x4 acc[CTW];
#pragma unroll
  for (int t = 0; t < CTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  const float L2E = 1.4426950408889634f;

  auto body = [&](Frag (&f)[2][KSW], int c) {
    // partial scores over this wave's columns
    f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0;
#pragma unroll
    for (int ks = 0; ks < KSW; ++ks) {
      s0 = mma16(f[0][ks], qf[ks], s0);
      s1 = mma16(f[1][ks], qf[ks], s1);
    }
    // the slice into the wave's transpose tile (its reads of the previous chunk precede in order)
#pragma unroll
    for (int ks = 0; ks < KSW; ++ks) {
      char* pb = tile + (ks >> 1) * PANEL;
      const int cc = (ks & 1) * 4 + (lane >> 4);
      *reinterpret_cast<Frag*>(pb + swz(lane & 15, cc)) = f[0][ks];
      *reinterpret_cast<Frag*>(pb + swz(16 + (lane & 15), cc)) = f[1][ks];
    }
    load_chunk(f, c + NR);  // the registers are free: refill NR chunks ahead (unconditionally: a
                            // load under a branch makes hipcc drain every load at the loop head)
    f32x4* rb = red + (c & 1) * NW * 2 * 64;
    rb[(wave * 2 + 0) * 64 + lane] = s0;
    rb[(wave * 2 + 1) * 64 + lane] = s1;
    __syncthreads();
    s0 = rb[lane];
    s1 = rb[64 + lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      s0 += rb[(w * 2 + 0) * 64 + lane];
      s1 += rb[(w * 2 + 1) * 64 + lane];
    }
    const int kb = k_lo + c * CK + 4 * (lane >> 4);
    if (k_lo + (c + 1) * CK > k_hi) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (kb + e >= k_hi) s0[e] = -INFINITY;
        if (kb + 16 + e >= k_hi) s1[e] = -INFINITY;
      }
    }
    float cm = fmaxf(fmaxf(fmaxf(s0[0], s0[1]), fmaxf(s0[2], s0[3])), fmaxf(fmaxf(s1[0], s1[1]), fmaxf(s1[2], s1[3])));
    cm = xor16_max(cm);
    cm = xor32_max(cm);
    const float mnew = fmaxf(m_run, cm);
    const float alpha = __builtin_amdgcn_exp2f((m_run - mnew) * L2E);
    m_run = mnew;
    const float mb = mnew * L2E;
    float ls = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s0[e] = __builtin_amdgcn_exp2f(fmaf(s0[e], L2E, -mb));
      s1[e] = __builtin_amdgcn_exp2f(fmaf(s1[e], L2E, -mb));
      ls += s0[e] + s1[e];
    }
    l_run = l_run * alpha + ls;
    const Frag pf = pack_p<T>(s0, s1);
    if (__any(alpha != 1.f)) {   // rescale only when some head's max moved (exact: alpha is 1 otherwise)
#pragma unroll
      for (int t = 0; t < CTW; ++t) acc[t] *= alpha;
    }
#pragma unroll
    for (int t = 0; t < CTW; ++t) {
      const int c0 = t * 16;
      const Frag ef = tr_frag<T>(tile + (c0 >> 6) * PANEL, 0, ((c0 & 63) >> 4) * 2, lane);
      acc[t] = mma16(ef, pf, acc[t]);
    }
    XPROBE(2 + min(c, 7));
  };

  if (nch > 0) {
    // chunks in groups of NR; a short last group gets fully masked chunks (p = 0, running max kept)
    if constexpr (NR == 2) {
      Frag fa[2][KSW], fb[2][KSW];
      load_chunk(fa, 0);
      load_chunk(fb, 1);
      XPROBE(1);
      for (int c = 0; c < nch; c += 2) {
        body(fa, c);
        body(fb, c + 1);
      }
    } else {
      Frag fa[2][KSW], fb[2][KSW], fc[2][KSW];
      load_chunk(fa, 0);
      load_chunk(fb, 1);
      load_chunk(fc, 2);
      for (int c = 0; c < nch; c += 3) {
        body(fa, c);
        body(fb, c + 1);
        body(fc, c + 2);
      }
    }
  }
  // ---- range partials: lane holds Uᵀ[cw0 + 16t + 4(lane>>4) + e][head lane&15]
  l_run = xor16_add(l_run);
  l_run = xor32_add(l_run);
  XPROBE(10);
  if (hq < a.H) {
    const long slot = ((long)b * a.nsplit + split) * a.H + hq;
    if constexpr (P16) {   // Σ_j p_j e_j / Σ_j p_j in T (a convex combination of encoder values): 8 B per lane
      T* pp = reinterpret_cast<T*>(a.part) + slot * D + cw0 + 4 * (lane >> 4);
      const float il = l_run > 0.f ? 1.f / l_run : 0.f;   // an empty range publishes Σ p = 0 (weight 0)
      typedef short s4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int t = 0; t < CTW; ++t) {
        s4 hv;
#pragma unroll
        for (int e = 0; e < 4; ++e) hv[e] = __builtin_bit_cast(short, DT<T>::fromf(acc[t][e] * il));
        *reinterpret_cast<s4*>(pp + t * 16) = hv;
      }
    } else {
      float* pp = a.part + slot * D + cw0 + 4 * (lane >> 4);
#pragma unroll
      for (int t = 0; t < CTW; ++t) *reinterpret_cast<f32x4*>(pp + t * 16) = acc[t];
    }
    if (wave == 0 && lane < 16) *reinterpret_cast<float2*>(a.ml + slot * 2) = float2{m_run, l_run};
  }
#ifdef WCB_XENC_PROBE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  XPROBE(11);
#else
  if (a.stamp.base) {
    __syncthreads();
    if (tid == 0) stamp_commit(a.stamp, t_start);
  }
#endif
}

template <typename T, int D>
__global__ __launch_bounds__(256) void xenc_merge_kernel(XencArgs a, T* u, long ldu) {
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int ns = a.nsplit;
  // every load is issued unconditionally (index clamped, weight 0 beyond nsplit): a load under a
  // run-time condition makes hipcc wait for each one in turn
  __shared__ float2 sv[kXencMaxSplit];
  if (tid < kXencMaxSplit)
    sv[tid] = tid < ns ? *reinterpret_cast<const float2*>(a.ml + (((long)b * ns + tid) * a.H + h) * 2) : float2{0.f, 0.f};
  __syncthreads();
  float2 v[kXencMaxSplit];
#pragma unroll
  for (int s = 0; s < kXencMaxSplit; ++s) v[s] = sv[s];
  float mx = -INFINITY;
#pragma unroll
  for (int s = 0; s < kXencMaxSplit; ++s)
    if (s < ns && v[s].y > 0.f) mx = fmaxf(mx, v[s].x);
  float w[kXencMaxSplit];
  float L = 0.f;
#pragma unroll
  for (int s = 0; s < kXencMaxSplit; ++s) {
    w[s] = (s < ns && v[s].y > 0.f) ? __expf(v[s].x - mx) : 0.f;   // empty ranges publish Σp = 0
    L += w[s] * v[s].y;
  }
  const float inv = 1.f / L;
  const float* pp = a.part + ((long)b * ns * a.H + h) * D;
  for (int c = tid * 4; c < D; c += 1024) {
    f32x4 pv[kXencMaxSplit];
#pragma unroll
    for (int s = 0; s < kXencMaxSplit; ++s) pv[s] = *reinterpret_cast<const f32x4*>(pp + (long)min(s, ns - 1) * a.H * D + c);
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kXencMaxSplit; ++s) acc += w[s] * pv[s];
    acc *= inv;
    typedef short s4 __attribute__((ext_vector_type(4)));
    s4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = __builtin_bit_cast(short, DT<T>::fromf(acc[e]));
    *reinterpret_cast<s4*>(u + (long)b * ldu + (long)h * D + c) = o;
  }
}

// xenc_merge_v_kernel: the range merge and the value projection in one launch (replaces
// xenc_merge_kernel + the grouped W_v decode GEMM: one dependent launch fewer per layer).
// Workgroup = (head h, RPW rows): u = Σ_s w_s·part_s / L as in xenc_merge_kernel (rounded to T, as the
// unfused path stores it), kept in LDS; then o = W_v,h·u + b_v as 16×16×32 MFMAs — wave w takes outputs
// 16w .. 16w + 15 of the head as the A rows, the rows' u the B columns 0 .. RPW-1, K = D in D/32 steps
// (u is exactly representable in T, so the B operand is u itself). Every weight load is issued before
// the partials (they do not depend on them). The MFMA form replaced VALU dot products (r04 probe: 7.6k
// cycles of the launch): 7.55 -> 7.08 us per C2 launch in the bench's serialised pass.
// OS (output splits): the head's 64 outputs over OS workgroups (OS = 2: waves 0-1 own the 32 outputs of
// this workgroup, waves 2-3 help with the range merge only): each workgroup reads W_v,h / OS, so twice the
// rows (RPW) per workgroup keep the grid while the weight bytes per workgroup halve. Same arithmetic per output.
template <typename T, int D, int MS, int RPW, bool P16 = false, int OS = 1>
__global__ __launch_bounds__(256) void xenc_merge_v_kernel(XencArgs a, const T* wv, const T* wfm, const float* bv, T* out, long ldo) {
  using Frag = typename DT<T>::frag;
  constexpr int KS = D / 32;
  static_assert(D <= 1024 && D % 32 == 0, "one 4-column group per thread");
  static_assert(RPW <= 16, "the rows are the B columns of one MFMA");
  static_assert(OS == 1 || OS == 2, "output splits");
  const int h = blockIdx.x / OS, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int otile = (blockIdx.x % OS) * (4 / OS) + wave;   // this wave's 16-output tile of the head
  const bool owner = wave < 4 / OS;
  const int ns = a.nsplit;
  __shared__ float2 sv[RPW][MS];
  __shared__ __attribute__((aligned(16))) float us[RPW][D];
  MPROBE(0);
  // W_v,h rows 16·otile + (lane & 15), k = 32·ks + 8·(lane >> 4): the A fragments of the wave's outputs
  // (fragment-major copy when given: tile h·4 + otile, 1 KiB contiguous per wave-instruction; the same values)
  Frag wf[KS];
  if (owner) {
    const T* wr = wfm ? wfm + ((long)(h * 4 + otile) * KS * 64 + lane) * 8
                      : wv + (long)(h * 64 + 16 * otile + (lane & 15)) * D + 8 * (lane >> 4);
    const int kstep = wfm ? 512 : 32;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wf[ks] = load_frag<T>(wr + ks * kstep);
  }
  const int c = min(tid * 4, D - 4);
  using PV = typename std::conditional<P16, uint2, f32x4>::type;   // P16: four T values, decoded after the loads
  PV pv[RPW][MS];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int b = min(blockIdx.y * RPW + r, a.rows - 1);
    if constexpr (P16) {
      const T* pp = reinterpret_cast<const T*>(a.part) + ((long)b * ns * a.H + h) * D;
#pragma unroll
      for (int s = 0; s < MS; ++s) pv[r][s] = *reinterpret_cast<const uint2*>(pp + (long)min(s, ns - 1) * a.H * D + c);
    } else {
      const float* pp = a.part + ((long)b * ns * a.H + h) * D;
#pragma unroll
      for (int s = 0; s < MS; ++s) pv[r][s] = *reinterpret_cast<const f32x4*>(pp + (long)min(s, ns - 1) * a.H * D + c);
    }
    const float2 mlv = *reinterpret_cast<const float2*>(a.ml + (((long)b * ns + min(tid, ns - 1)) * a.H + h) * 2);
    if (tid < MS) sv[r][tid] = tid < ns ? mlv : float2{0.f, 0.f};
  }
  MPROBE(1);
  __syncthreads();
  MPROBE(2);
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    float2 v[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) v[s] = sv[r][s];
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < MS; ++s)
      if (s < ns && v[s].y > 0.f) mx = fmaxf(mx, v[s].x);
    float w[MS];
    float L = 0.f;
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      w[s] = (s < ns && v[s].y > 0.f) ? __expf(v[s].x - mx) : 0.f;   // empty ranges publish Σp = 0
      L += w[s] * v[s].y;
    }
    const float inv = 1.f / L;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      if constexpr (P16) {   // normalised partials: weight w_s·Σp_s
        const uint2 q = pv[r][s];
        const uint32_t hw[4] = {q.x & 0xffffu, q.x >> 16, q.y & 0xffffu, q.y >> 16};
        f32x4 x;
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = DT<T>::tof(__builtin_bit_cast(T, (uint16_t)hw[e]));
        acc += (w[s] * v[s].y) * x;
      } else {
        acc += w[s] * pv[r][s];
      }
    }
    acc *= inv;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = DT<T>::tof(DT<T>::fromf(acc[e]));   // u in T, as stored unfused
    if (tid * 4 < D) *reinterpret_cast<f32x4*>(&us[r][c]) = acc;
  }
  __syncthreads();
  MPROBE(3);
  if (!owner) return;
  // B: column lane & 15 = row r of this workgroup (zero past RPW), k = 32·ks + 8·(lane >> 4)
  const int r = lane & 15;
  f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    Frag uf = Frag{};
    if (r < RPW) {
      const f32x4 u0 = *reinterpret_cast<const f32x4*>(&us[r][ks * 32 + 8 * (lane >> 4)]);
      const f32x4 u1 = *reinterpret_cast<const f32x4*>(&us[r][ks * 32 + 8 * (lane >> 4) + 4]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uf[e] = __builtin_bit_cast(typename std::remove_reference<decltype(uf[0])>::type, DT<T>::fromf(u0[e]));
        uf[4 + e] = __builtin_bit_cast(typename std::remove_reference<decltype(uf[0])>::type, DT<T>::fromf(u1[e]));
      }
    }
    o = mma16(wf[ks], uf, o);
  }
  // C: lane holds outputs 16·otile + 4·(lane >> 4) + e of row lane & 15
  const int b = blockIdx.y * RPW + r;
  if (r < RPW && b < a.rows) {
    const int n = h * 64 + 16 * otile + 4 * (lane >> 4);
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(bv + n);
    typedef short s4 __attribute__((ext_vector_type(4)));
    s4 hv;
#pragma unroll
    for (int e = 0; e < 4; ++e) hv[e] = __builtin_bit_cast(short, DT<T>::fromf(o[e] + b4[e]));
    *reinterpret_cast<s4*>(out + (long)b * ldo + n) = hv;
  }
#ifdef WCB_XENC_PROBE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  MPROBE(4);
#endif
}

// The encoder output [B][S][D] → the fragment-major chunk layout of attn_xenc_reg_kernel<.., FM>:
// [B][ceil(S/32) chunks][NW waves][2 halves][KSW k-steps][64 lanes][8], element (lane, e) of (chunk g,
// wave w, half h, k-step ks) = enc[b][32g + 16h + (lane & 15)][w·CW + 32ks + 8(lane >> 4) + e] (zero
// past S): the lane layout of the kernel's row loads, stored so one wave-instruction reads 1 KiB.
template <typename T, int D>
__global__ __launch_bounds__(256) void xenc_fm_kernel(const T* __restrict__ src, T* __restrict__ dst, int S, long n16) {
  using C = XregCfg<D>;
  constexpr int NW = C::NW, KSW = C::KSW, CW = C::CW;
  const int nchunk = (S + kXencCK - 1) / kXencCK;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) {
    long r = i;
    const int lane = (int)(r % 64); r /= 64;
    const int ks = (int)(r % KSW); r /= KSW;
    const int hf = (int)(r % 2); r /= 2;
    const int w = (int)(r % NW); r /= NW;
    const int g = (int)(r % nchunk);
    const long clip = r / nchunk;
    const int key = g * kXencCK + hf * 16 + (lane & 15);
    const int col = w * CW + 8 * (lane >> 4) + 32 * ks;
    s16x8 v = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (key < S) v = *reinterpret_cast<const s16x8*>(src + (clip * S + key) * D + col);
    *reinterpret_cast<s16x8*>(dst + i * 8) = v;
  }
}

long xenc_fm_elems(int B, int S, int D) { return (long)B * ((S + kXencCK - 1) / kXencCK) * kXencCK * D; }

template <typename T>
static void launch_fm_t(const void* src, void* dst, int B, int S, int D, hipStream_t s) {
  const long n16 = xenc_fm_elems(B, S, D) / 8;
  const dim3 grid((unsigned)std::min<long>((n16 + 255) / 256, 4096));
#define WCB_FM(DD) case DD: WCB_LAUNCH((xenc_fm_kernel<T, DD>), grid, dim3(256), 0, s, (const T*)src, (T*)dst, S, n16); break;
  switch (D) { WCB_FM(64) WCB_FM(128) WCB_FM(256) WCB_FM(384) WCB_FM(512) WCB_FM(768) WCB_FM(1024) default: break; }
#undef WCB_FM
}

void xenc_to_fm(DType t, const void* src, void* dst, int B, int S, int D, hipStream_t s) {
  if (t == kBF16) launch_fm_t<bf16_t>(src, dst, B, S, D, s);
  else if (t == kF16) launch_fm_t<f16_t>(src, dst, B, S, D, s);
}

bool xenc_supported(DType t, int D) {
  return (t == kBF16 || t == kF16) && (D == 384 || D == 768 || D == 1024 || D == 64 || D == 128 || D == 256 || D == 512);
}

template <typename T, int D>
static void launch_xenc(const XencArgs& a, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)attn_xenc_kernel<T, D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              XencCfg<D>::LDS);
    (void)hipFuncSetAttribute((const void*)attn_xenc_reg_kernel<T, D, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              XregCfg<D>::LDS);
    (void)hipFuncSetAttribute((const void*)attn_xenc_reg_kernel<T, D, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              XregCfg<D>::LDS);
    (void)hipFuncSetAttribute((const void*)attn_xenc_reg_kernel<T, D, 2, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              XregCfg<D>::LDS);
    (void)hipFuncSetAttribute((const void*)attn_xenc_reg_kernel<T, D, 3, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              XregCfg<D>::LDS);
    attr_set = true;
  }
  if (a.part16) {   // 16-bit normalised range partials (the register-ring variant 1)
    static bool attr16 = false;
    if (!attr16) {
      (void)hipFuncSetAttribute((const void*)attn_xenc_reg_kernel<T, D, 2, 4, true, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, XregCfg<D>::LDS);
      (void)hipFuncSetAttribute((const void*)attn_xenc_reg_kernel<T, D, 2, 4, false, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, XregCfg<D>::LDS);
      attr16 = true;
    }
    if (a.fm) WCB_LAUNCH((attn_xenc_reg_kernel<T, D, 2, 4, true, true>), dim3(a.nsplit, a.rows), dim3(XregCfg<D>::NW * 64), XregCfg<D>::LDS, s, a);
    else WCB_LAUNCH((attn_xenc_reg_kernel<T, D, 2, 4, false, true>), dim3(a.nsplit, a.rows), dim3(XregCfg<D>::NW * 64), XregCfg<D>::LDS, s, a);
    return;
  }
  if (a.fm) {   // the fragment-major chunk layout (register-ring variants 1 and 2 only)
    if (a.variant == 2)
      WCB_LAUNCH((attn_xenc_reg_kernel<T, D, 3, 4, true>), dim3(a.nsplit, a.rows), dim3(XregCfg<D>::NW * 64), XregCfg<D>::LDS, s, a);
    else
      WCB_LAUNCH((attn_xenc_reg_kernel<T, D, 2, 4, true>), dim3(a.nsplit, a.rows), dim3(XregCfg<D>::NW * 64), XregCfg<D>::LDS, s, a);
    return;
  }
  if constexpr (D % (8 * 32) == 0 && D >= 512) {
    static bool attr8 = false;
    if (!attr8) {
      (void)hipFuncSetAttribute((const void*)attn_xenc_reg_kernel<T, D, 2, 8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, XregCfg<D, 8>::LDS);
      attr8 = true;
    }
    if (a.variant == 3) {
      constexpr int kThreads = XregCfg<D, 8>::NW * 64, kLds = XregCfg<D, 8>::LDS;
      WCB_LAUNCH((attn_xenc_reg_kernel<T, D, 2, 8>), dim3(a.nsplit, a.rows), dim3(kThreads), kLds, s, a);
      return;
    }
  }
  if (a.variant == 0)
    WCB_LAUNCH((attn_xenc_kernel<T, D>), dim3(a.nsplit, a.rows), dim3(kXencNW * 64), XencCfg<D>::LDS, s, a);
  else if (a.variant == 2)
    WCB_LAUNCH((attn_xenc_reg_kernel<T, D, 3>), dim3(a.nsplit, a.rows), dim3(XregCfg<D>::NW * 64),
                       XregCfg<D>::LDS, s, a);
  else
    WCB_LAUNCH((attn_xenc_reg_kernel<T, D, 2>), dim3(a.nsplit, a.rows), dim3(XregCfg<D>::NW * 64),
                       XregCfg<D>::LDS, s, a);
}

template <typename T>
static void launch_xenc_t(const XencArgs& a, hipStream_t s) {
  switch (a.D) {
    case 64: launch_xenc<T, 64>(a, s); break;
    case 128: launch_xenc<T, 128>(a, s); break;
    case 256: launch_xenc<T, 256>(a, s); break;
    case 384: launch_xenc<T, 384>(a, s); break;
    case 512: launch_xenc<T, 512>(a, s); break;
    case 768: launch_xenc<T, 768>(a, s); break;
    case 1024: launch_xenc<T, 1024>(a, s); break;
    default: break;
  }
}

void xenc_attention(DType t, const XencArgs& a, hipStream_t s) {
  if (t == kBF16) launch_xenc_t<bf16_t>(a, s);
  else if (t == kF16) launch_xenc_t<f16_t>(a, s);
}

template <typename T>
static void launch_merge_t(const XencArgs& a, void* u, long ldu, hipStream_t s) {
  const dim3 grid(a.H, a.rows);
#define WCB_XC(DD) case DD: WCB_LAUNCH((xenc_merge_kernel<T, DD>), grid, dim3(256), 0, s, a, (T*)u, ldu); break;
  switch (a.D) { WCB_XC(64) WCB_XC(128) WCB_XC(256) WCB_XC(384) WCB_XC(512) WCB_XC(768) WCB_XC(1024) default: break; }
#undef WCB_XC
}

void xenc_merge(DType t, const XencArgs& a, void* u, long ldu, hipStream_t s) {
  if (t == kBF16) launch_merge_t<bf16_t>(a, u, ldu, s);
  else if (t == kF16) launch_merge_t<f16_t>(a, u, ldu, s);
}

template <typename T>
static void launch_merge_v_t(const XencArgs& a, const void* wv, const void* wfm, const float* bv, void* o, long ldo, hipStream_t s) {
  // two rows per workgroup (the head's W_v,h fragments serve both: half the weight re-reads; 4 measured
  // slower); MS: the partial loads per thread (the key-range count rounded up to 8 or 16; ranges past
  // nsplit carry weight 0)
  const dim3 grid(a.H, (a.rows + 1) / 2);
  const dim3 grid2(a.H * 2, (a.rows + 3) / 4);   // merge_os 2: the head's outputs over two workgroups, 4 rows each
#define WCB_XC(DD)                                                                                                    \
  case DD:                                                                                                            \
    if (a.merge_os == 2 && a.part16 && a.nsplit <= 8) WCB_LAUNCH((xenc_merge_v_kernel<T, DD, 8, 4, true, 2>), grid2, dim3(256), 0, s, a, (const T*)wv, (const T*)wfm, bv, (T*)o, ldo); \
    else if (a.part16 && a.nsplit <= 8) WCB_LAUNCH((xenc_merge_v_kernel<T, DD, 8, 2, true>), grid, dim3(256), 0, s, a, (const T*)wv, (const T*)wfm, bv, (T*)o, ldo); \
    else if (a.part16) WCB_LAUNCH((xenc_merge_v_kernel<T, DD, kXencMaxSplit, 2, true>), grid, dim3(256), 0, s, a, (const T*)wv, (const T*)wfm, bv, (T*)o, ldo); \
    else if (a.nsplit <= 8) WCB_LAUNCH((xenc_merge_v_kernel<T, DD, 8, 2>), grid, dim3(256), 0, s, a, (const T*)wv, (const T*)wfm, bv, (T*)o, ldo); \
    else WCB_LAUNCH((xenc_merge_v_kernel<T, DD, kXencMaxSplit, 2>), grid, dim3(256), 0, s, a, (const T*)wv, (const T*)wfm, bv, (T*)o, ldo);   \
    break;
  switch (a.D) { WCB_XC(128) WCB_XC(256) WCB_XC(384) WCB_XC(512) WCB_XC(768) WCB_XC(1024) default: break; }
#undef WCB_XC
}

void xenc_merge_v(DType t, const XencArgs& a, const void* wv, const float* bv, void* o, long ldo, hipStream_t s,
                  const void* wv_fm) {
  if (t == kBF16) launch_merge_v_t<bf16_t>(a, wv, wv_fm, bv, o, ldo, s);
  else if (t == kF16) launch_merge_v_t<f16_t>(a, wv, wv_fm, bv, o, ldo, s);
}

}  // namespace wcb
