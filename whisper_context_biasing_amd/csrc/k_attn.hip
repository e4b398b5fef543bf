// Attention kernels (head_dim 64 for every Whisper size).
//
// attn_flash_kernel — encoder self-attention, non-causal, S = 1500 keys
//   ([tf] modeling_whisper.py:284-356 with the SDPA backend; q is pre-scaled by head_dim^-0.5 —
//   folded exactly into q_proj since 0.125 is a power of two). 16-bit T only.
//   Workgroup = 4 waves × 32 query rows; K/V tiles of 64 keys double-buffered in LDS via
//   global_load_lds with an XOR-swizzled source address. "Swapped" products keep the softmax
//   lane-local: Sᵀ = K·Qᵀ puts one query per lane column, Oᵀ = Vᵀ·Pᵀ consumes the Sᵀ accumulator
//   registers directly as the B operand (permuted k order, matched by the Vᵀ fragment), Vᵀ
//   fragments come from ds_read_b64_tr_b16 transposed LDS reads. Online softmax in f32.
//
// attn_decode_kernel — one query row per workgroup (decoder self-attention over the KV cache,
//   decoder cross-attention over the precomputed encoder K/V, and the f32 "exact" encoder path).
//   8 lanes per key (16 B of K and V each), one pass with an online softmax, optional split-KV
//   over workgroups. HBM-bound on the K/V read.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "self_attn.h"

namespace wcb {

// Single pass over the keys (flash-decoding): every lane group of 8 lanes owns one key per load
// (16 B of K and of V per lane), a wave covers 64 keys per iteration with all 16 K/V loads in flight
// at once, the online softmax runs at wave level (running max / denominator, the accumulator
// rescaled when the max moves), waves combine in LDS, key chunks (split-KV) combine through the
// last-arriver hand-off below.
//
// Split-KV: workgroup (i·nsplit + c, b·H + h) handles key chunk c. With nsplit > 1 each chunk
// publishes (max, Σexp, Σexp·v[64]) with write-through (sc1) stores, drains them (vmcnt(0)) and takes
// an agent-scope ticket; the chunk that draws the last ticket reads every partial with sc1 loads,
// combines them in chunk order (deterministic) and resets the ticket (cdna_hip_programming.md §6
// Guideline 16, first row of the measured hand-off table).
// PHYS (beam search): key j of row b lives in cache row phys[(row0 + b)·phys_ld + j] (k_beam.hip).
template <typename T, int NW, int U, bool PHYS = false>
__global__ __launch_bounds__(NW * 64) void attn_decode_kernel(AttnArgs a) {
  __shared__ float wo[NW][64];
  __shared__ float wm[NW], wl[NW];
  const int nsplit = a.nsplit > 0 ? a.nsplit : 1;
  const int i = blockIdx.x / nsplit, chunk = blockIdx.x % nsplit;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long t_start = a.stamp.base ? stamp_now() : 0;
  const int seg = lane & 7, kg = lane >> 3;
  const int nk_all = (a.nkeys_dev ? (*a.nkeys_dev + a.nkeys_add) : a.nkeys) + (a.causal ? i : 0);
  const int per = (nk_all + nsplit - 1) / nsplit;
  const int j_lo = chunk * per, j_hi = min(nk_all, j_lo + per);
  const int nk = max(j_hi - j_lo, 0);
  const T* q = reinterpret_cast<const T*>(a.q) + ((long)b * a.q_Sb + i) * a.ldq + h * 64;
  const long krow = PHYS ? 0L : (long)((a.row0 + b) / a.b_div) * a.k_sb;
  const int* prow = PHYS ? a.phys + (long)(a.row0 + b) * a.phys_ld + j_lo : nullptr;
  const T* kb = reinterpret_cast<const T*>(a.k) + krow + (long)h * a.k_sh + (long)j_lo * a.k_sk + seg * 8;
  const T* vb = reinterpret_cast<const T*>(a.v) + krow + (long)h * a.k_sh + (long)j_lo * a.k_sk + seg * 8;
  auto koff = [&](int j) -> long { return (long)j * a.k_sk + (PHYS ? (long)prow[j] * a.k_sb : 0L); };
  float qv[8];
  load8f<T>(q + seg * 8, qv);

  // U keys per lane group per iteration
  constexpr int WSPAN = 8 * U, GSPAN = NW * WSPAN;
  float m = -INFINITY, l = 0.f;              // wave-uniform running max; per-lane partial Σp
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = wave * WSPAN; j0 < nk; j0 += GSPAN) {
    float kv[U][8], vv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) load8f<T>(kb + koff(min(j0 + u * 8 + kg, nk - 1)), kv[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) load8f<T>(vb + koff(min(j0 + u * 8 + kg, nk - 1)), vv[u]);
    float sc[U];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(qv[e], kv[u][e], d);
#pragma unroll
      for (int x = 1; x < 8; x <<= 1) d += __shfl_xor(d, x, 64);
      sc[u] = (j0 + u * 8 + kg < nk) ? d : -INFINITY;
      mx = fmaxf(mx, sc[u]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 8, 64));
    mx = xor16_max(mx);
    mx = xor32_max(mx);
    const float mn = fmaxf(m, mx);           // finite: the first iteration has ≥ 1 valid key
    const float r = __expf(m - mn);          // 0 on the first iteration (m = −inf)
    m = mn;
    l *= r;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] *= r;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float p = __expf(sc[u] - m);
      l += p;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(p, vv[u][e], o[e]);
    }
  }
  // reduce over the 8 lane groups (each group holds its own keys' p and p·v)
  l += __shfl_xor(l, 8, 64);
  l = xor16_add(l);
  l = xor32_add(l);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] += __shfl_xor(o[e], 8, 64);
    o[e] = xor16_add(o[e]);
    o[e] = xor32_add(o[e]);
  }
  if (kg == 0)
#pragma unroll
    for (int e = 0; e < 8; ++e) wo[wave][seg * 8 + e] = o[e];
  if (lane == 0) { wm[wave] = m; wl[wave] = l; }
  __syncthreads();
  if (wave != 0) return;
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < NW; ++w) M = fmaxf(M, wm[w]);
  float L = 0.f, acc = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const float sw = wl[w] > 0.f ? __expf(wm[w] - M) : 0.f;   // waves without keys hold l = 0
    L += wl[w] * sw;
    acc += wo[w][lane] * sw;
  }
  T* out = reinterpret_cast<T*>(a.o) + ((long)b * a.o_Sb + i) * a.ldo + h * 64;
  if (nsplit == 1) {
    out[lane] = DT<T>::fromf(acc / L);
    if (lane == 0) stamp_commit(a.stamp, t_start);
    return;
  }
  // ---- split-KV hand-off: publish this chunk's partial, last arriver combines
  const long slot = ((long)bh * a.Sq + i);
  float* part = a.part + slot * nsplit * 66;
  float* mine = part + chunk * 66;
  __hip_atomic_store(mine + 2 + lane, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 0) {
    __hip_atomic_store(mine, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = atomicAdd(a.ticket + slot, 1);
  old = __shfl(old, 0, 64);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (old != nsplit - 1) {
    if (lane == 0) stamp_commit(a.stamp, t_start);
    return;
  }
  float MM = -INFINITY;
  for (int c = 0; c < nsplit; ++c) {
    const float mc = __hip_atomic_load(part + c * 66, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float lc = __hip_atomic_load(part + c * 66 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lc > 0.f && mc > MM) MM = mc;
  }
  float LL = 0.f, OO = 0.f;
  for (int c = 0; c < nsplit; ++c) {
    const float mc = __hip_atomic_load(part + c * 66, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float lc = __hip_atomic_load(part + c * 66 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float oc = __hip_atomic_load(part + c * 66 + 2 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float w = lc > 0.f ? __expf(mc - MM) : 0.f;    // empty chunks publish l = 0
    LL += lc * w;
    OO += oc * w;
  }
  out[lane] = DT<T>::fromf(OO / LL);
  if (lane == 0) {
    __hip_atomic_store(a.ticket + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stamp_commit(a.stamp, t_start);
  }
}

// Two-pass variant (variant 0, the default for the cross-attention): pass 1 streams K and keeps the
// scores in LDS, exact max, pass 2 exponentiates, pass 3 streams V. 8 waves, 8 keys per lane group
// in flight. Measured in the decode graph (2 row groups of 16 rows) slightly ahead of the single-pass
// kernel above: fewer live registers, more waves per CU.
constexpr int kMaxKeys = 2048;
template <typename T, int NW>
__global__ __launch_bounds__(NW * 64) void attn_decode2p_kernel(AttnArgs a) {
  __shared__ float sc[kMaxKeys];
  __shared__ float red[NW][64 + 1];
  __shared__ float stat[2];
  const int nsplit = a.nsplit > 0 ? a.nsplit : 1;
  const int i = blockIdx.x / nsplit, chunk = blockIdx.x % nsplit;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long t_start = a.stamp.base ? stamp_now() : 0;
  const int seg = lane & 7, kg = lane >> 3;
  const int nk_all = (a.nkeys_dev ? (*a.nkeys_dev + a.nkeys_add) : a.nkeys) + (a.causal ? i : 0);
  const int per = (nk_all + nsplit - 1) / nsplit;
  const int j_lo = chunk * per, j_hi = min(nk_all, j_lo + per);
  const int nk = max(j_hi - j_lo, 0);
  const T* q = reinterpret_cast<const T*>(a.q) + ((long)b * a.q_Sb + i) * a.ldq + h * 64;
  const long krow = (long)((a.row0 + b) / a.b_div) * a.k_sb;
  const T* kb = reinterpret_cast<const T*>(a.k) + krow + (long)h * a.k_sh + (long)j_lo * a.k_sk + seg * 8;
  const T* vb = reinterpret_cast<const T*>(a.v) + krow + (long)h * a.k_sh + (long)j_lo * a.k_sk + seg * 8;
  float qv[8];
  load8f<T>(q + seg * 8, qv);

  // pass 1: scores. 8 lanes per key (16 B each), U keys per lane in flight (memory-level
  // parallelism: the K/V stream is the HBM-bound part of the decode step)
  constexpr int U = 8;
  constexpr int WSPAN = 8 * U, GSPAN = NW * WSPAN;
  float mx = -INFINITY;
  for (int j0 = wave * WSPAN; j0 < nk; j0 += GSPAN) {
    float kv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) load8f<T>(kb + (long)min(j0 + u * 8 + kg, nk - 1) * a.k_sk, kv[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float dsum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum = fmaf(qv[e], kv[u][e], dsum);
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) dsum += __shfl_xor(dsum, o, 64);
      const int j = j0 + u * 8 + kg;
      if (j < nk) { if (seg == 0) sc[j] = dsum; mx = fmaxf(mx, dsum); }
    }
  }
  mx = wave_max(mx);
  if (lane == 0) red[wave][0] = mx;
  __syncthreads();
  if (tid == 0) {
    float m = red[0][0];
    for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w][0]);
    stat[0] = m;
  }
  __syncthreads();
  const float m = stat[0];
  // pass 2: exponentials + denominator
  float ssum = 0.f;
  for (int j = tid; j < nk; j += NW * 64) {
    const float p = __expf(sc[j] - m);
    sc[j] = p;
    ssum += p;
  }
  ssum = wave_sum(ssum);
  __syncthreads();
  if (lane == 0) red[wave][1] = ssum;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int w = 0; w < NW; ++w) s += red[w][1];
    stat[1] = s;
  }
  // pass 3: o = P·V
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = wave * WSPAN; j0 < nk; j0 += GSPAN) {
    float vv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) load8f<T>(vb + (long)min(j0 + u * 8 + kg, nk - 1) * a.k_sk, vv[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * 8 + kg;
      const float p = j < nk ? sc[j] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(p, vv[u][e], o[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] += __shfl_xor(o[e], 8, 64);
    o[e] = xor16_add(o[e]);
    o[e] = xor32_add(o[e]);
  }
  __syncthreads();
  if (kg == 0)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wave][seg * 8 + e] = o[e];
  __syncthreads();
  if (wave != 0) return;
  float acc = 0.f;
  for (int w = 0; w < NW; ++w) acc += red[w][lane];
  T* out = reinterpret_cast<T*>(a.o) + ((long)b * a.o_Sb + i) * a.ldo + h * 64;
  if (nsplit == 1) {
    out[lane] = DT<T>::fromf(acc / stat[1]);
    if (lane == 0) stamp_commit(a.stamp, t_start);
    return;
  }
  // ---- split-KV hand-off: publish this chunk's partial, last arriver combines
  const long slot = ((long)bh * a.Sq + i);
  float* part = a.part + slot * nsplit * 66;
  float* mine = part + chunk * 66;
  __hip_atomic_store(mine + 2 + lane, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 0) {
    __hip_atomic_store(mine, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 1, stat[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = atomicAdd(a.ticket + slot, 1);
  old = __shfl(old, 0, 64);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (old != nsplit - 1) {
    if (lane == 0) stamp_commit(a.stamp, t_start);
    return;
  }
  float M = -INFINITY;
  for (int c = 0; c < nsplit; ++c) {
    const float mc = __hip_atomic_load(part + c * 66, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (mc > M) M = mc;
  }
  float L = 0.f, O = 0.f;
  for (int c = 0; c < nsplit; ++c) {
    const float mc = __hip_atomic_load(part + c * 66, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float lc = __hip_atomic_load(part + c * 66 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float oc = __hip_atomic_load(part + c * 66 + 2 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float w = lc > 0.f ? __expf(mc - M) : 0.f;    // empty chunks publish l = 0
    L += lc * w;
    O += oc * w;
  }
  out[lane] = DT<T>::fromf(O / L);
  if (lane == 0) {
    __hip_atomic_store(a.ticket + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stamp_commit(a.stamp, t_start);
  }
}

// Decoder self-attention of one new token (Sq = 1, no split, keys in place): one wave per (row,
// head). The first 64 keys' K and V rows are requested together with the key count (which lives in
// device memory: the step graph is replayed) — one memory round trip instead of a dependent pair;
// rows past the count (clamped to the cache capacity kv_rows) are loaded and masked. Longer
// contexts continue in 64-key chunks with an online softmax. 8 lanes per key (16 B each), 8 keys
// per load, 8 loads of K and of V per lane in flight.
// PHYS (beam search): key j of row b lives in cache row phys[(row0 + b)·phys_ld + j]; lane j of the
// wave loads the map entry of key j0 + j once per 64-key chunk and the K/V row offsets are shuffled
// from it (one dependent round trip per chunk, not one per key group). Skipping the key groups past
// the device-side count by a branch measured slower (C3 22.8 -> 38.3 µs); clamping their index to the
// last key (no branch) keeps the loads but collapses them onto one cache line.
template <typename T, bool PHYS>
__global__ __launch_bounds__(64) void attn_self_kernel(AttnArgs a) {
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H, lane = threadIdx.x;
  const int seg = lane & 7, kg = lane >> 3;
  const long base = (PHYS ? 0L : (long)((a.row0 + b) / a.b_div) * a.k_sb) + (long)h * a.k_sh + seg * 8;
  const T* kb = reinterpret_cast<const T*>(a.k) + base;
  const T* vb = reinterpret_cast<const T*>(a.v) + base;
  const T* q = reinterpret_cast<const T*>(a.q) + (long)b * a.q_Sb * a.ldq + h * 64;
  const int cap = a.kv_rows - 1;
  const int* prow = PHYS ? a.phys + (long)(a.row0 + b) * a.phys_ld : nullptr;
  int pj = PHYS ? prow[min(lane, cap)] : 0;
  auto koff = [&](int j, int u) -> long {   // element offset of key j = j0 + 8u + kg of this lane
    return (long)j * a.k_sk + (PHYS ? (long)__shfl(pj, u * 8 + kg, 64) * a.k_sb : 0L);
  };
  float qv[8], kv[8][8], vv[8][8];
  load8f<T>(q + seg * 8, qv);
  const int nk = a.nkeys_dev ? (*a.nkeys_dev + a.nkeys_add) : a.nkeys;
  if constexpr (PHYS) {
    // the key count arrives with the map (the same round trip): keys past it re-read key nk − 1
    // (one cache line for all of them) instead of fetching rows that are masked anyway
    const int kl = min(nk, a.kv_rows) - 1;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int kk = min(u * 8 + kg, kl);
      load8f<T>(kb + (long)kk * a.k_sk + (long)__shfl(pj, kk, 64) * a.k_sb, kv[u]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int kk = min(u * 8 + kg, kl);
      load8f<T>(vb + (long)kk * a.k_sk + (long)__shfl(pj, kk, 64) * a.k_sb, vv[u]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) load8f<T>(kb + koff(min(u * 8 + kg, cap), u), kv[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u) load8f<T>(vb + koff(min(u * 8 + kg, cap), u), vv[u]);
  }
  float m = -INFINITY, l = 0.f;
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nk; j0 += 64) {
    if (j0) {
      if constexpr (PHYS) pj = prow[min(min(j0 + lane, nk - 1), cap)];
#pragma unroll
      for (int u = 0; u < 8; ++u) load8f<T>(kb + koff(min(min(j0 + u * 8 + kg, nk - 1), cap), u), kv[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u) load8f<T>(vb + koff(min(min(j0 + u * 8 + kg, nk - 1), cap), u), vv[u]);
    }
    float sc[8];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(qv[e], kv[u][e], d);
#pragma unroll
      for (int x = 1; x < 8; x <<= 1) d += __shfl_xor(d, x, 64);
      sc[u] = (j0 + u * 8 + kg < nk) ? d : -INFINITY;
      mx = fmaxf(mx, sc[u]);
    }
    const float mn = fmaxf(m, wave_max(mx));
    const float r = __expf(m - mn);   // 0 on the first chunk (m = -inf)
    l *= r;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] *= r;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      // keys past the count were loaded speculatively (rows left by an earlier call, possibly
      // non-finite): they contribute nothing, not even 0·v
      const bool live = j0 + u * 8 + kg < nk;
      const float p = live ? __expf(sc[u] - mn) : 0.f;
      if (seg == 0) l += p;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = live ? fmaf(p, vv[u][e], o[e]) : o[e];
    }
    m = mn;
  }
  l = wave_sum(l);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] += __shfl_xor(o[e], 8, 64);
    o[e] = xor16_add(o[e]);
    o[e] = xor32_add(o[e]);
  }
  if (kg == 0) {
    float r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = o[e] / l;
    store8<T>(reinterpret_cast<T*>(a.o) + (long)b * a.o_Sb * a.ldo + h * 64 + seg * 8, r);
  }
}

// attn_self_kernel<T, false> (greedy rows, keys in place) with a compact argument block: the
// AttnArgs form took three dependent scalar round trips (kernel arguments, the device-side key count,
// the remaining arguments) before its K/V loads were issued; here every argument arrives in one
// scalar batch, the q / K / V loads go out first and the key count after them. Same arithmetic,
// bit-identical outputs.
struct SelfLean {
  const void* q; const void* k; const void* v; void* o;
  const int* nkeys_dev;
  long k_sb, k_sh;
  int ldq, ldo, H, cap, nkeys_add, row0, b_div, npairs;
};

template <typename T, int WPG = 1>
__global__ __launch_bounds__(64 * WPG) void attn_self_lean_kernel(SelfLean a) {
  // WPG (row, head) pairs per workgroup, one per wave (pairs past the batch re-run the last one)
  const int pair = min(blockIdx.y * WPG + (int)(threadIdx.x >> 6), a.npairs - 1);
  const int b = pair / a.H, h = pair % a.H;
  const long base = (long)((a.row0 + b) / a.b_div) * a.k_sb + (long)h * a.k_sh;
  self_attn_wave<T>(reinterpret_cast<const T*>(a.q) + (long)b * a.ldq + h * 64,
                           reinterpret_cast<const T*>(a.k) + base, reinterpret_cast<const T*>(a.v) + base, a.cap,
                           [&] { return __builtin_amdgcn_readfirstlane(__builtin_nontemporal_load(a.nkeys_dev)) + a.nkeys_add; },
                           reinterpret_cast<T*>(a.o) + (long)b * a.ldo + h * 64);
}

template <typename T>
static void launch_decode(const AttnArgs& b, dim3 grid, int variant, hipStream_t s) {
  if (b.kv_rows > 0 && b.Sq == 1 && b.nsplit == 1) {   // decoder self-attention, one new token
    if (!b.phys && b.nkeys_dev && b.k_sk == 64 && b.q_Sb == 1 && b.o_Sb == 1 && sizeof(T) == 2) {
      SelfLean c;
      c.q = b.q; c.k = b.k; c.v = b.v; c.o = b.o; c.nkeys_dev = b.nkeys_dev;
      c.k_sb = b.k_sb; c.k_sh = b.k_sh; c.ldq = (int)b.ldq; c.ldo = (int)b.ldo; c.H = b.H;
      c.cap = b.kv_rows - 1; c.nkeys_add = b.nkeys_add; c.row0 = b.row0; c.b_div = b.b_div > 0 ? b.b_div : 1;
      c.npairs = (int)grid.y;
      // one (row, head) pair per 64-thread workgroup (4 per 256-thread workgroup measured 0.5 ms slower per
      // 72-token C2 call, tools/decode_ab.py)
      WCB_LAUNCH((attn_self_lean_kernel<T, 1>), dim3(1, grid.y), dim3(64), 0, s, c);
      return;
    }
    if (b.phys) WCB_LAUNCH((attn_self_kernel<T, true>), dim3(1, grid.y), dim3(64), 0, s, b);
    else WCB_LAUNCH((attn_self_kernel<T, false>), dim3(1, grid.y), dim3(64), 0, s, b);
    return;
  }
  if (b.phys) {   // beam-search self-attention: keys through the row map
    WCB_LAUNCH((attn_decode_kernel<T, 4, 8, true>), grid, dim3(256), 0, s, b);
    return;
  }
  switch (variant) {
    case 0: WCB_LAUNCH((attn_decode2p_kernel<T, 8>), grid, dim3(512), 0, s, b); break;
    case 1: WCB_LAUNCH((attn_decode_kernel<T, 4, 8>), grid, dim3(256), 0, s, b); break;
    case 2: WCB_LAUNCH((attn_decode_kernel<T, 4, 4>), grid, dim3(256), 0, s, b); break;
    case 3: WCB_LAUNCH((attn_decode_kernel<T, 8, 4>), grid, dim3(512), 0, s, b); break;
    case 4: WCB_LAUNCH((attn_decode_kernel<T, 8, 8>), grid, dim3(512), 0, s, b); break;
    default: WCB_LAUNCH((attn_decode_kernel<T, 16, 4>), grid, dim3(1024), 0, s, b); break;
  }
}

void attention_decode(DType t, const AttnArgs& a, hipStream_t s) {
  const int ns = (a.part && a.ticket && a.nsplit > 1) ? a.nsplit : 1;
  AttnArgs b = a;
  b.nsplit = ns;
  const dim3 grid(a.Sq * ns, a.B * a.H);
  switch (t) {
    case kBF16: launch_decode<bf16_t>(b, grid, a.variant, s); break;
    case kF16: launch_decode<f16_t>(b, grid, a.variant, s); break;
    case kF32: launch_decode<float>(b, grid, a.variant, s); break;
  }
}

// --------------------------------------------------------------------------------- flash (MFMA)
// Registers: scores and softmax of every query fragment first, then P·V with one 16-row block of Vᵀ
// fragments live at a time; 32 queries per wave fit 3 waves per SIMD (152 VGPRs), 64 queries per wave
// 2 (the encoder default: half the K/Vᵀ LDS reads per MFMA; 3 spills).
// Softmax exponentials are bare v_exp_f32 (__builtin_amdgcn_exp2f): libm's exp2f wraps each one in a
// denormal range fix-up (compare, two selects, ldexp) — 4 extra VALU per score on a VALU-bound loop;
// the arguments are ≤ 0 here and results below 2^-126 contribute nothing.
// NS LDS stages (NS - 1 K/V tiles in flight behind the one being multiplied). 2 everywhere: a
// third stage measured 3.6 % slower on the beam cross-attention (C3: 90.9 vs 87.7 µs per launch).
template <typename T, int QW, int NS>
__global__ __launch_bounds__(256, QW == 2 ? 3 : 2) void attn_flash_kernel(AttnArgs a) {
  using Frag = typename DT<T>::frag;
  constexpr int QB = 4 * QW * 16;     // query rows per workgroup
  __shared__ __attribute__((aligned(16))) char lds[NS][2][64 * 128];   // [stage][K|V][64 keys x 128 B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int S = a.nkeys;
  // XCD grouping (a.xcd_nqb > 0, 1-D grid): workgroup w runs on XCD w % 8 (round-robin dispatch), so
  // (set, head) = (w / 8 / nqb)·8 + w % 8 puts every query block of one (set, head) on one XCD and its
  // K/V is fetched into one L2 instead of eight (bijective for B·H % 8 == 0)
  int bxx = blockIdx.x, bh = blockIdx.y;
  if (a.xcd_nqb > 0) {
    const int w = blockIdx.x, slot = w >> 3;
    bh = (slot / a.xcd_nqb) * 8 + (w & 7);
    bxx = slot % a.xcd_nqb;
  }
  const int b = bh / a.H, h = bh % a.H;
  // key split (a.nsplit > 1, few-query launches): workgroup (query block, split) takes a contiguous
  // range of 64-key tiles and publishes unnormalised partials; flash_merge_kernel combines them
  const int nsplit = a.nsplit > 1 ? a.nsplit : 1;
  const int split = bxx % nsplit;
  const int q0 = (bxx / nsplit) * QB + wave * QW * 16;
  const int nt_all = (S + 63) / 64, per_t = (nt_all + nsplit - 1) / nsplit;
  const int t_lo = min(split * per_t, nt_all), nt = min(nt_all, t_lo + per_t) - t_lo;
  const T* Q = reinterpret_cast<const T*>(a.q);
  const T* K = reinterpret_cast<const T*>(a.k) + (long)b * a.k_sb + (long)h * a.k_sh;
  const T* V = reinterpret_cast<const T*>(a.v) + (long)b * a.k_sb + (long)h * a.k_sh;

  // Q as the B operand of Sᵀ = K·Qᵀ: lane holds Q[q0 + qi*16 + (lane&15)][ks*32 + 8(lane>>4) .. +7]
  Frag qf[QW][2];
#pragma unroll
  for (int qi = 0; qi < QW; ++qi) {
    const int qr = min(q0 + qi * 16 + (lane & 15), a.Sq - 1);
    const T* qp = Q + ((long)b * a.q_Sb + qr) * a.ldq + h * 64 + 8 * (lane >> 4);
    qf[qi][0] = load_frag<T>(qp);
    qf[qi][1] = load_frag<T>(qp + 32);
  }
  // glds sources: each wave moves rows [wave*16, wave*16+16) of the K and V tiles (2 x 1 KiB each)
  const int lr0 = wave * 16 + (lane >> 3), lc = lane & 7;
  auto stage = [&](int st, int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = lr0 + i * 8;
      const int key = min((t_lo + kt) * 64 + r, S - 1);
      const int c = lc ^ ((r >> 1) & 7);
      glds16a(K + (long)key * a.k_sk + c * 8, &lds[st][0][(wave * 16 + i * 8) * 128]);
      glds16a(V + (long)key * a.k_sk + c * 8, &lds[st][1][(wave * 16 + i * 8) * 128]);
    }
  };

  f32x4 o[QW][4];
  float mrow[QW], lrow[QW];
#pragma unroll
  for (int qi = 0; qi < QW; ++qi) {
    mrow[qi] = -INFINITY; lrow[qi] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[qi][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float L2E = 1.4426950408889634f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // Q retired: only LDS-DMA is counted below
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nt) stage(p, p);
  int st = 0;
  // One K/V tile. TAIL: the tile reaches past the last key (only the very last tile can): its score
  // masking lives in that instantiation alone — the compares and selects of a run-time `if` were
  // hoisted by hipcc into every iteration (≈ 45 VALU / SALU instructions per query fragment per tile)
  auto tile = [&](int kt, auto tail_tag) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    // tile kt landed (4 LDS-DMA per wave per tile; the younger tiles stay in flight), then the
    // barrier publishes every wave's part and frees the stage read in iteration kt - 1
    const int ahead = min(nt - 1 - kt, NS - 2);
    if (NS >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (NS >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + NS - 1 < nt) stage((st + NS - 1) % NS, kt + NS - 1);
    const char* kt_l = lds[st][0];
    const char* vt_l = lds[st][1];
    st = st + 1 == NS ? 0 : st + 1;
    // K fragments (A operand of Sᵀ): rows = keys 16mf + (lane&15), k = dd
    Frag kf[4][2];
#pragma unroll
    for (int mf = 0; mf < 4; ++mf)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int r = mf * 16 + (lane & 15);
        kf[mf][ks] = *reinterpret_cast<const Frag*>(kt_l + swz(r, ks * 4 + (lane >> 4)));
      }
    const int kabs = (t_lo + kt) * 64;   // first key of this tile
    // scores and softmax of every query fragment first, then P·V with the Vᵀ fragments of one
    // 16-row dd block live at a time (read once, used by every query fragment): 8 VGPRs of Vᵀ instead
    // of 32 keeps the kernel at 3 waves per SIMD
    Frag pf[QW][2];
#pragma unroll
    for (int qi = 0; qi < QW; ++qi) {
      f32x4 s[4];
#pragma unroll
      for (int mf = 0; mf < 4; ++mf) {
        s[mf] = mma16(kf[mf][0], qf[qi][0], f32x4{0.f, 0.f, 0.f, 0.f});
        s[mf] = mma16(kf[mf][1], qf[qi][1], s[mf]);
      }
      if constexpr (TAIL) {
#pragma unroll
        for (int mf = 0; mf < 4; ++mf)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (kabs + mf * 16 + 4 * (lane >> 4) + e >= S) s[mf][e] = -INFINITY;
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int e = 0; e < 4; ++e) tmax = fmaxf(tmax, s[mf][e]);
      tmax = xor16_max(tmax);
      tmax = xor32_max(tmax);
      float ls = 0.f;
      const float mnew = fmaxf(mrow[qi], tmax);
      const float alpha = __builtin_amdgcn_exp2f((mrow[qi] - mnew) * L2E);
      mrow[qi] = mnew;
      const float mb = mnew * L2E;
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int e = 0; e < 4; ++e) { s[mf][e] = __builtin_amdgcn_exp2f(fmaf(s[mf][e], L2E, -mb)); ls += s[mf][e]; }
      lrow[qi] = lrow[qi] * alpha + ls;
      if (__any(alpha != 1.f)) {   // the accumulator rescale only when some row's max moved (exact)
#pragma unroll
        for (int j = 0; j < 4; ++j) o[qi][j] *= alpha;
      }
      pf[qi][0] = pack_p<T>(s[0], s[1]);
      pf[qi][1] = pack_p<T>(s[2], s[3]);
    }
    // Vᵀ fragments (A operand of Oᵀ): rows = dd 16mf + (lane&15), k = keys (permuted)
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      const Frag v0 = tr_frag<T>(vt_l, 0, mf * 2, lane), v1 = tr_frag<T>(vt_l, 32, mf * 2, lane);
#pragma unroll
      for (int qi = 0; qi < QW; ++qi) {
        o[qi][mf] = mma16(v0, pf[qi][0], o[qi][mf]);
        o[qi][mf] = mma16(v1, pf[qi][1], o[qi][mf]);
      }
    }
  };
  // every tile but a partial last one without masking code, then that one (if any)
  const int nt_full = nt > 0 && (t_lo + nt) * 64 > S ? nt - 1 : nt;   // (an empty key range: no tile)
  for (int kt = 0; kt < nt_full; ++kt) tile(kt, std::false_type{});
  if (nt_full < nt) tile(nt_full, std::true_type{});
  // epilogue: lane holds Oᵀ[dd = 16mf + 4(lane>>4) + e][q = lane&15]
#pragma unroll
  for (int qi = 0; qi < QW; ++qi) {
    float l = lrow[qi];
    l = xor16_add(l);
    l = xor32_add(l);
    const float inv = 1.f / l;
    const int qr = q0 + qi * 16 + (lane & 15);
    if (qr >= a.Sq) continue;
    if (nsplit > 1) {   // partial (max, Σp, Σp·v) of this key range: [b·H + h][q][split][66] f32
      float* pp = a.part + (((long)bh * a.Sq + qr) * nsplit + split) * 66;
      if (lane < 16) { pp[0] = mrow[qi]; pp[1] = l; }
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
        *reinterpret_cast<f32x4*>(pp + 2 + mf * 16 + 4 * (lane >> 4)) = o[qi][mf];
      continue;
    }
    T* op = reinterpret_cast<T*>(a.o) + ((long)b * a.o_Sb + qr) * a.ldo + h * 64 + 4 * (lane >> 4);
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      typedef short s4 __attribute__((ext_vector_type(4)));
      s4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const T tv = DT<T>::fromf(o[qi][mf][e] * inv);
        w[e] = __builtin_bit_cast(short, tv);
      }
      *reinterpret_cast<s4*>(op + mf * 16) = w;
    }
  }
}

// Combine the key-range partials of one (set, head, query) in split order (deterministic): one wave,
// lane = output column.
template <typename T>
__global__ __launch_bounds__(64) void flash_merge_kernel(AttnArgs a) {
  const long slot = blockIdx.x;   // (b·H + h)·Sq + q
  const int lane = threadIdx.x, ns = a.nsplit;
  const float* pp = a.part + slot * ns * 66;
  float M = -INFINITY;
  for (int c = 0; c < ns; ++c) M = fmaxf(M, pp[c * 66]);
  float L = 0.f, O = 0.f;
  for (int c = 0; c < ns; ++c) {
    const float lc = pp[c * 66 + 1];
    const float w = lc > 0.f ? __expf(pp[c * 66] - M) : 0.f;   // empty ranges publish l = 0
    L += lc * w;
    O += pp[c * 66 + 2 + lane] * w;
  }
  const int q = (int)(slot % a.Sq), bh = (int)(slot / a.Sq), b = bh / a.H, h = bh % a.H;
  reinterpret_cast<T*>(a.o)[((long)b * a.o_Sb + q) * a.ldo + h * 64 + lane] = DT<T>::fromf(O / L);
}

// attn_beam_kernel — beam-search cross-attention: the Sq <= 16 beam rows of one clip against its
// precomputed K/V, one workgroup per (clip, head). The flash kernel above gives each of its 4 waves
// 16 query rows of the block, so with 5 beams 3 of its 4 waves compute on padding; here the KEYS are
// split instead: wave w streams its own contiguous 1/NWV of the clip's keys through a private LDS-DMA
// ring (NSW stages of one 64-key K and V tile; only the issuing wave reads them, so the loop needs no
// workgroup barrier — its own counted vmcnt orders the reads), with the 16 query slots of the clip
// (the same swapped products and lane-local online softmax as the flash kernel). The waves' (max,
// Σp, Σp·v) are merged in wave order through LDS at the end (deterministic); no key-range partials
// leave the workgroup. [tf] modeling_whisper.py:284-356 (cross-attention), generation/utils.py:3208
// (beams share the clip's encoder states).
template <typename T, int NWV, int NSW>
__global__ __launch_bounds__(NWV * 64) void attn_beam_kernel(AttnArgs a) {
  using Frag = typename DT<T>::frag;
  extern __shared__ __attribute__((aligned(16))) char lds_dyn[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  char* ring = lds_dyn + wave * NSW * 2 * 64 * 128;              // this wave's stages [NSW][K|V][64 x 128 B]
  const int S = a.nkeys;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int nt_all = (S + 63) / 64, per_w = (nt_all + NWV - 1) / NWV;
  const int t_lo = min(wave * per_w, nt_all), nt = min(nt_all, t_lo + per_w) - t_lo;
  const T* Q = reinterpret_cast<const T*>(a.q);
  const T* K = reinterpret_cast<const T*>(a.k) + (long)b * a.k_sb + (long)h * a.k_sh;
  const T* V = reinterpret_cast<const T*>(a.v) + (long)b * a.k_sb + (long)h * a.k_sh;
  Frag qf[2];
  {
    const int qr = min(lane & 15, a.Sq - 1);
    const T* qp = Q + ((long)b * a.q_Sb + qr) * a.ldq + h * 64 + 8 * (lane >> 4);
    qf[0] = load_frag<T>(qp);
    qf[1] = load_frag<T>(qp + 32);
  }
  // one tile = 64 rows of K and of V, 8 x 1 KiB wave-instructions each (row r = 8i + (lane >> 3))
  auto stage = [&](int st, int kt) {
    char* base = ring + st * 2 * 64 * 128;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = i * 8 + (lane >> 3);
      const int key = min((t_lo + kt) * 64 + r, S - 1);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      glds16a(K + (long)key * a.k_sk + c * 8, base + i * 1024);
      glds16a(V + (long)key * a.k_sk + c * 8, base + 64 * 128 + i * 1024);
    }
  };
  f32x4 o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow = -INFINITY, lrow = 0.f;
  const float L2E = 1.4426950408889634f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // Q retired: only LDS-DMA is counted below
#pragma unroll
  for (int p = 0; p < NSW - 1; ++p)
    if (p < nt) stage(p, p);
  int st = 0;
  for (int kt = 0; kt < nt; ++kt) {
    const int ahead = min(nt - 1 - kt, NSW - 2);       // younger tiles of this wave still in flight
    if (NSW >= 5 && ahead >= 3) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    else if (NSW >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if (NSW >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the stage read in iteration kt - 1 is free: its fragments were consumed by that iteration's MFMAs
    if (kt + NSW - 1 < nt) stage((st + NSW - 1) % NSW, kt + NSW - 1);
    const char* kt_l = ring + st * 2 * 64 * 128;
    const char* vt_l = kt_l + 64 * 128;
    st = st + 1 == NSW ? 0 : st + 1;
    Frag kf[4][2];
#pragma unroll
    for (int mf = 0; mf < 4; ++mf)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) kf[mf][ks] = *reinterpret_cast<const Frag*>(kt_l + swz(mf * 16 + (lane & 15), ks * 4 + (lane >> 4)));
    const int kabs = (t_lo + kt) * 64;
    f32x4 sc[4];
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      sc[mf] = mma16(kf[mf][0], qf[0], f32x4{0.f, 0.f, 0.f, 0.f});
      sc[mf] = mma16(kf[mf][1], qf[1], sc[mf]);
    }
    if (kabs + 64 > S) {
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (kabs + mf * 16 + 4 * (lane >> 4) + e >= S) sc[mf][e] = -INFINITY;
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int mf = 0; mf < 4; ++mf)
#pragma unroll
      for (int e = 0; e < 4; ++e) tmax = fmaxf(tmax, sc[mf][e]);
    tmax = xor16_max(tmax);
    tmax = xor32_max(tmax);
    const float mnew = fmaxf(mrow, tmax);
    const float alpha = __builtin_amdgcn_exp2f((mrow - mnew) * L2E);
    mrow = mnew;
    const float mb = mnew * L2E;
    float ls = 0.f;
#pragma unroll
    for (int mf = 0; mf < 4; ++mf)
#pragma unroll
      for (int e = 0; e < 4; ++e) { sc[mf][e] = __builtin_amdgcn_exp2f(fmaf(sc[mf][e], L2E, -mb)); ls += sc[mf][e]; }
    lrow = lrow * alpha + ls;
    if (__any(alpha != 1.f)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] *= alpha;
    }
    const Frag p0 = pack_p<T>(sc[0], sc[1]), p1 = pack_p<T>(sc[2], sc[3]);
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      o[mf] = mma16(tr_frag<T>(vt_l, 0, mf * 2, lane), p0, o[mf]);
      o[mf] = mma16(tr_frag<T>(vt_l, 32, mf * 2, lane), p1, o[mf]);
    }
  }
  // ---- merge the waves' partials (wave order): lane holds Oᵀ[dd = 16mf + 4(lane>>4) + e][q = lane&15]
  lrow = xor16_add(lrow);
  lrow = xor32_add(lrow);
  __syncthreads();                                     // every wave is done with its ring: reuse it
  f32x4* ob = reinterpret_cast<f32x4*>(lds_dyn);       // [NWV][4][64]
  float2* ml = reinterpret_cast<float2*>(lds_dyn + NWV * 4 * 64 * 16);   // [NWV][16]
#pragma unroll
  for (int mf = 0; mf < 4; ++mf) ob[(wave * 4 + mf) * 64 + lane] = o[mf];
  if (lane < 16) ml[wave * 16 + lane] = float2{nt > 0 ? mrow : -INFINITY, nt > 0 ? lrow : 0.f};
  __syncthreads();
  if (wave != 0) return;
  const int q = lane & 15;
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < NWV; ++w) { const float2 t = ml[w * 16 + q]; if (t.y > 0.f) M = fmaxf(M, t.x); }
  float L = 0.f, wgt[NWV];
#pragma unroll
  for (int w = 0; w < NWV; ++w) {
    const float2 t = ml[w * 16 + q];
    wgt[w] = t.y > 0.f ? __builtin_amdgcn_exp2f((t.x - M) * L2E) : 0.f;
    L += wgt[w] * t.y;
  }
  const float inv = 1.f / L;
  if (q >= a.Sq) return;
  T* op = reinterpret_cast<T*>(a.o) + ((long)b * a.o_Sb + q) * a.ldo + h * 64 + 4 * (lane >> 4);
#pragma unroll
  for (int mf = 0; mf < 4; ++mf) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < NWV; ++w) acc += wgt[w] * ob[(w * 4 + mf) * 64 + lane];
    typedef short s4 __attribute__((ext_vector_type(4)));
    s4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = __builtin_bit_cast(short, DT<T>::fromf(acc[e] * inv));
    *reinterpret_cast<s4*>(op + mf * 16) = v;
  }
}

template <typename T, int NWV, int NSW>
static void launch_beam(const AttnArgs& a, hipStream_t s) {
  constexpr int lds = NWV * NSW * 2 * 64 * 128;
  static_assert(lds >= NWV * 4 * 64 * 16 + NWV * 16 * 8 && lds <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)attn_beam_kernel<T, NWV, NSW>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  WCB_LAUNCH((attn_beam_kernel<T, NWV, NSW>), dim3(a.B * a.H), dim3(NWV * 64), lds, s, a);
}

template <typename T>
static void launch_flash(const AttnArgs& a, hipStream_t s) {
  if (a.Sq <= 16 && a.variant >= 7 && a.variant <= 9) {   // beam rows of a clip, keys split over the waves
    // 7: 4 waves x 2 stages, 8: 2 waves x 4 stages, 9: 2 waves x 5 stages (128 / 128 / 160 KiB of LDS)
    if (a.variant == 7) launch_beam<T, 4, 2>(a, s);
    else if (a.variant == 8) launch_beam<T, 2, 4>(a, s);
    else launch_beam<T, 2, 5>(a, s);
  } else if (a.Sq <= 16) {   // a few query rows per K/V set (the beams of one clip): 16 queries per wave
    const int ns = (a.part && a.nsplit > 1) ? a.nsplit : 1;
    AttnArgs b = a;
    b.nsplit = ns;
    const dim3 grid((a.Sq + 63) / 64 * ns, a.B * a.H);
    WCB_LAUNCH((attn_flash_kernel<T, 1, 2>), grid, dim3(256), 0, s, b);
    if (ns > 1) WCB_LAUNCH(flash_merge_kernel<T>, dim3(a.B * a.H * a.Sq), dim3(64), 0, s, b);
  } else {   // one key range (the key split is the few-query form only); XCD-grouped query blocks
    AttnArgs b = a;
    b.nsplit = 1;
    const int qb = a.variant == 4 ? 256 : 128, nqb = (a.Sq + qb - 1) / qb, BH = a.B * a.H;
    const bool xg = nqb > 1 && BH % 8 == 0;
    b.xcd_nqb = xg ? nqb : 0;
    const dim3 grid = xg ? dim3(nqb * BH) : dim3(nqb, BH);
    // encoder tilings (option enc_flash): 64 queries per wave (4, default) or 32 (2)
    if (a.variant == 4) WCB_LAUNCH((attn_flash_kernel<T, 4, 2>), grid, dim3(256), 0, s, b);
    else WCB_LAUNCH((attn_flash_kernel<T, 2, 2>), grid, dim3(256), 0, s, b);
  }
}

// Non-causal attention of Sq query rows per (set b, head) over nkeys keys of that set: the encoder
// self-attention (Sq = nkeys = 1500) and the beam-search cross-attention (the nb beam rows of a clip
// against its precomputed K/V: each (clip, head) K/V block is streamed once for all of its beams).
bool attention_flash(DType t, const AttnArgs& a, hipStream_t s) {
  switch (t) {
    case kBF16: launch_flash<bf16_t>(a, s); return true;
    case kF16: launch_flash<f16_t>(a, s); return true;
    default: return false;
  }
}

}  // namespace wcb
