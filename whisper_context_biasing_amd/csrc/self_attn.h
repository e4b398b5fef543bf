// Decoder self-attention of one new token for one (row, head) pair on one wave
// ([tf] modeling_whisper.py:284-356, the decoder's self_attn with a KV cache): the body of the
// stand-alone kernel (k_attn.hip attn_self_lean_kernel).
// 8 lanes per key (16 B of K and of V each), 8 keys per load, the first 64 keys requested before the
// key count is known (rows past it clamped to the cache capacity `cap` and masked); longer contexts
// continue in 64-key chunks with an online softmax.
#pragma once
#include "common.h"

namespace wcb {

// q, o: the pair's 64 values; k0 / v0: its key 0 (keys 64 elements apart); nkeys(): the key count,
// called after the first K / V loads are issued
template <typename T, typename NK>
WCB_DEV void self_attn_wave(const T* q, const T* k0, const T* v0, int cap, NK&& nkeys, T* o) {
  const int lane = threadIdx.x & 63, seg = lane & 7, kg = lane >> 3;
  const T* kb = k0 + seg * 8;
  const T* vb = v0 + seg * 8;
  // K / V stay in their 16-bit bits until use (converted per product: exact), q in f32
  using Frag = typename DT<T>::frag;
  auto cv = [](const Frag& f, int e) -> float {
    if constexpr (__is_same(T, bf16_t)) return bf16_to_f((bf16_t)f[e]);
    else return float(f[e]);
  };
  float qv[8];
  Frag kv[8], vv[8];
  load8f<T>(q + seg * 8, qv);
#pragma unroll
  for (int u = 0; u < 8; ++u) kv[u] = load_frag<T>(kb + (long)min(u * 8 + kg, cap) * 64);
#pragma unroll
  for (int u = 0; u < 8; ++u) vv[u] = load_frag<T>(vb + (long)min(u * 8 + kg, cap) * 64);
  const int nk = nkeys();
  float m = -INFINITY, l = 0.f;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nk; j0 += 64) {
    if (j0) {
#pragma unroll
      for (int u = 0; u < 8; ++u) kv[u] = load_frag<T>(kb + (long)min(min(j0 + u * 8 + kg, nk - 1), cap) * 64);
#pragma unroll
      for (int u = 0; u < 8; ++u) vv[u] = load_frag<T>(vb + (long)min(min(j0 + u * 8 + kg, nk - 1), cap) * 64);
    }
    float sc[8];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(qv[e], cv(kv[u], e), d);
#pragma unroll
      for (int x = 1; x < 8; x <<= 1) d += __shfl_xor(d, x, 64);
      sc[u] = (j0 + u * 8 + kg < nk) ? d : -INFINITY;
      mx = fmaxf(mx, sc[u]);
    }
    const float mn = fmaxf(m, wave_max(mx));
    const float r = __expf(m - mn);
    l *= r;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= r;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool live = j0 + u * 8 + kg < nk;
      const float p = live ? __expf(sc[u] - mn) : 0.f;
      if (seg == 0) l += p;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = live ? fmaf(p, cv(vv[u], e), acc[e]) : acc[e];
    }
    m = mn;
  }
  l = wave_sum(l);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    acc[e] += __shfl_xor(acc[e], 8, 64);
    acc[e] = xor16_add(acc[e]);
    acc[e] = xor32_add(acc[e]);
  }
  if (kg == 0) {
    float r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = acc[e] / l;
    store8<T>(o + seg * 8, r);
  }
}

}  // namespace wcb
