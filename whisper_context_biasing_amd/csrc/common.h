// Shared device helpers for libwcb (gfx950 / CDNA4 only).
//
// Element types: bf16 (uint16 bits), f16 (_Float16), f32. Every kernel is templated on the
// activation/weight type T and computes in f32. MFMA fragments use ONE lane layout for all three
// types (lane l holds A[row l&15][k = 8*(l>>4) + j], j = 0..7, of a 16x16x32 step):
//   bf16 / f16 : one v_mfma_f32_16x16x32_{bf16,f16}
//   f32        : eight v_mfma_f32_16x16x4_f32 (exact f32 fma chains) — MFMA j consumes element j of
//                every lane, i.e. k = 8g + j over the four lane groups g; summing j = 0..7 covers
//                all 32 k, so A and B only have to share the permutation (they do).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"

typedef uint16_t bf16_t;
typedef _Float16 f16_t;
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

#define WCB_DEV __device__ __forceinline__

WCB_DEV float bf16_to_f(bf16_t v) { return __uint_as_float(uint32_t(v) << 16); }
// round-to-nearest-even; a plain __bf16 cast lowers to v_cvt_pk_bf16_f32 on gfx950 (NaN stays NaN)
WCB_DEV bf16_t f_to_bf16(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

template <typename T> struct DT;
template <> struct DT<bf16_t> {
  using frag = s16x8;
  static constexpr int kBytes = 2;
  WCB_DEV static float tof(bf16_t v) { return bf16_to_f(v); }
  WCB_DEV static bf16_t fromf(float f) { return f_to_bf16(f); }
};
template <> struct DT<f16_t> {
  using frag = h16x8;
  static constexpr int kBytes = 2;
  WCB_DEV static float tof(f16_t v) { return float(v); }
  WCB_DEV static f16_t fromf(float f) { return f16_t(f); }
};
template <> struct DT<float> {
  using frag = f32x8;
  static constexpr int kBytes = 4;
  WCB_DEV static float tof(float v) { return v; }
  WCB_DEV static float fromf(float f) { return f; }
};

// Cross-row lane exchanges without an LDS round trip: __shfl_xor(x, 16 | 32) lowers to
// ds_bpermute_b32 (an LDS-unit instruction and an lgkmcnt wait); gfx950's v_permlane16_swap /
// v_permlane32_swap swap rows in the VALU. (r[0], r[1]) at lane l = (x[l], x[l ^ 16]) in one order or
// the other, and f32 add / max are commutative, so these equal x + __shfl_xor(x, 16) (etc.) bit for bit.
WCB_DEV float xor16_add(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
WCB_DEV float xor32_add(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
WCB_DEV float xor16_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
WCB_DEV float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// In-launch hand-off between the workgroups of one group (MI355X_MICROARCH.md "Valid forms", row 1 of
// the measured sc1 table; cdna_hip_programming.md §6 G16): the producers store the handed-off bytes
// with sc1 (write-through) stores — st_sc1 — and call group_arrive_wait; it drains every wave's
// stores (vmcnt(0)), joins the workgroup, lets one lane add to the group's counter (agent scope) and
// poll it with sc1 loads until all n members of this generation arrived, and releases the other waves
// at a second workgroup barrier (no release / acquire fence: every handed-off byte is an sc1 store
// drained before the add and an sc1 load after the poll — the guide's measured row-1 form). Readers load the bytes
// with sc1 loads only (ld_sc1). Counters are 64-bit and monotonic (generation = the value an add
// returned / n; 2^64 arrivals do not wrap in any run). The spin is bounded (a co-residency failure cannot
// hang the GPU): running it out sets *err, which the host reports as an error at wcb_synchronize.
WCB_DEV void st_sc1(void* p, uint64_t v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
WCB_DEV uint64_t ld_sc1(const void* p) {
  return __hip_atomic_load(reinterpret_cast<uint64_t*>(const_cast<void*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
WCB_DEV void group_arrive_wait(unsigned long long* cnt, unsigned long long n, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long old = __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = (old / n + 1) * n;
    bool ok = false;
    for (int spin = 0; spin < (1 << 22); ++spin) {
      if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) { ok = true; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!ok) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
}

// A8 bias boost (oracle/bias_ref.py): x + lam·units as one f32 product and one f32 add, never a
// fused multiply-add, so every kernel rounds exactly like the oracle
WCB_DEV float bias_bonus(float x, float lam, int units) { return __fadd_rn(x, __fmul_rn(lam, (float)units)); }

WCB_DEV f32x4 mma16(const s16x8& a, const s16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
WCB_DEV f32x4 mma16(const h16x8& a, const h16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
WCB_DEV f32x4 mma16(const f32x8& a, const f32x8& b, f32x4 c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], c, 0, 0, 0);
  return c;
}

// Load one fragment (8 consecutive elements) from global or LDS memory.
template <typename T>
WCB_DEV typename DT<T>::frag load_frag(const T* p) {
  return *reinterpret_cast<const typename DT<T>::frag*>(p);
}

WCB_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

WCB_DEV float wave_sum(float v) {   // xor 32, 16, 8, 4, 2, 1 (the row swaps in the VALU)
  v = xor32_add(v);
  v = xor16_add(v);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
WCB_DEV float wave_max(float v) {
  v = xor32_max(v);
  v = xor16_max(v);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Store 8 consecutive f32 values as T.
template <typename T> WCB_DEV void store8(T* dst, const float* v);
template <> WCB_DEV void store8<bf16_t>(bf16_t* dst, const float* v) {
  s16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (short)f_to_bf16(v[j]);
  *reinterpret_cast<s16x8*>(dst) = o;
}
template <> WCB_DEV void store8<f16_t>(f16_t* dst, const float* v) {
  h16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f16_t(v[j]);
  *reinterpret_cast<h16x8*>(dst) = o;
}
template <> WCB_DEV void store8<float>(float* dst, const float* v) {
  *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
template <typename T> WCB_DEV void load8f(const T* src, float* v) {
  auto f = load_frag<T>(src);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if constexpr (sizeof(T) == 2) {
      if constexpr (DT<T>::kBytes == 2 && __is_same(T, bf16_t)) v[j] = bf16_to_f((bf16_t)f[j]);
      else v[j] = float(f[j]);
    } else {
      v[j] = f[j];
    }
  }
}

// Per-launch device time stamps (profiling of kernels replayed inside a hipGraph, where HIP events
// cannot bracket one node). A launch owns kStampSub sub-slots; workgroup w folds its
// (~t_start, t_end) into sub-slot w % kStampSub with atomicMax (sub-slots keep same-address atomic
// contention low), stamp_reduce takes max(t_end) − min(t_start) over them. s_memrealtime ticks
// (100 MHz). Launch slot = pos·stride + idx; slots start zeroed.
WCB_DEV unsigned long long stamp_now() { return __builtin_amdgcn_s_memrealtime(); }
WCB_DEV void stamp_commit(const wcb::Stamp& s, unsigned long long t0) {
  if (!s.base) return;
  const unsigned long long t1 = stamp_now();
  const int wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  unsigned long long* slot =
      s.base + 2 * (((long)(*s.pos) * s.stride + s.idx) * wcb::kStampSub + (wg % wcb::kStampSub));
  atomicMax(slot, ~t0);
  atomicMax(slot + 1, t1);
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5 "XCD swizzle").
WCB_DEV int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// ---- 16-bit K/V tiles in LDS: 128-byte rows (64 columns), 16-byte chunk c of row r stored at chunk
// slot c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 row reads and ds_read_b64_tr_b16 reads); the
// swizzle is applied to the global SOURCE address of the global_load_lds that fills the tile.
namespace wcb {
WCB_DEV void glds16a(const void* gptr, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(gptr, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
WCB_DEV int swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <typename T>
WCB_DEV typename DT<T>::frag tr_frag(const char* vt, int r0, int col_chunk2, int lane) {
  // 16-bit transposed read: group h = lane>>4, lane 4q+p of the group supplies row r0+4h+q,
  // columns 4p..4p+3 of the 16-column block (chunk pair col_chunk2, col_chunk2+1).
  const int h = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r1 = r0 + 4 * h + q, r2 = r1 + 16;
  const int c = col_chunk2 + (p >> 1), byte = (p & 1) * 8;
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(vt + swz(r1, c) + byte));
  const s4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(vt + swz(r2, c) + byte));
  typename DT<T>::frag f;
  if constexpr (__is_same(T, bf16_t)) {
    f = s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  } else {
    const s16x8 t8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    f = __builtin_bit_cast(h16x8, t8);
  }
  return f;
}

template <typename T>
WCB_DEV typename DT<T>::frag pack_p(const f32x4& lo, const f32x4& hi) {
  typename DT<T>::frag f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if constexpr (__is_same(T, bf16_t)) { f[e] = (short)f_to_bf16(lo[e]); f[e + 4] = (short)f_to_bf16(hi[e]); }
    else { f[e] = f16_t(lo[e]); f[e + 4] = f16_t(hi[e]); }
  }
  return f;
}

}  // namespace wcb
