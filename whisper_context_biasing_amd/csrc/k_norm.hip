// LayerNorm, token+position embedding and small fills.
//
// LayerNorm restates nn.LayerNorm(d, eps=1e-5) as used by every Whisper block
// ([tf] modeling_whisper.py:379-413, 448-505, final norms :642 / :790). One wave per row: the f32
// residual-stream row is read once into registers (vectorised by VEC), mean and variance are
// wave-shuffle reductions, the normalised row is written in the activation type T.
// embed restates WhisperDecoder's `embed_tokens(ids) + embed_positions(position_ids)`
// ([tf] modeling_whisper.py:737-762) for one decode step with the position read on device.
#include "common.h"
#include "kernels.h"

namespace wcb {

template <typename T, int VEC, int CH>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ b, T* __restrict__ y, int M, int d) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + (long)row * d;
  float v[CH][VEC];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int base = (c * 64 + lane) * VEC;
    if (base < d) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[c][e] = xr[base + e];
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[c][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) s += v[c][e];
  }
  const float mean = wave_sum(s) / d;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int base = (c * 64 + lane) * VEC;
    if (base < d)
#pragma unroll
      for (int e = 0; e < VEC; ++e) { const float t = v[c][e] - mean; q += t * t; }
  }
  const float rstd = rsqrtf(wave_sum(q) / d + 1e-5f);
  T* yr = y + (long)row * d;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int base = (c * 64 + lane) * VEC;
    if (base < d)
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        yr[base + e] = DT<T>::fromf((v[c][e] - mean) * rstd * w[base + e] + b[base + e]);
  }
}

template <typename T>
static void layernorm_t(const float* x, const float* w, const float* b, void* y, int M, int d, hipStream_t s) {
  const dim3 grid((M + 3) / 4), blk(256);
  T* yy = reinterpret_cast<T*>(y);
  // every Whisper width is a multiple of 64: d/64 elements per lane, grouped VEC at a time
  if (d % 256 == 0 && d <= 2048) {
    if (d <= 1024) WCB_LAUNCH((layernorm_kernel<T, 4, 4>), grid, blk, 0, s, x, w, b, yy, M, d);
    else WCB_LAUNCH((layernorm_kernel<T, 4, 8>), grid, blk, 0, s, x, w, b, yy, M, d);
  } else if (d % 128 == 0 && d <= 1024) {
    WCB_LAUNCH((layernorm_kernel<T, 2, 8>), grid, blk, 0, s, x, w, b, yy, M, d);
  } else {
    WCB_LAUNCH((layernorm_kernel<T, 1, 32>), grid, blk, 0, s, x, w, b, yy, M, d);
  }
}

void layernorm(DType t, const float* x, const float* w, const float* b, void* y, int M, int d, hipStream_t s) {
  switch (t) {
    case kBF16: layernorm_t<bf16_t>(x, w, b, y, M, d, s); break;
    case kF16: layernorm_t<f16_t>(x, w, b, y, M, d, s); break;
    case kF32: layernorm_t<float>(x, w, b, y, M, d, s); break;
  }
}

// also publishes the per-16-column partial sums (Σx, Σx²) of the new row for the fused LayerNorm
// of the first decoder GEMM (deterministic fixed-order sums, see k_gemm.hip st_in)
template <typename T>
__global__ __launch_bounds__(256) void embed_kernel(const T* __restrict__ emb, const T* __restrict__ pemb, const int* __restrict__ ids,
                                                    const int* __restrict__ pos, float* __restrict__ x, float* __restrict__ st,
                                                    int M, int d, T* __restrict__ x16, int V, int rps, int st_w,
                                                    T* __restrict__ x16fm, int fm_nw, int fm_kpw) {
  const int row = blockIdx.x;
  const int p = *pos + row % rps;
  const int raw = ids[row];
  const long id = raw >= 0 && raw < V ? raw : 0;   // never index past the table (ids are produced on device)
  for (int c0 = 0; c0 < d; c0 += 256) {
    const int c = c0 + threadIdx.x;
    float v = 0.f;
    if (c < d) {
      v = DT<T>::tof(emb[id * d + c]) + DT<T>::tof(pemb[(long)p * d + c]);
      x[(long)row * d + c] = v;
      if (x16) x16[(long)row * d + c] = DT<T>::fromf(v);
      if (x16fm) {   // fragment-major copy for the lean LN-fused projections (gemm_impl.h dec_lean_kernel AFM)
        const int kw = fm_kpw * 32, w2 = c / kw, ks2 = (c % kw) >> 5, lg = (c & 31) >> 3;
        x16fm[((((long)(row >> 4) * fm_nw + w2) * fm_kpw + ks2) * 64 + lg * 16 + (row & 15)) * 8 + (c & 7)] = DT<T>::fromf(v);
      }
    }
    if (st) {
      // one partial per group of st_w lanes (= columns), fixed butterfly order
      float s1 = v, s2 = v * v;
      if (st_w == 32) {
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
      } else {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
      }
      if (c < d && (c & (st_w - 1)) == 0) {
        st[((long)row * (d / st_w) + c / st_w) * 2] = s1;
        st[((long)row * (d / st_w) + c / st_w) * 2 + 1] = s2;
      }
    }
  }
}

void embed(DType t, const void* emb, const void* pemb, const int* ids, const int* pos, float* x, float* st, int M,
           int d, hipStream_t s, void* x16, int V, int rps, int st_w, void* x16fm) {
  rps = rps > 1 ? rps : 1;
  int nw = 0, kpw = 0;
  if (x16fm && !lean_cfg(d, nw, kpw)) x16fm = nullptr;
  switch (t) {
    case kBF16: WCB_LAUNCH(embed_kernel<bf16_t>, dim3(M), dim3(256), 0, s, (const bf16_t*)emb,
                                   (const bf16_t*)pemb, ids, pos, x, st, M, d, (bf16_t*)x16, V, rps, st_w, (bf16_t*)x16fm, nw, kpw); break;
    case kF16: WCB_LAUNCH(embed_kernel<f16_t>, dim3(M), dim3(256), 0, s, (const f16_t*)emb,
                                  (const f16_t*)pemb, ids, pos, x, st, M, d, (f16_t*)x16, V, rps, st_w, (f16_t*)x16fm, nw, kpw); break;
    case kF32: WCB_LAUNCH(embed_kernel<float>, dim3(M), dim3(256), 0, s, (const float*)emb,
                                  (const float*)pemb, ids, pos, x, st, M, d, (float*)x16, V, rps, st_w, (float*)nullptr, 0, 0); break;
  }
}

__global__ void fill_i32_kernel(int* p, int v, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v;
}
void fill_i32(int* p, int v, long n, hipStream_t s) {
  const int grid = (int)min((n + 255) / 256, 1024L);
  WCB_LAUNCH(fill_i32_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, p, v, n);
}

__global__ __launch_bounds__(64) void stamp_reduce_kernel(unsigned long long* slots, long n, unsigned long long* acc) {
  const long i = blockIdx.x * 64L + threadIdx.x;
  unsigned long long ticks = 0, used = 0;
  if (i < n) {
    unsigned long long* s = slots + 2 * i * kStampSub;
    unsigned long long nt0 = 0, t1 = 0;
    for (int k = 0; k < kStampSub; ++k) {
      nt0 = max(nt0, s[2 * k]);
      t1 = max(t1, s[2 * k + 1]);
      s[2 * k] = 0; s[2 * k + 1] = 0;
    }
    if (t1 != 0) { ticks = t1 - ~nt0; used = 1; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    ticks += __shfl_xor(ticks, o, 64);
    used += __shfl_xor(used, o, 64);
  }
  if (threadIdx.x == 0 && used) { atomicAdd(acc, ticks); atomicAdd(acc + 1, used); }
}
void stamp_reduce(unsigned long long* slots, long n, unsigned long long* acc, hipStream_t s) {
  WCB_LAUNCH(stamp_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, slots, n, acc);
}

}  // namespace wcb
