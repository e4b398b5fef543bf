// Weight staging and repacking on the device (wcb_load_weights / wcb_finalize_weights).
//
// Every parameter is staged as a dense f32 device tensor: borrowed device views (any of f32 / bf16 /
// f16, strided, up to 4-D) are gathered by view_to_f32_kernel without leaving the GPU; host arrays
// (wcb_set_weight) are copied up once. wcb_finalize_weights then builds the owned layouts (fused
// QKV, conv im2col order, the W_k,hᵀ panels, the cross-K/V stack, ...) with repack_kernel: a 3-D
// strided gather with a scale, rounded once to the model dtype — the same round-to-nearest-even the
// host packing used, so weights are bit-identical whichever way they arrived.

#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace wcb {

template <typename S>
__global__ __launch_bounds__(256) void view_to_f32_kernel(const S* __restrict__ src, WeightView v, float* __restrict__ dst) {
  const long n = v.shape[0] * v.shape[1] * v.shape[2] * v.shape[3];
  for (long o = blockIdx.x * 256L + threadIdx.x; o < n; o += (long)gridDim.x * 256) {
    long r = o;
    const long i3 = r % v.shape[3]; r /= v.shape[3];
    const long i2 = r % v.shape[2]; r /= v.shape[2];
    const long i1 = r % v.shape[1];
    const long i0 = r / v.shape[1];
    dst[o] = DT<S>::tof(src[i0 * v.stride[0] + i1 * v.stride[1] + i2 * v.stride[2] + i3 * v.stride[3]]);
  }
}

void view_to_f32(DType t, const void* src, const WeightView& v, float* dst, hipStream_t s) {
  const long n = v.shape[0] * v.shape[1] * v.shape[2] * v.shape[3];
  const int grid = (int)std::min<long>((n + 255) / 256, 4096);
  switch (t) {
    case kBF16: WCB_LAUNCH(view_to_f32_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)src, v, dst); break;
    case kF16: WCB_LAUNCH(view_to_f32_kernel<f16_t>, dim3(grid), dim3(256), 0, s, (const f16_t*)src, v, dst); break;
    case kF32: WCB_LAUNCH(view_to_f32_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)src, v, dst); break;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void repack_kernel(RepackArgs a) {
  const long n = (long)a.n[0] * a.n[1] * a.n[2];
  for (long o = blockIdx.x * 256L + threadIdx.x; o < n; o += (long)gridDim.x * 256) {
    const long i2 = o % a.n[2], i1 = (o / a.n[2]) % a.n[1], i0 = o / ((long)a.n[1] * a.n[2]);
    const float v = a.src[i0 * a.s[0] + i1 * a.s[1] + i2 * a.s[2]] * a.scale;
    reinterpret_cast<T*>(a.dst)[i0 * a.t[0] + i1 * a.t[1] + i2 * a.t[2]] = DT<T>::fromf(v);
  }
}

void repack(DType t, const RepackArgs& a, hipStream_t s) {
  const long n = (long)a.n[0] * a.n[1] * a.n[2];
  const int grid = (int)std::min<long>((n + 255) / 256, 4096);
  switch (t) {
    case kBF16: WCB_LAUNCH(repack_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, a); break;
    case kF16: WCB_LAUNCH(repack_kernel<f16_t>, dim3(grid), dim3(256), 0, s, a); break;
    case kF32: WCB_LAUNCH(repack_kernel<float>, dim3(grid), dim3(256), 0, s, a); break;
  }
}

// *count += #{i : a[i] != (b ? b[i] : 0)} (tied-weight and zero-bias checks)
__global__ __launch_bounds__(256) void count_diff_kernel(const float* a, const float* b, long n, int* count) {
  int c = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) c += a[i] != (b ? b[i] : 0.f);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, c);
}

void count_diff(const float* a, const float* b, long n, int* count, hipStream_t s) {
  const int grid = (int)std::min<long>((n + 255) / 256, 1024);
  WCB_LAUNCH(count_diff_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, a, b, n, count);
}

// LayerNorm folded into the projection that consumes it (decode rows > 64, gemm_impl.h LNF):
// u[n] = Σ_k γ_k W[n][k] and c[n] = Σ_k β_k W[n][k] + bias[n] (f32, fixed-order wave sums), so that
// LN(x)·Wᵀ + bias = r·(Σ_k x_k γ_k W[n][k] − μ·u[n]) + c[n] for a row with mean μ, 1/σ = r.
template <typename T>
__global__ __launch_bounds__(64) void ln_fold_kernel(const T* W, int K, const float* gam, const float* bet,
                                                     const float* bias, float* u, float* c) {
  const int n = blockIdx.x, lane = threadIdx.x;
  const T* w = W + (long)n * K;
  float su = 0.f, sc = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float x = DT<T>::tof(w[k]);
    su = gam ? fmaf(gam[k], x, su) : su + x;
    sc = bet ? fmaf(bet[k], x, sc) : sc;
  }
  su = wave_sum(su);
  sc = wave_sum(sc);
  if (lane == 0) {
    u[n] = su;
    if (c) c[n] = sc + (bias ? bias[n] : 0.f);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void scale_cols_kernel(const T* W, long n_el, int K, const float* gam, T* Wg) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n_el; i += (long)gridDim.x * 256)
    Wg[i] = DT<T>::fromf(gam[i % K] * DT<T>::tof(W[i]));
}

void scale_cols(DType t, const void* W, int N, int K, const float* gam, void* Wg, hipStream_t s) {
  const long n = (long)N * K;
  const dim3 grid((unsigned)std::min<long>((n + 255) / 256, 8192));
  switch (t) {
    case kBF16: WCB_LAUNCH(scale_cols_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)W, n, K, gam, (bf16_t*)Wg); break;
    case kF16: WCB_LAUNCH(scale_cols_kernel<f16_t>, grid, dim3(256), 0, s, (const f16_t*)W, n, K, gam, (f16_t*)Wg); break;
    case kF32: WCB_LAUNCH(scale_cols_kernel<float>, grid, dim3(256), 0, s, (const float*)W, n, K, gam, (float*)Wg); break;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void frag_major_kernel(const T* W, long n_el, int K, int nw, int kpw, T* dst) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n_el; i += (long)gridDim.x * 256) {
    const int e = (int)(i & 7), lane = (int)((i >> 3) & 63);
    long r = i >> 9;                       // (ct, wave, ks)
    const int ks = (int)(r % kpw); r /= kpw;
    const int wave = (int)(r % nw);
    const long ct = r / nw;
    const long n = ct * 16 + (lane & 15);
    const int k = wave * kpw * 32 + ks * 32 + 8 * (lane >> 4) + e;
    dst[i] = W[n * K + k];
  }
}

void frag_major(DType t, const void* W, int N, int K, int nw, int kpw, void* dst, hipStream_t s) {
  const long n = (long)N * K;
  const dim3 grid((unsigned)std::min<long>((n + 255) / 256, 8192));
  switch (t) {
    case kBF16: WCB_LAUNCH(frag_major_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)W, n, K, nw, kpw, (bf16_t*)dst); break;
    case kF16: WCB_LAUNCH(frag_major_kernel<f16_t>, grid, dim3(256), 0, s, (const f16_t*)W, n, K, nw, kpw, (f16_t*)dst); break;
    case kF32: break;
  }
}

void ln_fold(DType t, const void* W, int N, int K, const float* gam, const float* bet, const float* bias, float* u,
             float* c, hipStream_t s) {
  switch (t) {
    case kBF16: WCB_LAUNCH(ln_fold_kernel<bf16_t>, dim3(N), dim3(64), 0, s, (const bf16_t*)W, K, gam, bet, bias, u, c); break;
    case kF16: WCB_LAUNCH(ln_fold_kernel<f16_t>, dim3(N), dim3(64), 0, s, (const f16_t*)W, K, gam, bet, bias, u, c); break;
    case kF32: WCB_LAUNCH(ln_fold_kernel<float>, dim3(N), dim3(64), 0, s, (const float*)W, K, gam, bet, bias, u, c); break;
  }
}

}  // namespace wcb
