// Log-mel front end, restating `_torch_extract_fbank_features`
// ([tf] feature_extraction_whisper.py:135-168; caller data_utils/data_loader.py:171-172):
//   zero-pad/trim to 480000 samples → STFT(n_fft 400, hop 160, periodic Hann, center=True, reflect)
//   → |X|² (last frame dropped) → slaney mel (sparse: ≤ ~25 bins per filter) → clamp(1e-10).log10
//   → per-clip max → max(x, max − 8) → (x + 4) / 4.
//
// logmel_power_mel_kernel: one workgroup = 64 frames of one clip. The 10,480-sample window span is
// staged once in LDS (reflect padding resolved at load), the windowed 400-point real DFT runs as
// an exact-f32 MFMA product (v_mfma_f32_16x16x4_f32; each wave: the 64 frames x a quarter of the
// columns) of the frame matrix with a [416 × 416] table
// whose columns interleave (cos, −sin) per bin, so |X|² of a bin is lane ⊕ 1 in the accumulator
// (one shuffle). Power goes to LDS, the sparse mel filters are applied from it, log10 is written
// and the clip maximum reduced with one atomicMax (order-preserving int encoding of the float).
#include "common.h"
#include "kernels.h"

namespace wcb {

constexpr int kNFFT = 400, kHop = 160, kFrames = 3000, kNSamp = 480000;
constexpr int kFPB = 64;                         // frames per workgroup
constexpr int kSpan = (kFPB - 1) * kHop + 416;   // samples staged (K padded to 416)
constexpr int kNCol = 416;                       // 201 bins × (re, im) = 402, padded to 26·16
constexpr int kBins = 201;

WCB_DEV unsigned ord_enc(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
WCB_DEV float ord_dec(unsigned u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }

// SPLIT: the DFT products as bf16 MFMAs of 3-part splits of both operands (x = xh + xm + xl, t = th + tm +
// tl, each part the RNE bf16 of the remainder): x·t = xh·th + xh·tm + xm·th + xh·tl + xl·th + xm·tm + O(2^-24)
// (the six 16x16x32 bf16 MFMAs of a 32-deep k-step cost ~1/5 of the eight 16x16x4 f32 ones); not
// bit-identical to the f32 form, ~f32 accurate.
template <bool SPLIT>
__global__ __launch_bounds__(256) void logmel_power_mel_kernel(const float* __restrict__ pcm, long pcm_stride, int n_valid,
                                                               const float* __restrict__ dft, const uint16_t* __restrict__ dft3,
                                                               const int* __restrict__ mel_lo,
                                                               const int* __restrict__ mel_hi, const float* __restrict__ mel_w,
                                                               int n_mel, float* __restrict__ out, unsigned* __restrict__ clip_max) {
  constexpr int kPowLd = kBins + 3;
  constexpr int kLdsFloats = (kSpan > kFPB * kPowLd) ? kSpan : kFPB * kPowLd;
  __shared__ __attribute__((aligned(16))) float lds[kLdsFloats];
  __shared__ float wmax[4];
  const int b = blockIdx.y, f0 = blockIdx.x * kFPB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* x = pcm + (long)b * pcm_stride;
  const int nv = min(n_valid, kNSamp);
  // stage samples [f0*160 - 200, f0*160 - 200 + kSpan) with reflect padding of the 480000 signal
  const int s0 = f0 * kHop - kNFFT / 2;
  for (int i = tid; i < kSpan; i += 256) {
    int j = s0 + i;
    if (j < 0) j = -j;
    if (j >= kNSamp) j = 2 * (kNSamp - 1) - j;
    j = max(0, min(j, kNSamp - 1));
    lds[i] = j < nv ? x[j] : 0.f;
  }
  __syncthreads();
  // DFT: every wave takes all 64 frames of the workgroup (4 row fragments) against its share of the 26
  // column fragments (7, 7, 6, 6): each table fragment read from L2 feeds 4 row fragments (the earlier
  // split, 16 frames x all 26 column fragments per wave, re-read the 692 KB table 4x as often). The K
  // order of every output element is unchanged: bit-identical.
  constexpr int kCF = 26, kCW = 7;                       // column fragments, per wave (at most)
  static_assert(kCF == 2 * kCW + 2 * (kCW - 1) && kCF * 16 == kNCol, "the waves' column shares cover the table");
  const int cf0 = wave < 2 ? wave * kCW : 2 * kCW + (wave - 2) * (kCW - 1);
  const int ncf = wave < 2 ? kCW : kCW - 1;
  f32x4 acc[4][kCW];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < kCW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (SPLIT) {
    constexpr long kPart = (long)kNCol * kNCol;
    const uint16_t* brow = dft3 + (long)(cf0 * 16 + (lane & 15)) * kNCol + 8 * (lane >> 4);
    for (int kb = 0; kb < kNCol; kb += 32) {
      s16x8 ah[4], am[4], al[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float* arow = lds + (i * 16 + (lane & 15)) * kHop + 8 * (lane >> 4) + kb;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = arow[e];
          const bf16_t h = f_to_bf16(v);
          const float r1 = v - bf16_to_f(h);
          const bf16_t m = f_to_bf16(r1);
          const bf16_t l = f_to_bf16(r1 - bf16_to_f(m));
          ah[i][e] = (short)h; am[i][e] = (short)m; al[i][e] = (short)l;
        }
      }
#pragma unroll
      for (int j = 0; j < kCW; ++j) {
        if (j < ncf) {
          const uint16_t* bp = brow + (long)j * 16 * kNCol + kb;
          const s16x8 bh = *reinterpret_cast<const s16x8*>(bp);
          const s16x8 bm = *reinterpret_cast<const s16x8*>(bp + kPart);
          const s16x8 bl = *reinterpret_cast<const s16x8*>(bp + 2 * kPart);
#pragma unroll
          for (int i = 0; i < 4; ++i) {   // small terms first
            f32x4 c = acc[i][j];
            c = mma16(am[i], bm, c);
            c = mma16(al[i], bh, c);
            c = mma16(ah[i], bl, c);
            c = mma16(am[i], bh, c);
            c = mma16(ah[i], bm, c);
            acc[i][j] = mma16(ah[i], bh, c);
          }
        }
      }
    }
  } else {
  const float* brow = dft + (long)(cf0 * 16 + (lane & 15)) * kNCol + 8 * (lane >> 4);
  for (int kb = 0; kb < kNCol; kb += 32) {
    f32x8 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float* arow = lds + (i * 16 + (lane & 15)) * kHop + 8 * (lane >> 4) + kb;
#pragma unroll
      for (int e = 0; e < 8; ++e) a[i][e] = arow[e];
    }
#pragma unroll
    for (int j = 0; j < kCW; ++j) {
      if (j < ncf) {
        const f32x8 bf = *reinterpret_cast<const f32x8*>(brow + (long)j * 16 * kNCol + kb);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] = mma16(a[i], bf, acc[i][j]);
      }
    }
  }
  }
  __syncthreads();   // samples no longer needed: reuse LDS for the power spectrum
  // acc[i][j][e]: frame row 16i + (lane>>4)*4 + e, column 16(cf0 + j) + (lane&15): even = re, odd = im
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < kCW; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = acc[i][j][e];
        const float p = v * v + __shfl_xor(v, 1, 64) * __shfl_xor(v, 1, 64);
        const int col = (cf0 + j) * 16 + (lane & 15);
        if (j < ncf && (col & 1) == 0 && (col >> 1) < kBins)
          lds[(i * 16 + (lane >> 4) * 4 + e) * kPowLd + (col >> 1)] = p;
      }
  __syncthreads();
  // mel + log10: thread -> (mel m, frame f) with frames fastest (coalesced output rows)
  float lmax = -INFINITY;
  for (int idx = tid; idx < n_mel * kFPB; idx += 256) {
    const int m = idx / kFPB, f = idx % kFPB;
    if (f0 + f >= kFrames) continue;
    const int lo = mel_lo[m], hi = mel_hi[m];
    float s = 0.f;
    for (int k = lo; k < hi; ++k) s = fmaf(mel_w[m * 32 + (k - lo)], lds[f * kPowLd + k], s);
    const float lg = log10f(fmaxf(s, 1e-10f));
    out[((long)b * n_mel + m) * kFrames + f0 + f] = lg;
    lmax = fmaxf(lmax, lg);
  }
  lmax = wave_max(lmax);
  if (lane == 0) wmax[wave] = lmax;
  __syncthreads();
  if (tid == 0) atomicMax(clip_max + b, ord_enc(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]))));
}

__global__ void logmel_normalize_kernel(float* mel, const unsigned* clip_max, int n_per_clip, long total) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const float mx = ord_dec(clip_max[i / n_per_clip]);
    mel[i] = (fmaxf(mel[i], mx - 8.0f) + 4.0f) / 4.0f;
  }
}

void logmel_power_mel(const float* pcm, long pcm_stride, int n_samples, int B, const float* dft, const void* dft3,
                      const int* mel_lo, const int* mel_hi, const float* mel_w, int n_mel, float* mel_out,
                      unsigned* clip_max, hipStream_t s) {
  (void)hipMemsetAsync(clip_max, 0, sizeof(unsigned) * B, s);
  const dim3 grid((kFrames + kFPB - 1) / kFPB, B);
  if (dft3)
    WCB_LAUNCH(logmel_power_mel_kernel<true>, grid, dim3(256), 0, s, pcm, pcm_stride, n_samples, dft,
               reinterpret_cast<const uint16_t*>(dft3), mel_lo, mel_hi, mel_w, n_mel, mel_out, clip_max);
  else
    WCB_LAUNCH(logmel_power_mel_kernel<false>, grid, dim3(256), 0, s, pcm, pcm_stride, n_samples, dft,
               nullptr, mel_lo, mel_hi, mel_w, n_mel, mel_out, clip_max);
}

void logmel_normalize(float* mel, const unsigned* clip_max, int B, int n_mel, hipStream_t s) {
  const long total = (long)B * n_mel * kFrames;
  WCB_LAUNCH(logmel_normalize_kernel, dim3(2048), dim3(256), 0, s, mel, clip_max, n_mel * kFrames, total);
}

// mel f32 [B][n_mel][3000] → T [B][3002][n_mel] (rows 0 and 3001 zero: conv1 padding=1),
// so conv1 becomes a GEMM whose row t is the contiguous 3·n_mel window starting at row t.
template <typename T>
__global__ void mel_to_conv_input_kernel(const float* __restrict__ mel, int n_mel, T* __restrict__ xt, long clip_stride) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z, t0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int c = c0 + i / 64, t = t0 + i % 64;
    tile[i / 64][i % 64] = (c < n_mel && t < kFrames) ? mel[((long)b * n_mel + c) * kFrames + t] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int t = t0 + i / 64, c = c0 + i % 64;
    if (t < kFrames && c < n_mel) xt[(long)b * clip_stride + (long)(t + 1) * n_mel + c] = DT<T>::fromf(tile[i % 64][i / 64]);
  }
  if (blockIdx.x == 0 && blockIdx.y == 0)
    for (int c = threadIdx.x; c < n_mel; c += 256) {
      xt[(long)b * clip_stride + c] = DT<T>::fromf(0.f);
      xt[(long)b * clip_stride + (long)(kFrames + 1) * n_mel + c] = DT<T>::fromf(0.f);
    }
}

void mel_to_conv_input(DType t, const float* mel, int B, int n_mel, void* xt, long clip_stride, hipStream_t s) {
  const dim3 grid((kFrames + 63) / 64, (n_mel + 63) / 64, B);
  switch (t) {
    case kBF16: WCB_LAUNCH(mel_to_conv_input_kernel<bf16_t>, grid, dim3(256), 0, s, mel, n_mel, (bf16_t*)xt, clip_stride); break;
    case kF16: WCB_LAUNCH(mel_to_conv_input_kernel<f16_t>, grid, dim3(256), 0, s, mel, n_mel, (f16_t*)xt, clip_stride); break;
    case kF32: WCB_LAUNCH(mel_to_conv_input_kernel<float>, grid, dim3(256), 0, s, mel, n_mel, (float*)xt, clip_stride); break;
  }
}

}  // namespace wcb
