// Bias-weighted cross entropy of the reference forward (models/whisper_medical.py:113-156), fused.
//
// The reference builds a [B,T] weight map in a Python triple loop (every bias span compared against
// every label window, :118-133), then materialises log_softmax over the whole [B·T, V] logits
// (:136), gathers the label column (:142) and takes Σ(−logp·w·valid) / (Σvalid + 1e-8) (:145-151).
// Here one workgroup owns one label position (b, j):
//   * span coverage: the workgroup's threads test every (span n, start s) with s ≤ j < s + len_n
//     against the label row (the reference sets w = bias_weight on every token of a matched window;
//     a token covered by any match gets bias_weight, which is what the repeated assignments leave);
//   * one streaming pass over the logits row: per-thread online (max, Σexp) in f32, combined by
//     wave shuffles then through LDS, so each logit is read from HBM exactly once (the row is
//     V·4 B; nothing of size V is written back);
//   * −logp[label] = logsumexp − x[label], times w·valid, written per position.
// A single-workgroup reduction then sums the positions in a fixed order (deterministic) and
// divides by the valid count (+1e-8 on the weighted path; plain mean for nn.CrossEntropyLoss).
// HBM-bound: algorithmic bytes = B·T·V·4 (+ labels/spans, negligible).
#include "common.h"
#include "kernels.h"

namespace wcb {

namespace {
constexpr int kWceThreads = 256;
constexpr int kWceWaves = kWceThreads / 64;
}

__global__ __launch_bounds__(kWceThreads) void wce_row_kernel(WceArgs a) {
  const int r = blockIdx.x;                  // label position b·T + j
  const int b = r / a.T, j = r - b * a.T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float s_m[kWceWaves], s_s[kWceWaves];
  __shared__ int s_cov;
  if (tid == 0) s_cov = 0;
  __syncthreads();

  const int* lab = a.labels + (long)b * a.T;
  const int label = lab[j];
  // span coverage (only on the weighted path)
  if (a.use_spans) {
    const int total = a.N * a.Lmax;          // (span, offset of j inside the window)
    bool hit = false;
    for (int q = tid; q < total && !hit; q += kWceThreads) {
      const int n = q / a.Lmax, off = q - n * a.Lmax;
      const int len = a.span_len[(long)b * a.N + n];
      if (len <= 0 || off >= len) continue;
      const int s0 = j - off;
      if (s0 < 0 || s0 + len > a.T) continue;
      const int* sp = a.spans + ((long)b * a.N + n) * a.Lmax;
      bool eq = true;
      for (int i = 0; i < len && eq; ++i) eq = lab[s0 + i] == sp[i];
      hit = eq;
    }
    if (hit) atomicOr(&s_cov, 1);
  }

  const float* x = a.logits + (long)r * a.ld;
  float m = -INFINITY, s = 0.f;
  const int V = a.V;
  // 4-wide loads where the row is 16-byte aligned
  const bool vec = ((a.ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.logits) & 15) == 0);
  int c0 = 0;
  if (vec) {
    const int nv = V >> 2;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    for (int i = tid; i < nv; i += kWceThreads) {
      const float4 v = x4[i];
      const float mx = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
      if (mx > m) { s *= __expf(m - mx); m = mx; }
      s += __expf(v.x - m) + __expf(v.y - m) + __expf(v.z - m) + __expf(v.w - m);
    }
    c0 = nv << 2;
  }
  for (int i = c0 + tid; i < V; i += kWceThreads) {
    const float v = x[i];
    if (v > m) { s *= __expf(m - v); m = v; }
    s += __expf(v - m);
  }
  // combine (m, s) over the wave, then over the waves
  const float wm = wave_max(m);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - wm);
  s = wave_sum(s);
  if (lane == 0) { s_m[wave] = wm; s_s[wave] = s; }
  __syncthreads();
  if (tid == 0) {
    float M = s_m[0];
    for (int w = 1; w < kWceWaves; ++w) M = fmaxf(M, s_m[w]);
    float S = 0.f;
    for (int w = 0; w < kWceWaves; ++w) S += s_s[w] * __expf(s_m[w] - M);
    const bool valid = label != -100;
    float out = 0.f;
    if (valid) {
      const float lse = M + __logf(S);
      const float w = s_cov ? a.bias_weight : 1.f;
      out = (lse - x[label]) * w;
    }
    a.per_token[r] = out;
  }
}

// Fixed-order sum of the per-position terms and of the valid count; one workgroup.
__global__ __launch_bounds__(1024) void wce_reduce_kernel(WceArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double s_sum[16];
  __shared__ int s_cnt[16];
  const int R = a.B * a.T;
  double sum = 0.0;
  int cnt = 0;
  for (int i = tid; i < R; i += 1024) {
    sum += (double)a.per_token[i];
    cnt += a.labels[i] != -100;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sum += __shfl_xor(sum, o, 64);
    cnt += __shfl_xor(cnt, o, 64);
  }
  if (lane == 0) { s_sum[wave] = sum; s_cnt[wave] = cnt; }
  __syncthreads();
  if (tid == 0) {
    double S = 0.0;
    int C = 0;
    for (int w = 0; w < 16; ++w) { S += s_sum[w]; C += s_cnt[w]; }
    a.loss[0] = a.use_spans ? (float)(S / ((double)C + 1e-8)) : (float)(S / (double)C);
    if (a.count) a.count[0] = C;
  }
}

void weighted_ce(const WceArgs& a, hipStream_t s) {
  WCB_LAUNCH(wce_row_kernel, dim3(a.B * a.T), dim3(kWceThreads), 0, s, a);
  WCB_LAUNCH(wce_reduce_kernel, dim3(1), dim3(1024), 0, s, a);
}

}  // namespace wcb
