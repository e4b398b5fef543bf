// Beam search (A9) on the device: HF `_beam_search` ([tf] generation/utils.py:3208-3524, helpers
// :3008-3204) with the A8 bias boost and the MinNewTokens EOS mask as log-prob processors
// ([tf] utils.py:3388-3389). Oracle: oracle/beam_np.py.
//
// Rows r = b·nb + i (utterance b, running beam i). Per decode step:
//   beam_topk_kernel  one workgroup (4-16 waves) per row over the f32 logits row: log_softmax (max, Σexp), the
//                     boost (lam·(k - d + root bit) on the vocabulary, the exact lam·n(s, v) on the
//                     tokens of trans(state), which an LDS bitmap excludes from the vocabulary
//                     pass; oracle/bias_ref.py) and EOS mask, plus the
//                     beam's running score, then the row's top-K (K = 2·nb) by (score desc, token
//                     asc). HBM-bound: 4·V bytes per row (the later passes hit L2).
//   beam_step_kernel  one workgroup per utterance: the top-K of its nb·K row candidates (the global
//                     top-K over nb·V lies in their union, and per-row token order equals the
//                     flat-index order beam·V + token), running / finished updates (length penalty,
//                     -1e9 masks, early-stop heuristic), sequences, AC states, the self-attention key
//                     map, and the batch-wide stop test by the last arriving utterance.
// KV-cache reorder without copies (K9): row i's key/value at position t lives in cache row
// phys[i][t] (the row that computed it). A step writes position `pos` of every row in its own cache
// row, so choosing parents is a gather of nb·T ints per utterance instead of moving 2·L·t·d
// elements per row; the self-attention kernel reads each key through the map.
#include "common.h"
#include "kernels.h"

#include <stdexcept>
#include <type_traits>

namespace wcb {

namespace {
constexpr int kTopK = 16;                     // per-thread candidate list; K = 2·nb <= 16
constexpr int kBitWords = kBeamMaxVocab / 32;
constexpr float kNeg = -1.0e9f;

WCB_DEV bool beam_better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

// δ(s, tok): trans(s) entry if present, else the root child, else the root (k_select.hip)
WCB_DEV int ac_delta(const BeamArgs& a, int s, int tok) {
  for (int t = a.trans_off[s]; t < a.trans_off[s + 1]; ++t)
    if (a.trans_tok[t] == tok) return a.trans_dst[t];
  const int c = (tok >= 0 && tok < a.V) ? a.root_child[tok] : -1;
  return c >= 0 ? c : 0;
}

template <int NW>
WCB_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int q = 1; q < NW; ++q) r = fmaxf(r, red[q]);
  __syncthreads();
  return r;
}
template <int NW>
WCB_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int q = 1; q < NW; ++q) r += red[q];
  __syncthreads();
  return r;
}
}  // namespace

__global__ __launch_bounds__(256) void beam_init_kernel(BeamArgs a) {
  const int r = blockIdx.x, i = r % a.nb;
  const int Lg = a.Lt - a.P;
  for (int t = threadIdx.x; t < a.T; t += blockDim.x) a.phys[(long)r * a.T + t] = r;
  for (int t = threadIdx.x; t < Lg; t += blockDim.x) {
    a.run_seq[(long)r * Lg + t] = a.pad;
    a.fin_seq[(long)r * Lg + t] = a.pad;
  }
  if (threadIdx.x == 0) {
    a.run_sc[r] = i == 0 ? 0.f : kNeg;        // only beam 0 seeds the first step
    a.fin_sc[r] = kNeg;
    a.fin_done[r] = 0;
    a.fin_len[r] = 0;
    a.state[r] = 0;
    if (i == 0) { a.flags[2 * (r / a.nb)] = 1; a.flags[2 * (r / a.nb) + 1] = 0; }
  }
}

// NT threads per row (16 waves when the rows leave CUs idle: one wave per SIMD cannot hide the
// serial compare-exchange chain of a list insert, which every element of a wave pays when any lane
// inserts), KL = the per-thread list length (K rounded up: the chain is KL steps long)
template <int NT, int KL>
__global__ __launch_bounds__(NT) void beam_topk_kernel(BeamArgs a) {
  constexpr int NW = NT / 64;
  if (*a.all_done) return;                    // frozen once the search has stopped
  __shared__ uint32_t bits[kBitWords];
  __shared__ uint32_t tbits[kBitWords];       // tokens of trans(state): scored in their own pass
  __shared__ float red[NW];
  __shared__ float wv[NW];
  __shared__ int wi[NW], wt[NW];
  __shared__ float thr_v;
  __shared__ int thr_i;
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* row = a.logits + (long)r * a.ld;
  // the row as float4 (a.ld is a multiple of 4: the padded vocabulary), UB loads in flight per lane
  const f32x4* row4 = reinterpret_cast<const f32x4*>(row);
  const int V4 = a.V >> 2;
  constexpr int UB = 4;
  auto load4 = [&](int i) -> f32x4 {   // float4 i of the row, -inf past the vocabulary
    if (i < V4) return row4[i];
    f32x4 x;
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = 4 * i + e < a.V ? row[4 * i + e] : -INFINITY;
    return x;
  };
  const int n4 = (a.V + 3) >> 2;
  // one pass for max and Σexp (per lane: a running max, the sum rescaled when a batch raises it)
  float m = -INFINITY, s = 0.f;
  for (int i0 = tid; i0 < n4; i0 += NT * UB) {
    f32x4 x[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) x[u] = i0 + u * NT < n4 ? load4(i0 + u * NT) : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    float bm = m;
#pragma unroll
    for (int u = 0; u < UB; ++u) bm = fmaxf(bm, fmaxf(fmaxf(x[u][0], x[u][1]), fmaxf(x[u][2], x[u][3])));
    if (bm > m) { s = m == -INFINITY ? 0.f : s * expf(m - bm); m = bm; }
    if (m == -INFINITY) continue;
#pragma unroll
    for (int u = 0; u < UB; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += expf(x[u][e] - m);
  }
  const float mrow = block_max<NW>(m, red);
  s = m == -INFINITY ? 0.f : s * expf(m - mrow);   // lane sums onto the row max
  m = mrow;
  const float lsum = logf(block_sum<NW>(s, red));
  const bool boost = a.lam != 0.f;
  const int st = a.state[r];
  int rb = 0, sd = 0, sk = 0;
  if (boost) {
    const int nw = (a.V + 31) >> 5;
    for (int k = tid; k < nw; k += NT) { bits[k] = a.root_bits[k]; tbits[k] = 0u; }
    __syncthreads();
    for (int t = a.trans_off[st] + tid; t < a.trans_off[st + 1]; t += NT) {
      const int v = a.trans_tok[t];
      atomicOr(&tbits[v >> 5], 1u << (v & 31));
    }
    __syncthreads();
    sd = a.st_depth[st];
    sk = a.st_keep[st];
    rb = sk - sd;
  }
  const bool mask_eos = *a.step < a.min_new;
  const float rsc = a.run_sc[r];
  float lv[KL];
  int li[KL];
#pragma unroll
  for (int k = 0; k < KL; ++k) { lv[k] = -INFINITY; li[k] = 0x7fffffff; }
  auto insert = [&](float x, int v) {
    if (beam_better(x, v, lv[KL - 1], li[KL - 1])) {
      float pv = x;
      int pi = v;
#pragma unroll
      for (int k = 0; k < KL; ++k) {
        if (beam_better(pv, pi, lv[k], li[k])) {
          const float tv = lv[k];
          const int ti = li[k];
          lv[k] = pv; li[k] = pi; pv = tv; pi = ti;
        }
      }
    }
  };
  // the row's scores, f(score, token) per element: the vocabulary pass, then trans(state)
  auto scan = [&](auto&& f) {
    for (int i0 = tid; i0 < n4; i0 += NT * UB) {
      f32x4 xs[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) xs[u] = i0 + u * NT < n4 ? load4(i0 + u * NT) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < UB; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int v = 4 * (i0 + u * NT) + e;
          if (v >= a.V) continue;
          float x = (xs[u][e] - m) - lsum;                               // log_softmax
          if (boost) {                                                   // bias boost processor
            if ((tbits[v >> 5] >> (v & 31)) & 1u) continue;              // scored below
            x = bias_bonus(x, a.lam, rb + (int)((bits[v >> 5] >> (v & 31)) & 1u));
          }
          if (mask_eos && v == a.eos) x = -INFINITY;                     // MinNewTokens processor
          f(x + rsc, v);                                                 // + running beam score
        }
    }
    if (boost) {   // trans(state): the exact n(s, v) = d' - d + min(k, d + 1 - d')
      for (int t = a.trans_off[st] + tid; t < a.trans_off[st + 1]; t += NT) {
        const int v = a.trans_tok[t];
        const int d2 = a.st_depth[a.trans_dst[t]];
        float x = bias_bonus((row[v] - m) - lsum, a.lam, d2 - sd + min(sk, sd + 1 - d2));
        if (mask_eos && v == a.eos) x = -INFINITY;
        f(x + rsc, v);
      }
    }
  };
  // Threshold (when K <= NW): the K-th best of the NW wave maxima. They are K distinct elements at or
  // above it, so the row's top-K is too, and the list pass inserts only elements at or above it: a
  // few per wave instead of a serial insert chain on nearly every element. The top-K is unchanged.
  float tv = -INFINITY;
  int ti = 0x7fffffff;
  if (NW >= 8 && a.K <= NW) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    scan([&](float x, int v) { if (beam_better(x, v, bv, bi)) { bv = x; bi = v; } });
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (beam_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { wv[w] = bv; wi[w] = bi; }
    if (tid == 0) { thr_v = -INFINITY; thr_i = 0x7fffffff; }
    __syncthreads();
    if (tid < NW) {   // the wave maximum of rank K - 1 (NaN-free maxima are distinct elements)
      bv = wv[tid];
      bi = wi[tid];
      int rank = 0;
      for (int j = 0; j < NW; ++j) rank += beam_better(wv[j], wi[j], bv, bi) ? 1 : 0;
      if (rank == a.K - 1) { thr_v = bv; thr_i = bi; }
    }
    __syncthreads();
    tv = thr_v;
    ti = thr_i;
  }
  scan([&](float x, int v) { if (!beam_better(tv, ti, x, v)) insert(x, v); });
  int head = 0;
  for (int k = 0; k < a.K; ++k) {   // K rounds: block argmax over the threads' list heads
    float hv = -INFINITY;
    int hi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < KL; ++q)
      if (q == head) { hv = lv[q]; hi = li[q]; }
    int ht = tid;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(hv, o, 64);
      const int oi = __shfl_xor(hi, o, 64), ot = __shfl_xor(ht, o, 64);
      if (beam_better(ov, oi, hv, hi)) { hv = ov; hi = oi; ht = ot; }
    }
    if (lane == 0) { wv[w] = hv; wi[w] = hi; wt[w] = ht; }
    __syncthreads();
    float bv = wv[0];
    int bi = wi[0], bt = wt[0];
#pragma unroll
    for (int q = 1; q < NW; ++q)
      if (beam_better(wv[q], wi[q], bv, bi)) { bv = wv[q]; bi = wi[q]; bt = wt[q]; }
    if (tid == bt) ++head;
    // an all-NaN row leaves bi = INT_MAX: keep the candidate index inside the vocabulary
    if (tid == 0) { a.cand_val[(long)r * a.K + k] = bv; a.cand_tok[(long)r * a.K + k] = bi >= 0 && bi < a.V ? bi : a.eos; }
    __syncthreads();
  }
}

// Chunked top-K (nchunk > 1): each row's vocabulary split into nchunk chunks of CH4 float4 (a multiple of 8:
// chunk token ranges are 32-aligned, whole bitmap words), one workgroup per (chunk, row) in two launches —
// (1) the chunk's (max, Σexp); (2) the row's log-sum-exp from all chunk partials (fixed order, the same in
// every chunk's workgroup), then the chunk's top-K by (score desc, token asc) with the same per-element
// score as beam_topk_kernel. beam_step_kernel takes the top-K over the nb·nchunk·K candidates of an
// utterance (the row top-K lies in the union of its chunks' top-K). 5120 workgroups at C3's 320 rows where
// the per-row kernel ran 320 serial row scans.
WCB_DEV int beam_ch4(const BeamArgs& a) {
  const int n4 = (a.V + 3) >> 2;
  return ((n4 + a.nchunk - 1) / a.nchunk + 7) & ~7;
}

template <int NT>
__global__ __launch_bounds__(NT) void beam_chunk_stats_kernel(BeamArgs a) {
  constexpr int NW = NT / 64;
  if (*a.all_done) return;
  __shared__ float red[NW];
  const int c = blockIdx.x, r = blockIdx.y, tid = threadIdx.x;
  const float* row = a.logits + (long)r * a.ld;
  const f32x4* row4 = reinterpret_cast<const f32x4*>(row);
  const int V4 = a.V >> 2, n4 = (a.V + 3) >> 2, ch4 = beam_ch4(a);
  const int i_lo = c * ch4, i_hi = min(i_lo + ch4, n4);
  float m = -INFINITY, s = 0.f;
  for (int i = i_lo + tid; i < i_hi; i += NT) {
    f32x4 x;
    if (i < V4) x = row4[i];
    else {
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = 4 * i + e < a.V ? row[4 * i + e] : -INFINITY;
    }
    const float bm = fmaxf(m, fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])));
    if (bm > m) { s = m == -INFINITY ? 0.f : s * expf(m - bm); m = bm; }
    if (m == -INFINITY) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) s += expf(x[e] - m);
  }
  const float mc = block_max<NW>(m, red);
  s = m == -INFINITY ? 0.f : s * expf(m - mc);
  const float sc = block_sum<NW>(s, red);
  if (tid == 0) *reinterpret_cast<float2*>(a.chunk_stats + ((long)r * a.nchunk + c) * 2) = float2{mc, sc};
}

template <int NT, int KL>
__global__ __launch_bounds__(NT) void beam_topk_chunk_kernel(BeamArgs a) {
  constexpr int NW = NT / 64;
  constexpr int kW = 4 * 1024 / 32;          // bitmap words of a chunk (<= 1024 float4 = 4096 tokens, 32-aligned)
  if (*a.all_done) return;
  __shared__ uint32_t bits[kW], tbits[kW];
  __shared__ float wv[NW], row_ml[2];
  __shared__ int wi[NW], wt[NW];
  const int c = blockIdx.x, r = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* row = a.logits + (long)r * a.ld;
  const f32x4* row4 = reinterpret_cast<const f32x4*>(row);
  const int V4 = a.V >> 2, n4 = (a.V + 3) >> 2, ch4 = beam_ch4(a);
  const int i_lo = c * ch4, i_hi = min(i_lo + ch4, n4);
  const int v_lo = 4 * i_lo, v_hi = min(4 * i_hi, a.V), w_lo = v_lo >> 5;
  // the row's log-sum-exp from the chunk partials (wave 0, fixed butterfly: identical in every chunk)
  if (w == 0) {
    float2 p = float2{-INFINITY, 0.f};
    if (lane < a.nchunk) p = *reinterpret_cast<const float2*>(a.chunk_stats + ((long)r * a.nchunk + lane) * 2);
    const float m = wave_max(p.x);
    const float t = (p.x == -INFINITY || m == -INFINITY) ? 0.f : p.y * expf(p.x - m);
    const float ssum = wave_sum(t);
    if (lane == 0) { row_ml[0] = m; row_ml[1] = logf(ssum); }
  }
  const bool boost = a.lam != 0.f;
  const int st = a.state[r];
  int rb = 0, sd = 0, sk = 0;
  if (boost) {
    const int nwc = ((v_hi + 31) >> 5) - w_lo;
    for (int k = tid; k < nwc; k += NT) { bits[k] = a.root_bits[w_lo + k]; tbits[k] = 0u; }
    __syncthreads();
    for (int t = a.trans_off[st] + tid; t < a.trans_off[st + 1]; t += NT) {
      const int v = a.trans_tok[t];
      if (v >= v_lo && v < v_hi) atomicOr(&tbits[(v >> 5) - w_lo], 1u << (v & 31));
    }
    sd = a.st_depth[st];
    sk = a.st_keep[st];
    rb = sk - sd;
  }
  __syncthreads();
  const float m = row_ml[0], lsum = row_ml[1];
  const bool mask_eos = *a.step < a.min_new;
  const float rsc = a.run_sc[r];
  float lv[KL];
  int li[KL];
#pragma unroll
  for (int k = 0; k < KL; ++k) { lv[k] = -INFINITY; li[k] = 0x7fffffff; }
  auto insert = [&](float x, int v) {
    if (beam_better(x, v, lv[KL - 1], li[KL - 1])) {
      float pv = x;
      int pi = v;
#pragma unroll
      for (int k = 0; k < KL; ++k) {
        if (beam_better(pv, pi, lv[k], li[k])) {
          const float tv = lv[k];
          const int ti = li[k];
          lv[k] = pv; li[k] = pi; pv = tv; pi = ti;
        }
      }
    }
  };
  // the chunk's scores (beam_topk_kernel's per-element arithmetic): the vocabulary pass, then trans(state)
  for (int i = i_lo + tid; i < i_hi; i += NT) {
    f32x4 xs;
    if (i < V4) xs = row4[i];
    else {
#pragma unroll
      for (int e = 0; e < 4; ++e) xs[e] = 4 * i + e < a.V ? row[4 * i + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int v = 4 * i + e;
      if (v >= a.V) continue;
      float x = (xs[e] - m) - lsum;                                       // log_softmax
      if (boost) {                                                        // bias boost processor
        const int wd = (v >> 5) - w_lo;
        if ((tbits[wd] >> (v & 31)) & 1u) continue;                       // scored below
        x = bias_bonus(x, a.lam, rb + (int)((bits[wd] >> (v & 31)) & 1u));
      }
      if (mask_eos && v == a.eos) x = -INFINITY;                          // MinNewTokens processor
      insert(x + rsc, v);                                                 // + running beam score
    }
  }
  if (boost) {   // trans(state) tokens of this chunk: the exact n(s, v) = d' - d + min(k, d + 1 - d')
    for (int t = a.trans_off[st] + tid; t < a.trans_off[st + 1]; t += NT) {
      const int v = a.trans_tok[t];
      if (v < v_lo || v >= v_hi) continue;
      const int d2 = a.st_depth[a.trans_dst[t]];
      float x = bias_bonus((row[v] - m) - lsum, a.lam, d2 - sd + min(sk, sd + 1 - d2));
      if (mask_eos && v == a.eos) x = -INFINITY;
      insert(x + rsc, v);
    }
  }
  int head = 0;
  for (int k = 0; k < a.K; ++k) {   // K rounds: block argmax over the threads' list heads
    float hv = -INFINITY;
    int hi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < KL; ++q)
      if (q == head) { hv = lv[q]; hi = li[q]; }
    int ht = tid;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(hv, o, 64);
      const int oi = __shfl_xor(hi, o, 64), ot = __shfl_xor(ht, o, 64);
      if (beam_better(ov, oi, hv, hi)) { hv = ov; hi = oi; ht = ot; }
    }
    if (lane == 0) { wv[w] = hv; wi[w] = hi; wt[w] = ht; }
    __syncthreads();
    float bv = wv[0];
    int bi = wi[0], bt = wt[0];
#pragma unroll
    for (int q = 1; q < NW; ++q)
      if (beam_better(wv[q], wi[q], bv, bi)) { bv = wv[q]; bi = wi[q]; bt = wt[q]; }
    if (tid == bt) ++head;
    // fewer than K elements (or an all-NaN chunk): the index stays inside the vocabulary
    if (tid == 0) {
      const long o = ((long)r * a.nchunk + c) * a.K + k;
      a.cand_val[o] = bv;
      a.cand_tok[o] = bi >= 0 && bi < a.V ? bi : a.eos;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void beam_step_kernel(BeamArgs a) {
  if (*a.all_done) {   // frozen search: a step changes nothing, so every beam extends itself by pad
    if (threadIdx.x < a.nb) {
      const int r = blockIdx.x * a.nb + threadIdx.x;
      if (a.parent) a.parent[r] = threadIdx.x;
      a.next_ids[r] = a.pad;
    }
    return;
  }
  __shared__ float tv[kTopK], rlp[kTopK], flv[kTopK];
  __shared__ int tb[kTopK], tt[kTopK], hit[kTopK];
  __shared__ int sel[kMaxBeams], fsrc[kMaxBeams], st_old[kMaxBeams];
  __shared__ float fsc_old[kMaxBeams];
  __shared__ int fdone_old[kMaxBeams], flen_old[kMaxBeams];
  __shared__ int seq_old[kMaxBeams][kBeamMaxLen];
  __shared__ int fin_old[kMaxBeams][kBeamMaxLen];
  __shared__ int phys_old[kMaxBeams][kBeamMaxLen];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int nb = a.nb, K = a.K, R0 = b * nb;
  const int step = *a.step;
  const int cur = a.P + step;                 // tokens in every running sequence before this one
  const int Lg = a.Lt - a.P;
  const int unsat_old = a.flags[2 * b];
  // ---- phase 1 (wave 0): top-K of the nb·nchunk·K candidates by (score desc, beam·V + token asc);
  // candidate j of the utterance at lane j % 64, slot j / 64 (kCandPL slots: nb·nchunk·K <= 64·kCandPL)
  if (tid < 64) {
    constexpr int kCandPL = 2 * kBeamChunks;
    const int per_row = a.nchunk * K, nc = nb * per_row;
    float cv[kCandPL];
    int cf[kCandPL];
#pragma unroll
    for (int q = 0; q < kCandPL; ++q) {
      const int j = q * 64 + lane;
      cv[q] = -INFINITY; cf[q] = 0x7fffffff;
      if (j < nc) {
        const int rr = j / per_row;
        cv[q] = a.cand_val[(long)R0 * per_row + j];
        cf[q] = rr * a.V + a.cand_tok[(long)R0 * per_row + j];
      }
    }
    for (int k = 0; k < K; ++k) {
      float bv = cv[0];
      int bf = cf[0];
#pragma unroll
      for (int q = 1; q < kCandPL; ++q)
        if (beam_better(cv[q], cf[q], bv, bf)) { bv = cv[q]; bf = cf[q]; }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int of = __shfl_xor(bf, o, 64);
        if (beam_better(ov, of, bv, bf)) { bv = ov; bf = of; }
      }
      bool gone = false;   // the winner leaves its lane (the first slot holding it)
#pragma unroll
      for (int q = 0; q < kCandPL; ++q)
        if (!gone && cf[q] == bf && cv[q] == bv) { cv[q] = -INFINITY; cf[q] = 0x7fffffff; gone = true; }
      if (lane == 0) { tv[k] = bv; tb[k] = bf / a.V; tt[k] = bf % a.V; }
    }
  }
  // old state of the utterance into LDS (new rows are gathers of old rows)
  for (int e = tid; e < nb * step; e += 256) {
    const int i = e / step, t = e % step;
    seq_old[i][t] = a.run_seq[(long)(R0 + i) * Lg + t];
    fin_old[i][t] = a.fin_seq[(long)(R0 + i) * Lg + t];
  }
  for (int e = tid; e < nb * cur; e += 256) {
    const int i = e / cur, t = e % cur;
    phys_old[i][t] = a.phys[(long)(R0 + i) * a.T + t];
  }
  if (tid < nb) {
    st_old[tid] = a.state[R0 + tid];
    fsc_old[tid] = a.fin_sc[R0 + tid];
    fdone_old[tid] = a.fin_done[R0 + tid];
    flen_old[tid] = a.fin_len[R0 + tid];
  }
  __syncthreads();
  // ---- phase 2: stopping criteria, running scores, finished-candidate scores
  if (tid < K) {
    const int k = tid;
    const bool h = tt[k] == a.eos || cur + 1 >= a.Lt;
    hit[k] = h;
    rlp[k] = h ? tv[k] + kNeg : tv[k];
    const float den = (float)pow((double)(cur + 1 - a.P), (double)a.len_pen);
    float fl = tv[k] / den;
    if (!unsat_old) fl = fl + kNeg;
    const bool did = h && k < nb;
    if (!did) fl = fl + kNeg;
    flv[k] = fl;
  }
  __syncthreads();
  if (tid < K) {   // running beams: rank among the K by (rlp desc, k asc)
    const int k = tid;
    int rank = 0;
    for (int q = 0; q < K; ++q) rank += beam_better(rlp[q], q, rlp[k], k);
    if (rank < nb) sel[rank] = k;
  } else if (tid >= 64 && tid < 64 + nb + K) {   // finished: merge old nb and new K, keep nb
    const int m = tid - 64;
    const float vm = m < nb ? fsc_old[m] : flv[m - nb];
    int rank = 0;
    for (int q = 0; q < nb + K; ++q) {
      const float vq = q < nb ? fsc_old[q] : flv[q - nb];
      rank += beam_better(vq, q, vm, m);
    }
    if (rank < nb) fsrc[rank] = m;
  }
  __syncthreads();
  // ---- phase 3: write the new running and finished beams
  for (int e = tid; e < nb * (step + 1); e += 256) {
    const int i = e / (step + 1), t = e % (step + 1);
    const int k = sel[i];
    a.run_seq[(long)(R0 + i) * Lg + t] = t < step ? seq_old[tb[k]][t] : tt[k];
    const int m = fsrc[i];
    int fv;
    if (m < nb) fv = t < step ? fin_old[m][t] : a.pad;   // old finished sequences end before `step`
    else fv = t < step ? seq_old[tb[m - nb]][t] : tt[m - nb];
    a.fin_seq[(long)(R0 + i) * Lg + t] = fv;
  }
  for (int e = tid; e < nb * cur; e += 256) {
    const int i = e / cur, t = e % cur;
    a.phys[(long)(R0 + i) * a.T + t] = phys_old[tb[sel[i]]][t];
  }
  if (tid < nb) {
    const int i = tid, k = sel[i];
    if (cur < a.T) a.phys[(long)(R0 + i) * a.T + cur] = R0 + i;   // the next step writes its own row
    a.next_ids[R0 + i] = tt[k];
    if (a.parent) a.parent[R0 + i] = tb[k];
    a.run_sc[R0 + i] = rlp[k];
    a.state[R0 + i] = a.lam != 0.f ? ac_delta(a, st_old[tb[k]], tt[k]) : 0;
    const int m = fsrc[i];
    if (m < nb) {
      a.fin_sc[R0 + i] = fsc_old[m];
      a.fin_done[R0 + i] = fdone_old[m];
      a.fin_len[R0 + i] = flen_old[m];
    } else {
      a.fin_sc[R0 + i] = flv[m - nb];
      a.fin_done[R0 + i] = (hit[m - nb] && (m - nb) < nb) ? 1 : 0;
      a.fin_len[R0 + i] = step + 1;
    }
  }
  __syncthreads();
  // ---- phase 4: early-stop heuristic (early_stopping = False) and the batch-wide stop test
  if (tid == 0) {
    const float den = (float)pow((double)(cur + 1 - a.P), (double)a.len_pen);
    const float best = rlp[sel[0]] / den;
    float mn = INFINITY;
    for (int j = 0; j < nb; ++j) {
      const int m = fsrc[j];
      mn = fminf(mn, m < nb ? fsc_old[m] : flv[m - nb]);
    }
    bool any = false;
    for (int j = 0; j < nb; ++j) {
      const int m = fsrc[j];
      const bool done = m < nb ? fdone_old[m] != 0 : (hit[m - nb] && (m - nb) < nb);
      any |= best > (done ? mn : kNeg);
    }
    bool allhit = true;
    for (int k = 0; k < K; ++k) allhit &= hit[k] != 0;
    __hip_atomic_store(a.flags + 2 * b, (unsat_old && any) ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.flags + 2 * b + 1, allhit ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the flags went out write-through (sc1); drained before the ticket, read back with sc1 loads by the
    // utterance whose add returns last (MI355X_MICROARCH.md "Valid forms", row 1): no fences
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (atomicAdd(a.ticket, 1) == a.B - 1) {    // every utterance has arrived
      bool any_unsat = false, all_hit = true;
      for (int u = 0; u < a.B; ++u) {
        any_unsat |= __hip_atomic_load(a.flags + 2 * u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        all_hit &= __hip_atomic_load(a.flags + 2 * u + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
      }
      *a.step = step + 1;
      *a.pos = *a.pos + 1;
      if ((!any_unsat || all_hit) && *a.all_done == 0) *a.all_done = step + 1;
      *a.ticket = 0;
    }
  }
}

// out[b][t] = best finished sequence of utterance b (pad after its length); *out_len = max length
__global__ __launch_bounds__(256) void beam_output_kernel(BeamArgs a) {
  const int b = blockIdx.x, r = b * a.nb;
  const int Lg = a.Lt - a.P;
  const int len = a.fin_len[r];
  for (int t = threadIdx.x; t < a.out_ld; t += blockDim.x)
    a.out_ids[(long)b * a.out_ld + t] = (t < len && t < Lg) ? a.fin_seq[(long)r * Lg + t] : a.pad;
  if (threadIdx.x == 0) atomicMax(a.out_len, len);
}

void beam_init(const BeamArgs& a, hipStream_t s) {
  WCB_LAUNCH(beam_init_kernel, dim3(a.B * a.nb), dim3(256), 0, s, a);
}
void beam_select(const BeamArgs& a, hipStream_t s) {
  const int rows = a.B * a.nb;
  if (a.nchunk > 1) {   // chunked: (max, Σexp) per chunk, then the chunk top-K lists
    if (a.nchunk > kBeamChunks || a.nb * a.K > 2 * 64 || a.nb * a.nchunk * a.K > 64 * 2 * kBeamChunks)
      throw std::runtime_error("internal error: chunked beam top-K beyond its candidate budget");
    if ((((a.V + 3) / 4 + a.nchunk - 1) / a.nchunk + 7) / 8 * 8 > 1024)
      throw std::runtime_error("internal error: chunked beam top-K: vocabulary chunk above 4096 tokens");
    WCB_LAUNCH((beam_chunk_stats_kernel<256>), dim3(a.nchunk, rows), dim3(256), 0, s, a);
    auto chunk = [&](auto kl) {
      constexpr int KL = decltype(kl)::value;
      WCB_LAUNCH((beam_topk_chunk_kernel<256, KL>), dim3(a.nchunk, rows), dim3(256), 0, s, a);
    };
    if (a.K <= 4) chunk(std::integral_constant<int, 4>{});
    else if (a.K <= 8) chunk(std::integral_constant<int, 8>{});
    else if (a.K <= 12) chunk(std::integral_constant<int, 12>{});
    else chunk(std::integral_constant<int, 16>{});
    WCB_LAUNCH(beam_step_kernel, dim3(a.B), dim3(256), 0, s, a);
    return;
  }
  // 16 waves per row while the rows fit one per CU (C5: 80 rows), 8 up to two per CU (C3: 320)
  auto topk = [&](auto kl) {
    constexpr int KL = decltype(kl)::value;
    if (rows <= 256) WCB_LAUNCH((beam_topk_kernel<1024, KL>), dim3(rows), dim3(1024), 0, s, a);
    else if (rows <= 1024) WCB_LAUNCH((beam_topk_kernel<512, KL>), dim3(rows), dim3(512), 0, s, a);
    else WCB_LAUNCH((beam_topk_kernel<256, KL>), dim3(rows), dim3(256), 0, s, a);
  };
  if (a.K <= 4) topk(std::integral_constant<int, 4>{});
  else if (a.K <= 8) topk(std::integral_constant<int, 8>{});
  else if (a.K <= 12) topk(std::integral_constant<int, 12>{});
  else topk(std::integral_constant<int, 16>{});
  WCB_LAUNCH(beam_step_kernel, dim3(a.B), dim3(256), 0, s, a);
}
void beam_output(const BeamArgs& a, hipStream_t s) {
  WCB_LAUNCH(beam_output_kernel, dim3(a.B), dim3(256), 0, s, a);
}

}  // namespace wcb
