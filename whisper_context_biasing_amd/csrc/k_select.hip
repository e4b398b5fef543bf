// Greedy token selection fused with the bias-list log-prob boost and the generate() bookkeeping.
//
// Semantics (restating the greedy step of [tf] generation/utils.py:2894-2936 plus the build-defined
// A8 boost, oracle/bias_ref.py):
//   score[v] = logit[v] + lam * n(s, v)               (f32 product, f32 add: bias_bonus)
//   n(s, v)  = d' - d + min(k, d + 1 - d')            d = depth(s), k = keep(s), d' = depth(delta(s, v))
//   score[eos] = -inf while step < min_new_tokens     (MinNewTokens semantics, benchmark mode)
//   tok = argmax(score), lowest index on ties (torch.argmax); finished rows emit pad;
//   finished |= tok == eos; s <- delta(s, tok).       lam == 0 → plain greedy, bit-identical.
// delta(s, v) = trans(s) entry if v is listed (lands deeper than depth 1), else the root child
// root_child[v] (only word-start tokens may start a match: the host leaves the others at -1), else
// the root. So n = k - d for every token, + 1 on the root children (the root bitmap), and the exact
// value on the few tokens of trans(s). The vocabulary-wide pass (or the LM-head epilogue) reads the
// logits once applying lam·(rowbase + root bit), rowbase = k - d of the row's state; the per-row
// finalize re-scores only trans(s) — exact because lam >= 0 (checked on the host) and n on a trans
// token is never below the vocabulary-pass value, so an underestimated copy never wins.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace wcb {

WCB_DEV bool better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

__global__ __launch_bounds__(256) void select_partial_kernel(SelectArgs a) {
  const int m = blockIdx.y, c = blockIdx.x;
  const int chunk = (a.V + a.nchunk - 1) / a.nchunk;
  const int v0 = c * chunk, v1 = min(a.V, v0 + chunk);
  const float* row = a.logits + (long)m * a.ld;
  const bool mask_eos = *a.step < a.min_new;
  const int rb = a.rowbase[m];
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = v0 + threadIdx.x; v < v1; v += 256) {
    float x = row[v];
    if (a.lam != 0.f) x = bias_bonus(x, a.lam, rb + (int)((a.root_bits[v >> 5] >> (v & 31)) & 1u));
    if (mask_eos && v == a.eos) x = -INFINITY;
    if (better(x, v, bv, bi)) { bv = x; bi = v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sv[w] = bv; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float best = sv[0];
    int bidx = si[0];
    for (int k = 1; k < 4; ++k)
      if (better(sv[k], si[k], best, bidx)) { best = sv[k]; bidx = si[k]; }
    a.part_val[m * a.nchunk + c] = best;
    a.part_idx[m * a.nchunk + c] = bidx;
  }
}

// One wave per row; the last row to finish (atomic ticket) advances the step/position counters.
// EMB: the row's next-step input embedding in the same launch (k_norm.hip embed_kernel's arithmetic and
// stats grouping, 64 columns per pass).
template <typename T, bool EMB>
__global__ __launch_bounds__(64) void select_finalize_kernel(SelectArgs a) {
  const int m = blockIdx.x, lane = threadIdx.x;
  const int step = *a.step;
  const int pos0 = EMB ? *a.pos : 0;   // read before this row's ticket: the last arriver advances it
  const bool mask_eos = step < a.min_new;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = lane; c < a.nchunk; c += 64) {
    const float v = a.part_val[m * a.nchunk + c];
    const int i = a.part_idx[m * a.nchunk + c];
    if (better(v, i, bv, bi)) { bv = v; bi = i; }
  }
  const int s = a.state[m];
  const int t0 = a.trans_off[s], t1 = a.trans_off[s + 1];
  if (a.lam != 0.f) {
    const float* row = a.logits + (long)m * a.ld;
    const int d = a.st_depth[s], k = a.st_keep[s];
    for (int t = t0 + lane; t < t1; t += 64) {
      const int v = a.trans_tok[t];
      const int d2 = a.st_depth[a.trans_dst[t]];
      float x = bias_bonus(row[v], a.lam, d2 - d + min(k, d + 1 - d2));
      if (mask_eos && v == a.eos) x = -INFINITY;
      if (better(x, v, bv, bi)) { bv = x; bi = v; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  const bool fin = a.finished[m] != 0;
  // a row with no comparable value (all NaN) keeps bi = INT_MAX: emit EOS rather than an index past
  // the vocabulary (the next step's embedding lookup must stay in bounds)
  const int tok = fin ? a.pad : (bi >= 0 && bi < a.V ? bi : a.eos);
  // AC transition: tok in trans(s) → its target, else the root child, else root
  int dst = -1;
  for (int t = t0 + lane; t < t1; t += 64)
    if (a.trans_tok[t] == tok) dst = a.trans_dst[t];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dst = max(dst, __shfl_xor(dst, o, 64));
  if constexpr (EMB) {
    // 8 consecutive columns per lane (16-byte accesses of T; the fragment-major copy holds them
    // contiguously too), the optional per-st_w-column partials in embed_kernel's lane-butterfly order
    const int d = a.d, p = min(pos0 + 1, a.n_pos - 1);
    const T* er = reinterpret_cast<const T*>(a.emb) + (long)tok * d;
    const T* pr = reinterpret_cast<const T*>(a.pemb) + (long)p * d;
    if (a.st) {   // (older skinny consumers only) one column per lane, as embed_kernel
      for (int c0 = 0; c0 < d; c0 += 64) {
        const int c = c0 + lane;
        const float v = DT<T>::tof(er[c]) + DT<T>::tof(pr[c]);
        float s1 = v, s2 = v * v;
        if (a.st_w == 32) {
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
        } else {
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
        }
        if ((c & (a.st_w - 1)) == 0) {
          a.st[((long)m * (d / a.st_w) + c / a.st_w) * 2] = s1;
          a.st[((long)m * (d / a.st_w) + c / a.st_w) * 2 + 1] = s2;
        }
      }
    }
    for (int c = lane * 8; c < d; c += 512) {   // (d % 8 == 0)
      float v[8];
      float ev[8], pv[8];
      load8f<T>(er + c, ev);
      load8f<T>(pr + c, pv);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ev[e] + pv[e];
      float* xr = a.x + (long)m * d + c;
      *reinterpret_cast<f32x4*>(xr) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(xr + 4) = f32x4{v[4], v[5], v[6], v[7]};
      if (a.x16) store8<T>(reinterpret_cast<T*>(a.x16) + (long)m * d + c, v);
      if (a.x16fm) {
        const int kw = a.fm_kpw * 32, w2 = c / kw, ks2 = (c % kw) >> 5, lg = (c & 31) >> 3;
        store8<T>(reinterpret_cast<T*>(a.x16fm) + ((((long)(m >> 4) * a.fm_nw + w2) * a.fm_kpw + ks2) * 64 + lg * 16 + (m & 15)) * 8, v);
      }
    }
  }
  if (lane == 0) {
    if (dst < 0) dst = (tok >= 0 && tok < a.V && a.root_child[tok] >= 0) ? a.root_child[tok] : 0;
    a.state[m] = dst;
    a.rowbase[m] = a.st_keep[dst] - a.st_depth[dst];
    a.next_ids[m] = tok;
    a.out_ids[(long)m * a.out_ld + step] = tok;
    if (a.out_score) a.out_score[m] = fin ? 0.f : bv;
    const bool nf = fin || tok == a.eos;
    a.finished[m] = nf ? 1 : 0;
    // one 64-bit counter: arrivals in the low word, unfinished rows in the high word, so the row that
    // arrives last reads the complete count from the value its own add returns — no fence (the other
    // rows' stores are read only by later launches, behind the kernel boundary)
    const unsigned long long old = atomicAdd(a.ticket_unfin, 1ull + (nf ? 0ull : (1ull << 32)));
    if ((unsigned)(old & 0xffffffffull) == (unsigned)(a.M - 1)) {   // every row has arrived
      const int nun = (int)(old >> 32) + (nf ? 0 : 1);
      *a.step = step + 1;
      *a.pos = *a.pos + 1;
      if (nun == 0 && *a.all_done == 0) *a.all_done = step + 1;
      *a.ticket_unfin = 0ull;
    }
  }
}

// Causal prefill (runtime.cpp prefill): the token ids of positions *pos .. *pos + np - 1 of every
// row, rows (row, position) row-major; ld 0 = one prefix shared by every row.
__global__ void prefill_ids_kernel(int* ids, const int* src, int R, int np, int ld, const int* pos) {
  const int p = *pos;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < R * np; i += gridDim.x * blockDim.x)
    ids[i] = src[(long)(i / np) * ld + p + i % np];
}
void prefill_ids(int* ids, const int* src, int R, int np, int ld, const int* pos, hipStream_t s) {
  const int grid = std::min((R * np + 255) / 256, 256);
  WCB_LAUNCH(prefill_ids_kernel, dim3(grid), dim3(256), 0, s, ids, src, R, np, ld, pos);
}
__global__ void add_i32_kernel(int* p, int v) {
  if (threadIdx.x == 0) *p += v;
}
void add_i32(int* p, int v, hipStream_t s) { WCB_LAUNCH(add_i32_kernel, dim3(1), dim3(64), 0, s, p, v); }

// Teacher forcing / prompt prefill: next_ids[b] = forced[b·ld + (*pos) + 1]; pos += 1.
__global__ void advance_forced_kernel(int* next_ids, const int* forced, int M, int ld, int* pos) {
  const int p = *pos;
  __syncthreads();
  for (int b = threadIdx.x; b < M; b += blockDim.x) next_ids[b] = forced[(long)b * ld + p + 1];
  __syncthreads();
  if (threadIdx.x == 0) *pos = p + 1;
}
void advance_forced(int* next_ids, const int* forced, int M, int ld, int* pos, hipStream_t s) {
  WCB_LAUNCH(advance_forced_kernel, dim3(1), dim3(256), 0, s, next_ids, forced, M, ld, pos);
}

// next_ids[b] = src[b·ld + col]
__global__ void gather_col_kernel(int* dst, const int* src, int M, int ld, int col) {
  for (int b = threadIdx.x; b < M; b += blockDim.x) dst[b] = src[(long)b * ld + col];
}
void gather_col(int* dst, const int* src, int M, int ld, int col, hipStream_t s) {
  WCB_LAUNCH(gather_col_kernel, dim3(1), dim3(256), 0, s, dst, src, M, ld, col);
}

struct IntChunk { int n; int v[256]; };
__global__ void write_i32_kernel(int* dst, IntChunk c) {
  for (int i = threadIdx.x; i < c.n; i += blockDim.x) dst[i] = c.v[i];
}
void write_i32(int* dst, const int* host_src, int n, hipStream_t s) {
  for (int o = 0; o < n; o += 256) {
    IntChunk c;
    c.n = n - o < 256 ? n - o : 256;
    for (int i = 0; i < c.n; ++i) c.v[i] = host_src[o + i];
    WCB_LAUNCH(write_i32_kernel, dim3(1), dim3(256), 0, s, dst + o, c);
  }
}

void select_finalize(const SelectArgs& a, hipStream_t s) {
  if (!a.emb) {
    WCB_LAUNCH((select_finalize_kernel<float, false>), dim3(a.M), dim3(64), 0, s, a);
  } else if (a.dtype == kBF16) {
    WCB_LAUNCH((select_finalize_kernel<bf16_t, true>), dim3(a.M), dim3(64), 0, s, a);
  } else if (a.dtype == kF16) {
    WCB_LAUNCH((select_finalize_kernel<f16_t, true>), dim3(a.M), dim3(64), 0, s, a);
  } else {
    WCB_LAUNCH((select_finalize_kernel<float, true>), dim3(a.M), dim3(64), 0, s, a);
  }
}

void select_greedy(const SelectArgs& a, hipStream_t s) {
  WCB_LAUNCH(select_partial_kernel, dim3(a.nchunk, a.M), dim3(256), 0, s, a);
  select_finalize(a, s);
}

}  // namespace wcb
