// Host-side launch interface of the libwcb device kernels (internal; the public C-ABI is include/wcb.h).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace wcb {

// Profiling pass only: while `start`/`stop` are set (runtime.cpp, wcb_handle::timed), every launch in
// the scope goes through hipExtLaunchKernel with the event pair attached to the dispatch itself, so the
// pair carries the kernel's own begin/end timestamps (the same source rocprofv3's kernel trace reads),
// not an enqueue-to-completion interval. `start` marks the first launch of the scope, `stop` the last.
struct LaunchTimer {
  hipEvent_t start = nullptr, stop = nullptr;
  int n = 0;
  const void* fn = nullptr;   // first kernel of the scope and its total grid in threads (rocprofv3)
  long grid = 0;
};
inline thread_local LaunchTimer g_launch_timer;

#define WCB_LAUNCH(K, G, B, SH, S, ...)                                                              \
  do {                                                                                               \
    ::wcb::LaunchTimer& lt_ = ::wcb::g_launch_timer;                                                 \
    if (lt_.stop) {                                                                                  \
      if (!lt_.n) {                                                                                  \
        lt_.fn = reinterpret_cast<const void*>(K);                                                   \
        const dim3 g_ = dim3(G), b_ = dim3(B);                                                       \
        lt_.grid = (long)g_.x * g_.y * g_.z * b_.x * b_.y * b_.z;                                    \
      }                                                                                              \
      hipExtLaunchKernelGGL(K, G, B, SH, S, lt_.n ? nullptr : lt_.start, lt_.stop, 0, __VA_ARGS__);  \
      ++lt_.n;                                                                                       \
    } else {                                                                                         \
      hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                                               \
    }                                                                                                \
  } while (0)

enum DType : int { kBF16 = 0, kF16 = 1, kF32 = 2 };

// C[M,N] = epilogue(A[M,K] · W[N,K]ᵀ).  A row m lives at A + (m / a_Mb)·a_strideB + (m % a_Mb)·lda
// (a_Mb == 0: A + m·lda)
// (elements): one formula covers plain row-major operands, per-clip batched operands and the
// overlapping im2col rows of the two conv-stem convolutions.
struct GemmArgs {
  const void* A = nullptr; long lda = 0; int a_Mb = 0; long a_strideB = 0;   // a_Mb 0: plain rows
  const void* W = nullptr; long ldw = 0;
  int M = 0, N = 0, K = 0;
  const float* bias = nullptr;     // [N] f32
  const float* ln_w = nullptr;     // fused LayerNorm of the f32 A rows (skinny path): gamma, beta
  const float* ln_b = nullptr;
  int act = 0;                     // 0 none, 1 gelu(erf)
  const float* resid = nullptr;    // f32, same addressing as out (mode 0), may alias out
  const float* addrow = nullptr;   // f32 [c_Mb][N] row table added after act (encoder positions)
  void* out = nullptr; int out_f32 = 0;
  int mode = 0;                    // 0 rows, 1 head-split, 2 decode qkv (q rows + kv-cache append)
  long ldc = 0; int c_Mb = 0; long c_strideB = 0;
  int hs_S = 0, hs_H = 0, hs_B = 0;        // mode 1: [g][B][H][S][64]; mode 2: rows of the cache
  const int* pos = nullptr; int kv_T = 0;  // mode 2: cache position (device) and cache length
  void* kv_out = nullptr; int n_split = 0; // mode 2: columns >= n_split go to the cache
  int kv_rps = 0;                          // mode 2 prefill: row m → cache row m / kv_rps, position *pos + m % kv_rps
  int tile = 0;                            // MFMA tile kernel for a decode-row GEMM (> 64 rows; A pre-normalised)
  // decode-step fusions (skinny path)
  const float* st_in = nullptr;    // LN row statistics partials [M][st_nb][2] (Σx, Σx²) of A
  float* st_out = nullptr;         // partials of the written f32 rows (residual GEMMs, NF = 1)
  int st_nb = 0;                   // 16-column blocks per row (d / 16)
  float* sel_val = nullptr; int* sel_idx = nullptr;   // LM head: per-(row, workgroup) argmax partial
  const uint32_t* sel_root_bits = nullptr; float sel_lam = 0.f;
  const int* sel_rowbase = nullptr;   // per row k - d of its bias state: bonus lam·(base + root bit)
  int sel_eos = -1; const int* sel_step = nullptr; int sel_min_new = 0;
  // grouped A (skinny path, block-diagonal weights): the A row of output column block n0 starts
  // (n0 / a_grp_n) · a_grp_off elements further (q'_h = W_k,hᵀ q_h: K = 64 columns of head h)
  int a_grp_n = 0; long a_grp_off = 0;
  int skinny = 0;                  // decode projection: the skinny kernel whatever M (row blocks over grid.y)
  int ring_kt = 1;                 // tile 2: 64-deep K sub-tiles per LDS-ring stage (1 or 2)
  int wide = 0;                    // tile 2, K = d_model: gemm_wide_kernel tile config 10·FM + FN (0: ring tiles)
  int walkers = 0;                 // LM head column walkers per row block (0: kDecWalkers)
  // decode GEMM (gemm_dec_kernel): a T-typed copy of the f32 rows the epilogue writes (the
  // residual stream x → x16, read back as the LN-fused A operand of the next projection), and the
  // LN-fused A read from such a copy instead of the f32 rows (lda elements per row)
  void* out16 = nullptr;
  const void* ln_a16 = nullptr;
  // folded LayerNorm (ring tiles, decode rows > 64, gemm_impl.h LNF): A = the 16-bit residual rows x,
  // W = W' = W·diag(γ), ln_u = Σ_k W'[n][k], bias = ln_c = Σ_k β_k W[n][k] + b[n]; out = r·(acc − μ·ln_u[n]) + bias
  // with (μ, r) from rst_in: per row rst_nb = K / 32 partial sums (Σx, Σx²) of 32 columns each
  const float* ln_u = nullptr;
  const float* ln_c = nullptr;     // Σ_k β_k W[n][k] + bias[n] (becomes `bias` when the fold is taken)
  const void* ln_wg = nullptr;     // W' = W·diag(γ) in the model dtype (becomes `W` when the fold is taken)
  const void* ln_wg_fm = nullptr;  // W' fragment-major (the wide beam-row tiles; becomes `W_fm` with the fold)
  int lean_fold = 0;               // lean LN-fused projections: the folded form (W' fragment-major, c, u)
  int lean_mf2 = 0;                // lean projections: 32-row workgroups wherever M > 16 (default: N >= 2048 LN-fused)
  // greedy cross query (folded, lean): q'_h = W_k,hᵀ q_h in the same launch without a hand-off
  // (gemm_impl.h dec_xqk_kernel): W_kt fragment-major, q' rows [M][hs_H·K] (the q rows are not written)
  const void* xqk_wk = nullptr; void* xqk_out = nullptr; int xqk_nch = 0;   // (q' column chunks per head; 0: 8)
  const float* rst_in = nullptr; int rst_nb = 0;
  float* rst_out = nullptr;        // ring-tile residual writers: [M][N / 32] float2 partials of the written f32 rows
  // f16 encoder layers: the layer output is clamped to ±(finfo(f16).max − 1000)
  // ([tf] modeling_whisper.py:409-411); 0 = off
  float clamp = 0.f;
  // decode projection: the lean single-tile kernel (gemm_impl.h dec_lean_kernel, bit-identical to
  // gemm_dec_kernel) where its shape / epilogue table covers the launch; W_fm = the weight's
  // fragment-major copy (frag_major, same K split) when the runtime built one
  int lean = 0;
  const void* W_fm = nullptr;
  // lean path, fragment-major activations (fc1 → fc2): c_fm = write the output in the layout its
  // consumer (K = this N, lean_cfg split) reads; a_fm = A is in that layout for this launch's split
  int c_fm = 0, a_fm = 0;
  // lean residual writers: also the 16-bit rows in the fragment-major layout of the LN-fused consumers
  // (their A: a_fm with ln_a16 = this copy)
  void* out16_fm = nullptr;
  // LM head (greedy select, fragment-major embedding): the final LayerNorm of the rows in a launch of
  // its own into this scratch ([M][K] 16-bit, same arithmetic as the fused form: bit-identical), the
  // vocabulary walk then without it (tools/dec_kernel_bench: the fused LayerNorm cost each of the 512
  // walkers 10 µs of a 31 µs launch)
  void* ln_scratch = nullptr;
  // LDS-ring tiles (encoder GEMMs): tile order in bands of `raster` row panels, column tiles outer
  // within a band (0: row-major tile order)
  int raster = 0;
  // 16-bit encoder GEMMs: the ping-pong kernel (gemm_impl.h gemm_pp_kernel) where it covers the launch
  int pp = 0;
  // lean LN-fused cross-attention query (EPI 0): q'_h = W_k,hᵀ q_h in the same launch (kq_w = W_kt's
  // fragment-major copy, kq_out [M][kq_ld] = [M][H·d], heads in hs_H). kq_cnt: the launch's arrival
  // counters ([row blocks][hs_H], 64-bit, zeroed once at allocation, monotonic: 2^64 arrivals never wrap);
  // kq_err: a word set when a hand-off wait ran out its spin bound (the host reports it at synchronize).
  // Set only where the lean kernel takes the launch (gemm() throws otherwise).
  unsigned long long* kq_cnt = nullptr; int* kq_err = nullptr;
  const void* kq_w = nullptr; void* kq_out = nullptr; long kq_ld = 0;
  // profiling (stamps pass): the launch's first-workgroup start / last-workgroup end, recorded by the lean
  // kernel inside the replayed decode graph (common.h stamp_commit); null base: off
  struct Stamp* lstamp = nullptr;
};

void gemm(DType t, const GemmArgs& g, hipStream_t s);
constexpr int kLnfMaxK = 1280;   // widest K of the ring tiles' folded LayerNorm (GemmArgs::ln_wg)

// LayerNorm over rows of f32 x[M][d] → T y[M][d] (w, b f32).
void layernorm(DType t, const float* x, const float* w, const float* b, void* y, int M, int d,
               hipStream_t s);

// x[r][:] = emb[ids[r]][:] + pos_emb[*pos + r_pos][:] (f32 out), r_pos = r % rows_per_seq.
// stats: per-st_w-column partial sums (Σx, Σx²) of the new rows (16: the older skinny consumers; 32:
// the ring tiles' folded LayerNorm, GemmArgs::rst_in)
// x16fm: also the 16-bit rows in the fragment-major layout of the lean LN-fused projections (lean_cfg(d))
void embed(DType t, const void* emb, const void* pos_emb, const int* ids, const int* pos, float* x,
           float* stats, int M, int d, hipStream_t s, void* x16 = nullptr, int V = 1 << 30, int rps = 1, int st_w = 16,
           void* x16fm = nullptr);
// prefill: ids[r·np + t] = src[r·ld + *pos + t] (ld 0: one prefix row shared by every row)
void prefill_ids(int* ids, const int* src, int R, int np, int ld, const int* pos, hipStream_t s);
void add_i32(int* p, int v, hipStream_t s);   // *p += v (one thread)
// LM-head argmax partials per row: gemm_dec_kernel walks the vocabulary with kDecWalkers workgroups
// per row block and writes one partial per walker; the older skinny kernel one per 64 columns.
constexpr int kDecWalkers = 512;
bool gemm_dec_supported(DType t, int K);
int lm_head_partials(DType t, int K, int vocab, int walkers = kDecWalkers);

// Attention over heads of 64. q row for (b, i): q + (b·q_Sb + i)·ldq + h·64.
// key j of (b, h): k + b·k_sb + h·k_sh + j·k_sk (same strides for v).
// nkeys: if nkeys_dev != null → *nkeys_dev + nkeys_add (self-attention), else nkeys.
// Per-launch device time stamps for kernels replayed inside the decode hipGraph (see common.h).
constexpr int kStampSub = 64;
struct Stamp {
  unsigned long long* base = nullptr; const int* pos = nullptr; int stride = 0, idx = 0;
};

struct AttnArgs {
  const void* q = nullptr; long ldq = 0; long q_Sb = 0; int Sq = 1;
  const void* k = nullptr; const void* v = nullptr; long k_sb = 0, k_sh = 0, k_sk = 0;
  void* o = nullptr; long ldo = 0; long o_Sb = 0;
  int B = 0, H = 0;
  int nkeys = 0; const int* nkeys_dev = nullptr; int nkeys_add = 0;
  // split-KV (decode): nsplit key chunks per query row, partials [B·H·Sq][nsplit][66] f32, tickets
  // [B·H·Sq] int (zero-initialised; the combining chunk resets its ticket)
  int nsplit = 1; float* part = nullptr; int* ticket = nullptr;
  Stamp stamp;   // profiling (decode graph): per-launch start/end stamps
  int variant = 1;   // decode kernel variant (k_attn.hip launch_decode)
  // K/V row of query row b (decode kernels): phys ? phys[(row0 + b)·phys_ld + j] (beam search: the
  // cache row that computed key j) : (row0 + b) / b_div (beams sharing one clip's cross K/V)
  int row0 = 0, b_div = 1;
  const int* phys = nullptr; long phys_ld = 0;
  int causal = 0;    // decode kernels, Sq > 1 (prefill): query i sees the first nkeys(+dev) + i keys
  int q_log2 = 0;    // flash (encoder variant 6): q is pre-scaled by log2(e)
  int xcd_nqb = 0;   // flash, > 0: 1-D grid, the xcd_nqb query blocks of one (set, head) on one XCD
                     // (they share its K/V through that XCD's L2); requires B·H % 8 == 0
  int kv_rows = 0;   // > 0: K/V rows allocated per (row, head) — the one-token self-attention kernel
                     // loads the first keys before the device key count arrives, clamped to this
};
void attention_decode(DType t, const AttnArgs& a, hipStream_t s);   // VALU, any T, any Sq
bool attention_flash(DType t, const AttnArgs& a, hipStream_t s);    // MFMA encoder (16-bit T)

// Decoder cross-attention in encoder space (k_xenc.hip). Whisper's cross-attention key projection
// has no bias, so q_h·(enc W_kᵀ)_hᵀ = (W_k,hᵀ q_h)·encᵀ and Σ p·(enc W_vᵀ + b_v) = (Σ p·enc) W_vᵀ + b_v:
// the step streams the encoder output once per layer instead of the per-layer K and V.
constexpr int kXencMaxSplit = 16;
struct XencArgs {
  const void* enc = nullptr; long enc_sb = 0;   // [rows][S][D] model dtype, enc_sb elements per row
  const void* qp = nullptr;                     // [rows][H][D] q'_h = W_k,hᵀ q_h (q pre-scaled)
  int rows = 0, H = 0, D = 0, S = 0;
  int nsplit = 1;                               // key ranges per row (<= kXencMaxSplit)
  float* part = nullptr;                        // [rows][nsplit][H][D] Σ_j p_j enc_j (range-local max)
  float* ml = nullptr;                          // [rows][nsplit][H][2] (max, Σ p)
  Stamp stamp;
  int variant = 1;                              // 1 register chunk ring, 0 LDS-DMA chunk ring
  int row0 = 0, rows_per_enc = 1;               // row b reads encoder output (row0 + b) / rows_per_enc
  int fm = 0;                                   // enc in the fragment-major chunk layout (xenc_to_fm; variants 1, 2)
  // range partials in the model dtype, each normalised by its own Σ p (part then holds [rows][nsplit][H][D]
  // T values: half the bytes), the (max, Σ p) pairs in f32 as before. fm variants + xenc_merge_v only
  int part16 = 0;
  int merge_os = 1;          // xenc_merge_v_kernel: a head's 64 outputs over merge_os workgroups (1 or 2)
};
bool xenc_supported(DType t, int D);
// enc [B][S][D] → the fragment-major chunk layout of the register-ring kernel (xenc_fm_elems(B, S, D)
// elements: S rounded up to whole 32-key chunks, zero rows past S)
void xenc_to_fm(DType t, const void* src, void* dst, int B, int S, int D, hipStream_t s);
long xenc_fm_elems(int B, int S, int D);
void xenc_attention(DType t, const XencArgs& a, hipStream_t s);
// u[r][h·D + c] = (Σ_s w_s part[r][s][h][c]) / L  (model dtype; ldu elements per row)
void xenc_merge(DType t, const XencArgs& a, void* u, long ldu, hipStream_t s);
// merge + value projection fused (D % 128 == 0): o[row][h·64 + j] = W_v,h·u_h + b_v, T
// wv_fm (nullable): W_v in the fragment-major layout of frag_major(W_v, d, d, 1, d / 32) — each weight
// wave-instruction of the merge then reads 1 KiB contiguous
void xenc_merge_v(DType t, const XencArgs& a, const void* wv, const float* bv, void* o, long ldo, hipStream_t s,
                  const void* wv_fm = nullptr);

// log-mel front end
// dft3 (nullable): the table as three bf16 parts [3][416][416] — the DFT as split-bf16 MFMAs instead of f32
void logmel_power_mel(const float* pcm, long pcm_stride, int n_samples, int B, const float* dft, const void* dft3,
                      const int* mel_lo, const int* mel_hi, const float* mel_w, int n_mel,
                      float* mel_out, unsigned* clip_max, hipStream_t s);
void logmel_normalize(float* mel, const unsigned* clip_max, int B, int n_mel, hipStream_t s);
void mel_to_conv_input(DType t, const float* mel, int B, int n_mel, void* xt, long clip_stride,
                       hipStream_t s);

// greedy selection with bias-list boost (see csrc/k_select.hip for the semantics)
struct SelectArgs {
  const float* logits = nullptr; long ld = 0; int M = 0; int V = 0;
  float lam = 0.f; const uint32_t* root_bits = nullptr;
  const int* trans_off = nullptr; const int* trans_tok = nullptr; const int* trans_dst = nullptr;
  const int* root_child = nullptr;
  const int* st_depth = nullptr; const int* st_keep = nullptr;   // per automaton state
  int* state = nullptr; int* finished = nullptr;
  int* rowbase = nullptr;            // per row k - d of the new state (read by the next LM head)
  int eos = 0, pad = 0; int min_new = 0;
  int* step = nullptr;               // device counter of generated tokens (read + incremented)
  int* pos = nullptr;                // device decoder position (incremented)
  int* next_ids = nullptr; int* out_ids = nullptr; int out_ld = 0;
  float* part_val = nullptr; int* part_idx = nullptr; int nchunk = 0;
  int* all_done = nullptr;
  unsigned long long* ticket_unfin = nullptr;   // arrivals | unfinished << 32, zero between steps (reset by the last row)
  float* out_score = nullptr;        // optional: the chosen token's (boosted) logit per row (0 for finished rows)
  // the next step's embedding written by the finalize (emb non-null; DType dtype): x [M][d] f32 =
  // emb[tok] + pemb[min(pos + 1, n_pos - 1)], its T copy x16, the fragment-major T copy x16fm (fm_nw,
  // fm_kpw; nullable) and the per-st_w-column (Σx, Σx²) partials st (nullable) — embed()'s outputs bit
  // for bit, one launch fewer per step
  const void* emb = nullptr; const void* pemb = nullptr; int n_pos = 0, d = 0, dtype = 0;
  float* x = nullptr; void* x16 = nullptr; void* x16fm = nullptr; int fm_nw = 0, fm_kpw = 0;
  float* st = nullptr; int st_w = 16;
};
void select_greedy(const SelectArgs& a, hipStream_t s);          // vocabulary pass + finalize
void select_finalize(const SelectArgs& a, hipStream_t s);        // partials already written (fused LM head)
void advance_forced(int* next_ids, const int* forced, int M, int ld, int* pos, hipStream_t s);
void gather_col(int* dst, const int* src, int M, int ld, int col, hipStream_t s);

// Beam search (k_beam.hip): HF _beam_search with the A8 boost / MinNewTokens as log-prob processors.
// Rows r = b·nb + i (utterance b, running beam i); sequences hold generated tokens only.
constexpr int kMaxBeams = 8;
constexpr int kBeamMaxLen = 448;       // max_target_positions of every Whisper size
constexpr int kBeamMaxVocab = 53248;   // LDS boost bitmap
constexpr int kBeamChunks = 16;        // vocabulary chunks per row of the chunked beam top-K
struct BeamArgs {
  const float* logits = nullptr; long ld = 0; int V = 0;
  int B = 0, nb = 0, K = 0;            // utterances, beams, candidates kept per step (2·nb)
  int P = 0, Lt = 0, T = 0;            // prefix length, max total length, cache positions (phys row)
  int eos = 0, pad = 0, min_new = 0;
  float lam = 0.f, len_pen = 1.f;
  const uint32_t* root_bits = nullptr; const int* root_child = nullptr;
  const int* trans_off = nullptr; const int* trans_tok = nullptr; const int* trans_dst = nullptr;
  const int* st_depth = nullptr; const int* st_keep = nullptr;
  int* step = nullptr; int* pos = nullptr; int* all_done = nullptr; int* ticket = nullptr;
  int* next_ids = nullptr; int* state = nullptr;        // [R]
  float* run_sc = nullptr; int* run_seq = nullptr;      // [R], [R][Lt-P]
  int* phys = nullptr;                                  // [R][T] cache row of every key position
  float* cand_val = nullptr; int* cand_tok = nullptr;   // [R][nchunk][K] top-K per (row, vocabulary chunk)
  int nchunk = 1;                                       // vocabulary chunks per row (k_beam.hip beam_select)
  float* chunk_stats = nullptr;                         // [R][nchunk] (max, Σexp) of each chunk (nchunk > 1)
  float* fin_sc = nullptr; int* fin_done = nullptr; int* fin_len = nullptr; int* fin_seq = nullptr;  // [B·nb](·(Lt-P))
  int* flags = nullptr;                                 // [B][2]: heuristic unsatisfied, all K hit
  int* out_ids = nullptr; int out_ld = 0; int* out_len = nullptr;
  int* parent = nullptr;                                // [R] (nullable): the beam each running beam extends
};
void beam_init(const BeamArgs& a, hipStream_t s);
void beam_select(const BeamArgs& a, hipStream_t s);   // per-row top-K + per-utterance step
void beam_output(const BeamArgs& a, hipStream_t s);   // best finished sequence per utterance

// Bias-weighted cross entropy (k_loss.hip; models/whisper_medical.py:113-156).
struct WceArgs {
  const float* logits = nullptr; long ld = 0;          // [B·T][ld] f32, V columns used
  int B = 0, T = 0, V = 0;
  const int* labels = nullptr;                         // [B][T], -100 = ignore
  const int* spans = nullptr; const int* span_len = nullptr;   // [B][N][Lmax], [B][N] (0 = empty)
  int N = 0, Lmax = 0, use_spans = 0;
  float bias_weight = 1.f;
  float* per_token = nullptr;                          // [B·T] −logp[label]·w·valid
  float* loss = nullptr; int* count = nullptr;         // scalar loss, valid-label count (nullable)
};
void weighted_ce(const WceArgs& a, hipStream_t s);

// weight staging / repacking (k_weights.hip)
struct WeightView { long shape[4] = {1, 1, 1, 1}; long stride[4] = {0, 0, 0, 0}; };   // elements
void view_to_f32(DType t, const void* src, const WeightView& v, float* dst, hipStream_t s);   // dense f32
// dst[i0·t0 + i1·t1 + i2·t2] = T(scale · src[i0·s0 + i1·s1 + i2·s2]) over n0 × n1 × n2 (T = model dtype or f32)
struct RepackArgs { void* dst = nullptr; const float* src = nullptr; int n[3] = {1, 1, 1}; long s[3] = {0, 0, 0};
                    long t[3] = {0, 0, 0}; float scale = 1.f; };
void repack(DType t, const RepackArgs& a, hipStream_t s);
void count_diff(const float* a, const float* b, long n, int* count, hipStream_t s);   // b null: nonzeros
// u[n] = Σ_k γ_k W[n][k], c[n] = Σ_k β_k W[n][k] + bias[n] (the LayerNorm fold of gemm_impl.h LNF;
// gam null: γ = 1; bet / c null: no c)
void ln_fold(DType t, const void* W, int N, int K, const float* gam, const float* bet, const float* bias, float* u,
             float* c, hipStream_t s);

// Wg[n][k] = T(γ_k · W[n][k]) (the folded LayerNorm's weights)
void scale_cols(DType t, const void* W, int N, int K, const float* gam, void* Wg, hipStream_t s);
// Fragment-major copy of a 16-bit weight [N][K] (N % 16 == 0) for the lean decode projections
// (gemm_impl.h dec_lean_kernel, WFM): dst[ct][wave][ks][lane][8] = W[16·ct + lane % 16][wave·kpw·32 +
// ks·32 + 8·(lane / 16) + e], so every weight wave-instruction reads 1 KiB contiguous (the row-major
// MFMA B-fragment loads touch 16 rows × 64 B)
void frag_major(DType t, const void* W, int N, int K, int nw, int kpw, void* dst, hipStream_t s);
// (waves, k-steps per wave) of the lean decode projection at this K (false: not covered): the 16-bit
// rows of gemm_impl.h launch_dec_mf, so the lean and general decode kernels split K alike
inline bool lean_cfg(int K, int& nw, int& kpw) {
  switch (K) {
    case 64: nw = 2; kpw = 1; return true;
    case 512: nw = 4; kpw = 4; return true;
    case 768: nw = 4; kpw = 6; return true;
    case 1024: nw = 4; kpw = 8; return true;
    case 1280: nw = 8; kpw = 5; return true;
    case 2048: nw = 8; kpw = 8; return true;
    case 3072: nw = 8; kpw = 12; return true;
    case 4096: nw = 16; kpw = 8; return true;
    case 5120: nw = 16; kpw = 10; return true;
    default: return false;
  }
}
void fill_i32(int* p, int v, long n, hipStream_t s);
// dst[0..n) = host values, passed by value in the kernel arguments (stream-ordered, no host buffer
// lifetime or pageable-copy ordering to worry about)
void write_i32(int* dst, const int* host_src, int n, hipStream_t s);
// Per launch slot (kStampSub sub-slots each): add max(end) − min(start) to acc[0] (ticks) and 1 to
// acc[1] if the slot was used; then zero the n launch slots.
void stamp_reduce(unsigned long long* slots, long n, unsigned long long* acc, hipStream_t s);

}  // namespace wcb
