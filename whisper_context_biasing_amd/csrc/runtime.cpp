// libwcb host runtime: C-ABI entry points (include/wcb.h), weight repacking, workspaces, the
// encoder pipeline, the hipGraph-replayed greedy decode loop, the bias-list automaton builder and
// per-kernel time accounting.
//
// Maps onto the reference as follows:
//   wcb_log_mel   ↔ WhisperFeatureExtractor.__call__   (data_utils/data_loader.py:171-172)
//   wcb_encode    ↔ WhisperEncoder.forward             ([tf] modeling_whisper.py:592-646)
//   wcb_generate  ↔ model.generate(input_features, max_length) (scripts/evaluation.py:173-206,
//                   [tf] trainer_seq2seq.py:329, [tf] generation/utils.py:2783-2944 greedy loop)
//   wcb_forward   ↔ WhisperForConditionalGenerationWeightCE.forward (models/whisper_medical.py:45-111)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cxxabi.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <thread>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>
#include <cstdlib>
#include <deque>
#include <atomic>

#include "../../include/wcb.h"
#include "kernels.h"

using namespace wcb;

namespace {

struct WcbError : std::runtime_error {
  int code;
  WcbError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess)                                                                      \
      throw WcbError(WCB_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_));             \
  } while (0)
#define REQUIRE(c, msg)                                       \
  do {                                                        \
    if (!(c)) throw WcbError(WCB_ERR_ARG, std::string(msg)); \
  } while (0)

constexpr int kFrames = 3000, kNCol = 416, kNSamp = 480000;
constexpr int kXSplit = 8;   // max cross-attention key chunks per (row, head) (partials buffer size)

int esize(int dt) { return dt == WCB_F32 ? 4 : 2; }

// host f32 → device element bits
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    HIPCHK(hipMalloc(&p, b));
    // zeroed and complete before any (non-blocking) library stream can touch it
    HIPCHK(hipMemsetAsync(p, 0, b, nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));
    bytes = b;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename X> X* as() const { return reinterpret_cast<X*>(p); }
};

struct LayerW {
  void* qkv_w = nullptr; float* qkv_b = nullptr;   // [3d][d] (q rows pre-scaled by 1/8), bias (k = 0)
  void* o_w = nullptr; float* o_b = nullptr;
  float *ln1_w = nullptr, *ln1_b = nullptr;
  void* xq_w = nullptr; float* xq_b = nullptr;     // decoder cross-attention q (pre-scaled)
  void* xo_w = nullptr; float* xo_b = nullptr;
  float *lnx_w = nullptr, *lnx_b = nullptr;
  void* fc1_w = nullptr; float* fc1_b = nullptr;
  void* fc2_w = nullptr; float* fc2_b = nullptr;
  float *ln2_w = nullptr, *ln2_b = nullptr;
  // decoder, 16-bit: the pre-block LayerNorms folded into their consumers for rows > 64 (ring LNF,
  // gemm_impl.h): W' = W·diag(γ) (T), u = Σ_k W'[n][k], c = Σ_k β_k W[n][k] + bias, for QKV (ln1),
  // cross-q (lnx), fc1 (ln2)
  void *qkv_wg = nullptr, *xq_wg = nullptr, *fc1_wg = nullptr;
  float *ln1_u = nullptr, *ln1_c = nullptr, *lnx_u = nullptr, *lnx_c = nullptr, *ln2_u = nullptr, *ln2_c = nullptr;
  // encoder-space cross-attention (k_xenc.hip): W_k,hᵀ repacked [H][d][64], W_v [d][d], b_v
  void* xkt_w = nullptr; void* xv_w = nullptr; float* xv_b = nullptr;
  // decoder, 16-bit: fragment-major copies for the lean decode projections (kernels.h frag_major)
  void *qkv_fm = nullptr, *o_fm = nullptr, *xq_fm = nullptr, *xkt_fm = nullptr, *xo_fm = nullptr, *fc1_fm = nullptr,
       *fc2_fm = nullptr;
  void* xv_fm = nullptr;   // W_v for the greedy range merge (xenc_merge_v_kernel's A-fragment order)
  void *qkv_wgfm = nullptr, *xq_wgfm = nullptr, *fc1_wgfm = nullptr;   // folded weights fragment-major (beam_wide / beam_wfm)
};

struct ProfEntry {
  std::string name;
  int64_t launches = 0;
  double ms = 0, flops = 0, bytes = 0;
  const void* fn = nullptr;   // kernel of the class's first launch and its grid in threads
  long grid = 0;
};

}  // namespace

struct wcb_bias {
  int n_states = 1;
  int vocab = 0;
  uint64_t id = 0;                  // decode-graph cache key (never reused, unlike the address)
  wcb_handle* owner = nullptr;      // the handle whose decode graphs may hold these device buffers
  DevBuf root_bits, root_child, trans_off, trans_tok, trans_dst;
  DevBuf st_depth, st_keep;         // per state: trie depth, deepest completed phrase on its path
};

// lean decode projection classes stamped inside the replayed decode graph (stamps pass), by region
static const char* const kLeanStampClass[] = {"dec_xattn", "dec_qkv", "dec_out", "dec_xq", "dec_xo", "dec_fc1", "dec_fc2",
                                              "dec_kq"};
static int lean_stamp_region(const char* cls) {
  for (int r = 1; r < 8; ++r)
    if (!strcmp(cls, kLeanStampClass[r])) return r;
  return 0;
}

// Decode state of one in-flight generate call. Two contexts (one per cross-K/V buffer) let call
// i+1 decode on its own stream while call i is still decoding: two latency-bound step chains share
// the GPU instead of one.
struct DecCtx {
  static constexpr int kMaxSub = 8;             // row groups of <= 64 rows (beam search: B·nb rows)
  hipStream_t hs = nullptr;                     // decode stream of this context
  hipStream_t sub[kMaxSub] = {};                // row-group chains (fork/join inside the step graph)
  hipEvent_t ev_fork = nullptr, ev_join[kMaxSub] = {};
  int dec_B = 0, dec_T = 0;
  DevBuf kvself, dx, dx16, dx16fm, dh, dq, dqp, du, datt, dffn, dstats, drst, xpart, xml, xticket, logits, part_val, part_idx, ints,
      pids, outbuf, forced, beam;
  DevBuf kq_cnt;   // 64-bit arrival counters of the fused xq+kq launches [L][kMaxSub][4 row blocks][H] (monotonic)
  int nchunk = 64;
  hipGraphExec_t gexec = nullptr;               // captured decode step
  hipGraphExec_t gexec_k = nullptr;             // steps_per_graph consecutive decode steps in one graph
  int* done_h = nullptr;                        // pinned: the "all rows finished" step of the last 2 chunks
  hipEvent_t ev_poll[2] = {};
  std::string gkey;
};

struct wcb_handle {
  wcb_model_desc d{};
  DType dt = kBF16;
  int device = 0;
  std::string err;
  hipStream_t he = nullptr;   // front end + encoder + cross-K/V stream (overlaps the previous batch's decode)
  // Decode contexts in flight: call i decodes in context i % nctx from cross-K/V buffer i % nctx while
  // the encoder stream already works on the next call. Measured: 2 contexts, one chain each.
  static constexpr int kMaxCtx = 4;
  int nctx = 2;
  hipEvent_t ev_xkv[kMaxCtx] = {}, ev_dec[kMaxCtx] = {};   // cross-K/V buffer k written / decode reading it done
  int gen_count = 0;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  static constexpr int kMaxSub = DecCtx::kMaxSub;
  DecCtx dc[kMaxCtx];
  int n_sub = 1;   // row groups per decode step on concurrent streams (fork/join inside the graph);
                   // with two decode contexts in flight one chain each measured best
  // Cross-attention: one workgroup per (row, head) over all 1500 keys. Measured (tools/xattn_bench.py,
  // head-major K/V cycling 12 layers): split-KV hand-offs cost more than they hide at 16-32 rows.
  int xsplit = 1;
  // cross-attention kernel variant over precomputed K/V (k_attn.hip launch_decode), fixed at create
  // from the model — never from the batch, whose composition must not change a clip's tokens (the
  // two kernels sum in different orders): the single-pass kernel (1) for 20 heads (large-v3, C5:
  // 1076 -> 1110 audio-s/s), the two-pass kernel (0) otherwise (medium, C3: 2435 vs 2048 with 1)
  int xvariant = 0;
  // beam-search cross-attention on the flash kernel (16-bit, the rows of a clip grouped): key ranges
  // per (clip, head), merged by flash_merge_kernel. Fixed per handle (never from the batch). Measured
  // (audio-s/s, splits 1 / 2 / 4): C3 4491 / 4531 / 4452, C5 1405 / 1484 / 1485.
  int flash_split = 2;
  // the same with the clip's keys split over the 4 waves of one (clip, head) workgroup, merged in the
  // workgroup (option "beam_xattn" 1..3; 0, default = the flash kernel above, whose 4 waves split
  // 16-query blocks — with 5 beams three of them compute on padding, yet it measured as fast: the
  // launch streams 393 MB of K/V per layer at C3, ~5.3 TB/s, bandwidth- not compute-bound)
  int beam_xattn = 0;   // measured: C3 4.37 / 4.41 ms/token (1 / 0), C5 3.60 / 3.49: within noise / worse
  // decode rows > 64 (16-bit): pre-block LayerNorms folded into the ring-tile projections (option
  // "ln_fold" 1: γ folded into the weights, (μ, r) from the residual writers' per-32-column partial
  // sums, applied in the epilogue — no per-element work in the K loop, no LayerNorm launch) or a
  // LayerNorm launch before each projection (0). (Round 2's in-loop form — A scaled by γ and the row
  // sums accumulated inside the K loop — measured slower than the launch and is gone.)
  int ln_fold = 1;
  // greedy cross-attention (encoder space): range merge and W_v in one launch (option "merge_v";
  // C2 16,570 vs 16,259 audio-s/s for the two launches)
  int merge_v = 1;
  // greedy cross-attention: range partials in the model dtype, normalised per range (option "xpart16";
  // half the partial bytes the attention writes and the merge reads; (max, Σp) stay f32). Measured: C2
  // 19,607 / 19,555 vs 19,276 / 19,395 audio-s/s (interleaved, one box); the GPU suite (goldens, bf16
  // margin gates) green with it
  int xpart16 = 1;
  // greedy cross-attention query (<= 64 rows, encoder space, lean path): q'_h = W_k,hᵀ q_h inside the
  // LN-fused q_proj launch (option "xq_kq" 1; gemm_impl.h dec_lean_kernel FZ 2) or as a launch of its
  // own (0, default; bit-identical). Serialised, the fused launch is the faster (6.9 vs 4.4 + 3.0 µs);
  // inside the pipelined graph its in-launch hand-off stretches to 9.3 µs with the other chain and the
  // encoder beside it, and the C2 bench measured 19,084 (two launches) vs 18,999 (fused), mean of five
  // interleaved pairs
  int xq_kq = 0;
  // decode rows > 64: 64-deep K sub-tiles per ring stage of the 64x32 / 32x32 tiles (option "ring_kt",
  // 1 or 2; C5 1,594 -> 1,644 audio-s/s)
  int ring_kt = 2;
  // decode rows 65-96 (C5's 80 beam rows), K = d_model: out / xo / xq / fc1 on the wide single-burst tiles
  // (gemm_impl.h gemm_wide_kernel) instead of the ring tiles (option "beam_wide", set before finalize).
  // tools/beam_gemm_bench.py (80 rows, d = 1280, cold weights): out 6.3 -> 5.3 µs (16 x 32 tiles,
  // fragment-major W), fc1 13.5 -> 9.8 µs (32 x 32); QKV stays on the ring (7.5 vs 9.4); at C3's 320 rows
  // the ring tiles win every shape. C5 bench 2,478 / 2,485 vs 2,446 / 2,429 audio-s/s (interleaved)
  int beam_wide = 1;
  // decode rows > 64, ring tiles: the weights read from fragment-major copies (option "beam_wfm", set
  // before finalize: the folded QKV / xq / fc1 weights get such copies too) and the tile order (option
  // "beam_raster": bands of n row panels with the column tiles outer, so the row tiles sharing a weight
  // tile run on one XCD; 0 = row panels outer)
  int beam_wfm = 0;
  // <= 64 rows (greedy), the LN-fused lean projections (QKV, xq, fc1): the LayerNorm folded into the weights
  // (W·diag(γ) fragment-major, c, u: the beam tiles' algebra) instead of normalising the A rows in the kernel
  // (option "lean_fold", set before finalize). C2 bench 19,777 / 20,001 / 19,974 vs 19,527 / 19,553 / 19,692
  // audio-s/s (interleaved): the MFMAs start as soon as the rows land, the statistics ride the partial-tile
  // barrier — the in-kernel LayerNorm cost its launches ~1.1 µs each (xq 3.89 vs out 2.78 µs in-graph)
  int lean_fold = 1;
  // greedy cross query: the q projection and q'_h = W_k,hᵀ q_h in one launch, each workgroup recomputing its
  // head's q_h (gemm_impl.h dec_xqk_kernel; option "xqk"; needs lean_fold) instead of xq → kq: one launch
  // boundary less per layer, no hand-off. C2 20,423 / 20,431 / 20,382 vs 20,243 / 20,295 / 20,097 (interleaved)
  int xqk = 1;
  // q' column chunks per head of the fused cross query (option "xqk_chunks": 2, 4, 8, 16; C2: 4 within noise of
  // 8, 2 and 16 slower)
  int xqk_nch = 8;
  // greedy range merge + W_v (16-bit partials): a head's 64 outputs over 1 or 2 workgroups (option "merge_os";
  // 2 measured slower: C2 20,114 / 20,074 / 20,080 vs 20,325 / 20,343 / 20,300, interleaved)
  int merge_os = 1;
  // greedy LM head: column walkers per row block (option "lm_walkers", before finalize; = the argmax
  // partials per row select_finalize reduces). C2 (interleaved pairs): 256 walkers 20,464-20,644 vs 512
  // 20,353-20,395 audio-s/s; 128 and 1024 no better than 512, 384 equal to 256 — fewer walkers re-read and
  // re-normalise the rows fewer times, and the walk of ~13 tiles each still hides its weight stream
  int lm_walkers = 256;
  // log-mel DFT: the f32 products as six bf16 MFMA products of 3-part splits (hi, mid, lo; the dropped terms
  // below 2^-24 relative) instead of f32 MFMAs (option "mel_split")
  int mel_split = 0;
  // lean projections on 32-row workgroups wherever the chain has > 16 rows (option "lean_mf2"; default:
  // only the LN-fused N >= 2048 ones). Measured 2.7 % slower at C2 (19,803-19,948 vs 20,424-20,521)
  int lean_mf2 = 0;
  // beam top-K: each row's vocabulary in kBeamChunks chunks, one workgroup per (chunk, row) (option
  // "beam_chunks" 1) or one workgroup per row (0, default; k_beam.hip beam_select). Measured: C3 6,160 vs
  // 6,228, C5 2,517 vs 2,518 audio-s/s — the per-row kernel's 320 (80) long workgroups already run beside
  // the other decode context's launches, so spreading the scan over the chip only adds contention
  int beam_chunks = 0;
  int beam_raster = 0;
  // greedy LM head: the final LayerNorm in a launch of its own (option "lm_ln_split" 1) or inside the
  // column walk (0, default: with the f32 copies of the A rows no longer held across the statistics
  // barrier the fused walker is 22.46 vs 22.19 µs + the LayerNorm launch, tools/dec_kernel_bench.hip)
  int lm_ln_split = 0;
  // encoder flash attention tiling (option "enc_flash"): 2 = 32 queries per wave, 4 = 64 queries per
  // wave. Measured (tools/microbench.py, small / medium encoder shapes, µs): 2: 358 / 878, 4: 313 / 808
  // (3 / 4 LDS stages at 32 queries measured 328 / 887 and 399 / 1041: removed)
  int enc_flash_qw = 4;
  // Cross-attention formulation: 1 = encoder space (k_xenc.hip: the step streams the encoder output,
  // no cross-K/V precompute; 16-bit dtypes, d <= 1024), 0 = precomputed per-layer K/V (f32 "exact"
  // mode, large-v3). Fixed at create (WCB_XMODE overrides where supported).
  int xmode = 1;
  // beam search (num_beams > 1) reads precomputed per-clip cross-K/V (xmode 0) even when greedy uses
  // the encoder-space kernel: its per-row work is smaller and the beams of a clip share the K/V
  // (measured on C3, medium beam 5: 1805 vs 1414 audio-s/s). WCB_BEAM_XMODE=1 keeps encoder space.
  int beam_xmode = 0;
  // decoder rows per decode chain (WCB_GROUP_ROWS). One chain for every row count by default: the
  // beam configurations decode faster as one chain of 80-320-row launches than as 64-row chains on
  // parallel streams (measured: C3 1814 -> 2215, C5 864 -> 983 audio-s/s; profiles/r01c_sweep_grp_*)
  int group_rows = 512;
  // key ranges per row of the encoder-space kernel (rows x ranges workgroups). With 16-bit partials
  // (xpart16) measured C2 6: 19,496 / 19,581, 8: 19,356 / 19,301, 10: 18,246, 12: 18,743, 16: 18,120
  int xenc_split = 6;
  // the decode's copy of the encoder output in the fragment-major chunk layout (k_xenc.hip
  // xenc_fm_kernel): 1 KiB contiguous per load wave-instruction of the register-ring kernel, where the
  // row layout touches 16 rows x 64 B (option "xenc_fm"; variants 1 and 2; bit-identical)
  int xenc_fm = 1;
  int xenc_variant = 1; // attn_xenc kernel variant (k_xenc.hip)
  // decoder LayerNorm input of the fused LN projections: 1 = the T-typed copy of the residual stream
  // the producers write beside the f32 rows (half the bytes per projection workgroup; C2 decode 1.066
  // vs 1.110 ms/token), 0 = the f32 rows (f32 mode). WCB_LN16 overrides.
  int ln16 = 1;
  int vocab_pad = 0;    // LM-head rows padded to a multiple of 128 (zero rows): the MFMA tile path's N
  int steps_per_graph = 8;   // decode steps captured per replayed graph (option "steps_per_graph")
  // decode projections of <= 64 rows on dec_lean_kernel (gemm_impl.h; bit-identical to
  // gemm_dec_kernel, one kernel-argument round trip and one load burst per launch; option "lean")
  int lean = 1;
  // lean path: the residual writers (embedding, out / xo / fc2 projections) also write the 16-bit rows
  // fragment-major for the LayerNorm-fused consumers (QKV, xq, fc1); option "lean_x"
  int lean_x = 1;
  struct wcb_state* step_state = nullptr;   // the active step-wise decode (wcb_decode_begin), if any
  // encoder GEMM tile order (option "enc_raster"): bands of n row panels with the column tiles outer
  // (GemmArgs::raster; 0 = row-major). 8 measured best with the round-3 ring kernel (whisper-small:
  // QKV 185 -> 177, fc1 297 -> 281, out 118 -> 116 us, fc2 within noise; profiles/r03f_enc_gemm_bench.txt)
  int enc_raster = 8;
  // encoder GEMMs (option "enc_gemm"): the ping-pong kernel (gemm_impl.h gemm_pp_kernel), 256-wide tiles
  // and 192-wide where those leave fewer tile rounds (4, default: C2 out 90.4 -> 89.2, fc2 273.4 -> 261.2 µs
  // against the LDS-ring kernel's 256x192 tiles, tools/enc_bench.py gemm; the bench line within noise),
  // the LDS-ring kernel for those (1), or the LDS-ring kernel everywhere (0)
  int enc_gemm = 4;
  // decode projections on gemm_dec_kernel (K supported): the LayerNorm consumers compute their row
  // statistics from the rows they load, so the producers publish no per-16-column partial sums
  bool dec_gemm = false;
  std::map<std::string, DevBuf> staged;   // every parameter as a dense f32 device tensor until finalize
  std::vector<DevBuf> owned;
  bool ready = false;
  int dbg_enc_layers = -1;   // debug: run only this many encoder layers (-1 = all)
  // weights
  void *conv1_w = nullptr, *conv2_w = nullptr;
  float *conv1_b = nullptr, *conv2_b = nullptr, *enc_pos = nullptr;
  int k1pad = 0;
  std::vector<LayerW> enc, dec;
  float *enc_ln_w = nullptr, *enc_ln_b = nullptr, *dec_ln_w = nullptr, *dec_ln_b = nullptr;
  void* xkv_w = nullptr; float* xkv_b = nullptr;
  void *tok_emb = nullptr, *dec_pos = nullptr;
  void* tok_emb_fm = nullptr;   // 16-bit: fragment-major copy of tok_emb for the greedy LM head
  // mel tables
  DevBuf dft, dft3, mel_lo, mel_hi, mel_w, clip_max;
  // encoder workspace
  int enc_B = 0;
  DevBuf xt, hbuf, x, h, qkv, att, ffn, encout;
  // per decode context: cross-K/V (xmode 0) or the encoder output (xmode 1); buffer k is read by
  // decode context k while the encoder stream fills the next one
  DevBuf xkv2[kMaxCtx];
  // default (empty) bias automaton
  std::unique_ptr<wcb_bias> empty_bias;
  std::vector<wcb_bias*> biases;     // live automatons created on this handle (lifetime, wcb.h)
  // device error word: set by a kernel whose in-launch hand-off wait ran out its spin bound (common.h
  // group_arrive_wait); read and cleared by wcb_synchronize (and the blocking calls that wait anyway)
  DevBuf dev_err;
  // profiling
  bool prof = false, prof_stamps = false;
  std::vector<ProfEntry> prof_e;
  std::deque<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> prof_pending;
  std::vector<hipEvent_t> ev_pool;
  DevBuf stamps, stamp_acc;                   // decode device stamps (graph nodes): cross-attention + the lean projections
  // stamp regions per decode context: 0 the cross-attention, 1.. the lean projection classes
  static constexpr int kStampRegions = 8;
  unsigned long long* stamp_base(int buf, int region) {
    return stamps.as<unsigned long long>() + ((size_t)buf * kStampRegions + region) * stamp_slots() * 2 * kStampSub;
  }
  double xattn_bytes = 0, xattn_flops = 0;    // algorithmic work of the stamped launches
  long stamp_slots() const { return (long)d.n_text_ctx * d.n_layers * kMaxSub; }   // per context

  int H() const { return d.n_heads; }
  int S() const { return d.n_audio_ctx; }

  void* upload(const void* src, size_t bytes) {
    owned.emplace_back();
    owned.back().ensure(bytes);
    HIPCHK(hipMemcpy(owned.back().p, src, bytes, hipMemcpyHostToDevice));
    return owned.back().p;
  }
  float* upload_f(const std::vector<float>& v) { return reinterpret_cast<float*>(upload(v.data(), v.size() * 4)); }
  void* own(size_t bytes) {
    owned.emplace_back();
    owned.back().ensure(bytes);
    return owned.back().p;
  }
  // staged parameter `name` (f32 device), element count checked
  const float* W(const std::string& name, size_t expect) {
    auto it = staged.find(name);
    if (it == staged.end()) throw WcbError(WCB_ERR_STATE, "missing weight " + name);
    if (it->second.bytes != expect * 4)
      throw WcbError(WCB_ERR_ARG, "weight " + name + " has " + std::to_string(it->second.bytes / 4) +
                                      " elements, expected " + std::to_string(expect));
    return it->second.as<float>();
  }

  // ---------------------------------------------------------------- profiling helpers
  int prof_id(const char* name) {
    for (size_t i = 0; i < prof_e.size(); ++i)
      if (prof_e[i].name == name) return (int)i;
    prof_e.push_back(ProfEntry{name});
    return (int)prof_e.size() - 1;
  }
  hipEvent_t get_ev() {
    if (!ev_pool.empty()) { auto e = ev_pool.back(); ev_pool.pop_back(); return e; }
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    return e;
  }
  template <typename F>
  void timed(const char* name, double flops, double bytes, hipStream_t st, F&& f) {
    if (!prof) { f(); return; }
    const int id = prof_id(name);
    hipEvent_t a = get_ev(), b = get_ev();
    g_launch_timer = LaunchTimer{a, b, 0};   // kernel begin/end timestamps (kernels.h, WCB_LAUNCH)
    try {
      f();
    } catch (...) {
      g_launch_timer = LaunchTimer{};
      throw;
    }
    const int n = g_launch_timer.n;
    if (n && !prof_e[id].fn) {
      prof_e[id].fn = g_launch_timer.fn;
      prof_e[id].grid = g_launch_timer.grid;
    }
    g_launch_timer = LaunchTimer{};
    if (n == 0) {   // nothing launched (copies / memsets only): a zero-width interval
      HIPCHK(hipEventRecord(a, st));
      HIPCHK(hipEventRecord(b, st));
    }
    prof_e[id].launches += 1;
    prof_e[id].flops += flops;
    prof_e[id].bytes += bytes;
    prof_pending.push_back({id, {a, b}});
  }
  // an enclosing interval (e.g. the whole decode loop) from plain stream events: enqueue-to-completion,
  // used for totals only, never for a per-launch duration
  template <typename F>
  void timed_wall(const char* name, hipStream_t st, F&& f) {
    if (!prof) { f(); return; }
    const int id = prof_id(name);
    hipEvent_t a = get_ev(), b = get_ev();
    HIPCHK(hipEventRecord(a, st));
    f();
    HIPCHK(hipEventRecord(b, st));
    prof_e[id].launches += 1;
    prof_pending.push_back({id, {a, b}});
  }
  void prof_collect() {
    while (!prof_pending.empty()) {
      auto& p = prof_pending.front();
      HIPCHK(hipEventSynchronize(p.second.second));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, p.second.first, p.second.second));
      prof_e[p.first].ms += ms;
      ev_pool.push_back(p.second.first);
      ev_pool.push_back(p.second.second);
      prof_pending.pop_front();
    }
  }
};

namespace {

thread_local std::string g_err;
std::atomic<uint64_t> g_next_bias_id{1};

template <typename F>
int guarded(wcb_handle* h, F&& f) {
  try {
    f();
    return WCB_OK;
  } catch (const WcbError& e) {
    (h ? h->err : g_err) = e.what();
    return e.code;
  } catch (const std::exception& e) {
    (h ? h->err : g_err) = e.what();
    return WCB_ERR_ARG;
  }
}

// ---------------------------------------------------------------------------- mel tables
double hz_to_mel(double f) { return f >= 1000.0 ? 15.0 + std::log(f / 1000.0) * (27.0 / std::log(6.4)) : 3.0 * f / 200.0; }
double mel_to_hz(double m) { return m >= 15.0 ? 1000.0 * std::exp((std::log(6.4) / 27.0) * (m - 15.0)) : 200.0 * m / 3.0; }

// Slaney filters [201][n_mel] as [tf] audio_utils.py:638-729 (norm="slaney", mel_scale="slaney")
std::vector<double> mel_filters(int n_mel) {
  const int nf = 201;
  std::vector<double> mf(n_mel + 2), ff(n_mel + 2), fft(nf), out((size_t)nf * n_mel, 0.0);
  const double mmin = hz_to_mel(0.0), mmax = hz_to_mel(8000.0);
  for (int i = 0; i < n_mel + 2; ++i) {
    // np.linspace: start + i*step, last point exactly stop
    mf[i] = (i == n_mel + 1) ? mmax : mmin + i * ((mmax - mmin) / (n_mel + 1));
    ff[i] = mel_to_hz(mf[i]);
  }
  for (int k = 0; k < nf; ++k) fft[k] = (k == nf - 1) ? 8000.0 : k * (8000.0 / (nf - 1));
  for (int k = 0; k < nf; ++k)
    for (int m = 0; m < n_mel; ++m) {
      const double down = -(ff[m] - fft[k]) / (ff[m + 1] - ff[m]);
      const double up = (ff[m + 2] - fft[k]) / (ff[m + 2] - ff[m + 1]);
      const double v = std::max(0.0, std::min(down, up));
      out[(size_t)k * n_mel + m] = v * (2.0 / (ff[m + 2] - ff[m]));
    }
  return out;
}

}  // namespace

// ======================================================================================= C ABI
extern "C" {

const char* wcb_last_error(const wcb_handle* h) { return h ? h->err.c_str() : g_err.c_str(); }

int wcb_create(const wcb_model_desc* desc, int device, wcb_handle** out) {
  return guarded(nullptr, [&] {
    REQUIRE(desc && out, "null argument");
    REQUIRE(desc->d_model % 64 == 0 && desc->d_model / desc->n_heads == 64, "head_dim must be 64");
    REQUIRE(desc->dtype >= 0 && desc->dtype <= 2, "dtype");
    REQUIRE(desc->n_mel == 80 || desc->n_mel == 128, "n_mel must be 80 or 128");
    REQUIRE(desc->n_audio_ctx * 2 == kFrames, "n_audio_ctx must be 1500");
    HIPCHK(hipSetDevice(device));
    auto h = std::make_unique<wcb_handle>();
    h->d = *desc;
    h->dt = DType(desc->dtype);
    h->device = device;
    HIPCHK(hipStreamCreateWithPriority(&h->he, hipStreamNonBlocking, 0));
    // decode streams: created on first use (ensure_ctx_streams), one per decode context in use. HIP
    // maps streams onto a small pool of hardware queues (GPU_MAX_HW_QUEUES, 4 by default); a context
    // whose queue is shared with the caller's stream inherits the caller's cross-stream waits (the
    // sync_out of every front-end call), which serialised the two decode chains (measured: C2 step
    // 102-139 ms when the library's streams predated the caller's, 52 ms otherwise). Streams that are
    // never used take no queue.
    for (int ci = 0; ci < wcb_handle::kMaxCtx; ++ci) {
      DecCtx& D = h->dc[ci];
      HIPCHK(hipEventCreateWithFlags(&D.ev_fork, hipEventDisableTiming));
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&D.done_h), 2 * sizeof(int), hipHostMallocDefault));
      for (hipEvent_t& e : D.ev_poll) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      for (int i = 0; i < DecCtx::kMaxSub; ++i) HIPCHK(hipEventCreateWithFlags(&D.ev_join[i], hipEventDisableTiming));
    }
    for (int i = 0; i < wcb_handle::kMaxCtx; ++i) {
      HIPCHK(hipEventCreateWithFlags(&h->ev_xkv[i], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&h->ev_dec[i], hipEventDisableTiming));
    }
    HIPCHK(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming));
    h->xvariant = desc->n_heads >= 20 ? 1 : 0;
    h->xmode = xenc_supported(h->dt, desc->d_model) ? 1 : 0;
    h->beam_xmode = 0;
    if (h->dt == kF32) h->ln16 = 0;   // f32 "exact" mode: the copy would be the f32 rows themselves
    h->dec_gemm = gemm_dec_supported(h->dt, desc->d_model);
    // DFT table [416 cols][416 k]: col 2b = win·cos(2πbk/400), col 2b+1 = −win·sin(2πbk/400)
    std::vector<float> dft((size_t)kNCol * kNCol, 0.f);
    for (int c = 0; c < 402; ++c) {
      const int bin = c >> 1;
      for (int k = 0; k < 400; ++k) {
        const double win = 0.5 - 0.5 * std::cos(2.0 * M_PI * k / 400.0);
        const double ang = 2.0 * M_PI * (double)((long)bin * k % 400) / 400.0;
        dft[(size_t)c * kNCol + k] = (float)(win * ((c & 1) ? -std::sin(ang) : std::cos(ang)));
      }
    }
    h->dft.ensure(dft.size() * 4);
    HIPCHK(hipMemcpy(h->dft.p, dft.data(), dft.size() * 4, hipMemcpyHostToDevice));
    {   // the same table as three bf16 parts (hi, mid, lo: each the RNE bf16 of the remainder of the double
        // value): the split-bf16 DFT (k_logmel.hip SPLIT) multiplies with these
      auto bf = [](double v, double& back) -> uint16_t {
        const float f = (float)v;
        uint32_t u;
        std::memcpy(&u, &f, 4);
        u += 0x7fffu + ((u >> 16) & 1u);   // round to nearest even (finite values only)
        const uint16_t hbits = (uint16_t)(u >> 16);
        const uint32_t w = (uint32_t)hbits << 16;
        float g;
        std::memcpy(&g, &w, 4);
        back = g;
        return hbits;
      };
      std::vector<uint16_t> t3((size_t)3 * kNCol * kNCol, 0);
      for (int c = 0; c < 402; ++c) {
        const int bin = c >> 1;
        for (int k = 0; k < 400; ++k) {
          const double win = 0.5 - 0.5 * std::cos(2.0 * M_PI * k / 400.0);
          const double ang = 2.0 * M_PI * (double)((long)bin * k % 400) / 400.0;
          double r = win * ((c & 1) ? -std::sin(ang) : std::cos(ang)), back;
          for (int part = 0; part < 3; ++part) {
            t3[(size_t)part * kNCol * kNCol + (size_t)c * kNCol + k] = bf(r, back);
            r -= back;
          }
        }
      }
      h->dft3.ensure(t3.size() * 2);
      HIPCHK(hipMemcpy(h->dft3.p, t3.data(), t3.size() * 2, hipMemcpyHostToDevice));
    }
    const auto fb = mel_filters(desc->n_mel);
    std::vector<int> lo(desc->n_mel), hi(desc->n_mel);
    std::vector<float> w((size_t)desc->n_mel * 32, 0.f);
    for (int m = 0; m < desc->n_mel; ++m) {
      int a = -1, b = -1;
      for (int k = 0; k < 201; ++k)
        if ((float)fb[(size_t)k * desc->n_mel + m] != 0.f) { if (a < 0) a = k; b = k; }
      if (a < 0) { a = 0; b = -1; }
      REQUIRE(b - a + 1 <= 32, "mel filter wider than 32 bins");
      lo[m] = a;
      hi[m] = b + 1;
      for (int k = a; k <= b; ++k) w[(size_t)m * 32 + (k - a)] = (float)fb[(size_t)k * desc->n_mel + m];
    }
    h->mel_lo.ensure(lo.size() * 4);
    h->mel_hi.ensure(hi.size() * 4);
    h->mel_w.ensure(w.size() * 4);
    HIPCHK(hipMemcpy(h->mel_lo.p, lo.data(), lo.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->mel_hi.p, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->mel_w.p, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    // empty automaton (root only) so greedy without a bias list uses the same kernels
    auto eb = std::make_unique<wcb_bias>();
    eb->vocab = desc->vocab;
    const int nw = (desc->vocab + 31) / 32;
    eb->root_bits.ensure((size_t)nw * 4);
    eb->root_child.ensure((size_t)desc->vocab * 4);
    HIPCHK(hipMemsetAsync(eb->root_child.p, 0xff, (size_t)desc->vocab * 4, nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));
    std::vector<int> off = {0, 0};
    eb->trans_off.ensure(8);
    HIPCHK(hipMemcpy(eb->trans_off.p, off.data(), 8, hipMemcpyHostToDevice));
    eb->trans_tok.ensure(4);
    eb->trans_dst.ensure(4);
    eb->st_depth.ensure(4);   // root: depth 0, keep 0 (zeroed)
    eb->st_keep.ensure(4);
    h->empty_bias = std::move(eb);
    h->dev_err.ensure(4);
    *out = h.release();
  });
}

void wcb_destroy(wcb_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  for (wcb_bias* b : h->biases) b->owner = nullptr;   // still valid to destroy; no graph holds them now
  for (DecCtx& D : h->dc) {
    if (D.gexec) (void)hipGraphExecDestroy(D.gexec);
    if (D.gexec_k) (void)hipGraphExecDestroy(D.gexec_k);
    for (DevBuf* b : {&D.kvself, &D.dx, &D.dx16, &D.dx16fm, &D.dh, &D.dq, &D.dqp, &D.du, &D.datt, &D.dffn, &D.dstats, &D.drst, &D.xpart, &D.xml, &D.xticket,
                      &D.logits, &D.part_val, &D.part_idx, &D.ints, &D.outbuf, &D.forced, &D.beam, &D.kq_cnt})
      b->release();
    if (D.ev_fork) (void)hipEventDestroy(D.ev_fork);
    for (hipEvent_t e : D.ev_poll)
      if (e) (void)hipEventDestroy(e);
    if (D.done_h) (void)hipHostFree(D.done_h);
    for (int i = 0; i < DecCtx::kMaxSub; ++i) {
      if (D.ev_join[i]) (void)hipEventDestroy(D.ev_join[i]);
      if (D.sub[i]) (void)hipStreamDestroy(D.sub[i]);
    }
    if (D.hs) (void)hipStreamDestroy(D.hs);
  }
  for (auto& b : h->owned) b.release();
  for (DevBuf* b : {&h->dft, &h->dft3, &h->mel_lo, &h->mel_hi, &h->mel_w, &h->clip_max, &h->xt, &h->hbuf, &h->x, &h->h,
                    &h->qkv, &h->att, &h->ffn, &h->encout, &h->stamps, &h->stamp_acc, &h->dev_err})
    b->release();
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->ev_in) (void)hipEventDestroy(h->ev_in);
  if (h->ev_out) (void)hipEventDestroy(h->ev_out);
  if (h->he) (void)hipStreamDestroy(h->he);
  for (int i = 0; i < wcb_handle::kMaxCtx; ++i) {
    h->xkv2[i].release();
    if (h->ev_xkv[i]) (void)hipEventDestroy(h->ev_xkv[i]);
    if (h->ev_dec[i]) (void)hipEventDestroy(h->ev_dec[i]);
  }
  delete h;
}

namespace {
void quiesce(wcb_handle* h);
void drop_graphs(wcb_handle* h);
}  // namespace

int wcb_set_option(wcb_handle* h, const char* name, int value) {
  return guarded(h, [&] {
    REQUIRE(h && name, "bad argument");
    const std::string n = name;
    // An open step-wise decode carries device state across wcb_decode_step calls that the decode options
    // shaped (the next input's embedding and its fragment-major copy, the LayerNorm statistics the residual
    // writers published, the encoder-output layout): only the encoder-side and generate()-only options may
    // change under it (decode_contexts has its own check below).
    static const char* const kFreeWhileStepwise[] = {"decode_contexts", "enc_flash", "enc_gemm", "enc_raster",
                                                     "steps_per_graph", "kq_cnt_seed"};
    bool free_opt = false;
    for (const char* f : kFreeWhileStepwise) free_opt |= n == f;
    REQUIRE(free_opt || !h->step_state, "option " + n + ": a step-wise decode is active (wcb_decode_end first)");
    if (n == "xmode" || n == "beam_xmode") {
      REQUIRE(!h->ready, "option " + n + " selects the weight layouts: set it before wcb_finalize_weights");
      REQUIRE(value == 0 || value == 1, "option " + n + ": 0 or 1");
      // encoder space only where the kernel exists (16-bit, d <= 1024): elsewhere the K/V formulation
      if (n == "xmode") h->xmode = value && xenc_supported(h->dt, h->d.d_model);
      else h->beam_xmode = value && h->xmode;
      if (!h->xmode) h->beam_xmode = 0;
    } else if (n == "decode_contexts") {
      REQUIRE(value >= 1 && value <= wcb_handle::kMaxCtx, "option decode_contexts: 1..4");
      // the step-wise state owns context kMaxCtx-1: generate() may not cycle into it while it is open
      REQUIRE(!h->step_state || value < wcb_handle::kMaxCtx,
              "option decode_contexts: 4 while a step-wise decode is active (wcb_decode_end first)");
      h->nctx = value;
    } else if (n == "group_rows") {
      REQUIRE(value >= 16 && value <= 512, "option group_rows: 16..512");
      h->group_rows = value;
    } else if (n == "xenc_variant") {
      REQUIRE(value >= 0 && value <= 3, "option xenc_variant: 0..3");
      h->xenc_variant = value;
    } else if (n == "enc_flash") {
      REQUIRE(value == 2 || value == 4, "option enc_flash: 2 or 4");
      h->enc_flash_qw = value;
    } else if (n == "xenc_split") {
      REQUIRE(!h->ready, "option xenc_split: set before the weights are finalized");
      REQUIRE(value >= 1 && value <= kXencMaxSplit, "option xenc_split: 1..16");
      h->xenc_split = value;
    } else if (n == "lm_ln_split") {
      h->lm_ln_split = value != 0;
    } else if (n == "ring_kt") {
      REQUIRE(value == 1 || value == 2, "option ring_kt: 1 or 2");
      h->ring_kt = value;
    } else if (n == "kq_cnt_seed") {
      // test hook: every allocated arrival counter of the fused xq+kq launches set to 4·value (a generation
      // boundary of the 4-member groups), e.g. just below 2^31 or 2^32 to check that no counter width wraps
      REQUIRE(value >= 0, "option kq_cnt_seed: >= 0");
      quiesce(h);
      for (DecCtx& D : h->dc) {
        if (!D.kq_cnt.p) continue;
        std::vector<unsigned long long> v(D.kq_cnt.bytes / 8, 4ull * (unsigned long long)value);
        HIPCHK(hipMemcpy(D.kq_cnt.p, v.data(), v.size() * 8, hipMemcpyHostToDevice));
      }
    } else if (n == "steps_per_graph") {
      REQUIRE(value >= 1 && value <= 64, "option steps_per_graph: 1..64");
      h->steps_per_graph = value;
    } else if (n == "xenc_fm") {
      h->xenc_fm = value != 0;
    } else if (n == "xq_kq") {
      h->xq_kq = value != 0;
    } else if (n == "enc_gemm") {
      REQUIRE(value == 0 || value == 1 || value == 4 || value == 5, "option enc_gemm: 0, 1, 4 or 5");
      h->enc_gemm = value;
    } else if (n == "enc_raster") {
      REQUIRE(value >= 0 && value <= 64, "option enc_raster: 0..64");
      h->enc_raster = value;
    } else if (n == "lean") {
      // the lean path's fragment-major weight copies are built at finalize only when it is on
      REQUIRE(!h->ready, "option lean selects weight layouts: set it before wcb_finalize_weights");
      h->lean = value != 0;
    } else if (n == "lean_x") {
      h->lean_x = value != 0;
    } else if (n == "xpart16") {
      h->xpart16 = value != 0;
    } else if (n == "merge_v") {
      h->merge_v = value != 0;
    } else if (n == "ln_fold") {
      // the folded W·diag(γ) copies are built at finalize only when it is on
      REQUIRE(!h->ready, "option ln_fold selects weight layouts: set it before wcb_finalize_weights");
      h->ln_fold = value != 0;
    } else if (n == "lean_mf2") {
      h->lean_mf2 = value != 0;
    } else if (n == "mel_split") {
      h->mel_split = value != 0;
    } else if (n == "lm_walkers") {
      REQUIRE(!h->ready, "option lm_walkers sizes the argmax partials: set it before wcb_finalize_weights");
      REQUIRE(value == 128 || value == 192 || value == 256 || value == 384 || value == 512 || value == 1024,
              "option lm_walkers: 128, 192, 256, 384, 512 or 1024");
      h->lm_walkers = value;
    } else if (n == "merge_os") {
      REQUIRE(value == 1 || value == 2, "option merge_os: 1 or 2");
      h->merge_os = value;
    } else if (n == "xqk_chunks") {
      REQUIRE(value == 2 || value == 4 || value == 8 || value == 16, "option xqk_chunks: 2, 4, 8 or 16");
      h->xqk_nch = value;
    } else if (n == "xqk") {
      h->xqk = value != 0;
    } else if (n == "lean_fold") {
      REQUIRE(!h->ready, "option lean_fold selects weight layouts: set it before wcb_finalize_weights");
      h->lean_fold = value != 0;
    } else if (n == "beam_chunks") {
      h->beam_chunks = value != 0;
    } else if (n == "beam_wfm") {
      REQUIRE(!h->ready, "option beam_wfm selects weight layouts: set it before wcb_finalize_weights");
      h->beam_wfm = value != 0;
    } else if (n == "beam_raster") {
      REQUIRE(value >= 0 && value <= 64, "option beam_raster: 0..64");
      h->beam_raster = value;
    } else if (n == "beam_wide") {
      // the wide tiles read fragment-major copies of the folded xq / fc1 weights, built at finalize
      REQUIRE(!h->ready, "option beam_wide selects weight layouts: set it before wcb_finalize_weights");
      h->beam_wide = value != 0;
    } else if (n == "beam_xattn") {
      REQUIRE(value >= 0 && value <= 3, "option beam_xattn: 0..3");
      h->beam_xattn = value;
    } else if (n == "flash_split") {
      REQUIRE(value >= 1 && value <= kXSplit, "option flash_split: 1..8");
      h->flash_split = value;
    } else if (n == "xvariant") {
      REQUIRE(value >= 0 && value <= 5, "option xvariant: 0..5");
      h->xvariant = value;
    } else {
      throw WcbError(WCB_ERR_ARG, "unknown option " + n);
    }
    quiesce(h);
    drop_graphs(h);   // captured decode steps baked the old configuration in
  });
}

int wcb_set_weight(wcb_handle* h, const char* name, const float* data, const int64_t* shape, int ndim) {
  return guarded(h, [&] {
    REQUIRE(h && name && data && shape && ndim >= 1, "null argument");
    size_t n = 1;
    for (int i = 0; i < ndim; ++i) n *= (size_t)shape[i];
    HIPCHK(hipSetDevice(h->device));
    DevBuf& b = h->staged[name];
    b.release();
    b.ensure(n * 4);
    HIPCHK(hipMemcpy(b.p, data, n * 4, hipMemcpyHostToDevice));
  });
}

int wcb_load_weights(wcb_handle* h, const wcb_tensor_view* views, int n, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && (views || n == 0) && n >= 0, "bad argument");
    HIPCHK(hipSetDevice(h->device));
    const hipStream_t s = (hipStream_t)stream;
    for (int k = 0; k < n; ++k) {
      const wcb_tensor_view& v = views[k];
      REQUIRE(v.name && v.data && v.ndim >= 1 && v.ndim <= 4, "bad tensor view");
      REQUIRE(v.dtype == WCB_F32 || v.dtype == WCB_BF16 || v.dtype == WCB_F16, "tensor view dtype");
      WeightView w;   // right-aligned into 4 dims
      size_t cnt = 1;
      for (int i = 0; i < v.ndim; ++i) {
        REQUIRE(v.shape[i] >= 1, "tensor view shape");
        w.shape[4 - v.ndim + i] = v.shape[i];
        w.stride[4 - v.ndim + i] = v.stride[i];
        cnt *= (size_t)v.shape[i];
      }
      DevBuf& b = h->staged[v.name];
      b.release();
      b.ensure(cnt * 4);
      view_to_f32(DType(v.dtype), v.data, w, b.as<float>(), s);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));   // the borrowed views are not read after return
  });
}

int wcb_finalize_weights(wcb_handle* h) {
  return guarded(h, [&] {
    REQUIRE(h, "null handle");
    HIPCHK(hipSetDevice(h->device));
    const int d = h->d.d_model, L = h->d.n_layers, F = h->d.ffn, V = h->d.vocab, nm = h->d.n_mel, H = h->H();
    const size_t dd = (size_t)d * d, e = esize(h->d.dtype);
    HIPCHK(hipStreamSynchronize(h->he));
    const hipStream_t st = h->he;
    // owned model-dtype / f32 tensors built from the staged f32 parameters on the device
    auto rp = [&](bool f32, void* dst, const float* src, std::initializer_list<int> n, std::initializer_list<long> sv,
                  std::initializer_list<long> tv, float scale = 1.f) {
      RepackArgs a;
      a.dst = dst; a.src = src; a.scale = scale;
      std::copy(n.begin(), n.end(), a.n);
      std::copy(sv.begin(), sv.end(), a.s);
      std::copy(tv.begin(), tv.end(), a.t);
      repack(f32 ? kF32 : h->dt, a, st);
    };
    auto dense = [&](bool f32, const float* src, size_t cnt, float scale = 1.f) -> void* {
      void* p = h->own(cnt * (f32 ? 4 : e));
      rp(f32, p, src, {1, 1, (int)cnt}, {0, 0, 1}, {0, 0, 1}, scale);
      return p;
    };
    auto T_ = [&](const std::string& name, size_t cnt, float scale = 1.f) { return dense(false, h->W(name, cnt), cnt, scale); };
    auto F_ = [&](const std::string& name, size_t cnt, float scale = 1.f) {
      return reinterpret_cast<float*>(dense(true, h->W(name, cnt), cnt, scale));
    };
    DevBuf check;
    check.ensure(4);
    // conv1: W1[o][c][k] → [o][k·n_mel + c], K padded to a multiple of 64 with zeros
    h->k1pad = (3 * nm + 63) / 64 * 64;
    h->conv1_w = h->own((size_t)d * h->k1pad * e);   // zeroed on allocation (the K padding)
    rp(false, h->conv1_w, h->W("model.encoder.conv1.weight", (size_t)d * nm * 3), {d, 3, nm}, {(long)nm * 3, 1, 3},
       {(long)h->k1pad, nm, 1});
    h->conv1_b = F_("model.encoder.conv1.bias", d);
    // conv2: W2[o][c][k] → [o][k·d + c]
    h->conv2_w = h->own(dd * 3 * e);
    rp(false, h->conv2_w, h->W("model.encoder.conv2.weight", dd * 3), {d, 3, d}, {(long)d * 3, 1, 3}, {3L * d, d, 1});
    h->conv2_b = F_("model.encoder.conv2.bias", d);
    h->enc_pos = F_("model.encoder.embed_positions.weight", (size_t)h->S() * d);
    auto attn_qkv = [&](const std::string& p, LayerW& lw) {
      // q scaling head_dim^-0.5 = 0.125 (exact power of two: folding it is bit-identical)
      lw.qkv_w = h->own(3 * dd * e);
      rp(false, lw.qkv_w, h->W(p + "q_proj.weight", dd), {1, 1, (int)dd}, {0, 0, 1}, {0, 0, 1}, 0.125f);
      rp(false, (char*)lw.qkv_w + dd * e, h->W(p + "k_proj.weight", dd), {1, 1, (int)dd}, {0, 0, 1}, {0, 0, 1});
      rp(false, (char*)lw.qkv_w + 2 * dd * e, h->W(p + "v_proj.weight", dd), {1, 1, (int)dd}, {0, 0, 1}, {0, 0, 1});
      lw.qkv_b = reinterpret_cast<float*>(h->own(3 * (size_t)d * 4));   // k has no bias: zeros
      rp(true, lw.qkv_b, h->W(p + "q_proj.bias", d), {1, 1, d}, {0, 0, 1}, {0, 0, 1}, 0.125f);
      rp(true, lw.qkv_b + 2 * d, h->W(p + "v_proj.bias", d), {1, 1, d}, {0, 0, 1}, {0, 0, 1});
      lw.o_w = T_(p + "out_proj.weight", dd);
      lw.o_b = F_(p + "out_proj.bias", d);
    };
    auto mlp = [&](const std::string& p, LayerW& lw) {
      lw.ln1_w = F_(p + "self_attn_layer_norm.weight", d);
      lw.ln1_b = F_(p + "self_attn_layer_norm.bias", d);
      lw.ln2_w = F_(p + "final_layer_norm.weight", d);
      lw.ln2_b = F_(p + "final_layer_norm.bias", d);
      lw.fc1_w = T_(p + "fc1.weight", (size_t)F * d);
      lw.fc1_b = F_(p + "fc1.bias", F);
      lw.fc2_w = T_(p + "fc2.weight", (size_t)d * F);
      lw.fc2_b = F_(p + "fc2.bias", d);
    };
    auto zero_bias = [&](const std::string& name) {   // Whisper's encoder_attn.k_proj has no bias
      auto it = h->staged.find(name);
      if (it == h->staged.end()) return;
      count_diff(it->second.as<float>(), nullptr, (long)(it->second.bytes / 4), check.as<int>(), st);
    };
    h->enc.assign(L, LayerW{});
    h->dec.assign(L, LayerW{});
    const bool kv_stack = h->xmode == 0 || h->beam_xmode == 0;
    if (kv_stack) {
      h->xkv_w = h->own((size_t)2 * L * dd * e);
      h->xkv_b = reinterpret_cast<float*>(h->own((size_t)2 * L * d * 4));   // k rows: zero bias
    }
    for (int i = 0; i < L; ++i) {
      const std::string pe = "model.encoder.layers." + std::to_string(i) + ".";
      attn_qkv(pe + "self_attn.", h->enc[i]);
      mlp(pe, h->enc[i]);
      const std::string pd = "model.decoder.layers." + std::to_string(i) + ".";
      attn_qkv(pd + "self_attn.", h->dec[i]);
      mlp(pd, h->dec[i]);
      LayerW& lw = h->dec[i];
      lw.xq_w = T_(pd + "encoder_attn.q_proj.weight", dd, 0.125f);
      lw.xq_b = F_(pd + "encoder_attn.q_proj.bias", d, 0.125f);
      lw.xo_w = T_(pd + "encoder_attn.out_proj.weight", dd);
      lw.xo_b = F_(pd + "encoder_attn.out_proj.bias", d);
      lw.lnx_w = F_(pd + "encoder_attn_layer_norm.weight", d);
      lw.lnx_b = F_(pd + "encoder_attn_layer_norm.bias", d);
      const float* wk = h->W(pd + "encoder_attn.k_proj.weight", dd);
      const float* wv = h->W(pd + "encoder_attn.v_proj.weight", dd);
      const float* bv = h->W(pd + "encoder_attn.v_proj.bias", d);
      zero_bias(pd + "encoder_attn.k_proj.bias");
      if (h->xmode == 1) {
        // W_k,hᵀ: [H][d][64], element (h, c, i) = W_k[h·64 + i][c] (K = 64 contiguous for the MFMA)
        lw.xkt_w = h->own(dd * e);
        rp(false, lw.xkt_w, wk, {H, d, 64}, {64L * d, 1, d}, {(long)d * 64, 64, 1});
        lw.xv_w = dense(false, wv, dd);
        lw.xv_b = reinterpret_cast<float*>(dense(true, bv, d));
      }
      if (kv_stack) {   // cross K/V projection of every layer fused into one [2·L·d][d] weight: rows (l, k|v, d)
        rp(false, (char*)h->xkv_w + (size_t)(2 * i) * dd * e, wk, {1, 1, (int)dd}, {0, 0, 1}, {0, 0, 1});
        rp(false, (char*)h->xkv_w + (size_t)(2 * i + 1) * dd * e, wv, {1, 1, (int)dd}, {0, 0, 1}, {0, 0, 1});
        rp(true, h->xkv_b + (size_t)(2 * i + 1) * d, bv, {1, 1, d}, {0, 0, 1}, {0, 0, 1});
      }
    }
    if (h->dt != kF32) {
      for (int i = 0; i < L; ++i) {
        LayerW& lw = h->dec[i];
        // W' = W·diag(γ) rounded to T, u = Σ_k W'[n][k] (of the rounded W': the epilogue's μ·u then
        // removes exactly the mean the accumulator carries), c = Σ_k β_k W[n][k] + bias
        auto fold = [&](const void* W, int N, const float* gam, const float* bet, const float* bias, void*& Wg, float*& u,
                        float*& c) {
          Wg = h->own((size_t)N * d * e);
          u = reinterpret_cast<float*>(h->own((size_t)N * 4));
          c = reinterpret_cast<float*>(h->own((size_t)N * 4));
          scale_cols(h->dt, W, N, d, gam, Wg, st);
          ln_fold(h->dt, W, N, d, gam, bet, bias, u, c, st);          // c (u overwritten below)
          ln_fold(h->dt, Wg, N, d, nullptr, nullptr, nullptr, u, nullptr, st);
        };
        if (h->ln_fold) {   // (decode rows > 64 only; memory: QKV + xq + fc1 weights once more per layer)
          fold(lw.qkv_w, 3 * d, lw.ln1_w, lw.ln1_b, lw.qkv_b, lw.qkv_wg, lw.ln1_u, lw.ln1_c);
          fold(lw.xq_w, d, lw.lnx_w, lw.lnx_b, lw.xq_b, lw.xq_wg, lw.lnx_u, lw.lnx_c);
          fold(lw.fc1_w, F, lw.ln2_w, lw.ln2_b, lw.fc1_b, lw.fc1_wg, lw.ln2_u, lw.ln2_c);
        }
        // fragment-major copies for the lean decode projections (<= 64 rows): each weight wave-instruction
        // then reads 1 KiB contiguous (tools/dec_kernel_bench.hip: out 3.75 -> 3.16, fc2 8.39 -> 6.43 µs)
        auto fm = [&](const void* W, int N, int K) -> void* {
          int nw = 0, kpw = 0;
          if (!h->lean || !W || N % 16 || !lean_cfg(K, nw, kpw)) return nullptr;   // (lean path only)
          void* p = h->own((size_t)N * K * e);
          frag_major(h->dt, W, N, K, nw, kpw, p, st);
          return p;
        };
        lw.qkv_fm = fm(lw.qkv_w, 3 * d, d);
        lw.o_fm = fm(lw.o_w, d, d);
        lw.xq_fm = fm(lw.xq_w, d, d);
        lw.xo_fm = fm(lw.xo_w, d, d);
        lw.fc1_fm = fm(lw.fc1_w, F, d);
        lw.fc2_fm = fm(lw.fc2_w, d, F);
        if (lw.xkt_w) lw.xkt_fm = fm(lw.xkt_w, H * d, 64);
        if ((h->beam_wide || h->beam_wfm || h->lean_fold) && h->ln_fold) {   // the folded weights fragment-major
          lw.xq_wgfm = fm(lw.xq_wg, d, d);
          lw.fc1_wgfm = fm(lw.fc1_wg, F, d);
          if (h->beam_wfm || h->lean_fold) lw.qkv_wgfm = fm(lw.qkv_wg, 3 * d, d);
        }
        if (lw.xv_w && h->lean && h->dt != kF32 && d % 128 == 0 && d <= 1024) {   // 16 output rows per wave, all of K per wave
          lw.xv_fm = h->own((size_t)d * d * e);
          frag_major(h->dt, lw.xv_w, d, d, 1, d / 32, lw.xv_fm, st);
        }
      }
    }
    h->enc_ln_w = F_("model.encoder.layer_norm.weight", d);
    h->enc_ln_b = F_("model.encoder.layer_norm.bias", d);
    h->dec_ln_w = F_("model.decoder.layer_norm.weight", d);
    h->dec_ln_b = F_("model.decoder.layer_norm.bias", d);
    h->vocab_pad = (V + 127) / 128 * 128;   // zero rows past V (own() zeroes): logits columns ≥ V are 0
    h->tok_emb = h->own((size_t)h->vocab_pad * d * e);
    rp(false, h->tok_emb, h->W("model.decoder.embed_tokens.weight", (size_t)V * d), {1, 1, (int)((size_t)V * d)},
       {0, 0, 1}, {0, 0, 1});
    h->dec_pos = T_("model.decoder.embed_positions.weight", (size_t)h->d.n_text_ctx * d);
    if (h->dt != kF32) {   // the greedy LM head's column walk reads a fragment-major copy (zero rows past V)
      int nw = 0, kpw = 0;
      if (h->lean && lean_cfg(d, nw, kpw)) {
        h->tok_emb_fm = h->own((size_t)h->vocab_pad * d * e);
        frag_major(h->dt, h->tok_emb, h->vocab_pad, d, nw, kpw, h->tok_emb_fm, st);
      }
    }
    int bad_bias = 0, untied = 0;
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(&bad_bias, check.p, 4, hipMemcpyDeviceToHost));
    REQUIRE(bad_bias == 0, "encoder_attn.k_proj has no bias in Whisper ([tf] modeling_whisper.py:279)");
    if (h->staged.count("proj_out.weight")) {   // tied to the embedding (models/whisper_medical.py:14)
      HIPCHK(hipMemsetAsync(check.p, 0, 4, st));
      const size_t n = (size_t)V * d;
      count_diff(h->W("proj_out.weight", n), h->W("model.decoder.embed_tokens.weight", n), (long)n, check.as<int>(), st);
      HIPCHK(hipStreamSynchronize(st));
      HIPCHK(hipMemcpy(&untied, check.p, 4, hipMemcpyDeviceToHost));
      REQUIRE(untied == 0, "proj_out.weight must be tied to model.decoder.embed_tokens.weight");
    }
    HIPCHK(hipGetLastError());
    h->staged.clear();
    h->ready = true;
  });
}

}  // extern "C"

// ============================================================================== pipelines
namespace {

// caller stream → library stream `to` (inputs ready)
void sync_in(wcb_handle* h, void* stream, hipStream_t to) {
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipEventRecord(h->ev_in, (hipStream_t)stream));
  HIPCHK(hipStreamWaitEvent(to, h->ev_in, 0));
}
// library stream `from` → caller stream (outputs ready)
void sync_out(wcb_handle* h, void* stream, hipStream_t from) {
  HIPCHK(hipEventRecord(h->ev_out, from));
  HIPCHK(hipStreamWaitEvent((hipStream_t)stream, h->ev_out, 0));
  HIPCHK(hipGetLastError());
}
// the device error word (after the streams drained): a hand-off that ran out its bound means the launch's
// workgroups were not co-resident and its outputs are unsynchronised — an error, never silent
void check_dev_err(wcb_handle* h) {
  int e = 0;
  HIPCHK(hipMemcpy(&e, h->dev_err.p, 4, hipMemcpyDeviceToHost));
  if (e) {
    HIPCHK(hipMemset(h->dev_err.p, 0, 4));
    throw WcbError(WCB_ERR_HIP, "an in-launch hand-off wait timed out (workgroups not co-resident): outputs invalid");
  }
}
// drain every library stream (before any workspace reallocation)
void quiesce(wcb_handle* h) {
  HIPCHK(hipStreamSynchronize(h->he));
  for (DecCtx& D : h->dc)
    if (D.hs) HIPCHK(hipStreamSynchronize(D.hs));
}

void ensure_enc_ws(wcb_handle* h, int B) {
  if (B <= h->enc_B) return;
  quiesce(h);
  const size_t e = esize(h->d.dtype), d = h->d.d_model, S = h->S(), M = (size_t)B * S;
  h->xt.ensure(((size_t)B * (kFrames + 2) * h->d.n_mel + 256) * e);
  h->hbuf.ensure(((size_t)B * (kFrames + 1) * d + 256) * e);
  h->x.ensure(M * d * 4);
  h->h.ensure(M * d * e);
  h->qkv.ensure(M * 3 * d * e);
  h->att.ensure(M * d * e);
  h->ffn.ensure(M * h->d.ffn * e);
  h->encout.ensure(M * d * e);
  h->clip_max.ensure((size_t)B * 4);
  h->enc_B = B;
}

GemmArgs rowgemm(const void* A, long lda, const void* W, int M, int N, int K, void* out, long ldc) {
  GemmArgs g;
  g.A = A; g.lda = lda; g.W = W; g.ldw = K; g.M = M; g.N = N; g.K = K; g.out = out; g.ldc = ldc;
  return g;
}

// decode projections: always the skinny kernel (rows over grid.y), also for row groups > 64 rows
GemmArgs drow(const void* A, long lda, const void* W, int M, int N, int K, void* out, long ldc) {
  GemmArgs g = rowgemm(A, lda, W, M, N, K, out, ldc);
  g.skinny = 1;
  return g;
}

// algorithmic bytes of a decode-step GEMM: the weights once, the A rows, the written C rows
double gemm_bytes(const wcb_handle* h, const GemmArgs& g) {
  const double e = esize(h->d.dtype);
  const double a_bytes = g.ln_w && !g.ln_a16 ? 4.0 : e;
  const double c_bytes = g.out_f32 ? 4.0 : e;
  return (double)g.N * g.K * e + (double)g.M * g.K * a_bytes + (double)g.M * g.N * c_bytes;
}
// one decode-step GEMM launch; timed per class only in the eager profiling pass (events cannot
// bracket a node of a replayed graph)
void dgemm(wcb_handle* h, const char* cls, const GemmArgs& g, hipStream_t st) {
  h->timed(cls, 2.0 * g.M * g.N * g.K, gemm_bytes(h, g), st, [&] { gemm(h->dt, g, st); });
}

void run_gemm(wcb_handle* h, const char* cls, const GemmArgs& g0) {
  GemmArgs g = g0;
  g.raster = h->enc_raster;
  g.pp = h->enc_gemm;
  h->timed(cls, 2.0 * g.M * g.N * g.K, 0.0, h->he, [&] { gemm(h->dt, g, h->he); });
}

// WhisperEncoder.forward ([tf] modeling_whisper.py:592-646) on mel f32 [B][n_mel][3000]; the final
// LayerNorm writes [B][1500][d] to enc_out (h->encout when null)
void encode_impl(wcb_handle* h, const float* mel, int B, void* enc_out) {
  ensure_enc_ws(h, B);
  const int d = h->d.d_model, S = h->S(), nm = h->d.n_mel, H = h->H();
  const long M = (long)B * S;
  const size_t e = esize(h->d.dtype);
  const long xt_stride = (long)(kFrames + 2) * nm, hb_stride = (long)(kFrames + 1) * d;
  h->timed("mel_to_conv_input", 0, 0, h->he, [&] { mel_to_conv_input(h->dt, mel, B, nm, h->xt.p, xt_stride, h->he); });
  {  // conv1 + GELU → hbuf rows 1..3000 of every clip (row 0 = conv2's zero padding)
    GemmArgs g = rowgemm(h->xt.p, nm, h->conv1_w, B * kFrames, d, h->k1pad, (char*)h->hbuf.p + d * e, d);
    g.a_Mb = kFrames; g.a_strideB = xt_stride;
    g.c_Mb = kFrames; g.c_strideB = hb_stride;
    g.bias = h->conv1_b; g.act = 1;
    run_gemm(h, "enc_conv1", g);
  }
  {  // conv2 (stride 2) + GELU + positions → x (f32 residual stream)
    GemmArgs g = rowgemm(h->hbuf.p, 2L * d, h->conv2_w, (int)M, d, 3 * d, h->x.p, d);
    g.a_Mb = S; g.a_strideB = hb_stride;
    g.c_Mb = S; g.c_strideB = (long)S * d;   // c_Mb also indexes the position table
    g.bias = h->conv2_b; g.act = 1; g.addrow = h->enc_pos; g.out_f32 = 1;
    run_gemm(h, "enc_conv2", g);
  }
  const int nl = h->dbg_enc_layers >= 0 ? std::min(h->dbg_enc_layers, h->d.n_layers) : h->d.n_layers;
  for (int l = 0; l < nl; ++l) {
    const LayerW& w = h->enc[l];
    h->timed("layernorm", 0, M * d * (4.0 + e), h->he, [&] { layernorm(h->dt, h->x.as<float>(), w.ln1_w, w.ln1_b, h->h.p, (int)M, d, h->he); });
    GemmArgs q = rowgemm(h->h.p, d, w.qkv_w, (int)M, 3 * d, d, h->qkv.p, 3 * d);
    q.bias = w.qkv_b;
    run_gemm(h, "enc_qkv", q);
    AttnArgs a;
    a.q = h->qkv.p; a.ldq = 3 * d; a.q_Sb = S; a.Sq = S;
    a.k = (char*)h->qkv.p + d * e; a.v = (char*)h->qkv.p + 2 * d * e;
    a.k_sb = (long)S * 3 * d; a.k_sh = 64; a.k_sk = 3 * d;
    a.o = h->att.p; a.ldo = d; a.o_Sb = S; a.B = B; a.H = H; a.nkeys = S;
    a.variant = h->dt == kF32 ? 4 : h->enc_flash_qw;   // (f32: the VALU kernel below)
    h->timed("enc_attn", 4.0 * B * H * (double)S * S * 64, 0, h->he, [&] {
      if (!attention_flash(h->dt, a, h->he)) attention_decode(h->dt, a, h->he);
    });
    GemmArgs o = rowgemm(h->att.p, d, w.o_w, (int)M, d, d, h->x.p, d);
    o.bias = w.o_b; o.resid = h->x.as<float>(); o.out_f32 = 1;
    run_gemm(h, "enc_out", o);
    h->timed("layernorm", 0, M * d * (4.0 + e), h->he, [&] { layernorm(h->dt, h->x.as<float>(), w.ln2_w, w.ln2_b, h->h.p, (int)M, d, h->he); });
    GemmArgs f1 = rowgemm(h->h.p, d, w.fc1_w, (int)M, h->d.ffn, d, h->ffn.p, h->d.ffn);
    f1.bias = w.fc1_b; f1.act = 1;
    run_gemm(h, "enc_fc1", f1);
    GemmArgs f2 = rowgemm(h->ffn.p, h->d.ffn, w.fc2_w, (int)M, d, h->d.ffn, h->x.p, d);
    f2.bias = w.fc2_b; f2.resid = h->x.as<float>(); f2.out_f32 = 1;
    if (h->dt == kF16) f2.clamp = 65504.f - 1000.f;   // fp16 layer-output clamp (large-v3 fp16 config)
    run_gemm(h, "enc_fc2", f2);
  }
  void* dst = enc_out ? enc_out : h->encout.p;
  h->timed("layernorm", 0, M * d * (4.0 + e), h->he, [&] { layernorm(h->dt, h->x.as<float>(), h->enc_ln_w, h->enc_ln_b, dst, (int)M, d, h->he); });
}

// device ints of a decode context: I_TU = the greedy select's 64-bit arrival | unfinished counter (8-byte aligned)
enum { I_STEP = 0, I_POS = 1, I_DONE = 2, I_TICKET = 3, I_UNFIN = 4, I_TU = 6, I_NEXT = 16 };

void drop_graphs(wcb_handle* h) {
  for (DecCtx& D : h->dc) {
    if (D.gexec) (void)hipGraphExecDestroy(D.gexec);
    if (D.gexec_k) (void)hipGraphExecDestroy(D.gexec_k);
    D.gexec = D.gexec_k = nullptr;
    D.gkey.clear();
  }
}

// positions per prefill pass: up to kPrefillRows activation rows (bounds the row workspaces)
constexpr int kPrefillRows = 256;
int prefill_chunk(int R) { return std::max(1, kPrefillRows / std::max(R, 1)); }

// decode workspace: B decoder rows (clips x beams) reading `clips` encoder outputs; activation
// buffers for `rows` >= B rows (a prefill pass carries several positions per decoder row)
// contexts [c0, c1) (default: the generate() contexts 0 .. nctx-1; the step-wise decode state owns
// context kMaxCtx-1)
// the decode streams of contexts [c0, c1), created on first use at the highest priority (the decode
// chains are latency-bound and the next batch's encoder runs beside them: their workgroups dispatch
// ahead of encoder tiles); row-group streams only when n_sub > 1
hipStream_t make_dec_stream(wcb_handle* h) {
  hipStream_t s = nullptr;
  int prio_lo = 0, prio_hi = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  HIPCHK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio_hi));
  return s;
}

void ensure_ctx_streams(wcb_handle* h, int c0, int c1) {
  for (int ci = c0; ci < c1; ++ci) {
    DecCtx& D = h->dc[ci];
    if (D.hs && (h->n_sub <= 1 || D.sub[0])) continue;
    if (!D.hs) D.hs = make_dec_stream(h);
    for (int i = 0; i < DecCtx::kMaxSub && h->n_sub > 1; ++i)
      if (!D.sub[i]) D.sub[i] = make_dec_stream(h);
  }
}

void ensure_dec_ws(wcb_handle* h, int clips, int B, int T, int out_ld, int xmode, int rows = 0, int c0 = 0, int c1 = -1) {
  if (c1 < 0) c1 = h->nctx;
  ensure_ctx_streams(h, c0, c1);
  rows = std::max(rows, B);
  const size_t e = esize(h->d.dtype), d = h->d.d_model, L = h->d.n_layers, S = h->S();
  const DecCtx& D0 = h->dc[c1 - 1];   // every context of the range is sized together
  const size_t xbuf = xmode ? (size_t)xenc_fm_elems(clips, (int)S, (int)d) * e : 2 * L * (size_t)clips * S * d * e;
  const size_t need[] = {xbuf, 2 * L * (size_t)B * T * d * e, (size_t)rows * d * 4,
                         (size_t)rows * h->d.ffn * e, (size_t)B * h->vocab_pad * 4, (size_t)(I_NEXT + 4 * B + 16) * 4,
                         (size_t)B * out_ld * 4};
  const DevBuf* have[] = {&h->xkv2[c1 - 1], &D0.kvself, &D0.dx, &D0.dffn, &D0.logits, &D0.ints, &D0.outbuf};
  bool grow = false;
  for (int i = 0; i < 7; ++i) grow |= need[i] > have[i]->bytes;
  if (!grow && B <= D0.dec_B && T <= D0.dec_T) return;
  quiesce(h);
  drop_graphs(h);
  for (int ci = c0; ci < c1; ++ci) {
    DecCtx& D = h->dc[ci];
    h->xkv2[ci].ensure(need[0]);
    D.kvself.ensure(need[1]);
    D.dec_B = std::max(D.dec_B, B);
    D.dec_T = std::max(D.dec_T, T);
    D.dx.ensure((size_t)rows * d * 4);
    D.dx16.ensure((size_t)rows * d * e);
    D.dh.ensure((size_t)rows * d * e);
    D.dq.ensure((size_t)rows * d * e);
    D.datt.ensure((size_t)rows * d * e);
    // fragment-major copies: whole 16-row blocks, two blocks of slack (a 32-row workgroup past the rows)
    D.dffn.ensure(((size_t)(rows + 15) / 16 * 16 + 32) * h->d.ffn * e);
    D.dx16fm.ensure(((size_t)(rows + 15) / 16 * 16 + 32) * d * e);
    D.dstats.ensure((size_t)rows * (d / 16) * 2 * 4);
    D.drst.ensure((size_t)rows * (d / 32) * 2 * 4);
    D.xpart.ensure(std::max((size_t)rows * h->H() * kXSplit * 66, (size_t)rows * h->xenc_split * h->H() * d) * 4);
    D.xml.ensure((size_t)rows * h->xenc_split * h->H() * 2 * 4);
    D.dqp.ensure((size_t)rows * h->H() * d * e);
    D.du.ensure((size_t)rows * h->H() * d * e);
    D.xticket.ensure((size_t)rows * h->H() * 4);     // zeroed on allocation; combiners reset their slot
    D.kq_cnt.ensure((size_t)L * DecCtx::kMaxSub * 4 * h->H() * 8);   // zeroed on allocation, monotonic
    D.pids.ensure((size_t)rows * 4);
    D.logits.ensure((size_t)B * h->vocab_pad * 4);
    D.nchunk = lm_head_partials(h->dt, (int)d, h->d.vocab, h->lm_walkers);   // argmax partials per row of the LM head
    D.part_val.ensure((size_t)B * D.nchunk * 4);
    D.part_idx.ensure((size_t)B * D.nchunk * 4);
    D.ints.ensure(need[5]);
    D.outbuf.ensure(need[6]);
  }
}

// cross-attention K/V of every decoder layer from the encoder output (A4), once per clip:
// one GEMM [B·1500, d] × [2·L·d, d]ᵀ written head-split as [L·2][B][H][1500][64]
void cross_kv(wcb_handle* h, int B, int buf, const void* enc) {
  const int d = h->d.d_model, S = h->S(), L = h->d.n_layers;
  GemmArgs g = rowgemm(enc, d, h->xkv_w, B * S, 2 * L * d, d, h->xkv2[buf].p, 0);
  g.bias = h->xkv_b; g.mode = 1; g.hs_S = S; g.hs_H = h->H(); g.hs_B = B;
  run_gemm(h, "xkv_gemm", g);
}

// the encoder-space decode's encoder output (xmode 1) in decode buffer `buf` from the row layout
// [B][S][d] (fragment-major chunk layout when xenc_fm applies: the layout the register-ring kernel
// streams), on stream st
bool xenc_fm_on(const wcb_handle* h) { return h->xenc_fm && (h->xenc_variant == 1 || h->xenc_variant == 2); }
void fill_xenc(wcb_handle* h, int buf, const void* src, int B, hipStream_t st) {
  if (xenc_fm_on(h)) {
    h->timed("xenc_layout", 0, 2.0 * B * h->S() * h->d.d_model * esize(h->d.dtype), st,
             [&] { xenc_to_fm(h->dt, src, h->xkv2[buf].p, B, h->S(), h->d.d_model, st); });
  } else if (src != h->xkv2[buf].p) {
    HIPCHK(hipMemcpyAsync(h->xkv2[buf].p, src, (size_t)B * h->S() * h->d.d_model * esize(h->d.dtype),
                          hipMemcpyDeviceToDevice, st));
  }
}

struct StepCfg {
  int B, T, out_ld, buf;   // B: decoder rows (clips x beams); buf: which cross-K/V buffer the step reads
  bool lm_head, select;
  float* logits_out; long logits_ld;   // LM head destination
  const wcb_bias* bias; float lam; int min_new;
  const int* forced; int forced_ld;    // advance_forced source when !select
  int clips = 0, nb = 1;               // encoder outputs (0: B) and decoder rows per encoder output
  int xmode = 1;                       // cross-attention formulation of this call (wcb_handle::xmode)
  int host_pos = -1;                   // decoder position of this step when known on the host (eager)
  const int* phys = nullptr;           // beam search: cache row of every key position [B][T]
  const BeamArgs* beam = nullptr;      // beam search selection (replaces the greedy select)
  int rps = 1;                         // positions per decoder row in this pass (> 1: causal prefill)
  float* score_out = nullptr;          // greedy select: the chosen token's (boosted) logit per row (step-wise API)
  // greedy: the step's input embedding was written by the previous step's select_finalize (or by
  // step_embed before the first step), and this step's finalize writes the next one
  bool embedded = false;
};

// the residual's fragment-major copy applies (lean path): the lean LayerNorm table covers d, every
// LN consumer and residual writer has its weights' fragment-major copy, and the decode GEMMs publish
// no 16-column LayerNorm partials (the lean kernel writes none)
bool xfm_possible(const wcb_handle* h) {
  const int d = h->d.d_model;
  if (!h->lean || !h->lean_x || h->dt == kF32 || !h->ln16 || !h->dec_gemm) return false;
  if (d != 512 && d != 768 && d != 1024 && d != 1280) return false;
  for (const LayerW& w : h->dec)
    if (!w.qkv_fm || !w.o_fm || !w.xq_fm || !w.xo_fm || !w.fc1_fm || !w.fc2_fm) return false;
  return true;
}

// the folded LayerNorm of the > 64-row projections is available (16-bit, d a multiple of 32)
bool lnf_possible(const wcb_handle* h) {
  return h->ln_fold && h->dt != kF32 && h->d.d_model % 32 == 0 && h->d.d_model <= kLnfMaxK;
}

// Decoder layers + LM head for rows [b0, b0 + nb) of the batch on stream `st_`: WhisperDecoder.forward
// with a KV cache ([tf] modeling_whisper.py:690-795). Every position-dependent quantity is read on
// the device, so the launch sequence replays as a hipGraph. Row-indexed buffers are addressed with
// the row offset; the KV caches keep the full-batch layout ([kv][B][H][T][64]).
void decode_rows(wcb_handle* h, const StepCfg& c, int b0, int nb, int chain, hipStream_t st_) {
  DecCtx& D = h->dc[c.buf];
  const int d = h->d.d_model, S = h->S(), H = h->H(), L = h->d.n_layers, B = c.B, T = c.T;
  const size_t e = esize(h->d.dtype);
  int* ints = D.ints.as<int>();
  int* pos = ints + I_POS;
  // prefill (c.rps > 1): every decoder row carries rps consecutive positions, rows (row, position)
  // row-major; b0 / nb count decoder rows (KV-cache rows), r0 / M activation rows
  const int rps = c.rps > 1 ? c.rps : 1, r0 = b0 * rps, M = nb * rps;
  float* x = D.dx.as<float>() + (size_t)r0 * d;
  char* x16 = (char*)D.dx16.p + (size_t)r0 * d * e;       // T copy of x: the LN-fused A operand
  const void* lna = h->ln16 ? x16 : nullptr;
  const int nbk = d / 16;
  float* st = D.dstats.as<float>() + (size_t)r0 * nbk * 2;
  float* st_pub = h->dec_gemm ? nullptr : st;   // LN partial sums only for the older skinny consumers
  // > 64 rows, 16-bit, decode GEMMs supported: every residual writer is a ring tile that publishes
  // per-32-column (Σx, Σx²) of its rows (and the embedding does), so the LN consumers fold the
  // LayerNorm into their tiles (ln_fold) instead of a LayerNorm launch each
  float* rst = D.drst.as<float>() + (size_t)r0 * (d / 32) * 2;
  char* dq = (char*)D.dq.p + (size_t)r0 * d * e;
  char* datt = (char*)D.datt.p + (size_t)r0 * d * e;
  char* dffn = (char*)D.dffn.p + (size_t)r0 * h->d.ffn * e;
  // More than 64 activation rows (beam rows, prefill passes): a LayerNorm launch into dh, then the
  // MFMA tile GEMM — each weight tile read once per 128 rows, where the row-block decode kernel reads
  // the weights once per 16-32 rows. Grouped (block-diagonal) products stay on the decode kernel.
  // Only where the tile grid is wide enough to stream the weights from many CUs: the LM head, and the
  // N >= 2048 projections (QKV, fc1) at >= 192 rows (C3: 320 beam rows); the d-wide projections keep
  // the decode kernel (and keep writing the 16-bit residual copy its LayerNorm consumers read).
  const bool tiled = M > 64;
  const bool lnf_ok = tiled && h->dec_gemm && lnf_possible(h);
  // fragment-major operands (lean path): this chain's rows start a 16-row block of the copies
  const bool fm_ok = !tiled && h->lean && h->dt != kF32 && lna && r0 % 16 == 0 && M <= 64;
  // the residual's fragment-major copy (written by the embedding and every residual writer, read by
  // the LayerNorm-fused projections); decode_step's and prefill_step's embeddings write it for every
  // row whenever xfm_possible
  // (one position per row: the lean QKV appends one key per row)
  char* x16fm = fm_ok && rps == 1 && xfm_possible(h) ? (char*)D.dx16fm.p + (size_t)r0 * d * e : nullptr;
  char* dh = (char*)D.dh.p + (size_t)r0 * d * e;
  int cur_l = 0;   // the layer being issued (the lean launches' stamp slot)
  Stamp lst;
  auto proj = [&](const char* cls, GemmArgs g) {
    const bool lm = g.W == h->tok_emb;
    // > 64 rows, 16-bit: every non-grouped projection on the 32/64-row LDS-ring tiles (tile 2; C5's
    // 80 beam rows: 0.5 TB/s of weights on the row-block decode kernel, which holds A in registers
    // and re-reads the weights per 32 rows)
    const bool ring = h->dt != kF32 && !lm && !g.st_out;
    if (tiled && !g.a_grp_n && (lm || ring || (M >= 192 && g.N >= 2048))) {
      if (g.ln_w && ring && g.ln_u && g.ln_wg && lnf_ok && lna) {   // LayerNorm folded into the ring tiles
        g.A = lna; g.lda = d; g.W = g.ln_wg; g.ldw = g.K; g.W_fm = g.ln_wg_fm;
        g.bias = g.ln_c; g.ln_w = g.ln_b = nullptr; g.st_in = nullptr; g.ln_a16 = nullptr;
        g.rst_in = rst; g.rst_nb = d / 32;
      } else if (g.ln_w) {
        g.W_fm = nullptr;
        g.ln_u = nullptr;
        const float* xa = static_cast<const float*>(g.A);
        h->timed("dec_ln", 0, (double)M * d * (4.0 + e), st_,
                 [&] { layernorm(h->dt, xa, g.ln_w, g.ln_b, dh, M, d, st_); });
        g.A = dh; g.lda = d;
        g.ln_w = g.ln_b = nullptr; g.st_in = nullptr; g.ln_a16 = nullptr;
      }
      g.tile = ring ? 2 : 1; g.skinny = 0; g.ring_kt = h->ring_kt;
      if (ring && g.resid && g.out16 && lnf_ok) g.rst_out = rst;   // residual writer: stats for the next LN
      // <= 96 beam rows (C5's 80), K = d_model, fragment-major weights at hand: the wide single-burst
      // tiles for out / xo / xq (16 x 32) and fc1 (32 x 32); QKV keeps the ring (tools/beam_gemm_bench.py)
      g.a_fm = 0; g.c_fm = 0; g.out16_fm = nullptr;
      if (ring && h->beam_wide && M <= 96 && g.K == d && g.W_fm && !g.kv_out) {
        const std::string cn = cls;
        if (cn == "dec_out" || cn == "dec_xo" || cn == "dec_xq") g.wide = 12;
        else if (cn == "dec_fc1") g.wide = 22;
      }
      if (!g.wide && !h->beam_wfm) g.W_fm = nullptr;
      if (ring) g.raster = h->beam_raster;
    } else {
      g.lean = h->lean;   // <= 64 rows: the lean single-tile kernel where it covers the launch
      g.lean_fold = h->lean_fold && g.ln_w && g.ln_wg_fm && g.ln_u && g.ln_c;
      g.lean_mf2 = h->lean_mf2;
      const int region = h->prof_stamps ? lean_stamp_region(cls) : 0;
      if (region) {   // stamps pass: this launch's start / end inside the replayed graph
        lst.base = h->stamp_base(c.buf, region);
        lst.pos = pos; lst.stride = L * wcb_handle::kMaxSub; lst.idx = cur_l * wcb_handle::kMaxSub + chain;
        g.lstamp = &lst;
      }
    }
    dgemm(h, cls, g, st_);
  };
  const size_t cache_l = 2 * (size_t)B * H * T * 64;   // elements per layer (K then V)
  const int clips = c.clips ? c.clips : B;
  const size_t xkv_l = 2 * (size_t)clips * H * S * 64;
  for (int l = 0; l < L; ++l) {
    cur_l = l;
    const LayerW& w = h->dec[l];
    char* cache = (char*)D.kvself.p + (l * cache_l + (size_t)b0 * H * T * 64) * e;
    GemmArgs q = drow(x, d, w.qkv_w, M, 3 * d, d, dq, d);    // LayerNorm fused (f32 A rows)
    q.ln_w = w.ln1_w; q.ln_b = w.ln1_b; q.st_in = st; q.st_nb = nbk; q.ln_a16 = lna;
    q.bias = w.qkv_b; q.mode = 2; q.n_split = d; q.kv_out = cache; q.hs_B = B; q.hs_H = H; q.kv_T = T; q.pos = pos;
    q.kv_rps = rps; q.ln_u = w.ln1_u; q.ln_c = w.ln1_c; q.ln_wg = w.qkv_wg; q.W_fm = w.qkv_fm; q.ln_wg_fm = w.qkv_wgfm;
    if (x16fm) { q.ln_a16 = x16fm; q.a_fm = 1; }
    proj("dec_qkv", q);
    AttnArgs a;
    a.q = dq; a.ldq = d; a.q_Sb = rps; a.Sq = rps; a.causal = rps > 1;
    const char* cache0 = (char*)D.kvself.p + l * cache_l * e;   // K/V rows addressed absolutely
    a.k = cache0; a.v = cache0 + (size_t)B * H * T * 64 * e;
    a.k_sb = (long)H * T * 64; a.k_sh = (long)T * 64; a.k_sk = 64;
    a.row0 = b0; a.phys = c.phys; a.phys_ld = T;
    a.o = datt; a.ldo = d; a.o_Sb = rps; a.B = nb; a.H = H; a.nkeys_dev = pos; a.nkeys_add = 1;
    a.kv_rows = rps == 1 ? T : 0;
    {
      const double t_keys = c.host_pos >= 0 ? c.host_pos + 1 : 0;   // keys this step (eager pass)
      h->timed("dec_self_attn", 4.0 * nb * H * t_keys * 64, nb * H * t_keys * 128.0 * e, st_,
               [&] { attention_decode(h->dt, a, st_); });
    }
    GemmArgs o = drow(datt, d, w.o_w, M, d, d, x, d);
    o.bias = w.o_b; o.resid = x; o.out_f32 = 1; o.st_out = st_pub; o.st_nb = nbk; o.out16 = x16; o.W_fm = w.o_fm;
    o.out16_fm = x16fm;
    proj("dec_out", o);
    if (c.xmode == 1) {
      // cross attention in encoder space: q'_h = W_k,hᵀ q_h (block-diagonal GEMM, K = 64), one pass
      // over the encoder output per layer for all heads, range combine + W_v,h + b_v
      char* dqp = (char*)D.dqp.p + (size_t)r0 * H * d * e;
      GemmArgs xq = drow(x, d, w.xq_w, M, d, d, dq, d);
      xq.ln_w = w.lnx_w; xq.ln_b = w.lnx_b; xq.st_in = st; xq.st_nb = nbk; xq.ln_a16 = lna;
      xq.bias = w.xq_b; xq.ln_u = w.lnx_u; xq.ln_c = w.lnx_c; xq.ln_wg = w.xq_wg; xq.W_fm = w.xq_fm; xq.ln_wg_fm = w.xq_wgfm;
      if (x16fm) { xq.ln_a16 = x16fm; xq.a_fm = 1; }
      // q'_h = W_k,hᵀ q_h in the q_proj launch: the lean LN table's widths, both fragment-major copies
      const bool kqf = h->xq_kq && h->lean && fm_ok && w.xq_fm && w.xkt_fm && (d == 512 || d == 768 || d == 1024 || d == 1280);
      if (kqf) {
        xq.kq_w = w.xkt_fm; xq.kq_out = dqp; xq.kq_ld = (long)H * d; xq.hs_H = H;
        xq.kq_cnt = D.kq_cnt.as<unsigned long long>() + ((size_t)l * DecCtx::kMaxSub + chain) * 4 * H;
        xq.kq_err = h->dev_err.as<int>();
      }
      // q_h and q'_h in one launch without a hand-off (option xqk; the folded q_proj weights)
      const bool xqk = !kqf && h->xqk && h->lean && fm_ok && h->lean_fold && w.xq_wgfm && w.xkt_fm && w.lnx_u &&
                       H * 64 == d && (d == 512 || d == 768 || d == 1024 || d == 1280);
      if (xqk) { xq.xqk_wk = w.xkt_fm; xq.xqk_out = dqp; xq.hs_H = H; xq.xqk_nch = h->xqk_nch; }
      proj("dec_xq", xq);
      if (!kqf && !xqk) {
        GemmArgs kq = drow(dq, d, w.xkt_w, M, H * d, 64, dqp, (long)H * d);
        kq.a_grp_n = d; kq.a_grp_off = 64; kq.W_fm = w.xkt_fm;
        proj("dec_kq", kq);
      }
      XencArgs xa;
      xa.fm = xenc_fm_on(h);
      xa.enc = h->xkv2[c.buf].p; xa.enc_sb = xa.fm ? xenc_fm_elems(1, S, d) : (long)S * d;
      xa.row0 = r0; xa.rows_per_enc = c.nb * rps;   // beams (and prefill positions) of a clip share its encoder output
      xa.qp = dqp; xa.rows = M; xa.H = H; xa.D = d; xa.S = S; xa.nsplit = h->xenc_split;
      xa.variant = h->xenc_variant;
      xa.part = D.xpart.as<float>() + (size_t)r0 * h->xenc_split * H * d;
      xa.ml = D.xml.as<float>() + (size_t)r0 * h->xenc_split * H * 2;
      const bool fused_merge = h->merge_v && d % 128 == 0;
      xa.part16 = h->xpart16 && xa.fm && fused_merge;
      xa.merge_os = h->merge_os;
      if (h->prof_stamps) {
        xa.stamp.base = h->stamp_base(c.buf, 0);
        xa.stamp.pos = pos;
        xa.stamp.stride = L * wcb_handle::kMaxSub; xa.stamp.idx = l * wcb_handle::kMaxSub + chain;
      }
      // algorithmic bytes: every distinct clip's encoder output once (beams of a clip share it)
      h->timed("dec_xattn", 4.0 * M * H * (double)S * d, (double)nb / c.nb * S * d * e, st_,
               [&] { xenc_attention(h->dt, xa, st_); });
      if (fused_merge) {   // range merge + o_h = W_v,h u_h + b_v,h in one launch
        h->timed("dec_xmerge", 0, (double)M * H * d * h->xenc_split * (xa.part16 ? e : 4.0) + (double)d * d * e, st_,
                 [&] { xenc_merge_v(h->dt, xa, w.xv_w, w.xv_b, datt, d, st_, w.xv_fm); });
      } else {
        char* du = (char*)D.du.p + (size_t)r0 * H * d * e;
        h->timed("dec_xmerge", 0, (double)M * H * d * (h->xenc_split * 4.0 + e), st_,
                 [&] { xenc_merge(h->dt, xa, du, (long)H * d, st_); });
        GemmArgs vg = drow(du, (long)H * d, w.xv_w, M, d, d, datt, d);    // o_h = W_v,h u_h + b_v,h
        vg.a_grp_n = 64; vg.a_grp_off = d; vg.bias = w.xv_b;
        proj("dec_vg", vg);
      }
    } else {
      // cross attention over the precomputed encoder K/V
      GemmArgs xq = drow(x, d, w.xq_w, M, d, d, dq, d);
      xq.ln_w = w.lnx_w; xq.ln_b = w.lnx_b; xq.st_in = st; xq.st_nb = nbk; xq.ln_a16 = lna;
      xq.bias = w.xq_b; xq.ln_u = w.lnx_u; xq.ln_c = w.lnx_c; xq.ln_wg = w.xq_wg; xq.W_fm = w.xq_fm; xq.ln_wg_fm = w.xq_wgfm;
      if (x16fm) { xq.ln_a16 = x16fm; xq.a_fm = 1; }
      proj("dec_xq", xq);
      AttnArgs xa;
      const char* xkv = (const char*)h->xkv2[c.buf].p + l * xkv_l * e;
      xa.q = dq; xa.ldq = d; xa.q_Sb = 1; xa.Sq = 1;
      xa.k = xkv; xa.v = xkv + (size_t)clips * H * S * 64 * e;
      xa.row0 = r0; xa.b_div = c.nb * rps;     // beams (and prefill positions) of a clip share its cross K/V
      xa.k_sb = (long)H * S * 64; xa.k_sh = (long)S * 64; xa.k_sk = 64;
      xa.o = datt; xa.ldo = d; xa.o_Sb = 1; xa.B = M; xa.H = H; xa.nkeys = S;
      xa.nsplit = h->xsplit; xa.part = D.xpart.as<float>() + (size_t)r0 * H * kXSplit * 66;
      xa.ticket = D.xticket.as<int>() + (size_t)r0 * H;
      xa.variant = h->xvariant;   // fixed per handle: the same clip decodes alike in any batch
      if (h->prof_stamps) {
        xa.stamp.base = h->stamp_base(c.buf, 0);
        xa.stamp.pos = pos;
        xa.stamp.stride = L * wcb_handle::kMaxSub; xa.stamp.idx = l * wcb_handle::kMaxSub + chain;
      }
      // 16-bit, several rows per clip (beams, prefill positions), row group aligned to clips: the
      // MFMA flash kernel over (clip, head) blocks — each clip's K/V streamed once for all of its rows
      // (the per-row kernels re-read it once per beam). Chosen from the dtype and the decode shape,
      // never from the batch size.
      const int G = c.nb * rps;
      const bool grouped = h->dt != kF32 && G > 1 && r0 % G == 0 && M % G == 0;
      if (grouped) {
        xa.k = xkv + (size_t)(r0 / G) * xa.k_sb * e;
        xa.v = (const char*)xa.v + (size_t)(r0 / G) * xa.k_sb * e;
        xa.q_Sb = G; xa.Sq = G; xa.o_Sb = G; xa.B = M / G; xa.row0 = 0; xa.b_div = 1;
        xa.nsplit = h->flash_split; xa.ticket = nullptr;
        xa.part = D.xpart.as<float>() + (size_t)r0 * H * kXSplit * 66;
        if (h->beam_xattn && G <= 16) xa.variant = 6 + h->beam_xattn;   // keys split over the waves (attn_beam_kernel)
      }
      h->timed("dec_xattn", 4.0 * M * H * (double)S * 64, (double)nb / c.nb * H * S * 128.0 * e, st_, [&] {
        if (!grouped || !attention_flash(h->dt, xa, st_)) attention_decode(h->dt, xa, st_);
      });
    }
    GemmArgs xo = drow(datt, d, w.xo_w, M, d, d, x, d);
    xo.bias = w.xo_b; xo.resid = x; xo.out_f32 = 1; xo.st_out = st_pub; xo.st_nb = nbk; xo.out16 = x16; xo.W_fm = w.xo_fm;
    xo.out16_fm = x16fm;
    proj("dec_xo", xo);
    // MLP. Lean path (<= 64 rows, 16-bit): fc1 writes its output fragment-major in the layout fc2's
    // split of K = ffn reads (every A wave-instruction of fc2 then reads 1 KiB contiguous: its 98 KB of
    // activations per workgroup at d = 768 were the largest operand of the decode step)
    const bool afm = fm_ok && w.fc1_fm && w.fc2_fm &&
                     (d == 512 || d == 768 || d == 1024 || d == 1280) &&
                     (h->d.ffn == 2048 || h->d.ffn == 3072 || h->d.ffn == 4096 || h->d.ffn == 5120);
    GemmArgs f1 = drow(x, d, w.fc1_w, M, h->d.ffn, d, dffn, h->d.ffn);
    f1.ln_w = w.ln2_w; f1.ln_b = w.ln2_b; f1.st_in = st; f1.st_nb = nbk; f1.ln_a16 = lna;
    f1.bias = w.fc1_b; f1.act = 1; f1.ln_u = w.ln2_u; f1.ln_c = w.ln2_c; f1.ln_wg = w.fc1_wg; f1.W_fm = w.fc1_fm; f1.ln_wg_fm = w.fc1_wgfm;
    f1.c_fm = afm;
    if (x16fm) { f1.ln_a16 = x16fm; f1.a_fm = 1; }
    proj("dec_fc1", f1);
    GemmArgs f2 = drow(dffn, h->d.ffn, w.fc2_w, M, d, h->d.ffn, x, d);
    f2.bias = w.fc2_b; f2.resid = x; f2.out_f32 = 1; f2.st_out = st_pub; f2.st_nb = nbk; f2.out16 = x16; f2.W_fm = w.fc2_fm;
    f2.a_fm = afm;
    f2.out16_fm = x16fm;
    proj("dec_fc2", f2);
  }
  if (c.lm_head) {
    GemmArgs lm = drow(x, d, h->tok_emb, M, h->d.vocab, d, c.logits_out + (size_t)b0 * c.logits_ld, c.logits_ld);
    if (rps > 1) { lm.ldc = h->d.vocab; lm.c_Mb = rps; lm.c_strideB = c.logits_ld; }   // row (b, t) → b·ld + t·V
    // tile path: all vocab_pad columns (zero rows past V) into a logits buffer of that row stride
    const bool lm_tiled = tiled && rps == 1 && c.logits_ld >= h->vocab_pad;
    if (lm_tiled) lm.N = h->vocab_pad;
    lm.ln_w = h->dec_ln_w; lm.ln_b = h->dec_ln_b; lm.st_in = st; lm.st_nb = nbk; lm.ln_a16 = lna;
    if (h->lean) lm.W_fm = h->tok_emb_fm;
    if (h->lean && !tiled && rps == 1 && h->lm_ln_split) lm.ln_scratch = dh;   // the final LayerNorm in a launch of its own
    lm.out_f32 = 1;
    if (c.select && !c.beam) {   // argmax partials with the root boost + EOS mask fused into the LM head
      lm.walkers = h->lm_walkers;
      lm.sel_val = D.part_val.as<float>() + (size_t)b0 * D.nchunk;
      lm.sel_idx = D.part_idx.as<int>() + (size_t)b0 * D.nchunk;
      lm.sel_root_bits = c.bias->root_bits.as<uint32_t>(); lm.sel_lam = c.lam;
      lm.sel_rowbase = ints + I_NEXT + 3 * c.B + b0;   // per row k - d of its state (select_finalize)
      lm.sel_eos = h->d.eos_token_id; lm.sel_step = ints + I_STEP; lm.sel_min_new = c.min_new;
    }
    if (lm_tiled) {
      proj("lm_head", lm);
    } else {
      dgemm(h, "lm_head", lm, st_);
    }
  }
}

// One decode step for the whole batch: embedding, then the batch split into `h->n_sub` row groups
// whose layer chains run on separate streams (fork/join events, captured into the same graph) so
// the latency-bound projections of one group overlap the HBM-bound cross-attention of another;
// token selection (or teacher forcing) joins them.
// the decode step's input embedding (next_ids at the device position) into the residual rows, their
// 16-bit copies and LayerNorm partials
void step_embed(wcb_handle* h, const StepCfg& c) {
  DecCtx& D = h->dc[c.buf];
  const int d = h->d.d_model, B = c.B;
  int* ints = D.ints.as<int>();
  const bool r32 = h->dec_gemm && lnf_possible(h);   // 32-column stats for the folded LayerNorm (rows > 64)
  h->timed("dec_embed", 0, (double)B * d * (2.0 * esize(h->d.dtype) + 4), D.hs, [&] {
    embed(h->dt, h->tok_emb, h->dec_pos, ints + I_NEXT, ints + I_POS, D.dx.as<float>(),
          !h->dec_gemm ? D.dstats.as<float>() : r32 ? D.drst.as<float>() : nullptr, B, d, D.hs, D.dx16.p, h->d.vocab, 1,
          r32 ? 32 : 16, xfm_possible(h) ? D.dx16fm.p : nullptr);
  });
}

void decode_step(wcb_handle* h, const StepCfg& c) {
  DecCtx& D = h->dc[c.buf];
  const int d = h->d.d_model, B = c.B;
  int* ints = D.ints.as<int>();
  int* pos = ints + I_POS;
  int* next_ids = ints + I_NEXT;
  if (!c.embedded) step_embed(h, c);
  // rows per chain: the skinny projections split rows over grid.y, so a chain can take any number
  // of rows (WCB_GROUP_ROWS; more chains overlap latency, fewer re-read the weights less often)
  const int ngrp = (B + h->group_rows - 1) / h->group_rows;
  const int ns = std::max(ngrp, std::max(1, std::min(h->n_sub, B)));
  if (ns == 1 || !D.sub[0]) {        // one stream: row groups back to back
    for (int i = 0; i < ns; ++i) {
      const int b0 = (int)((long)B * i / ns), b1 = (int)((long)B * (i + 1) / ns);
      decode_rows(h, c, b0, b1 - b0, i, D.hs);
    }
  } else {
    HIPCHK(hipEventRecord(D.ev_fork, D.hs));
    for (int i = 0; i < ns; ++i) {
      const int b0 = (int)((long)B * i / ns), b1 = (int)((long)B * (i + 1) / ns);
      HIPCHK(hipStreamWaitEvent(D.sub[i], D.ev_fork, 0));
      decode_rows(h, c, b0, b1 - b0, i, D.sub[i]);
      HIPCHK(hipEventRecord(D.ev_join[i], D.sub[i]));
    }
    for (int i = 0; i < ns; ++i) HIPCHK(hipStreamWaitEvent(D.hs, D.ev_join[i], 0));
  }
  if (c.select && c.beam) {
    h->timed("dec_select", 0, (double)B * h->d.vocab * 4, D.hs, [&] { beam_select(*c.beam, D.hs); });
  } else if (c.select) {
    SelectArgs s;
    s.logits = c.logits_out; s.ld = c.logits_ld; s.M = B; s.V = h->d.vocab;
    s.lam = c.lam;
    s.root_bits = c.bias->root_bits.as<uint32_t>();
    s.trans_off = c.bias->trans_off.as<int>(); s.trans_tok = c.bias->trans_tok.as<int>();
    s.trans_dst = c.bias->trans_dst.as<int>(); s.root_child = c.bias->root_child.as<int>();
    s.st_depth = c.bias->st_depth.as<int>(); s.st_keep = c.bias->st_keep.as<int>();
    s.state = next_ids + B; s.finished = next_ids + 2 * B; s.rowbase = next_ids + 3 * B;
    s.eos = h->d.eos_token_id; s.pad = h->d.pad_token_id; s.min_new = c.min_new;
    s.step = ints + I_STEP; s.pos = pos; s.next_ids = next_ids;
    s.out_ids = D.outbuf.as<int>(); s.out_ld = c.out_ld;
    s.part_val = D.part_val.as<float>(); s.part_idx = D.part_idx.as<int>(); s.nchunk = D.nchunk;
    s.all_done = ints + I_DONE;
    s.ticket_unfin = reinterpret_cast<unsigned long long*>(ints + I_TU);
    s.out_score = c.score_out;
    if (c.embedded) {   // the next step's input embedding in the same launch (embed()'s outputs)
      const bool r32 = h->dec_gemm && lnf_possible(h);
      s.emb = h->tok_emb; s.pemb = h->dec_pos; s.n_pos = h->d.n_text_ctx; s.d = d; s.dtype = h->dt;
      s.x = D.dx.as<float>(); s.x16 = D.dx16.p;
      // (greedy decodes <= 64 rows: the decode-GEMM consumers compute their own LayerNorm statistics, so
      // the 32-column partials of the > 64-row folded path are not published; the older skinny consumers
      // still read 16-column ones)
      s.st = !h->dec_gemm ? D.dstats.as<float>() : nullptr; s.st_w = 16;
      (void)r32;
      int nw = 0, kpw = 0;
      if (xfm_possible(h) && lean_cfg(d, nw, kpw)) { s.x16fm = D.dx16fm.p; s.fm_nw = nw; s.fm_kpw = kpw; }
    }
    h->timed("dec_select", 0, (double)B * D.nchunk * 8, D.hs, [&] { select_finalize(s, D.hs); });
  } else {
    advance_forced(next_ids, c.forced, B, c.forced_ld, pos, D.hs);
  }
}

// Causal prefill of np positions (*pos .. *pos + np - 1) of every decoder row in ONE pass of the
// decoder (prompt tokens / teacher forcing): ids from src[row·ld + position] (ld 0: one prefix shared
// by every row), rows (row, position) row-major, the KV cache written at those positions, the
// self-attention causal over the cache, the cross-attention rows mapped to their clip; LM head on
// every row when c.lm_head. Advances *pos by np. Eager (its shapes change with np).
void prefill_step(wcb_handle* h, StepCfg c, int np, const int* src, int ld) {
  DecCtx& D = h->dc[c.buf];
  const int d = h->d.d_model, R = c.B, M = R * np;
  int* ints = D.ints.as<int>();
  int* pos = ints + I_POS;
  c.rps = np;
  c.select = false;
  c.phys = nullptr;   // prompt keys: every row's own cache row (beam_init's identity map)
  c.beam = nullptr;
  h->timed("dec_embed", 0, (double)M * d * (2.0 * esize(h->d.dtype) + 4), D.hs, [&] {
    prefill_ids(D.pids.as<int>(), src, R, np, ld, pos, D.hs);
    const bool r32 = h->dec_gemm && lnf_possible(h);
    embed(h->dt, h->tok_emb, h->dec_pos, D.pids.as<int>(), pos, D.dx.as<float>(), r32 ? D.drst.as<float>() : nullptr, M,
          d, D.hs, D.dx16.p, h->d.vocab, np, 32, xfm_possible(h) ? D.dx16fm.p : nullptr);
  });
  decode_rows(h, c, 0, R, 0, D.hs);
  add_i32(pos, np, D.hs);
}

// Beam-search state of decode context D (utterances B, nb beams each, R = B·nb rows): one buffer carved
// into [R] running / finished scores, finished flags and lengths, [R][Lg] running and finished
// sequences, [R][Tc] key map, [R][K] per-row candidates, [B][2] utterance flags, [R] parent beams.
// ensure_beam_buf sizes it (draining the streams first when it grows); beam_args carves it.
constexpr int kBeamBufs = 12;
void beam_words(int B, int nb, int Lg, int Tc, size_t* w) {
  const size_t R = (size_t)B * nb, K = 2 * (size_t)nb;
  const size_t C = kBeamChunks;   // candidate lists per (row, vocabulary chunk); chunk (max, Σexp)
  const size_t v[kBeamBufs] = {R, R, R, R, R * Lg, R * Lg, R * Tc, R * C * K, R * C * K, (size_t)B * 2, R, R * C * 2};
  std::copy(v, v + kBeamBufs, w);
}
void ensure_beam_buf(wcb_handle* h, DecCtx& D, int B, int nb, int Lg, int Tc) {
  size_t w[kBeamBufs], bytes = 0;
  beam_words(B, nb, Lg, Tc, w);
  for (size_t x : w) bytes += (x * 4 + 255) / 256 * 256;
  if (bytes > D.beam.bytes) { quiesce(h); D.beam.ensure(bytes); }
}
void beam_set_bias(BeamArgs& bm, const wcb_bias* bs) {
  bm.root_bits = bs->root_bits.as<uint32_t>(); bm.root_child = bs->root_child.as<int>();
  bm.trans_off = bs->trans_off.as<int>(); bm.trans_tok = bs->trans_tok.as<int>(); bm.trans_dst = bs->trans_dst.as<int>();
  bm.st_depth = bs->st_depth.as<int>(); bm.st_keep = bs->st_keep.as<int>();
}
// Lt: the total length cap (prefix + max new tokens, MaxLength), Tc: cache positions, Lg: max new tokens
BeamArgs beam_args(wcb_handle* h, DecCtx& D, int B, int nb, int P, int Lt, int Tc, int Lg, int min_new, float lam,
                   const wcb_bias* bs) {
  size_t w[kBeamBufs];
  beam_words(B, nb, Lg, Tc, w);
  char* p = (char*)D.beam.p;
  auto take = [&](int i) { char* q = p; p += (w[i] * 4 + 255) / 256 * 256; return q; };
  const int R = B * nb;
  int* ints = D.ints.as<int>();
  BeamArgs bm;
  bm.run_sc = (float*)take(0); bm.fin_sc = (float*)take(1); bm.fin_done = (int*)take(2); bm.fin_len = (int*)take(3);
  bm.run_seq = (int*)take(4); bm.fin_seq = (int*)take(5); bm.phys = (int*)take(6);
  bm.cand_val = (float*)take(7); bm.cand_tok = (int*)take(8); bm.flags = (int*)take(9); bm.parent = (int*)take(10);
  bm.chunk_stats = (float*)take(11);
  bm.nchunk = h->beam_chunks ? kBeamChunks : 1;
  bm.logits = D.logits.as<float>(); bm.ld = h->vocab_pad; bm.V = h->d.vocab;
  bm.B = B; bm.nb = nb; bm.K = 2 * nb; bm.P = P; bm.Lt = Lt; bm.T = Tc;
  bm.eos = h->d.eos_token_id; bm.pad = h->d.pad_token_id; bm.min_new = min_new;
  bm.lam = lam; bm.len_pen = 1.f;
  beam_set_bias(bm, bs);
  bm.step = ints + I_STEP; bm.pos = ints + I_POS; bm.all_done = ints + I_DONE; bm.ticket = ints + I_TICKET;
  bm.next_ids = ints + I_NEXT; bm.state = ints + I_NEXT + R;
  bm.out_ids = D.outbuf.as<int>(); bm.out_ld = Lg; bm.out_len = ints + I_UNFIN;
  return bm;
}

}  // namespace

extern "C" {

int wcb_log_mel(wcb_handle* h, const float* pcm, int B, int n_samples, int64_t pcm_stride, float* mel_out, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && pcm && mel_out && B > 0 && n_samples > 0, "bad argument");
    REQUIRE(pcm_stride >= std::min(n_samples, kNSamp), "pcm_stride < n_samples");
    if ((size_t)B * 4 > h->clip_max.bytes) { quiesce(h); h->clip_max.ensure((size_t)std::max(B, h->enc_B) * 4); }
    sync_in(h, stream, h->he);
    h->timed("log_mel", 0, (double)B * (std::min(n_samples, kNSamp) * 4.0 + h->d.n_mel * kFrames * 4.0 * 3), h->he, [&] {
      logmel_power_mel(pcm, (long)pcm_stride, n_samples, B, h->dft.as<float>(), h->mel_split ? h->dft3.p : nullptr,
                       h->mel_lo.as<int>(), h->mel_hi.as<int>(),
                       h->mel_w.as<float>(), h->d.n_mel, mel_out, h->clip_max.as<unsigned>(), h->he);
      logmel_normalize(mel_out, h->clip_max.as<unsigned>(), B, h->d.n_mel, h->he);
    });
    sync_out(h, stream, h->he);
  });
}

int wcb_encode(wcb_handle* h, const float* mel, int B, void* enc_out, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && mel && B > 0, "bad argument");
    if (!h->ready) throw WcbError(WCB_ERR_STATE, "weights not finalized");
    ensure_enc_ws(h, B);
    sync_in(h, stream, h->he);
    encode_impl(h, mel, B, enc_out);
    sync_out(h, stream, h->he);
  });
}

int wcb_generate(wcb_handle* h, const float* mel, int B, const wcb_gen_cfg* cfg, const wcb_bias* bias,
                 const int32_t* prefix, int prefix_len, int32_t* out_ids, int32_t* out_steps, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && cfg && out_ids && out_steps && B > 0, "bad argument");
    if (!h->ready) throw WcbError(WCB_ERR_STATE, "weights not finalized");
    const int nb = cfg->num_beams;
    REQUIRE(nb >= 1 && nb <= kMaxBeams, "num_beams must be in [1, 8]");
    const int R = B * nb;   // decoder rows: utterance b, beam i -> row b*nb + i
    REQUIRE(B <= 64, "batch > 64 per handle: split the batch");
    REQUIRE(R <= 64 * DecCtx::kMaxSub, "batch x num_beams > 512 rows per call: split the batch");
    REQUIRE(cfg->bias_boost >= 0.f, "bias_boost must be >= 0");
    REQUIRE(cfg->max_new_tokens >= 1, "max_new_tokens must be >= 1");
    REQUIRE(mel != nullptr, "mel is required");
    const int P = prefix ? prefix_len : 1;
    REQUIRE(P >= 1, "prefix_len must be >= 1");
    const int T = P + cfg->max_new_tokens;
    REQUIRE(T <= h->d.n_text_ctx + 1, "prefix + max_new_tokens exceeds max_target_positions");
    const wcb_bias* bs = bias ? bias : h->empty_bias.get();
    REQUIRE(bs == h->empty_bias.get() || bs->owner == h,
            "bias automaton was created on another handle (wcb_bias_create binds it to its handle)");
    REQUIRE(bs->vocab == h->d.vocab, "bias automaton built for another vocabulary");
    const bool fixed_len = cfg->min_new_tokens >= cfg->max_new_tokens;   // EOS masked: no host polling
    const int out_ld = cfg->max_new_tokens;
    const int Tc = std::min(T, h->d.n_text_ctx);
    if (nb > 1) {
      REQUIRE(cfg->max_new_tokens <= kBeamMaxLen && Tc <= kBeamMaxLen, "beam search: more than 448 positions");
      REQUIRE(cfg->bias_boost == 0.f || h->d.vocab <= kBeamMaxVocab, "beam search boost: vocabulary too large");
    }
    ensure_enc_ws(h, B);
    const int xm = nb > 1 ? h->beam_xmode : h->xmode;   // this call's cross-attention formulation
    ensure_dec_ws(h, B, R, Tc, out_ld, xm, P > 1 ? R * std::min(prefill_chunk(R), P - 1) : R);
    const int buf = h->gen_count++ % h->nctx;
    DecCtx& D = h->dc[buf];
    // beam state [R] / [R][max_new] / [R][Tc] / [R][K] / [B][2] in one buffer
    if (nb > 1) ensure_beam_buf(h, D, B, nb, cfg->max_new_tokens, Tc);
    // ---- encoder stream: front end → encoder → cross-K/V into buffer `buf` once the decode that
    //      last read that buffer has finished. It overlaps the previous call's decode.
    sync_in(h, stream, h->he);
    HIPCHK(hipStreamWaitEvent(h->he, h->ev_dec[buf], 0));
    if (xm == 1) {   // the decode reads the encoder output itself (re-laid out for the stream when xenc_fm)
      encode_impl(h, mel, B, xenc_fm_on(h) ? nullptr : h->xkv2[buf].p);
      if (xenc_fm_on(h)) fill_xenc(h, buf, h->encout.p, B, h->he);
    } else {
      encode_impl(h, mel, B, nullptr);
      h->timed_wall("xkv_gemm_total", h->he, [&] { cross_kv(h, B, buf, h->encout.p); });
    }
    HIPCHK(hipEventRecord(h->ev_xkv[buf], h->he));
    // ---- decode stream
    HIPCHK(hipStreamWaitEvent(D.hs, h->ev_xkv[buf], 0));
    int* ints = D.ints.as<int>();
    HIPCHK(hipMemsetAsync(ints, 0, (size_t)(I_NEXT + 4 * R) * 4, D.hs));
    if (prefix) {   // one prefix row shared by every decoder row (forced_ld = 0 below)
      if ((size_t)P * 4 > D.forced.bytes) { quiesce(h); D.forced.ensure((size_t)P * 4); }
      write_i32(D.forced.as<int>(), prefix, P, D.hs);
      gather_col(ints + I_NEXT, D.forced.as<int>(), R, 0, 0, D.hs);
    } else {
      fill_i32(ints + I_NEXT, h->d.decoder_start_token_id, R, D.hs);
    }
    BeamArgs bm;
    if (nb > 1) {
      bm = beam_args(h, D, B, nb, P, T, Tc, cfg->max_new_tokens, cfg->min_new_tokens, cfg->bias_boost, bs);
      beam_init(bm, D.hs);   // before the prefill: the self-attention reads keys through bm.phys
    }
    StepCfg sc{R, Tc, out_ld, buf, false, false, D.logits.as<float>(), (long)h->vocab_pad, bs, cfg->bias_boost,
               cfg->min_new_tokens, D.forced.as<int>(), 0};
    sc.clips = B;
    sc.nb = nb;
    sc.xmode = xm;
    if (nb > 1) { sc.phys = bm.phys; sc.beam = &bm; }
    // prompt positions 0 .. P-2 in causal prefill passes, then the last prompt token is the first
    // decode step's input
    for (int p0 = 0, np; p0 + 1 < P; p0 += np) {
      np = std::min(prefill_chunk(R), P - 1 - p0);
      prefill_step(h, sc, np, D.forced.as<int>(), 0);
    }
    if (P > 1) gather_col(ints + I_NEXT, D.forced.as<int>(), R, 0, P - 1, D.hs);
    sc.lm_head = true;
    sc.select = true;
    if (nb == 1) {   // greedy: every step's finalize embeds the next step's input; the first one here
      sc.embedded = true;
      step_embed(h, sc);
    }
    char key[256];
    snprintf(key, sizeof key, "%d/%d/%d/%d/%llu/%a/%d/%d/%d/%d", B, nb, Tc, out_ld, (unsigned long long)bs->id,
             cfg->bias_boost, cfg->min_new_tokens, h->n_sub, (int)h->prof_stamps, P);
    const int max_new = cfg->max_new_tokens;
    // per-launch HIP events (profiling bit 0) cannot bracket nodes of a replayed graph: eager launches
    const bool use_graph = cfg->use_graph && !h->prof;
    // The decode step replays as a hipGraph; steps_per_graph steps are captured into one graph so the
    // per-replay gap is paid once per chunk (every position-dependent value is read on the device, so
    // a multi-step graph is the single-step graph unrolled). Natural-EOS mode polls the device
    // "all finished" flag once per chunk.
    const int chunk = h->steps_per_graph;
    int done = 0, steps = 0;
    if (use_graph && (!D.gexec || D.gkey != key)) {
      if (D.gexec) { (void)hipGraphExecDestroy(D.gexec); D.gexec = nullptr; }
      if (D.gexec_k) { (void)hipGraphExecDestroy(D.gexec_k); D.gexec_k = nullptr; }
      const int ks[2] = {1, chunk};
      for (int ki = 0; ki < (chunk > 1 ? 2 : 1); ++ki) {   // the k-step graph only when it differs
        const int k = ks[ki];
        hipGraph_t graph;
        HIPCHK(hipStreamBeginCapture(D.hs, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < k; ++i) decode_step(h, sc);
        HIPCHK(hipStreamEndCapture(D.hs, &graph));
        HIPCHK(hipGraphInstantiate(k == 1 ? &D.gexec : &D.gexec_k, graph, nullptr, nullptr, 0));
        HIPCHK(hipGraphDestroy(graph));
      }
      D.gkey = key;
    }
    // Natural-EOS mode (reference decoding) polls the device "all finished" step one chunk behind:
    // chunk k+1 is queued before the host waits for chunk k's flag, so the GPU never idles on the
    // host (at most one chunk of extra steps after the last row finished; the output is cut at it).
    int pending = -1;   // slot of the chunk whose flag is in flight
    h->timed_wall("decode_loop", D.hs, [&] {
      while (steps < max_new) {
        const int n = std::min(chunk, max_new - steps);
        if (use_graph && n == chunk && D.gexec_k) {
          HIPCHK(hipGraphLaunch(D.gexec_k, D.hs));
        } else {
          for (int i = 0; i < n; ++i) {
            if (use_graph) {
              HIPCHK(hipGraphLaunch(D.gexec, D.hs));
            } else {
              sc.host_pos = P - 1 + steps + i;
              decode_step(h, sc);
            }
          }
        }
        steps += n;
        if (fixed_len) continue;
        const int slot = (pending + 1) & 1;
        HIPCHK(hipMemcpyAsync(D.done_h + slot, ints + I_DONE, 4, hipMemcpyDeviceToHost, D.hs));
        HIPCHK(hipEventRecord(D.ev_poll[slot], D.hs));
        if (pending >= 0) {
          HIPCHK(hipEventSynchronize(D.ev_poll[pending]));
          if (D.done_h[pending] > 0) { done = D.done_h[pending]; break; }
        }
        pending = slot;
      }
      if (!fixed_len && done <= 0 && pending >= 0) {
        HIPCHK(hipEventSynchronize(D.ev_poll[pending]));
        done = D.done_h[pending];
      }
    });
    if (done <= 0) done = steps;
    if (h->prof_stamps) {   // fold this call's cross-attention stamps into the device accumulator
      const double launches_rows = (double)(P - 1 + steps) * h->d.n_layers * R * h->H() * h->S();
      // algorithmic bytes: K and V (xmode 0) or the encoder output once for all heads (xmode 1), of
      // every distinct clip once (the beams of a clip share its rows: counted per clip, not per row)
      const double launches_clips = launches_rows / nb;
      h->xattn_bytes += xm ? launches_clips / h->H() * h->d.d_model * esize(h->d.dtype)
                                 : launches_clips * 64 * 2 * esize(h->d.dtype);
      h->xattn_flops += xm ? launches_rows * h->d.d_model * 4 : launches_rows * 64 * 4;
      for (int r = 0; r < wcb_handle::kStampRegions; ++r)
        stamp_reduce(h->stamp_base(buf, r), h->stamp_slots(), h->stamp_acc.as<unsigned long long>() + 2 * r, D.hs);
    }
    if (nb > 1) {   // best finished sequence of every utterance; its columns = the longest of them
      beam_output(bm, D.hs);
      HIPCHK(hipMemcpyAsync(out_ids, D.outbuf.p, (size_t)B * out_ld * 4, hipMemcpyDeviceToDevice, D.hs));
      if (cfg->async_out) {   // serving pipelines: every max_new column (pad past each best sequence), no
                              // host wait, so the next call's front end + encoder overlap this decode
        HIPCHK(hipEventRecord(h->ev_dec[buf], D.hs));
        *out_steps = max_new;
        return;
      }
      int olen = 0;
      HIPCHK(hipMemcpyAsync(&olen, ints + I_UNFIN, 4, hipMemcpyDeviceToHost, D.hs));
      HIPCHK(hipEventRecord(h->ev_dec[buf], D.hs));
      HIPCHK(hipStreamSynchronize(D.hs));
      if (h->xq_kq) check_dev_err(h);   // the in-launch hand-off's error word: outputs invalid if it is set
      *out_steps = std::min(olen, max_new);
      sync_out(h, stream, D.hs);
      return;
    }
    HIPCHK(hipMemcpyAsync(out_ids, D.outbuf.p, (size_t)B * out_ld * 4, hipMemcpyDeviceToDevice, D.hs));
    HIPCHK(hipEventRecord(h->ev_dec[buf], D.hs));
    *out_steps = std::min(done, max_new);
    if (!cfg->async_out) {
      // blocking calls with the in-launch hand-off on (option xq_kq) validate its error word before the ids
      // are handed out; async calls report it at wcb_synchronize
      if (h->xq_kq) { HIPCHK(hipStreamSynchronize(D.hs)); check_dev_err(h); }
      sync_out(h, stream, D.hs);
    }
  });
}

// ---- step-wise greedy decoding (SURVEY §8(b) wcb_decode_begin / wcb_decode_step): the decode step
// of wcb_generate, one token per call, on the decode context kMaxCtx-1 (its own stream and buffers,
// so generate() calls on contexts 0 .. nctx-1 are unaffected); eager launches (the caller inspects
// every step). One active state per handle.
struct wcb_state {
  wcb_handle* h = nullptr;
  int B = 0, P = 1, T = 0, steps = 0, max_new = 0, min_new = 0, xmode = 1;
  int fwd = 0;   // positions appended by wcb_forward_cached (a forward-cache state takes no decode steps)
  float lam = 0.f;
  uint64_t bias_id = 0;
  int nb = 1;    // beams per utterance (> 1: beam search, rows R = B·nb; the running beams in bm)
  BeamArgs bm;
};

// step-wise beam search: the beam path of wcb_generate one step per call (begin: cross-K/V of the
// given encoder output, beam state, causal prefill of the per-clip prefix on every beam row)
static void decode_begin_beams(wcb_handle* h, const void* enc, int B, int nb, const int32_t* prefix, int prefix_len,
                               int max_new_tokens, float bias_boost, int min_new_tokens, wcb_state** out, void* stream) {
  REQUIRE(h && enc && out && B > 0 && B <= 64, "bad argument (1 <= B <= 64, enc and out required)");
  if (!h->ready) throw WcbError(WCB_ERR_STATE, "weights not finalized");
  REQUIRE(nb >= 2 && nb <= kMaxBeams, "num_beams must be in [2, 8] (greedy: num_beams = 1)");
  const int R = B * nb;
  REQUIRE(R <= 64 * DecCtx::kMaxSub, "batch x num_beams > 512 rows: split the batch");
  REQUIRE(h->nctx < wcb_handle::kMaxCtx, "step-wise decoding needs a free decode context (decode_contexts <= 3)");
  REQUIRE(!h->step_state, "a step-wise decode is already active on this handle (wcb_decode_end first)");
  REQUIRE(bias_boost >= 0.f && min_new_tokens >= 0 && max_new_tokens >= 1,
          "bias_boost and min_new_tokens must be >= 0, max_new_tokens >= 1");
  REQUIRE(bias_boost == 0.f || h->d.vocab <= kBeamMaxVocab, "beam search boost: vocabulary too large");
  const int P = prefix ? prefix_len : 1;
  REQUIRE(P >= 1 && P < h->d.n_text_ctx, "prefix_len must be in [1, max_target_positions)");
  // generate(): the length cap is prefix + max_length, at most max_target_positions
  const int Lt = std::min(P + max_new_tokens, h->d.n_text_ctx), max_new = Lt - P, Tc = Lt;
  REQUIRE(Tc <= kBeamMaxLen, "beam search: more than 448 positions");
  const int ci = wcb_handle::kMaxCtx - 1;
  const int xm = h->beam_xmode;
  ensure_dec_ws(h, B, R, Tc, max_new, xm, P > 1 ? R * std::min(prefill_chunk(R), P - 1) : R, ci, ci + 1);
  DecCtx& D = h->dc[ci];
  ensure_beam_buf(h, D, B, nb, max_new, Tc);
  sync_in(h, stream, D.hs);
  if (xm == 1) {
    fill_xenc(h, ci, enc, B, D.hs);
  } else {
    sync_in(h, stream, h->he);
    cross_kv(h, B, ci, enc);                        // on the encoder stream
    HIPCHK(hipStreamSynchronize(h->he));
  }
  int* ints = D.ints.as<int>();
  HIPCHK(hipMemsetAsync(ints, 0, (size_t)(I_NEXT + 4 * R) * 4, D.hs));
  if (prefix) {   // per-clip prefixes [B][P] (host) on every beam row of the clip: [R][P]
    std::vector<int32_t> rows((size_t)R * P);
    for (int r = 0; r < R; ++r) std::copy(prefix + (size_t)(r / nb) * P, prefix + (size_t)(r / nb + 1) * P, rows.begin() + (size_t)r * P);
    if (rows.size() * 4 > D.forced.bytes) { quiesce(h); D.forced.ensure(rows.size() * 4); }
    HIPCHK(hipMemcpyAsync(D.forced.p, rows.data(), rows.size() * 4, hipMemcpyHostToDevice, D.hs));
    HIPCHK(hipStreamSynchronize(D.hs));   // pageable host source
  } else {
    fill_i32(ints + I_NEXT, h->d.decoder_start_token_id, R, D.hs);
  }
  // owned until the device work below succeeded (HIPCHK throws through here)
  std::unique_ptr<wcb_state> st(new wcb_state);
  st->h = h; st->B = B; st->P = P; st->T = Tc; st->max_new = max_new; st->min_new = min_new_tokens;
  st->xmode = xm; st->lam = bias_boost; st->nb = nb;
  st->bm = beam_args(h, D, B, nb, P, Lt, Tc, max_new, min_new_tokens, bias_boost, h->empty_bias.get());
  beam_init(st->bm, D.hs);   // before the prefill: the self-attention reads keys through the key map
  StepCfg sc{R, Tc, max_new, ci, false, false, D.logits.as<float>(), (long)h->vocab_pad, h->empty_bias.get(),
             bias_boost, min_new_tokens, D.forced.as<int>(), P};
  sc.clips = B;
  sc.nb = nb;
  sc.xmode = xm;
  sc.phys = st->bm.phys;
  for (int p0 = 0, np; p0 + 1 < P; p0 += np) {
    np = std::min(prefill_chunk(R), P - 1 - p0);
    prefill_step(h, sc, np, D.forced.as<int>(), P);
  }
  if (prefix) gather_col(ints + I_NEXT, D.forced.as<int>(), R, P, P - 1, D.hs);
  HIPCHK(hipStreamSynchronize(D.hs));
  h->step_state = st.release();
  *out = h->step_state;
  sync_out(h, stream, D.hs);
}

int wcb_decode_begin(wcb_handle* h, const void* enc, int B, int num_beams, const int32_t* prefix, int prefix_len,
                     float bias_boost, int min_new_tokens, wcb_state** out, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && enc && out && B > 0 && B <= 64, "bad argument (1 <= B <= 64, enc and out required)");
    if (!h->ready) throw WcbError(WCB_ERR_STATE, "weights not finalized");
    if (num_beams != 1) {   // beam search to the default length cap (generate()'s max_length 448)
      if (num_beams < 1) throw WcbError(WCB_ERR_ARG, "num_beams must be >= 1");
      return decode_begin_beams(h, enc, B, num_beams, prefix, prefix_len, h->d.n_text_ctx, bias_boost, min_new_tokens, out,
                                stream);
    }
    REQUIRE(h->nctx < wcb_handle::kMaxCtx, "step-wise decoding needs a free decode context (decode_contexts <= 3)");
    REQUIRE(!h->step_state, "a step-wise decode is already active on this handle (wcb_decode_end first)");
    REQUIRE(bias_boost >= 0.f && min_new_tokens >= 0, "bias_boost and min_new_tokens must be >= 0");
    const int P = prefix ? prefix_len : 1;
    REQUIRE(P >= 1 && P < h->d.n_text_ctx, "prefix_len must be in [1, max_target_positions)");
    const int ci = wcb_handle::kMaxCtx - 1;
    const int T = h->d.n_text_ctx, max_new = h->d.n_text_ctx - P;
    const int xm = h->xmode;
    ensure_dec_ws(h, B, B, T, max_new, xm, P > 1 ? B * std::min(prefill_chunk(B), P - 1) : B, ci, ci + 1);
    DecCtx& D = h->dc[ci];
    sync_in(h, stream, D.hs);
    // the caller's encoder output [B][1500][d] (model dtype) is copied / projected into owned buffers
    if (xm == 1) {
      fill_xenc(h, ci, enc, B, D.hs);
    } else {
      sync_in(h, stream, h->he);
      cross_kv(h, B, ci, enc);                        // on the encoder stream
      HIPCHK(hipStreamSynchronize(h->he));
    }
    int* ints = D.ints.as<int>();
    HIPCHK(hipMemsetAsync(ints, 0, (size_t)(I_NEXT + 4 * B) * 4, D.hs));
    if (prefix) {   // per-row prefixes [B][P] (host), positions 0 .. P-2 prefilled, P-1 is the first input
      if ((size_t)B * P * 4 > D.forced.bytes) { quiesce(h); D.forced.ensure((size_t)B * P * 4); }
      HIPCHK(hipMemcpyAsync(D.forced.p, prefix, (size_t)B * P * 4, hipMemcpyHostToDevice, D.hs));
      HIPCHK(hipStreamSynchronize(D.hs));   // pageable host source
    } else {
      fill_i32(ints + I_NEXT, h->d.decoder_start_token_id, B, D.hs);
    }
    StepCfg sc{B, T, max_new, ci, false, false, D.logits.as<float>(), (long)h->vocab_pad, h->empty_bias.get(),
               bias_boost, min_new_tokens, D.forced.as<int>(), P};
    sc.clips = B;
    sc.xmode = xm;
    for (int p0 = 0, np; p0 + 1 < P; p0 += np) {
      np = std::min(prefill_chunk(B), P - 1 - p0);
      prefill_step(h, sc, np, D.forced.as<int>(), P);
    }
    if (prefix) gather_col(ints + I_NEXT, D.forced.as<int>(), B, P, P - 1, D.hs);
    step_embed(h, sc);   // the first step's input (every step's finalize embeds the next one)
    HIPCHK(hipStreamSynchronize(D.hs));
    auto* st = new wcb_state;
    st->h = h; st->B = B; st->P = P; st->T = T; st->max_new = max_new; st->min_new = min_new_tokens;
    st->xmode = xm; st->lam = bias_boost;
    h->step_state = st;
    *out = st;
    sync_out(h, stream, D.hs);
  });
}

int wcb_decode_step(wcb_handle* h, wcb_state* st, const wcb_bias* bias, int32_t* next_ids, float* scores, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && st && st->h == h && h->step_state == st && next_ids, "bad argument (state of this handle, next_ids)");
    REQUIRE(st->fwd == 0, "wcb_decode_step on a forward cache (wcb_forward_cached state)");
    if (st->steps >= st->max_new) {
      // the length cap: refused, except for a finished beam search, whose steps are frozen (identity
      // parents, pad ids; the device position stopped at the last cache slot)
      bool frozen = false;
      if (st->nb > 1) {
        DecCtx& D = h->dc[wcb_handle::kMaxCtx - 1];
        int v = 0;
        HIPCHK(hipMemcpyAsync(&v, D.ints.as<int>() + I_DONE, 4, hipMemcpyDeviceToHost, D.hs));
        HIPCHK(hipStreamSynchronize(D.hs));
        frozen = v > 0;
      }
      REQUIRE(frozen, "max_target_positions reached");
    }
    const wcb_bias* bs = bias ? bias : h->empty_bias.get();
    REQUIRE(bs == h->empty_bias.get() || bs->owner == h, "bias automaton was created on another handle");
    REQUIRE(bs->vocab == h->d.vocab, "bias automaton built for another vocabulary");
    REQUIRE(st->steps == 0 || bs->id == st->bias_id, "the bias automaton must stay the same for the whole decode");
    const int ci = wcb_handle::kMaxCtx - 1;
    DecCtx& D = h->dc[ci];
    sync_in(h, stream, D.hs);
    const int R = st->B * st->nb;
    StepCfg sc{R, st->T, st->max_new, ci, true, true, D.logits.as<float>(), (long)h->vocab_pad, bs, st->lam,
               st->min_new, D.forced.as<int>(), 0};
    sc.clips = st->B;
    sc.xmode = st->xmode;
    sc.host_pos = st->P - 1 + st->steps;
    if (st->nb > 1) {   // beam step: the running beams' new tokens, their scores (running log-prob sums)
      beam_set_bias(st->bm, bs);
      sc.nb = st->nb;
      sc.phys = st->bm.phys;
      sc.beam = &st->bm;
    } else {
      sc.score_out = scores;
      sc.embedded = true;   // (wcb_decode_begin embedded the first input; each finalize embeds the next)
    }
    decode_step(h, sc);
    HIPCHK(hipMemcpyAsync(next_ids, D.ints.as<int>() + I_NEXT, (size_t)R * 4, hipMemcpyDeviceToDevice, D.hs));
    if (st->nb > 1 && scores)
      HIPCHK(hipMemcpyAsync(scores, st->bm.run_sc, (size_t)R * 4, hipMemcpyDeviceToDevice, D.hs));
    st->bias_id = bs->id;
    ++st->steps;
    sync_out(h, stream, D.hs);
  });
}

int wcb_decode_begin_beams(wcb_handle* h, const void* enc, int B, int num_beams, const int32_t* prefix, int prefix_len,
                           int max_new_tokens, float bias_boost, int min_new_tokens, wcb_state** out, void* stream) {
  return guarded(h, [&] {
    REQUIRE(num_beams >= 2, "wcb_decode_begin_beams: num_beams must be >= 2 (greedy: wcb_decode_begin)");
    decode_begin_beams(h, enc, B, num_beams, prefix, prefix_len, max_new_tokens, bias_boost, min_new_tokens, out, stream);
  });
}

int wcb_decode_parents(wcb_handle* h, wcb_state* st, int32_t* parents, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && st && st->h == h && h->step_state == st && parents, "bad argument (state of this handle, parents)");
    REQUIRE(st->nb > 1, "wcb_decode_parents: not a beam-search state");
    REQUIRE(st->steps > 0, "wcb_decode_parents: no step taken yet");
    DecCtx& D = h->dc[wcb_handle::kMaxCtx - 1];
    sync_in(h, stream, D.hs);
    HIPCHK(hipMemcpyAsync(parents, st->bm.parent, (size_t)st->B * st->nb * 4, hipMemcpyDeviceToDevice, D.hs));
    sync_out(h, stream, D.hs);
  });
}

int wcb_decode_info(wcb_handle* h, wcb_state* st, int32_t* max_new, int32_t* steps, int32_t* done) {
  return guarded(h, [&] {
    REQUIRE(h && st && st->h == h && h->step_state == st, "bad argument (state of this handle)");
    if (max_new) *max_new = st->max_new;
    if (steps) *steps = st->steps;
    if (done) {   // the device's all-finished flag (I_DONE: the step at which every utterance / row was done)
      DecCtx& D = h->dc[wcb_handle::kMaxCtx - 1];
      int v = 0;
      HIPCHK(hipMemcpyAsync(&v, D.ints.as<int>() + I_DONE, 4, hipMemcpyDeviceToHost, D.hs));
      HIPCHK(hipStreamSynchronize(D.hs));
      *done = v > 0 ? 1 : 0;
    }
  });
}

int wcb_decode_result(wcb_handle* h, wcb_state* st, int32_t* out_ids, int out_ld, int32_t* out_steps, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && st && st->h == h && h->step_state == st && out_ids && out_steps, "bad argument");
    REQUIRE(st->fwd == 0, "wcb_decode_result on a forward cache (wcb_forward_cached state)");
    DecCtx& D = h->dc[wcb_handle::kMaxCtx - 1];
    int* ints = D.ints.as<int>();
    sync_in(h, stream, D.hs);
    int n = st->steps;
    if (st->nb > 1) {   // the best finished sequence of every utterance so far (generate()'s beam output)
      HIPCHK(hipMemsetAsync(ints + I_UNFIN, 0, 4, D.hs));
      beam_output(st->bm, D.hs);
      int olen = 0;
      HIPCHK(hipMemcpyAsync(&olen, ints + I_UNFIN, 4, hipMemcpyDeviceToHost, D.hs));
      HIPCHK(hipStreamSynchronize(D.hs));
      n = std::min(olen, st->max_new);
    }
    // the library's output rows are st->max_new wide; the caller's out_ld columns must hold the n generated
    REQUIRE(out_ld >= n && out_ld >= 1, "wcb_decode_result: out_ld " + std::to_string(out_ld) + " < the " +
                                            std::to_string(n) + " generated columns (wcb_decode_info gives the width)");
    if (n > 0)
      HIPCHK(hipMemcpy2DAsync(out_ids, (size_t)out_ld * 4, D.outbuf.p, (size_t)st->max_new * 4, (size_t)n * 4,
                              st->B, hipMemcpyDeviceToDevice, D.hs));
    *out_steps = n;
    sync_out(h, stream, D.hs);
  });
}

int wcb_decode_end(wcb_handle* h, wcb_state* st) {
  return guarded(h, [&] {
    REQUIRE(h && st && st->h == h && h->step_state == st, "bad argument (state of this handle)");
    HIPCHK(hipStreamSynchronize(h->dc[wcb_handle::kMaxCtx - 1].hs));
    check_dev_err(h);
    h->step_state = nullptr;
    delete st;
  });
}

int wcb_synchronize(wcb_handle* h) {
  return guarded(h, [&] {
    REQUIRE(h, "null handle");
    quiesce(h);
    HIPCHK(hipGetLastError());
    check_dev_err(h);
  });
}

// teacher forcing on decode context `buf` once its encoder-side buffer is ready (ev_xkv[buf] recorded
// on the encoder stream): causal prefill of positions 0 .. T-1 of every row, logits of every position
static void forward_decode(wcb_handle* h, int buf, int B, const int32_t* dec_ids, int T, float* logits) {
  DecCtx& D = h->dc[buf];
  HIPCHK(hipStreamWaitEvent(D.hs, h->ev_xkv[buf], 0));
  int* ints = D.ints.as<int>();
  HIPCHK(hipMemsetAsync(ints, 0, (size_t)(I_NEXT + 4 * B) * 4, D.hs));
  for (int p0 = 0, np; p0 < T; p0 += np) {
    np = std::min(prefill_chunk(B), T - p0);
    StepCfg sc{B, T, 1, buf, true, false, logits + (size_t)p0 * h->d.vocab, (long)T * h->d.vocab, nullptr, 0.f,
               0, nullptr, 0};
    sc.xmode = h->xmode;
    prefill_step(h, sc, np, dec_ids, T);
  }
  HIPCHK(hipEventRecord(h->ev_dec[buf], D.hs));
}

int wcb_forward(wcb_handle* h, const float* mel, int B, const int32_t* dec_ids, int T, float* logits, void* enc_out,
                void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && mel && dec_ids && logits && B > 0 && T > 0, "bad argument");
    if (!h->ready) throw WcbError(WCB_ERR_STATE, "weights not finalized");
    REQUIRE(B <= 64, "batch > 64 per handle");
    REQUIRE(T <= h->d.n_text_ctx, "decoder_input_ids longer than max_target_positions");
    ensure_enc_ws(h, B);
    ensure_dec_ws(h, B, B, T, 1, h->xmode, B * std::min(prefill_chunk(B), T));
    const int buf = h->gen_count++ % h->nctx;
    sync_in(h, stream, h->he);
    HIPCHK(hipStreamWaitEvent(h->he, h->ev_dec[buf], 0));
    if (h->xmode == 1) {
      void* eo = enc_out ? enc_out : h->encout.p;
      encode_impl(h, mel, B, eo);
      fill_xenc(h, buf, eo, B, h->he);
    } else {
      void* eo = enc_out ? enc_out : h->encout.p;
      encode_impl(h, mel, B, eo);
      cross_kv(h, B, buf, eo);
    }
    HIPCHK(hipEventRecord(h->ev_xkv[buf], h->he));
    forward_decode(h, buf, B, dec_ids, T, logits);
    sync_out(h, stream, h->dc[buf].hs);
  });
}

int wcb_forward_enc(wcb_handle* h, const void* enc, int B, const int32_t* dec_ids, int T, float* logits, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && enc && dec_ids && logits && B > 0 && T > 0, "bad argument");
    if (!h->ready) throw WcbError(WCB_ERR_STATE, "weights not finalized");
    REQUIRE(B <= 64, "batch > 64 per handle");
    REQUIRE(T <= h->d.n_text_ctx, "decoder_input_ids longer than max_target_positions");
    ensure_dec_ws(h, B, B, T, 1, h->xmode, B * std::min(prefill_chunk(B), T));
    const int buf = h->gen_count++ % h->nctx;
    sync_in(h, stream, h->he);
    HIPCHK(hipStreamWaitEvent(h->he, h->ev_dec[buf], 0));
    // the given encoder output takes the place of encode_impl's: the same buffer (encoder space) or the
    // same cross-K/V GEMM over it (K/V formulation), so the logits equal wcb_forward's bit for bit
    if (h->xmode == 1) fill_xenc(h, buf, enc, B, h->he);
    else cross_kv(h, B, buf, enc);
    HIPCHK(hipEventRecord(h->ev_xkv[buf], h->he));
    forward_decode(h, buf, B, dec_ids, T, logits);
    sync_out(h, stream, h->dc[buf].hs);
  });
}

int wcb_forward_cached(wcb_handle* h, wcb_state* st, const int32_t* dec_ids, int T, float* logits, void* stream) {
  return guarded(h, [&] {
    REQUIRE(h && st && st->h == h && h->step_state == st && dec_ids && logits && T > 0,
            "bad argument (state of this handle, dec_ids, logits, T > 0)");
    REQUIRE(st->steps == 0, "wcb_forward_cached on a state that wcb_decode_step has advanced");
    REQUIRE(st->P == 1, "wcb_forward_cached needs a state begun without a prefix");
    REQUIRE(st->fwd + T <= st->T, "past_key_values + decoder_input_ids exceed max_target_positions");
    const int ci = wcb_handle::kMaxCtx - 1, B = st->B;
    ensure_dec_ws(h, B, B, st->T, st->max_new, st->xmode, B * std::min(prefill_chunk(B), T), ci, ci + 1);
    DecCtx& D = h->dc[ci];
    sync_in(h, stream, D.hs);
    // the new ids at their absolute positions of the [B][T] forced buffer (prefill_ids reads src[b·T + pos])
    if ((size_t)B * st->T * 4 > D.forced.bytes) { quiesce(h); D.forced.ensure((size_t)B * st->T * 4); }
    HIPCHK(hipMemcpy2DAsync(D.forced.as<int>() + st->fwd, (size_t)st->T * 4, dec_ids, (size_t)T * 4, (size_t)T * 4, B,
                            hipMemcpyDeviceToDevice, D.hs));
    for (int p0 = 0, np; p0 < T; p0 += np) {
      np = std::min(prefill_chunk(B), T - p0);
      StepCfg sc{B, st->T, 1, ci, true, false, logits + (size_t)p0 * h->d.vocab, (long)T * h->d.vocab, nullptr, 0.f,
                 0, nullptr, 0};
      sc.clips = B;
      sc.xmode = st->xmode;
      prefill_step(h, sc, np, D.forced.as<int>(), st->T);
    }
    st->fwd += T;
    sync_out(h, stream, D.hs);
  });
}

// ------------------------------------------------------------------------------ bias automaton
int wcb_bias_create(wcb_handle* h, const int32_t* tokens, const int32_t* offsets, int n_phrases,
                    const uint8_t* word_start, wcb_bias** out) {
  return guarded(h, [&] {
    REQUIRE(h && out && n_phrases >= 0 && (n_phrases == 0 || (tokens && offsets)), "bad argument");
    const int V = h->d.vocab;
    // trie
    std::vector<std::map<int, int>> ch(1);
    std::vector<int> depth(1, 0);
    std::vector<char> end(1, 0);
    for (int p = 0; p < n_phrases; ++p) {
      int s = 0;
      REQUIRE(offsets[p + 1] >= offsets[p], "offsets must be non-decreasing");
      for (int i = offsets[p]; i < offsets[p + 1]; ++i) {
        const int v = tokens[i];
        REQUIRE(v >= 0 && v < V, "bias token id out of range");
        auto it = ch[s].find(v);
        if (it == ch[s].end()) {
          ch.emplace_back();
          depth.push_back(depth[s] + 1);
          end.push_back(0);
          const int nn = (int)ch.size() - 1;
          ch[s][v] = nn;
          s = nn;
        } else {
          s = it->second;
        }
      }
      if (s) end[s] = 1;
    }
    const int ns = (int)ch.size();
    std::vector<int> fail(ns, 0), keep(ns, 0), order;
    order.reserve(ns);
    std::deque<int> q;
    for (auto& kv : ch[0]) {
      fail[kv.second] = 0;
      keep[kv.second] = end[kv.second] ? 1 : 0;
      q.push_back(kv.second);
    }
    while (!q.empty()) {
      const int s = q.front();
      q.pop_front();
      order.push_back(s);
      for (auto& kv : ch[s]) {
        keep[kv.second] = end[kv.second] ? depth[kv.second] : keep[s];
        int f = fail[s];
        while (f && !ch[f].count(kv.first)) f = fail[f];
        auto it = ch[f].find(kv.first);
        fail[kv.second] = (it != ch[f].end() && it->second != kv.second) ? it->second : 0;
        q.push_back(kv.second);
      }
    }
    // trans(s): every token whose transition from s lands at depth >= 2 (root children are the
    // vocabulary-wide bitmap). Walk the failure chain; the first (deepest) state owning the token wins.
    std::vector<int> off(ns + 1, 0), tok, dst;
    for (int s = 0; s < ns; ++s) {
      std::map<int, int> t;
      for (int f = s; f != 0; f = fail[f])
        for (auto& kv : ch[f])
          if (!t.count(kv.first)) t[kv.first] = kv.second;
      for (auto& kv : t)
        if (depth[kv.second] >= 2) { tok.push_back(kv.first); dst.push_back(kv.second); }
      off[s + 1] = (int)tok.size();
    }
    // root children: a match may START only at a word-start token (word_start == null: any token)
    std::vector<uint32_t> bits((V + 31) / 32, 0u);
    std::vector<int> rc(V, -1);
    for (auto& kv : ch[0])
      if (!word_start || word_start[kv.first]) {
        bits[kv.first >> 5] |= 1u << (kv.first & 31);
        rc[kv.first] = kv.second;
      }
    auto b = std::make_unique<wcb_bias>();
    b->n_states = ns;
    b->vocab = V;
    b->id = g_next_bias_id.fetch_add(1);   // process-wide: a graph key never names another handle's bias
    b->owner = h;
    HIPCHK(hipSetDevice(h->device));
    b->root_bits.ensure(bits.size() * 4);
    HIPCHK(hipMemcpy(b->root_bits.p, bits.data(), bits.size() * 4, hipMemcpyHostToDevice));
    b->root_child.ensure(rc.size() * 4);
    HIPCHK(hipMemcpy(b->root_child.p, rc.data(), rc.size() * 4, hipMemcpyHostToDevice));
    b->trans_off.ensure(off.size() * 4);
    HIPCHK(hipMemcpy(b->trans_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice));
    b->trans_tok.ensure(std::max<size_t>(tok.size(), 1) * 4);
    b->trans_dst.ensure(std::max<size_t>(dst.size(), 1) * 4);
    if (!tok.empty()) {
      HIPCHK(hipMemcpy(b->trans_tok.p, tok.data(), tok.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(b->trans_dst.p, dst.data(), dst.size() * 4, hipMemcpyHostToDevice));
    }
    b->st_depth.ensure((size_t)ns * 4);
    b->st_keep.ensure((size_t)ns * 4);
    HIPCHK(hipMemcpy(b->st_depth.p, depth.data(), (size_t)ns * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->st_keep.p, keep.data(), (size_t)ns * 4, hipMemcpyHostToDevice));
    h->biases.push_back(b.get());
    *out = b.release();
  });
}

// Lifetime (wcb.h): the decode graphs of the owning handle capture the automaton's device buffers.
// Destroying it waits for the handle's queued work and drops those graphs (they are re-captured by
// the next wcb_generate), so a graph can never replay reads of freed memory.
void wcb_bias_destroy(wcb_bias* b) {
  if (!b) return;
  if (wcb_handle* h = b->owner) {
    (void)hipSetDevice(h->device);
    try {
      quiesce(h);
    } catch (...) {
    }
    for (DecCtx& D : h->dc)
      if (D.gkey.find("/" + std::to_string(b->id) + "/") != std::string::npos) {
        if (D.gexec) (void)hipGraphExecDestroy(D.gexec);
        if (D.gexec_k) (void)hipGraphExecDestroy(D.gexec_k);
        D.gexec = D.gexec_k = nullptr;
        D.gkey.clear();
      }
    h->biases.erase(std::remove(h->biases.begin(), h->biases.end(), b), h->biases.end());
  }
  for (DevBuf* x : {&b->root_bits, &b->root_child, &b->trans_off, &b->trans_tok, &b->trans_dst, &b->st_depth, &b->st_keep})
    x->release();
  delete b;
}

int wcb_bias_num_states(const wcb_bias* b) { return b ? b->n_states : 0; }

int wcb_debug_copy(wcb_handle* h, const char* name, void* dst, int64_t bytes, int enc_layers) {
  return guarded(h, [&] {
    REQUIRE(h && name, "bad argument");
    h->dbg_enc_layers = enc_layers;
    const std::map<std::string, DevBuf*> bufs = {{"xt", &h->xt}, {"hbuf", &h->hbuf}, {"x", &h->x}, {"h", &h->h},
                                                 {"qkv", &h->qkv}, {"att", &h->att}, {"ffn", &h->ffn},
                                                 {"encout", &h->encout}, {"xkv", &h->xkv2[0]},
                                                 {"logits", &h->dc[0].logits}};
    if (bytes == 0) return;   // only set the layer limit
    REQUIRE(dst, "null dst");
    auto it = bufs.find(name);
    REQUIRE(it != bufs.end(), std::string("unknown buffer ") + name);
    REQUIRE((size_t)bytes <= it->second->bytes, "bytes exceeds buffer size");
    quiesce(h);
    HIPCHK(hipMemcpy(dst, it->second->p, (size_t)bytes, hipMemcpyDeviceToDevice));
  });
}

int wcb_profile_enable(wcb_handle* h, int enable) {
  return guarded(h, [&] {
    REQUIRE(h, "null handle");
    quiesce(h);
    h->prof_collect();
    h->prof = (enable & 1) != 0;          // HIP events around front-end / encoder launches
    h->prof_stamps = (enable & 2) != 0;   // device stamps in the decode cross-attention (graph nodes)
    h->prof_e.clear();
    h->xattn_bytes = h->xattn_flops = 0;
    if (h->prof_stamps) {
      const size_t sb = (size_t)h->nctx * wcb_handle::kStampRegions * h->stamp_slots() * 16 * kStampSub;
      h->stamps.ensure(sb);
      h->stamp_acc.ensure(16 * wcb_handle::kStampRegions);
      HIPCHK(hipMemsetAsync(h->stamps.p, 0, sb, nullptr));
      HIPCHK(hipMemsetAsync(h->stamp_acc.p, 0, 16 * wcb_handle::kStampRegions, nullptr));
      HIPCHK(hipStreamSynchronize(nullptr));
    }
  });
}

int wcb_profile_read(wcb_handle* h, int n, char (*names)[32], int64_t* launches, double* ms, double* flops, double* bytes) {
  int count = 0;
  const int rc = guarded(h, [&] {
    REQUIRE(h, "null handle");
    h->prof_collect();
    if (h->prof_stamps && h->stamp_acc.p) {   // decode cross-attention + lean projections: device-stamped launches
      quiesce(h);
      unsigned long long acc[2 * wcb_handle::kStampRegions] = {};
      HIPCHK(hipMemcpy(acc, h->stamp_acc.p, sizeof(acc), hipMemcpyDeviceToHost));
      if (acc[1]) {
        const int id = h->prof_id("dec_xattn");
        h->prof_e[id].launches = (int64_t)acc[1];
        h->prof_e[id].ms = (double)acc[0] / 1e5;   // 100 MHz s_memrealtime ticks
        h->prof_e[id].bytes = h->xattn_bytes;
        h->prof_e[id].flops = h->xattn_flops;
      }
      for (int r = 1; r < wcb_handle::kStampRegions; ++r) {
        if (!acc[2 * r + 1]) continue;
        const int id = h->prof_id((std::string(kLeanStampClass[r]) + "@graph").c_str());
        h->prof_e[id].launches = (int64_t)acc[2 * r + 1];
        h->prof_e[id].ms = (double)acc[2 * r] / 1e5;
      }
    }
    for (size_t i = 0; i < h->prof_e.size() && (int)i < n; ++i) {
      snprintf(names[i], 32, "%s", h->prof_e[i].name.c_str());
      launches[i] = h->prof_e[i].launches;
      ms[i] = h->prof_e[i].ms;
      flops[i] = h->prof_e[i].flops;
      bytes[i] = h->prof_e[i].bytes;
    }
    count = (int)h->prof_e.size();
  });
  return rc == WCB_OK ? count : rc;
}

int wcb_profile_kernel(wcb_handle* h, int i, char* name, int cap, int64_t* grid) {
  return guarded(h, [&] {
    REQUIRE(h && name && cap > 0, "bad argument");
    REQUIRE(i >= 0 && i < (int)h->prof_e.size(), "profile entry out of range");
    const ProfEntry& e = h->prof_e[i];
    std::string nm;
    if (e.fn) {
      const char* raw = hipKernelNameRefByPtr(e.fn, nullptr);
      if (raw) {
        int st = 0;
        char* dm = abi::__cxa_demangle(raw, nullptr, nullptr, &st);
        nm = (st == 0 && dm) ? dm : raw;
        free(dm);
      }
    }
    snprintf(name, (size_t)cap, "%s", nm.c_str());
    if (grid) *grid = e.grid;
  });
}

// ------------------------------------------------------------------------------ kernel-level ops
int wcb_op_gemm_kernel(int dtype, const void* A, const void* W, int M, int N, int K, const float* bias, int act,
                       const float* resid, void* out, int out_f32, int kernel, void* stream) {
  return guarded(nullptr, [&] {
    REQUIRE(A && W && out && M > 0 && N > 0 && K > 0, "bad argument");
    REQUIRE(N % 8 == 0, "N must be a multiple of 8");
    REQUIRE(K % (dtype == WCB_F32 ? 32 : 64) == 0, "K must be a multiple of the 128-byte K tile");
    REQUIRE((kernel >= 0 && kernel <= 7 && kernel != 3) || kernel == 106 || kernel == 107 ||
            (kernel % 100 >= 11 && kernel % 100 <= 52 && kernel < 200),
            "kernel: 0, 1, 2, 4, 5, 6, 7 or a wide tile config 11-52 (+100 on 6, 7 and the wide configs: W fragment-major)");
    const bool wfm = kernel >= 100;
    kernel %= 100;
    GemmArgs g = rowgemm(A, K, W, M, N, K, out, N);
    g.bias = bias; g.act = act; g.resid = resid; g.out_f32 = out_f32;
    g.raster = 8;
    if (kernel >= 6) {   // the decode-row (beam) tiles: 6 / 7 = LDS-ring tiles (7: row panels outer, the
                         // runtime's order before option beam_raster), 10·FM + FN = gemm_wide_kernel
      REQUIRE(M > 64 && dtype != WCB_F32, "decode-row tiles: 16-bit, M > 64");
      g.tile = 2; g.ring_kt = 2;
      if (kernel == 7) g.raster = 0;
      if (kernel <= 7 && wfm) g.W_fm = W;
      if (kernel > 7) {
        g.wide = kernel;
        if (wfm) g.W_fm = W;
        REQUIRE(!resid || resid == out, "wide tiles: the residual is updated in place (resid == out)");
      }
    } else {
      g.pp = kernel;
    }
    gemm(DType(dtype), g, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
  });
}

int wcb_op_gemm(int dtype, const void* A, const void* W, int M, int N, int K, const float* bias, int act,
                const float* resid, void* out, int out_f32, void* stream) {
  return wcb_op_gemm_kernel(dtype, A, W, M, N, K, bias, act, resid, out, out_f32, 1, stream);
}

int wcb_op_gemm_ln(int dtype, const float* X, const float* ln_w, const float* ln_b, const float* stats,
                   const void* W, int M, int N, int K, const float* bias, int act, void* out, int out_f32, void* stream) {
  return guarded(nullptr, [&] {
    REQUIRE(X && ln_w && ln_b && stats && W && out && M > 0 && M <= 64 && N > 0 && K % 16 == 0, "bad argument");
    GemmArgs g = rowgemm(X, K, W, M, N, K, out, N);
    g.ln_w = ln_w; g.ln_b = ln_b; g.st_in = stats; g.st_nb = K / 16;
    g.bias = bias; g.act = act; g.out_f32 = out_f32;
    gemm(DType(dtype), g, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
  });
}

int wcb_op_layernorm(int dtype, const float* x, const float* w, const float* b, void* y, int M, int d, void* stream) {
  return guarded(nullptr, [&] {
    REQUIRE(x && w && b && y && M > 0 && d > 0 && d % 64 == 0 && d <= 2048, "bad argument");
    layernorm(DType(dtype), x, w, b, y, M, d, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
  });
}

int wcb_op_attention_decode(int dtype, const void* q, const void* k, const void* v, void* o, int B, int H, int Sk,
                            int nsplit, int variant, void* stream) {
  return guarded(nullptr, [&] {
    REQUIRE(q && k && v && o && B > 0 && H > 0 && Sk > 0 && Sk <= 2048 && nsplit >= 1 && nsplit <= 64, "bad argument");
    AttnArgs a;   // decode layout: q/o [B][H·64], K/V head-major [B][H][Sk][64] (the cross-K/V layout)
    a.q = q; a.ldq = (long)H * 64; a.q_Sb = 1; a.Sq = 1;
    a.k = k; a.v = v; a.k_sb = (long)H * Sk * 64; a.k_sh = (long)Sk * 64; a.k_sk = 64;
    a.o = o; a.ldo = (long)H * 64; a.o_Sb = 1; a.B = B; a.H = H; a.nkeys = Sk;
    a.variant = variant;
    if (variant == 6 || variant == 7) a.kv_rows = Sk;   // the one-token self-attention kernel (speculative first keys)
    int* nk_dev = nullptr;
    if (variant == 7) {   // the key count read on the device (decode graphs): the lean self-attention kernel
      // per-call, stream-ordered scratch (a shared buffer would race between calls on different streams),
      // written by a kernel whose argument carries the value (no pageable host source)
      HIPCHK(hipMallocAsync(reinterpret_cast<void**>(&nk_dev), 4, (hipStream_t)stream));
      const int nk1 = Sk - 1;
      write_i32(nk_dev, &nk1, 1, (hipStream_t)stream);
      a.nkeys_dev = nk_dev; a.nkeys_add = 1;
    }
    static DevBuf part, ticket;
    if (nsplit > 1) {
      a.nsplit = nsplit;
      part.ensure((size_t)B * H * nsplit * 66 * 4);
      ticket.ensure((size_t)B * H * 4);
      a.part = part.as<float>();
      a.ticket = ticket.as<int>();
    }
    attention_decode(DType(dtype), a, (hipStream_t)stream);
    if (nk_dev) HIPCHK(hipFreeAsync(nk_dev, (hipStream_t)stream));
    HIPCHK(hipGetLastError());
  });
}

int wcb_op_cross_attention_enc(int dtype, const void* q, const void* enc, const void* wkt, const void* wv,
                               const float* bv, void* o, int B, int H, int S, int nsplit, int variant, void* stream) {
  return guarded(nullptr, [&] {
    const int d = H * 64;
    REQUIRE(q && enc && wkt && wv && bv && o && B > 0 && B <= 64 && H > 0 && S > 0 && nsplit >= 1 &&
                nsplit <= kXencMaxSplit, "bad argument");
    REQUIRE(xenc_supported(DType(dtype), d), "encoder-space cross-attention needs a 16-bit dtype and d <= 1024");
    static DevBuf qp, u, part, ml;   // workspaces of this test entry point
    const size_t e = esize(dtype);
    qp.ensure((size_t)B * H * d * e);
    u.ensure((size_t)B * H * d * e);
    part.ensure((size_t)B * nsplit * H * d * 4);
    ml.ensure((size_t)B * nsplit * H * 2 * 4);
    GemmArgs kq = rowgemm(q, d, wkt, B, H * d, 64, qp.p, (long)H * d);
    kq.a_grp_n = d; kq.a_grp_off = 64;
    gemm(DType(dtype), kq, (hipStream_t)stream);
    XencArgs xa;
    xa.enc = enc; xa.enc_sb = (long)S * d; xa.qp = qp.p; xa.rows = B; xa.H = H; xa.D = d; xa.S = S;
    xa.nsplit = nsplit; xa.part = part.as<float>(); xa.ml = ml.as<float>();
    xa.variant = variant % 100;
    xa.part16 = variant >= 1000 && d % 128 == 0;   // variant + 1000: 16-bit normalised range partials
    if (xa.part16) xa.variant = 1;
    xenc_attention(DType(dtype), xa, (hipStream_t)stream);
    if (d % 128 == 0 && (variant < 100 || variant >= 1000)) {   // the runtime's default: merge + W_v fused
      xenc_merge_v(DType(dtype), xa, wv, bv, o, d, (hipStream_t)stream);
    } else {   // variant + 100: merge kernel + grouped W_v GEMM (option merge_v = 0, and d = 64)
      xenc_merge(DType(dtype), xa, u.p, (long)H * d, (hipStream_t)stream);
      GemmArgs vg = rowgemm(u.p, (long)H * d, wv, B, d, d, o, d);
      vg.a_grp_n = 64; vg.a_grp_off = d; vg.bias = bv;
      gemm(DType(dtype), vg, (hipStream_t)stream);
    }
    HIPCHK(hipGetLastError());
  });
}

int wcb_op_weighted_ce(const float* logits, long ld, int B, int T, int V, const int32_t* labels,
                       const int32_t* spans, const int32_t* span_len, int N, int Lmax, float bias_weight,
                       float* per_token, float* loss, int32_t* count, void* stream) {
  return guarded(nullptr, [&] {
    REQUIRE(logits && labels && per_token && loss && B > 0 && T > 0 && V > 0 && ld >= V, "bad argument");
    REQUIRE(!spans || (span_len && N > 0 && Lmax > 0), "spans need span_len, N > 0 and Lmax > 0");
    WceArgs a;
    a.logits = logits; a.ld = ld; a.B = B; a.T = T; a.V = V; a.labels = labels;
    a.spans = spans; a.span_len = span_len; a.N = spans ? N : 0; a.Lmax = spans ? Lmax : 0;
    a.use_spans = spans ? 1 : 0; a.bias_weight = bias_weight;
    a.per_token = per_token; a.loss = loss; a.count = count;
    weighted_ce(a, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
  });
}

int wcb_op_attention(int dtype, const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk,
                     int flash, void* stream) {
  return guarded(nullptr, [&] {
    REQUIRE(q && k && v && o && B > 0 && H > 0 && Sq > 0 && Sk > 0 && Sk <= 2048, "bad argument");
    AttnArgs a;
    const long ld = (long)H * 64;
    a.q = q; a.ldq = ld; a.q_Sb = Sq; a.Sq = Sq;
    a.k = k; a.v = v; a.k_sb = (long)Sk * ld; a.k_sh = 64; a.k_sk = ld;
    a.o = o; a.ldo = ld; a.o_Sb = Sq; a.B = B; a.H = H; a.nkeys = Sk;
    const bool beam = flash >= 200 && flash <= 202;
    if (flash == 1 || flash == 100 || beam || flash < 0) {
      // 100: 64 queries per wave;
      // 200 / 201 / 202: the beam kernel (keys split over the waves, Sq <= 16; 4 waves x 2 stages, 2 x 4,
      // 2 x 5); -n: n key ranges + merge (Sq <= 16)
      a.variant = flash == 100 ? 4 : beam ? 7 + (flash - 200) : 1;
      REQUIRE(!beam || Sq <= 16, "the beam kernel takes at most 16 query rows per set");
      REQUIRE(dtype != WCB_F32, "flash attention needs a 16-bit dtype");
      static DevBuf fpart;
      if (flash < 0) {
        REQUIRE(-flash <= 8 && Sq <= 16, "flash key split: 1..8 ranges, Sq <= 16");
        a.nsplit = -flash;
        fpart.ensure((size_t)B * H * Sq * a.nsplit * 66 * 4);
        a.part = fpart.as<float>();
      }
      attention_flash(DType(dtype), a, (hipStream_t)stream);
    } else {
      static DevBuf part, ticket;   // split-KV workspace of this test entry point (zeroed on growth)
      if (flash > 1) {
        a.nsplit = flash;
        part.ensure((size_t)B * H * Sq * flash * 66 * 4);
        ticket.ensure((size_t)B * H * Sq * 4);
        a.part = part.as<float>();
        a.ticket = ticket.as<int>();
      }
      attention_decode(DType(dtype), a, (hipStream_t)stream);
    }
    HIPCHK(hipGetLastError());
  });
}

}  // extern "C"
