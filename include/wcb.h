/* libwcb — MI355X-native Whisper contextual-biasing inference path (C ABI).
 *
 * The reference exposes no native plugin API: its hot-path boundary is the Python class contract of
 * `WhisperForConditionalGenerationWeightCE` (models/whisper_medical.py:12-172) driven by
 * `scripts/evaluation.py:164-206` and the feature extractor call at data_utils/data_loader.py:171.
 * Each entry point below replaces one piece of that surface; the Python mirror
 * `whisper_context_biasing_amd.model.WhisperCB` binds them with ctypes.
 *
 * Conventions: return 0 on success, a negative wcb_status otherwise (message: wcb_last_error);
 * no exception crosses the ABI. Activation buffers are caller-owned DEVICE memory; weights,
 * workspaces and KV caches are library-owned. One handle per GPU; calls on one handle are
 * serialised by the caller. `stream` is a hipStream_t (NULL = default stream).
 */
#ifndef WCB_H_
#define WCB_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wcb_handle wcb_handle;
typedef struct wcb_bias wcb_bias;

enum wcb_status {
  WCB_OK = 0,
  WCB_ERR_ARG = -1,       /* invalid argument / shape (ValueError in the reference) */
  WCB_ERR_STATE = -2,     /* call out of order (e.g. weights not finalized) */
  WCB_ERR_HIP = -3,       /* HIP runtime error */
  WCB_ERR_UNSUPPORTED = -4
};

enum wcb_dtype { WCB_BF16 = 0, WCB_F16 = 1, WCB_F32 = 2 };

/* Model dimensions (HF WhisperConfig fields; encoder and decoder depth are equal for every size). */
typedef struct {
  int d_model, n_layers, n_heads, ffn, vocab, n_mel;
  int n_audio_ctx;   /* 1500 */
  int n_text_ctx;    /* 448 */
  int eos_token_id, pad_token_id, decoder_start_token_id;
  int dtype;         /* wcb_dtype of weights and activations (f32 accumulation everywhere) */
} wcb_model_desc;

/* Decode configuration (replaces the GenerationConfig of scripts/evaluation.py:173-179). */
typedef struct {
  int max_new_tokens;   /* generate(max_length=N) of the reference → at most N new tokens */
  int min_new_tokens;   /* EOS masked while fewer tokens were generated (benchmark mode) */
  int num_beams;        /* 1 = greedy (the reference eval setting) */
  float bias_boost;     /* lambda >= 0 of the bias-list boost; 0 = plain greedy bit-for-bit */
  int use_graph;        /* replay the decode step as a captured hipGraph */
  int async_out;        /* 1: do not make `stream` wait for the decode; outputs valid after
                           wcb_synchronize (lets the next call's front end + encoder overlap it) */
} wcb_gen_cfg;

/* replaces WhisperForConditionalGenerationWeightCE(config) (models/whisper_medical.py:16-22) */
int wcb_create(const wcb_model_desc* desc, int device, wcb_handle** out);
void wcb_destroy(wcb_handle* h);
const char* wcb_last_error(const wcb_handle* h);

/* alternative formulations the tests compare (defaults are fixed per model; no environment variables):
 *   "xmode" 0/1        decoder cross-attention over per-layer K/V, or in encoder space (before finalize)
 *   "beam_xmode" 0/1   the same for beam search (before finalize)
 *   "group_rows" n     decoder rows per layer chain (16..512)
 *   "xenc_variant" v   encoder-space kernel variant, "xvariant" v  K/V cross-attention kernel variant
 *   "flash_split" n    key ranges per (clip, head) of the beam-search cross-attention (flash kernel), 1..8
 *   "beam_xattn" v     beam-search cross-attention: keys split over the waves of one (clip, head) workgroup
 *                      (1: 4 waves x 2 LDS stages, 2: 2 x 4, 3: 2 x 5) or the flash kernel over key ranges (0)
 *   "ln_fold" 0/1      decode rows > 64 (16-bit): LayerNorm folded into the projection (1, default: finalize
 *                      keeps W·diag(γ) copies of QKV / cross-q / fc1, ≈ +1/4 of the decoder weights), or its own
 *                      launch (0); before finalize
 *   "merge_v" 0/1      greedy encoder-space cross-attention: range merge and W_v fused (1) or two launches
 *   "xpart16" 0/1      greedy encoder-space cross-attention (fused merge): the key-range partials stored in the
 *                      model dtype, each normalised by its own softmax sum, (max, sum) in f32 (1, default: half
 *                      the partial bytes) or unnormalised f32 partials (0)
 *   "xq_kq" 0/1        greedy encoder-space cross-attention query (lean path): q'_h = W_k,hᵀ q_h computed inside
 *                      the LN-fused q_proj launch (1) or as a launch of its own (0, default); bit-identical
 *   "lean" 0/1         decode projections of <= 64 rows (16-bit) on the lean single-tile kernel (1, default)
 *                      or the general decode GEMM (0); bit-identical. Before finalize: with it finalize keeps
 *                      fragment-major copies of the decoder projection weights and the token embedding (the
 *                      decoder weights once more in memory, e.g. ≈ +1.8 GB at large-v3 fp16)
 *   "lean_x" 0/1       lean path, one position per row: the residual writers also write the 16-bit rows
 *                      fragment-major for the LayerNorm-fused QKV / xq / fc1 (1, default); bit-identical
 *   "decode_contexts" n  decode contexts in flight (1..4): calls decode on n streams from n buffers (4 is
 *                      refused while a step-wise decode owns context 3)
 *   "steps_per_graph" n  decode steps captured per replayed hipGraph (1..64, default 8)
 *   "xenc_fm" 0/1      greedy encoder-space cross-attention reads the encoder output in the fragment-major chunk
 *                      layout (1, default; 1 KiB contiguous per load wave-instruction) or the row layout (0)
 *   "ring_kt" 1/2      decode rows > 64: 64-deep K sub-tiles per LDS-ring stage of the projection tiles
 *   "beam_wide" 0/1    decode rows 65-96 (C5's beam rows): out / xo / xq / fc1 on the wide single-burst tiles
 *                      with fragment-major weights (1, default) or the LDS-ring tiles (0); before finalize
 *   "beam_wfm" 0/1     decode rows > 64: the LDS-ring tiles read fragment-major weight copies (0, default);
 *                      before finalize
 *   "beam_raster" n    decode rows > 64: ring tile order in bands of n row panels, column tiles outer (0, default:
 *                      row panels outer)
 *   "lean_fold" 0/1    <= 64 rows: the LayerNorm-fused projections (QKV, cross-q, fc1) with the LayerNorm folded
 *                      into fragment-major W·diag(γ) copies (1, default) or normalised in the kernel (0); before
 *                      finalize
 *   "xqk" 0/1          greedy cross query (encoder space, lean, folded): q_h and q'_h = W_k,hᵀ q_h in one launch
 *                      with no hand-off, each workgroup recomputing its head's q_h (1, default) or the xq → kq
 *                      launches (0)
 *   "xqk_chunks" n     fused cross query: q' column chunks per head, each chunk's workgroup recomputing q_h (2, 4,
 *                      8 (default), 16); bit-identical
 *   "lean_mf2" 0/1     <= 64 rows: every lean projection on 32-row workgroups where the chain has > 16 rows (1) or
 *                      only the LN-fused N >= 2048 ones (0, default); bit-identical
 *   "mel_split" 0/1    log-mel DFT as split-bf16 MFMAs (1) or exact-f32 MFMAs (0, default); both within 2e-5 of
 *                      the reference feature extractor
 *   "lm_walkers" n     greedy LM head: column walkers per row block = argmax partials per row (128, 192, 256
 *                      (default), 384, 512, 1024; before finalize); the selected ids do not depend on it
 *   "merge_os" 1/2     greedy range merge + W_v: a head's 64 outputs in one workgroup of 2 rows (1, default) or
 *                      over two workgroups of 4 rows (2); bit-identical
 *   "beam_chunks" 0/1  beam top-K over 16 vocabulary chunks per row, one workgroup each (1) or one workgroup
 *                      per row (0, default)
 *   "xenc_split" n     key ranges per row of the greedy encoder-space cross-attention (1..16, before finalize)
 *   "enc_flash" v      encoder flash attention tiling: 2 (32 queries per wave), 4 (64 queries, default)
 *   "enc_raster" n     encoder GEMM tile order: bands of n row panels, column tiles outer (8, default;
 *                      0: row-major); bit-identical
 *   "enc_gemm" v       encoder GEMM kernels: 4 (default) the ping-pong kernel, 256- or 192-wide tiles by the
 *                      fewer tile rounds; 1 the LDS-ring kernel's 256x192 tiles where 192-wide wins; 0 the
 *                      LDS-ring kernel everywhere; 5 the ping-pong kernel's 192-wide tiles wherever N allows
 *                      (162 VGPRs: room on a CU for a decode workgroup beside it; measured 1 % slower)
 * While a step-wise decode is open (wcb_decode_begin .. wcb_decode_end) only decode_contexts, enc_flash,
 * enc_gemm, enc_raster and steps_per_graph may change: the others shape the state it carries between steps. */
int wcb_set_option(wcb_handle* h, const char* name, int value);

/* replaces from_pretrained / load_state_dict: one HF state-dict tensor (host f32, C order), staged
 * on the device. Names follow the reference's state dict (model.encoder.layers.{i}.self_attn.q_proj.weight,
 * ...). proj_out.weight is tied to model.decoder.embed_tokens.weight (models/whisper_medical.py:14). */
int wcb_set_weight(wcb_handle* h, const char* name, const float* data, const int64_t* shape, int ndim);

/* a BORROWED device tensor (e.g. a torch CUDA tensor or a view into an RCCL-broadcast blob) */
typedef struct wcb_tensor_view {
  const char* name;     /* HF state-dict name */
  const void* data;     /* device pointer of element [0,...,0] */
  int dtype;            /* wcb_dtype of the elements */
  int ndim;             /* 1..4 */
  int64_t shape[4];
  int64_t stride[4];    /* in elements */
} wcb_tensor_view;
/* stages n device tensors without a host round trip (gathered and widened to f32 on the device, on
 * `stream`); the views are not read after the call returns. Mixes freely with wcb_set_weight. */
int wcb_load_weights(wcb_handle* h, const wcb_tensor_view* views, int n, void* stream);
/* build the device layouts from the staged tensors on the device (fused QKV with q pre-scaled,
 * im2col conv weights, W_k,hᵀ panels, all-layer cross-KV stack), rounded once to the model dtype;
 * staging buffers are released. */
int wcb_finalize_weights(wcb_handle* h);

/* replaces WhisperFeatureExtractor.__call__ (data_utils/data_loader.py:171-172):
 * pcm f32 [B][pcm_stride] (first n_samples valid, zero-padded/trimmed to 480000)
 * → mel_out f32 [B][n_mel][3000]. */
int wcb_log_mel(wcb_handle* h, const float* pcm, int B, int n_samples, int64_t pcm_stride, float* mel_out,
                void* stream);

/* replaces WhisperEncoder.forward ([tf] modeling_whisper.py:592-646): mel f32 [B][n_mel][3000]
 * → enc_out [B][1500][d] in the model dtype (may be NULL: result kept internally for decode). */
int wcb_encode(wcb_handle* h, const float* mel, int B, void* enc_out, void* stream);

/* replaces model.generate(input_features, max_length=...) as called by
 * [tf] trainer_seq2seq.py:329: greedy (num_beams = 1) or HF beam search (num_beams 2..8,
 * [tf] generation/utils.py:3208) from [decoder_start] (+ optional prefix), bias boost,
 * out_ids int32 DEVICE [B][cfg->max_new_tokens] (finished rows padded with pad_token_id; beams: the
 * best finished sequence of each clip), *out_steps = number of generated columns (greedy: all rows
 * finished or max_new_tokens; beams: the longest best sequence — with async_out, max_new_tokens: the
 * length is not read back, columns past a clip's best sequence hold pad_token_id).
 * The front end/encoder run on one library stream and the decode on another, with two cross-K/V
 * buffers: call i+1's encoder overlaps call i's decode (async_out = 1 keeps `stream` free). */
int wcb_generate(wcb_handle* h, const float* mel, int B, const wcb_gen_cfg* cfg, const wcb_bias* bias,
                 const int32_t* prefix, int prefix_len, int32_t* out_ids, int32_t* out_steps, void* stream);

/* Step-wise decoding (SURVEY §8(b) wcb_decode_begin / wcb_decode_step): the decode step of wcb_generate
 * one token per call, for callers that inspect every step (the reference's surface is generate(); this is
 * the streaming form of it). `enc` = encoder output [B][1500][d] in the model dtype (DEVICE, copied /
 * projected at begin: not retained), `prefix` = per-utterance prompt [B][prefix_len] (HOST, NULL:
 * decoder_start_token_id only; positions 0 .. prefix_len-2 are prefilled, the last one is the first step's
 * input), EOS masked while fewer than min_new_tokens were generated. One active state per handle (it owns
 * decode context 3, so decode_contexts must be <= 3). The bias automaton must be the same (or NULL) at
 * every step of one decode.
 *  - greedy (num_beams = 1): wcb_decode_step writes next_ids [B] (int32, DEVICE) and, when non-NULL,
 *    scores [B] (f32, DEVICE: the chosen token's logit + bias boost; 0 for finished rows); finished rows
 *    emit pad_token_id.
 *  - beam search (num_beams = nb in 2..8, HF _beam_search, [tf] generation/utils.py:3208-3524, one
 *    iteration per step; rows R = B·nb, beam i of utterance b = row b·nb + i): wcb_decode_begin caps the
 *    length at max_target_positions as generate() does by default, wcb_decode_begin_beams at prefix +
 *    max_new_tokens (generate(max_length=...); the cap is a stopping criterion, so it changes the beams).
 *    wcb_decode_step writes the token each running beam appended, next_ids [R], and when non-NULL the
 *    running log-prob sums, scores [R]; wcb_decode_parents then gives parents [R] (int32, DEVICE): the
 *    beam (0..nb-1 of the same utterance) each running beam extends — the running sequences are the
 *    parents' sequences plus next_ids. Once every utterance is done a step changes nothing.
 *    Once every utterance is done (wcb_decode_info's *done) the search is frozen: a step writes parents =
 *    identity and next_ids = pad_token_id, so a consumer that extends its hypotheses every step is unchanged.
 *  - wcb_decode_info: *max_new = the state's column capacity (max_target_positions - prefix_len for
 *    wcb_decode_begin, max_new_tokens for wcb_decode_begin_beams), *steps = the steps taken, *done = 1 once
 *    every utterance (row) has finished (blocks on the decode stream for it); each pointer may be NULL.
 *  - wcb_decode_result: out_ids [B][out_ld] (int32, DEVICE) receives the n generated columns, *out_steps
 *    (host) = n: greedy, the steps taken (finished rows padded); beams, the best finished sequence of each
 *    utterance so far with n its longest length — after the steps generate() takes, exactly generate()'s
 *    output. out_ld < n is refused (WCB_ERR_ARG); out_ld = *max_new always holds the result. */
typedef struct wcb_state wcb_state;
int wcb_decode_begin(wcb_handle* h, const void* enc, int B, int num_beams, const int32_t* prefix, int prefix_len,
                     float bias_boost, int min_new_tokens, wcb_state** out, void* stream);
int wcb_decode_begin_beams(wcb_handle* h, const void* enc, int B, int num_beams, const int32_t* prefix, int prefix_len,
                           int max_new_tokens, float bias_boost, int min_new_tokens, wcb_state** out, void* stream);
int wcb_decode_step(wcb_handle* h, wcb_state* st, const wcb_bias* bias, int32_t* next_ids, float* scores, void* stream);
int wcb_decode_parents(wcb_handle* h, wcb_state* st, int32_t* parents, void* stream);
int wcb_decode_info(wcb_handle* h, wcb_state* st, int32_t* max_new, int32_t* steps, int32_t* done);
int wcb_decode_result(wcb_handle* h, wcb_state* st, int32_t* out_ids, int out_ld, int32_t* out_steps, void* stream);
int wcb_decode_end(wcb_handle* h, wcb_state* st);

/* wait for every queued front-end / encoder / decode operation of the handle */
int wcb_synchronize(wcb_handle* h);

/* replaces forward(input_features, decoder_input_ids) (models/whisper_medical.py:45-111):
 * dec_ids int32 DEVICE [B][T] → logits f32 DEVICE [B][T][vocab]; enc_out as in wcb_encode. */
int wcb_forward(wcb_handle* h, const float* mel, int B, const int32_t* dec_ids, int T, float* logits,
                void* enc_out, void* stream);

/* replaces forward(encoder_outputs=..., decoder_input_ids) (models/whisper_medical.py:54-55, 93-111, the
 * decoder on a given encoder output, no re-encode): enc = encoder output [B][1500][d] in the model dtype
 * (DEVICE, e.g. wcb_encode's enc_out; copied / projected, not retained) → logits as wcb_forward, bit for
 * bit the logits wcb_forward computes from the mel that produced enc. */
int wcb_forward_enc(wcb_handle* h, const void* enc, int B, const int32_t* dec_ids, int T, float* logits, void* stream);

/* replaces forward(..., use_cache=True) / forward(..., past_key_values=...) (models/whisper_medical.py:54-55,
 * 89-110: the decoder's self-attention KV cache carried between calls): `st` = a step-wise state begun with
 * wcb_decode_begin(enc, B, 1, NULL, ...) (it owns the encoder output and the cache); each call appends
 * positions [n, n + T) for dec_ids [B][T] (int32, DEVICE), n = the positions appended so far, and writes
 * their logits [B][T][vocab] (f32, DEVICE). A state used here takes no wcb_decode_step. */
int wcb_forward_cached(wcb_handle* h, wcb_state* st, const int32_t* dec_ids, int T, float* logits, void* stream);

/* bias list: n_phrases token sequences, phrase i = tokens[offsets[i] .. offsets[i+1]) (host
 * arrays), built into an Aho-Corasick automaton on the device. word_start (host, [vocab] bytes, or
 * NULL = every token) marks the tokens a match may START at — for a BPE vocabulary the tokens that
 * begin a word (leading space); tokenise phrases as they appear inside a transcript. Boost
 * semantics (oracle/bias_ref.py, k_select.hip): each token scores +lam·n(s, v) where n counts the
 * tokens the transition adds to the current match minus the dropped, unfinished ones (retraction);
 * completed phrases keep their bonus.
 * Lifetime: an automaton belongs to the handle that created it; wcb_bias_destroy waits for that
 * handle's queued work and drops the decode graphs that captured it (serialise it with the handle's
 * other calls, like every call on a handle). It may outlive the handle (destroy it afterwards). */
int wcb_bias_create(wcb_handle* h, const int32_t* tokens, const int32_t* offsets, int n_phrases,
                    const uint8_t* word_start, wcb_bias** out);
void wcb_bias_destroy(wcb_bias* b);
int wcb_bias_num_states(const wcb_bias* b);

/* per-kernel time accounting for the benchmark's roofline. enable bit 0: HIP events around every
 * front-end / encoder launch on its stream; bit 1: device time stamps (s_memrealtime) written by the
 * decode cross-attention kernel, which runs inside the replayed step graph where events cannot
 * bracket a single node. 0 disables; counters are reset. */
int wcb_profile_enable(wcb_handle* h, int enable);
/* fills up to n entries: name, launches, total milliseconds, algorithmic flops, algorithmic bytes */
int wcb_profile_read(wcb_handle* h, int n, char (*names)[32], int64_t* launches, double* ms,
                     double* flops, double* bytes);

/* entry i of wcb_profile_read: the (demangled) kernel symbol of the class's first launch and its grid
 * in threads (x·y·z), as rocprofv3 names them (Kernel_Name; Grid_Size = Grid_Size_X·Y·Z); "" when the class
 * launched nothing or was stamped on the device */
int wcb_profile_kernel(wcb_handle* h, int i, char* name, int cap, int64_t* grid);

/* debug: copy an internal workspace buffer (xt, hbuf, x, h, qkv, att, ffn, encout, xkv, logits)
 * into dst (device) after synchronising; enc_layers limits later encodes to that many layers
 * (-1 = all). bytes == 0 only sets the limit. */
int wcb_debug_copy(wcb_handle* h, const char* name, void* dst, int64_t bytes, int enc_layers);

/* ---- kernel-level entry points (parity tests and microbenchmarks) ---- */
/* out[M][N] = act(A[M][K] · W[N][K]ᵀ + bias) (+ resid), row-major, dtype of A/W = dtype */
int wcb_op_gemm(int dtype, const void* A, const void* W, int M, int N, int K, const float* bias, int act,
                const float* resid, void* out, int out_f32, void* stream);
/* the same with the encoder-GEMM kernel chosen: kernel 1 = the ping-pong kernel where it covers the shape
 * and is the faster one (16-bit, N % 256 == 0, K % 64 == 0, K >= 128, M >= 256; the LDS-ring kernel's
 * 256x192 tiles where those leave fewer tile rounds), 4 = the same with the ping-pong kernel's own 192-wide
 * tiles there (option "enc_gemm"), 2 / 5 = the ping-pong kernel's 256- / 192-wide tiles for every shape they
 * cover (residual epilogue included), 0 = the LDS-ring / tile kernels; decode-row (beam) tiles, 16-bit,
 * M > 64: 6 = the LDS-ring tiles, 10·FM + FN (11, 12, 21, 22, 41, 42, 51, 52) = the wide single-burst
 * tiles of 16·FM rows x 16·FN columns (K = 768, 1024 or 1280; resid, when given, must equal out; a shape
 * the wide tiles do not cover runs on the ring tiles), 100 + that: W given fragment-major
 * ([N / 16][K / 32][64 lanes][8]: element (n, k) at lane 16·((k % 32) / 8) + n % 16, slot k % 8) */
int wcb_op_gemm_kernel(int dtype, const void* A, const void* W, int M, int N, int K, const float* bias, int act,
                       const float* resid, void* out, int out_f32, int kernel, void* stream);
/* decode-step fused form: out[M][N] = act(LN(X) · W[N][K]ᵀ + bias), X f32 [M][K] (M <= 64), with the
 * LayerNorm row statistics taken from stats[M][K/16][2] = per-16-column (Σx, Σx²) partials */
int wcb_op_gemm_ln(int dtype, const float* X, const float* ln_w, const float* ln_b, const float* stats,
                   const void* W, int M, int N, int K, const float* bias, int act, void* out, int out_f32,
                   void* stream);
/* y[M][d] (dtype) = LayerNorm(x f32 [M][d]) * w + b, eps 1e-5 */
int wcb_op_layernorm(int dtype, const float* x, const float* w, const float* b, void* y, int M, int d,
                     void* stream);
/* o[B][Sq][H*64] = softmax(q kᵀ) v per head (q pre-scaled), k/v [B][Sk][H*64];
 * flash=1 selects the MFMA kernel (16-bit dtypes; Sq <= 16: the few-query form of beam search), 100 the
 * MFMA kernel with 64 queries per wave, 200 / 201 / 202 (Sq <= 16) the beam kernel (the keys of a (set,
 * head) split over its waves, merged in the workgroup: 4 waves x 2 LDS stages, 2 x 4, 2 x 5), -n (Sq <= 16)
 * the MFMA kernel over n key ranges merged in
 * fixed order; 0 the decode kernel; n >= 2 the decode kernel with n split-KV key chunks combined by the
 * last-arriving chunk. */
int wcb_op_attention(int dtype, const void* q, const void* k, const void* v, void* o, int B, int H, int Sq,
                     int Sk, int flash, void* stream);
/* decode attention in the runtime's layout: q/o [B][H*64], K/V head-major [B][H][Sk][64]; one query
 * per (row, head), nsplit key chunks (split-KV), kernel variant (k_attn.hip launch_decode; 6 = the
 * one-token self-attention kernel, nsplit 1; 7 = the same with the key count read on the device, as the
 * decode step runs it: the lean form for 16-bit). */
int wcb_op_attention_decode(int dtype, const void* q, const void* k, const void* v, void* o, int B, int H,
                            int Sk, int nsplit, int variant, void* stream);

/* decoder cross-attention in encoder space (k_xenc.hip), the xmode-1 decode path:
 * o[B][d] = Σ_h-blocks W_v,h softmax_j(q'_h · enc_j) enc_j + b_v with q'_h = W_k,hᵀ q_h;
 * q [B][H*64] (pre-scaled by 1/8), enc [B][S][d], wkt = W_k repacked [H][d][64] (element (h,c,i) =
 * W_k[h*64+i][c]), wv [d][d] (HF layout), bv f32 [d]; nsplit key ranges per row (1..16). 16-bit dtypes.
 * variant: attn_xenc kernel variant; + 100 = merge kernel + grouped W_v GEMM instead of the fused merge. */
int wcb_op_cross_attention_enc(int dtype, const void* q, const void* enc, const void* wkt, const void* wv,
                               const float* bv, void* o, int B, int H, int S, int nsplit, int variant, void* stream);

/* Bias-weighted cross entropy — replaces the loss block of
 * WhisperForConditionalGenerationWeightCE.forward (models/whisper_medical.py:113-156): weight
 * bias_weight on every label token covered by a contiguous match of one of its utterance's spans
 * (:118-133), −log_softmax(logits)[label]·w over labels ≠ −100, summed / (valid count + 1e-8)
 * (:136-151). spans == NULL: nn.CrossEntropyLoss(ignore_index=−100) mean (:152-155).
 * logits f32 [B·T][ld] (device), labels [B][T], spans [B][N][Lmax] with span_len [B][N] (0 = empty
 * span, skipped — :122-127); per_token [B·T] (device, caller-owned) receives −logp·w·valid;
 * loss (device f32 scalar) and count (device, nullable) the mean and the valid-label count.
 * Labels must be −100 or in [0, V). Async on `stream`; deterministic (fixed-order reduction). */
int wcb_op_weighted_ce(const float* logits, long ld, int B, int T, int V, const int32_t* labels,
                       const int32_t* spans, const int32_t* span_len, int N, int Lmax, float bias_weight,
                       float* per_token, float* loss, int32_t* count, void* stream);

/* Host-side scoring (csrc/metric.cpp, no GPU): the arithmetic of utils/compute_metric.py on
 * already-normalised text. wcb_wer_counts: per utterance i, errors[i] = word-level Levenshtein
 * distance between refs[i] and hyps[i] (whitespace-separated words) and ref_words[i] = |words(refs[i])|
 * — corpus WER = Σerrors / Σref_words, as evaluate's "wer" (jiwer) computes it at
 * compute_metric.py:159. n_threads <= 0: all hardware threads. wcb_bias_counts: compute_bias_wer's
 * per-utterance tallies (compute_metric.py:200-230): non-overlapping phrase counts in ref / pred. */
int wcb_wer_counts(const char* const* refs, const char* const* hyps, int n, int64_t* errors, int64_t* ref_words,
                   int n_threads);
int wcb_bias_counts(const char* ref, const char* pred, const char* const* phrases, int n_phrases,
                    int64_t* distance, int64_t* tokens);

#ifdef __cplusplus
}
#endif
#endif /* WCB_H_ */
