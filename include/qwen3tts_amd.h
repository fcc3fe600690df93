/*
 * qwen3tts_amd.h -- C ABI of the MI355X-native (gfx950) Qwen3-TTS hot path.
 *
 * Library: qwen3-tts_amd/lib/libqwen3tts_amd.so (built by qwen3-tts_amd/build.py / __graft_entry__.build()).
 *
 * The reference (kritsanan1/Qwen3-TTS = QwenLM/Qwen3-TTS 0.0.4) has NO native ABI: its hot path is PyTorch
 * eager code plus third-party kernels reached through nn.Linear / transformers' ALL_ATTENTION_FUNCTIONS
 * (SURVEY.md §2, §8b).  Each entry point below names the reference operator(s) it replaces
 * (M = qwen_tts/core/models/modeling_qwen3_tts.py, K = qwen_tts/core/tokenizer_12hz/modeling_qwen3_tts_tokenizer_v2.py).
 *
 * Conventions: plain device pointers + sizes, a hipStream_t passed as void*, int status return
 * (0 = ok, < 0 = QT_ERR_*; qt_last_error() is not needed: codes are exhaustive).  No allocation, no host
 * synchronisation, no global mutable state: every call is graph-capturable and reentrant.
 * Activations: row-major, channels-last.  dtype codes: QT_F32 / QT_BF16.
 */
#ifndef QWEN3TTS_AMD_H
#define QWEN3TTS_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

enum { QT_F32 = 0, QT_BF16 = 1 };
enum { QT_ACT_NONE = 0, QT_ACT_SILU = 1, QT_ACT_GELU = 2, QT_ACT_RELU = 3, QT_ACT_SIGMOID = 4,
       QT_ACT_RELU_TANH = 5 /* tanh(relu(x)): ECAPA attentive pooling M:232 */ };
enum { QT_AACT_NONE = 0, QT_AACT_ELU = 1 };  /* activation applied to the A operand as it is loaded */
enum { QT_PAD_ZERO = 0, QT_PAD_REFLECT = 1, QT_PAD_REPLICATE = 2 };
enum { QT_EPI_STORE = 0, QT_EPI_ADD = 1, QT_EPI_SWIGLU = 2 };
enum { QT_OK = 0, QT_ERR_ARG = -1, QT_ERR_SHAPE = -2, QT_ERR_DTYPE = -3, QT_ERR_LAUNCH = -4 };

/* ---------------------------------------------------------------------------------------------
 * qt_gemm: out[m][n] (=|+=) epi( rs[m] * sum_k W[n][k] * gamma[k] * A[m][k] + bias[n] ) * colscale[n]
 *
 * Replaces every nn.Linear / nn.Conv1d / nn.ConvTranspose1d of the hot path:
 *   talker & code predictor q/k/v/o, gate/up/down, codec_head, lm_head[g], small_to_mtp_projection,
 *   text_projection (M:740-751, 848-850, 1167-1174, 1575-1579);  codec pre_conv, transformer linears,
 *   ConvNeXt pwconv, decoder convs / transposed convs (K:159-242, 294-369, 492-493, 618-657, 838-864).
 * Fused prologues: RMSNorm (rmsnorm != 0 or gamma != NULL: out *= rsqrt(mean_k A^2 + eps) per row;
 * gamma scales A, or is folded into W at load time -- Qwen3TTSRMSNorm M:595-610 feeding the Linear), row gather
 * (a_index != NULL; nn.Embedding feeding the Linear), implicit im2col (taps > 0).
 * Fused epilogues: bias, SiLU / GELU, colscale (LayerScale K:393-405, ConvNeXt gamma K:236),
 * residual add (QT_EPI_ADD, M:1409/1417), SwiGLU (QT_EPI_SWIGLU; W rows interleaved 8 gate / 8 up per
 * 16-row tile, output width N/2; Qwen3TTSTalkerTextMLP M:842-855).
 * W must be pre-tiled by qt_tile_weight (layout in gemm.hip; rows padded to 16).  Columns n >= N are not
 * written (SwiGLU: N = 2*I, I % 8 == 0).
 * Conv mode (taps > 0): A is [batch][t_in][cin] (lda = row stride), output row m = b*t_out + t reads
 * input time t + t_off + j*dil for tap j (zero outside [0, t_in)), K = taps*cin_pad.
 * ------------------------------------------------------------------------------------------- */
typedef struct qt_gemm_args {
  int M, N, K;
  int a_dtype, w_dtype, o_dtype;
  const void* A;
  long long lda;
  const int* a_index;
  const void* W;
  const float* gamma;
  float eps;
  int rmsnorm;
  const float* bias;
  const float* colscale;
  int act;
  int epi;
  void* out;
  long long ldo;
  int taps, dil, cin, cin_pad, t_in, t_out, t_off;
  /* decode GEMV (M<=16) split-K: ws = zero-initialised device scratch of ws_bytes (>= QT_GEMM_WS_MIN),
   * owned by the caller and used by one stream at a time; splitk 0 = auto, 1 = off, n = force n.
   * Partials are reduced in a fixed order by the last-arriving block: results are deterministic. */
  void* ws; long long ws_bytes; int splitk;
  /* optional SnakeBeta on the A operand (K:577-615), per input channel: a' = a + inv_beta[c]*sin(alpha[c]*a)^2
   * (alpha / inv_beta pre-exponentiated); fuses the activation that precedes every codec conv */
  const float* snake_alpha; const float* snake_inv_beta;
  /* QT_AACT_ELU: ELU(alpha = 1) on every A element (zero padding stays zero) -- the nn.ELU that precedes every
   * MimiConv1d of the tokenizer encoder (transformers modeling_mimi.py MimiEncoder / MimiResnetBlock) */
  int a_act;
  /* optional bf16 copy of every element the epilogue stores (fp32 out, QT_EPI_STORE / QT_EPI_ADD; decode GEMV
   * shapes: M <= 16, or the skinny row-group GEMV path of 17..96 rows / <= 256 rows of a <= 2048-column output):
   * out2[m*ldo2 + n] = bf16(out[m*ldo + n]).  Decode writes the residual stream this way so the next
   * RMS-normalised GEMV reads its A operand at half the bytes (its MFMA rounds A to bf16 anyway). */
  void* out2; long long ldo2;
} qt_gemm_args;
#define QT_GEMM_WS_MIN (4 << 20)

int qt_gemm(const qt_gemm_args* args, void* stream);

/* Row-major [N][Kp] weight (Kp padded to 32 bf16 / 16 fp32) -> MFMA-fragment tiles (ceil(N/16)*16 rows). */
int qt_tile_weight(const void* src, int dtype, int N, int Kp, void* dst, void* stream);

/* ---------------------------------------------------------------------------------------------
 * qt_qkv_post: per-head q_norm / k_norm (RMSNorm over head_dim), rotate-half RoPE from cos/sin tables,
 * q written to q_out (fp32 [R][Hq*D]); k, v written into the KV cache at (row_batch[r], kv_pos[r]).
 * Replaces M:773-785 (q_norm/k_norm, apply_multimodal_rotary_pos_emb == 1-D rope for TTS, DynamicCache
 * .update) and K:323-333 (codec: no q/k norm).  qkv: fp32 [R][(Hq+2*Hkv)*D].
 * cache layout [B][Hkv][Lmax][D] in kv_dtype.  cos/sin tables: fp32 [npos][D/2].
 * ------------------------------------------------------------------------------------------- */
typedef struct qt_qkv_args {
  int R, Hq, Hkv, D;
  const float* qkv;
  const float* q_norm; const float* k_norm; float eps;
  const float* cos_tab; const float* sin_tab;
  const int* rope_pos; const int* row_batch; const int* kv_pos;
  float* q_out;
  void* k_cache; void* v_cache; int kv_dtype; int Lmax;
} qt_qkv_args;
int qt_qkv_post(const qt_qkv_args* args, void* stream);

/* ---------------------------------------------------------------------------------------------
 * qt_attention: per query row r, keys [max(row_start[r], row_len[r]-window), row_len[r]) of batch
 * row_batch[r]; GQA (Hq/Hkv q heads per kv head); softmax in fp32.  Replaces eager/sdpa/FA2 attention
 * (M:634-657, 787-801; K:121-144, 335-349 incl. the 72-frame sliding window).  out [R][Hq*D] (o_dtype).
 * ------------------------------------------------------------------------------------------- */
typedef struct qt_attn_args {
  int R, Hq, Hkv, D, Lmax, window;
  const float* q;
  const void* k_cache; const void* v_cache; int kv_dtype;
  const int* row_batch; const int* row_start; const int* row_len;
  void* out; int o_dtype;
  int max_keys;
} qt_attn_args;
int qt_attention(const qt_attn_args* args, void* stream);

/* ---------------------------------------------------------------------------------------------
 * qt_decode_attention: qt_qkv_post + qt_attention fused for rows whose key range ends at their own new
 * position (talker / code-predictor decode, M:773-801): per (row, kv head) q/k RMSNorm + RoPE, append of
 * the new k/v at kv_pos[r], then attention over keys [max(row_start[r], kv_pos[r]+1-window), kv_pos[r]].
 * out fp32 [R][Hq*D].  Rows must not read each other's new keys (one row per batch entry).
 * ------------------------------------------------------------------------------------------- */
typedef struct qt_decode_attn_args {
  int R, Hq, Hkv, D, Lmax, window;
  const float* qkv;
  const float* q_norm; const float* k_norm; float eps;
  const float* cos_tab; const float* sin_tab;
  const int* rope_pos; const int* row_batch; const int* kv_pos; const int* row_start;
  void* k_cache; void* v_cache; int kv_dtype;
  void* out; int o_dtype;  /* [R][Hq*D]; bf16 output = the rounding the next bf16 MFMA applies anyway */
  int const_pos;  /* >= 0: rope_pos = kv_pos = const_pos, row_start = 0, row_batch = r (code-predictor steps:
                     static positions as a launch constant, so no dependent load precedes the K/V stream) */
  int nsplit;     /* split-KV: each (row, kv head) runs on nsplit blocks over disjoint key ranges (<= 8; 0/1 = off);
                     the last block to arrive merges the partial softmax states in split order (deterministic) */
  void* ws; long long ws_bytes;  /* nsplit > 1: zero-initialised scratch >= qt_decode_attn_ws_bytes(), one stream */
} qt_decode_attn_args;
long long qt_decode_attn_ws_bytes(int R, int Hq, int Hkv, int D, int nsplit);
int qt_decode_attention(const qt_decode_attn_args* args, void* stream);
/* Short prefill whose keys are all new (the code predictor's per-frame 2-token prefill, M:1142-1160): rows
 * r = b*T + t at positions t = 0..T-1 of batch item b (T == 2), causal over the T keys, k/v appended to the
 * cache at 0..T-1.  Uses R, Hq, Hkv, D, Lmax, qkv, q_norm, k_norm, eps, cos/sin, caches, out, o_dtype of args.
 * One launch instead of qt_qkv_post + qt_attention. */
int qt_small_prefill_attention(const qt_decode_attn_args* args, int T, void* stream);

/* ---------------------------------------------------------------------------------------------
 * qt_decode_attn_oproj: qt_decode_attention + the o_proj GEMV + residual add in one launch, for short caches
 * (the code predictor's decode steps, M:930-958 attention -> o_proj -> M:1004 residual):
 *   x[r][n] += sum_k Wo[n][k] * attn(r)[k],  attn as qt_decode_attention computes it (rounded to the weight
 *   dtype, as the separate path stores it before the o_proj MFMA).
 * Row r is batch entry r; keys [row_start[r], kv_pos[r]] (or [0, const_pos] when const_pos >= 0); Hkv <= 8.
 * w_o: o_proj weight tiled by qt_tile_weight ([N][Hq*D], w_dtype == kv_dtype).  x: fp32 residual [R][ldx].
 * One block per (column group, row) recomputes the row's attention for every kv head and sums the per-head
 * partial products in head order inside the block (deterministic, no workspace).  Each block re-reads its
 * row's keys, so use it where keys are few (<= 64 cached keys).
 * ------------------------------------------------------------------------------------------- */
typedef struct qt_attn_oproj_args {
  int R, Hq, Hkv, D, Lmax;
  const float* qkv;                       /* fp32 [R][(Hq + 2*Hkv)*D] raw q/k/v projections */
  const float* q_norm; const float* k_norm; float eps;
  const float* cos_tab; const float* sin_tab;
  const int* rope_pos; const int* kv_pos; const int* row_start; int const_pos;
  void* k_cache; void* v_cache; int kv_dtype;
  const void* w_o; int w_dtype; int N;
  float* x; long long ldx;
  void* x16; long long ldx16;  /* optional bf16 copy of the updated residual rows (next RMS GEMV's A operand) */
} qt_attn_oproj_args;
int qt_decode_attn_oproj(const qt_attn_oproj_args* args, void* stream);

/* ---------------------------------------------------------------------------------------------
 * qt_mlp_decode: one decode step of the Qwen3 MLP with its residual, fused (M:655-668: down_proj(act(gate_proj
 * (x)) * up_proj(x)) after the post-attention RMSNorm, + residual): x[m] += W_down(silu(W_gate n(x)) * W_up n(x)).
 * M <= 16 rows (fp32 residual x, row stride ldx), H in {1024, 2048}, I % 32 == 0, H/16 <= I/32 <= 256;
 * bf16 weight tiles from qt_tile_weight: w_gu = gate/up interleaved 8+8 rows per tile with the RMSNorm gamma
 * folded in, w_down = [H][I].  ws: zero-initialised device scratch of >= qt_mlp_ws_bytes(M, H, I), used by
 * one stream at a time; err (optional device int) is set to 1 if the in-kernel arrival wait timed out.
 * Deterministic: partials are reduced in block order.
 * ------------------------------------------------------------------------------------------- */
typedef struct qt_mlp_args {
  int M, H, I;
  float* x; long long ldx;
  const void* w_gu; const void* w_down;
  float eps;
  void* ws; long long ws_bytes;
  int* err;
} qt_mlp_args;
long long qt_mlp_ws_bytes(int M, int H, int I);
/* ---------------------------------------------------------------------------------------------
 * qt_cp_mlp: one persistent launch (256 workgroups, one per CU) for a code-predictor decode step's
 *   x += down(SwiGLU(gate_up(rms(x16))));  x16 = bf16(x);  out3 = rms(x16) . W3
 * i.e. M:1000-1011 (post-attention RMSNorm, Qwen3TTSTalkerTextMLP, residual) followed by the next RMS-normalised
 * projection (the next layer's q/k/v, or the final norm + lm_head[g], M:1299), with the two all-to-all hand-offs
 * (SwiGLU output, new residual) inside the launch as tagged granules instead of kernel boundaries.  bf16 weight
 * tiles from qt_tile_weight (w_gu gate/up interleaved 8 + 8 rows per tile, RMSNorm gammas folded into w_gu / w3).
 * M <= 16 rows; H = 1024, I = 3072, N3 in {1024, 2048, 4096} (qt_cp_mlp_supported; needs >= 256 CUs).
 * tags: device scratch of qt_cp_mlp_tags_bytes(H, I), zeroed before the first launch of a tag sequence; the launch's
 * tag base is *epoch_ctr * epoch_mul + epoch_add (>= 1, distinct for every launch until the scratch is zeroed
 * again).  err: device int set to 1 if a hand-off wait timed out (results are then invalid; never hangs).
 * ------------------------------------------------------------------------------------------- */
typedef struct qt_cp_mlp_args {
  int M, H, I, N3;
  void* x16; long long ldx16;        /* bf16 residual shadow: read (gate/up A operand), rewritten with the new rows */
  float* x; long long ldx;           /* fp32 residual, += the down projection */
  const void* w_gu; const void* w_down; const void* w3;
  float eps;
  float* out3; long long ldo3;
  void* tags; long long tags_bytes;
  const int* epoch_ctr; int epoch_mul, epoch_add;
  int* err;
} qt_cp_mlp_args;
long long qt_cp_mlp_tags_bytes(int H, int I);
int qt_cp_mlp_supported(int M, int H, int I, int N3);
int qt_cp_mlp(const qt_cp_mlp_args* args, void* stream);
int qt_mlp_decode(const qt_mlp_args* args, void* stream);

/* ---------------------------------------------------------------------------------------------
 * qt_sample: transformers-4.57 logits processing + token choice, one row per block.
 * RepetitionPenalty (seen flags) -> MinNewTokens (mask eos while *n_generated < min_new_tokens) ->
 * SuppressTokens [suppress_lo, suppress_hi) except suppress_keep (+ eos when ignore_eos) ->
 * greedy argmax (lowest index on ties) or Temperature -> TopK -> TopP -> softmax -> inverse-CDF draw from
 * a Philox stream (seed, *step, substep, row).  Finished rows emit eos (HF pad = eos).  Replaces
 * GenerationMixin's processors / sampling for the talker (M:2044-2066) and the code predictor (M:1671-1680).
 * tok_out[r] gets the token; if codes != NULL also codes[r*codes_ld + (*step + codes_step_off)*codes_w + codes_col].
 * ------------------------------------------------------------------------------------------- */
typedef struct qt_sample_args {
  const float* logits; int R; int V; long long ld;
  unsigned char* seen; float rep_penalty;
  const int* n_generated; int min_new_tokens; int eos_id;
  int suppress_lo, suppress_hi, suppress_keep; int ignore_eos;
  unsigned char* finished;
  int do_sample; int top_k; float top_p; float temperature;
  unsigned long long seed; const int* step; int substep;
  int* tok_out;
  int* codes; long long codes_ld; int codes_w; int codes_col; int codes_step_off;
  int row_base;  /* global index of row 0: Philox stream id = row_base + r, so a batch split into row groups draws exactly the streams of the whole batch */
  /* optional next-step input: emb_out[r*emb_ld + i] = emb_table[tok*emb_dim + i], i < emb_dim (fp32) -- the
   * embedding of the chosen token (pre-projected when the model has small_to_mtp), written by the sampler */
  const float* emb_table; int emb_dim; float* emb_out; long long emb_ld;
  /* optional device seed (read when the sampler runs, so a captured graph draws a fresh Philox stream per
   * request without recapture); NULL -> `seed` above */
  const unsigned long long* seed_ptr;
  float debug_u;  /* < 0: off.  Tests only: replaces the unit uniform of the inverse-CDF draw (1.0 -> u = total) */
  void* emb_out16; long long emb_ld16;  /* optional bf16 copy of the emb_out row (next RMS-normalised GEMV's A) */
  /* optional second gathered row (with emb_table): emb2_out[r*emb2_ld + i] = emb2_table[tok*emb2_dim + i] -- the
   * code predictor's layer-0 q/k/v projection of every table row, precomputed, so the next step skips that GEMV */
  const float* emb2_table; int emb2_dim; float* emb2_out; long long emb2_ld;
  int algo;  /* top-k (<= 64) sampling path, tests / measurement: 0 auto (histogram, per-wave on fall-through),
              * 1 per-wave candidate lists only, 2 histogram (same as 0).  Same Philox draws, same tokens. */
  /* per-row counters (continuous batching, every row its own request): row r reads step[r * ctr_stride] and
   * n_generated[r * ctr_stride]; 0 = one counter shared by every row */
  int ctr_stride;
  /* optional per-row Philox stream id (NULL -> row_base + r): a request keeps the stream of its index in the
   * request list whichever batch slot decodes it */
  const int* philox_row;
} qt_sample_args;
int qt_sample(const qt_sample_args* args, void* stream);

/* Qwen3TTSRMSNorm (M:595-610 / K:372-390): out = gamma * (x * rsqrt(mean(x^2) + eps)), fp32 [M][N]. */
int qt_rmsnorm(const float* x, const float* gamma, float eps, float* out, int M, int N, void* stream);
/* qt_rmsnorm + a record of each normalised row at rec[m*rec_ld + (step[m*step_stride] + step_off)*N] (per-frame
 * hidden states written inside the captured frame graph at the device step counter(s)). */
int qt_rmsnorm_rec(const float* x, const float* gamma, float eps, float* out, int M, int N, float* rec,
                   long long rec_ld, const int* step, int step_off, int step_stride, void* stream);

/* out[m] = table[idx[m]] (fp32 out, table dtype), nn.Embedding row gather (M:1441, 1670). */
int qt_gather_rows(const void* table, int dtype, const int* idx, int M, int H, float* out, long long ldo, void* stream);

/* Talker decode input (M:1681-1692): x[b] = E0[codes[b,t,0]] + sum_g Ecp[g][codes[b,t,1+g]]
 * + (t < T ? trailing[b][t] : pad), t = step[b*step_stride].  codes: int32 [B][codes_ld] rows holding [F][G].
 * x16 (optional): bf16 copy of x ([B][H]), the A operand of the first layer's RMS-normalised QKV GEMV. */
int qt_frame_embed(const void* emb0, const void* emb_cp, int dtype, int V0, int Vcp, int G, int H,
                   const int* codes, long long codes_ld, const int* step, int step_stride, const float* trailing,
                   int T, const float* pad, float* x, void* x16, int B, void* stream);

/* counters[i] += 1 for i < n (end-of-frame step / position advance inside a captured graph). */
int qt_advance(int* counters, int n, void* stream);
/* per-row counters, field-major [nfields][B], field 0 = each row's frame index: row b advances every field by one
 * while counters[b] < cap (a finished batch slot awaiting its next request stays at frame cap).  The end-of-frame
 * advance of the replaced loop's `cache_position` / `rope_deltas` bookkeeping (M:1693-1711), per request. */
int qt_advance_rows(int* counters, int B, int nfields, int cap, void* stream);

/* ---- codec decoder helpers (K) ---- */
/* SplitResidualVectorQuantizer.decode table gather-sum (K:814-820): out[b][t][:] = sum_q tab_q[codes[b][t][q]],
 * group split: q < n_first -> out_first, else out_rest.  tables fp32 [Q][2048][dim] pre-divided by usage. */
int qt_rvq_gather(const float* tables, int Q, int n_first, int cb_size, int dim, const int* codes, int B, int T,
                  float* out_first, float* out_rest, void* stream);
/* SnakeBeta (K:577-615) channels-last: y = x + inv_beta[c] * sin(x * alpha[c])^2 (alpha/inv_beta pre-exp'd). */
int qt_snake(const void* x, void* y, int dtype, long long rows, int C, const float* alpha, const float* inv_beta,
             void* stream);
/* ConvNeXt depthwise causal conv k=7 + LayerNorm(eps) (K:210-232), channels-last [B][T][C] -> out (dtype). */
int qt_dwconv_ln(const void* x, int dtype, int B, int T, int C, const float* w, const float* b, const float* ln_w,
                 const float* ln_b, float eps, void* out, void* stream);
/* clamp(-1, 1) + dtype -> fp32 pcm (K:883). */
int qt_clamp_pcm(const void* x, int dtype, long long n, float* out, void* stream);

/* ---- voice-clone front end ----
 * T = transformers models/mimi/modeling_mimi.py (the tokenizer encoder, K:898-907, 960-990);
 * M:95-470, 1940-1954 = mel spectrogram + ECAPA-TDNN speaker encoder. */
/* Time-axis pad / copy, channels-last: out[b][t][c] (t < t_total) = src(x)[b][t - left][c] (+ x2 likewise),
 * src per mode for t - left outside [0, T): QT_PAD_ZERO -> 0, QT_PAD_REFLECT -> mirrored (torch "reflect"),
 * QT_PAD_REPLICATE -> edge row; rows >= T + left + right are zero.  Replaces the F.pad of MimiConv1d (T:327-347),
 * Conv1d(padding="same", padding_mode="reflect") (M:246-266) and mel_spectrogram's reflect pad (M:446-449);
 * x2 = the Res2Net running sum (M:114-119).  Strides are in elements (row = one time step). */
int qt_pad_time(const void* x, long long ldx, const void* x2, long long ldx2, int dtype, int B, int T, int C, int left,
                int right, int mode, int t_total, void* out, long long ldo, void* stream);
/* x[b][t][0..C) = 0 for v <= t < Tp (batch stride Tp*ldx): the right "extra" zero padding of a strided MimiConv1d
 * (T:269-279) when the buffer is longer than the valid length. */
int qt_zero_tail(void* x, int dtype, int B, int Tp, int v, int C, long long ldx, void* stream);
/* nn.LayerNorm (T:735-736): out = (x - mean) * rsqrt(var + eps) * w + b per row; x fp32, out dtype. */
int qt_layernorm(const float* x, long long ldx, const float* w, const float* b, float eps, void* out, int o_dtype,
                 long long ldo, int M, int N, void* stream);
/* Residual VQ encode (MimiResidualVectorQuantizer.encode T:1050-1068 / MimiEuclideanCodebook.quantize T:985-991):
 * per row r: res = x[r]; for q < Q: code = argmin_c |res - E_q[c]|^2 (lowest index on ties), res -= E_q[code];
 * codes[r*codes_ld + q] = code.  tab [Q][cb][D] (embed_sum / clamp(cluster_usage, 1e-5)), tabT = the same
 * transposed [Q][D][cb].  D <= 256, cb % 64 == 0.  ws: zero-initialised device scratch of
 * >= qt_rvq_encode_ws_bytes(R, D, cb) bytes, one stream at a time (arrival counters re-arm themselves).
 * Launches Q kernels (one per codebook stage); deterministic. */
long long qt_rvq_encode_ws_bytes(int R, int D, int cb);
int qt_rvq_encode(const float* x, long long ldx, const float* tab, const float* tabT, int Q, int cb, int D, int R,
                  int* codes, long long codes_ld, void* ws, long long ws_bytes, void* stream);
/* log-mel from a real DFT (M:451-468): spec [F][ld_spec] holds (re, im) pairs of nbin bins;
 * out[f][m] = log(max(sum_k basis[m][k] * sqrt(re^2 + im^2 + 1e-9), 1e-5)). */
int qt_mel_logmag(const float* spec, long long ld_spec, int F, int nbin, const float* basis, int nmel, float* out,
                  long long ldo, void* stream);
/* Per-(item, channel) statistics over time (AttentiveStatisticsPooling._compute_statistics M:204-207,
 * SqueezeExcitationBlock mean M:146): w = softmax_t(logits[b][t][c]) (logits != NULL) or 1/T;
 * mean = sum_t w x, std = sqrt(max(sum_t w (x - mean)^2, eps)); mean/std at out[b*ld_out + c] (std optional). */
int qt_time_stats(const void* x, int dtype, long long ldx, const float* logits, long long ldl, int B, int T, int C,
                  float eps, float* mean_out, float* std_out, long long ld_out, void* stream);
/* out[b][t][c] = x[b][t][c] * s[b*lds + c] + res[b][t][c] (SE excitation + block residual, M:150, 322). */
int qt_scale_add(const void* x, long long ldx, const float* s, long long lds, const void* res, long long ldr, int dtype,
                 int B, int T, int C, void* out, long long ldo, void* stream);
/* out[b][t][0..W) = v[b*ldv + 0..W) for all t < T (the mean / std broadcast of attentive pooling, M:225-227). */
int qt_bcast_rows(const float* v, long long ldv, int B, int T, int W, void* out, int o_dtype, long long ldo,
                  void* stream);

#ifdef __cplusplus
}
#endif
#endif
