/*
 * icap.h — C-ABI of libicap_hip.so, the MI355X-native (gfx950) hot path of the
 * prefix image-captioning trainer (reference: thenoobychocobo/gpt2-image-captioning).
 *
 * The reference has no FFI of its own: its seam is the Python module surface of
 * src/models.py / src/train.py, and all of its device arithmetic happens inside
 * HF transformers + ATen. Each entry point below replaces one piece of that
 * arithmetic; the reference call site it stands in for is cited per function
 * (paths relative to the reference root; HF/ = transformers/, TORCH/ = torch/).
 *
 * Conventions
 *  - Plain device pointers + int64 sizes/strides, no torch types. Strides are in
 *    ELEMENTS. Storage dtype is ICAP_F32 (parity mode) or ICAP_BF16 (perf mode);
 *    every kernel computes in fp32. Biases, LayerNorm affine params, optimizer
 *    state and loss outputs are always fp32.
 *  - `stream` is a hipStream_t passed as void*. Every call is asynchronous and
 *    stream-ordered; no call allocates, frees or synchronises, so a sequence of
 *    calls can be captured into a hipGraph. Caller-owned workspaces are sized by
 *    the *_workspace_bytes queries.
 *  - Return 0 on success, nonzero ICAP_ERR_* on failure; icap_last_error()
 *    returns a thread-local message for the last failure on the calling thread.
 *  - Dropout: keep(i) = hash(seed', offset + i) >= p*2^32, scale 1/(1-p); the
 *    index i is the row-major element index of the tensor the mask applies to,
 *    so forward and backward regenerate identical masks. p == 0 disables it.
 *    seed' = seed + (seed_ptr ? *seed_ptr * 0x9E3779B97F4A7C15 : 0): a device
 *    counter (icap_counter_increment) lets a captured graph draw fresh masks
 *    on every replay.
 */
#ifndef ICAP_H
#define ICAP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ICAP_FP8_MX: GEMM operands only (icap_gemm in_dtype): OCP e4m3fn bytes with one E8M0 scale per 32-element */
/* K block (OCP MX), the scales in the layout icap_quantize_mx writes (icap_gemm_args.a_scale / b_scale).      */
enum { ICAP_F32 = 0, ICAP_BF16 = 1, ICAP_FP8_MX = 2 };
enum {
  ICAP_ACT_NONE = 0,
  ICAP_ACT_GELU_NEW = 1,   /* HF/activations.py:59-66 (GPT-2 gelu_new)        */
  ICAP_ACT_RELU = 2,       /* TORCH/nn/modules/transformer.py (mapper FFN)     */
  ICAP_ACT_QUICK_GELU = 3, /* HF/activations.py:117-123 (CLIP)                 */
  ICAP_ACT_TANH = 4,       /* src/models.py:29 (MLPMappingNetwork activation)  */
  ICAP_ACT_GELU_ERF = 5    /* exact erf GELU (HF ViT hidden_act "gelu", src/embeddings/vit.py) */
};
enum { ICAP_OK = 0, ICAP_ERR_ARG = 1, ICAP_ERR_LAUNCH = 2 };

const char* icap_last_error(void);
int icap_version(void);
/* number of device kernels compiled into the library (>0 when the gfx950 code object loaded) */
int icap_device_arch_ok(void);

/* ------------------------------------------------------------------------- */
/* GEMM: C[M,N] = epi(alpha * A[M,K] . B[N,K]^T)                              */
/* Replaces every dense contraction of the path: GPT-2 Conv1D c_attn/c_proj/  */
/* c_fc/mlp.c_proj (HF/models/gpt2/modeling_gpt2.py:185,223,238-241;          */
/* HF/pytorch_utils.py:117-121), the tied LM head (modeling_gpt2.py:698),     */
/* the mapper Linear + encoder projections (src/models.py:119,129-139,154),   */
/* MLPMappingNetwork (src/models.py:52-56), CLIP patch-embed/q,k,v/out/fc1/fc2/*/
/* visual_projection (HF/models/clip/modeling_clip.py:148-154,280-350,751),   */
/* and every backward dX / dW product of train.py:145.                         */
/* Both operands are K-contiguous (row-major A, row-major B = "weight [out,in]").*/
/* Epilogue order (forward): v = alpha*acc + bias[n];                          */
/*   if aux: aux[m,n] = (act==TANH ? act(v) : v);  v = act(v);                 */
/*   v *= dropmask(m*N+n);  if resid: v += resid[m,n];  C = beta*C + v.        */
/* Backward epilogue (dact != NONE): v = alpha*acc * dropmask * act'(dact_src).*/
/* Constraints: K % 8 == 0 (bf16) / K % 4 == 0 (f32); lda,ldb multiples of 8/4;*/
/* beta != 0 only with f32 C.                                                  */
/* ------------------------------------------------------------------------- */
typedef struct {
  int64_t M, N, K;
  int32_t in_dtype;   /* dtype of A and B */
  int32_t c_dtype;    /* dtype of C, aux, resid, dact_src */
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc;
  float alpha, beta;
  const float* bias;  /* [N] or NULL */
  int32_t act;        /* ICAP_ACT_* forward activation */
  void* aux; int64_t ldaux;             /* store of pre-activation (or tanh output) or NULL */
  int32_t dact;                          /* backward: multiply by act'(dact_src) */
  const void* dact_src; int64_t ld_dact;
  const void* resid; int64_t ldr;        /* residual added last, or NULL */
  float drop_p; uint64_t seed; uint64_t offset;
  const uint64_t* seed_ptr;               /* optional device seed counter */
  /* split-K: fp32 scratch of >= splits*M*N*4 bytes (16-byte aligned) or NULL.   */
  /* split_k: 0 = automatic (launches that cannot fill the chip, N % 4 == 0,    */
  /* and only when the workspace is given), 1 = never, > 1 = forced.            */
  /* The partial sums are reduced in a fixed order (deterministic). The split   */
  /* count is a function of (M, N, K, dtype, trans_ab, m_hint) only — never of  */
  /* the workspace size or of the tickets: a workspace smaller than that split  */
  /* needs is ICAP_ERR_ARG, never a different summation order.                  */
  void* workspace; int64_t workspace_bytes; int32_t split_k;
  /* optional device-side row count (int32, <= M): only rows < *m_dev are     */
  /* computed and stored; the launch geometry stays sized for M, so a graph   */
  /* captured once serves every count (LM head over the compacted targets).   */
  const int32_t* m_dev;
  /* trans_ab != 0: both operands K-outer — A stored [K][lda] (element (m,k) at A[k*lda+m]), B stored      */
  /* [K][ldb] — the weight-gradient products dW = dY^T X over token rows (src/train.py:145 backward of   */
  /* every nn.Linear / Conv1D) without transposing either operand. bf16 inputs, lda >= M, ldb >= N.    */
  int32_t trans_ab;
  /* ln_gamma != NULL: A is replaced by LayerNorm(A) over its K columns first (row mean / variance, eps,    */
  /* then * ln_gamma[k] + ln_beta[k], rounded to the input dtype) — the decode step's ln_1 / ln_2 fused    */
  /* into the QKV / c_fc GEMMs (HF/models/gpt2/modeling_gpt2.py:281,301). Only for M <= 128 launches.     */
  const float* ln_gamma; const float* ln_beta; float ln_eps;
  /* path: 0 = automatic kernel choice; 1 = the 128-row tile kernels only; (2: the round-2 persistent ring    */
  /* kernel, measured slower and removed: rejected); 3 = the 256 x 256 8-phase kernel wherever its           */
  /* preconditions hold (bf16 A/B, no trans_ab / ln / beta /                                                   */
  /*     m_dev / split-K, M and N >= 256) —                                                                      */
  /* for A/B measurements and for tests that compare the two paths (identical MFMA chains: bitwise equal);    */
  /* 4 / 5 = the 256-row 8-phase kernel with 128- / 256-column tiles wherever its preconditions hold (bf16    */
  /*     A/B, no trans_ab / ln_gamma / split-K, M >= 256, K >= 64; m_dev and the LayerNorm hand-off allowed:   */
  /*     csrc/gemm8p.hip) — same use; 6 = the 256 x 128 tile kernel on the 3-stage ring (csrc/gemm_tile.h       */
  /*     variant 22) for unsplit bf16 row-major launches, M >= 256 — same use; 7 = 192 x 64 tiles (variant 24:  */
  /*     4 waves stacked in M) for bf16 row-major launches without a LayerNorm fold / consumer, M >= 192,       */
  /*     unsplit — same use; 8 / 9 / 10 = the split-role ring kernel (4 or 8 MFMA waves + 4 LDS-DMA waves,    */
  /*     one block per CU: csrc/gemm_tile.h ROLES) on 128 x 256 (variant 26) / 96 x 128 (variant 27) /          */
  /*     192 x 256 (variant 28) tiles for bf16 row-major launches without ln_gamma (9: no LayerNorm consumer),  */
  /*     unsplit unless split_k > 1 is given (not 28: fp32 slabs + the reduce pass, as the tile kernels, no     */
  /*     LayerNorm hand-off) — same use; 11 = the K-outer split-role kernel (variant 31, 128 x 128 tiles) for bf16 */
  /*     trans_ab launches, K split over slabs by its own rule unless split_k is given — same use; 12 = the     */
  /*     split-role ring on 160 x 128 tiles (variant 32, no LayerNorm consumer) — same use.                     */
  int32_t path;
  /* in_dtype == ICAP_FP8_MX: the E8M0 block scales of A (M rows) and B (N rows), K % 128 == 0, lda / ldb      */
  /* multiples of 16, 16-byte aligned. For a 128-element K stage s and 64-row group g, 256 bytes at offset      */
  /* (s * ceil(R/64) + g) * 256: row r's 4 block scales at ((r % 16) * 16 + ((r / 16) % 4) * 4) (R = M or N),   */
  /* i.e. K/32 * ceil(R/64) * 64 bytes. The product is sum_k a[m,k] 2^(sa-127) b[n,k] 2^(sb-127) in fp32       */
  /* (v_mfma_scale_f32_16x16x128_f8f6f4), then the same epilogue as bf16 / f32 inputs.                       */
  const uint8_t* a_scale; const uint8_t* b_scale;
  /* m_hint (with m_dev): the expected device row count, for the kernel choice only (0: M). Any count <= M is   */
  /* computed correctly whatever the hint; a captured graph keeps the choice made at capture.                   */
  int64_t m_hint;
  /* tickets (optional): int32 scratch of tickets_len entries, all ZERO before the first launch that uses it; every */
  /* launch leaves them zero. With it (and the workspace), automatic split-K over few output tiles (long K, fewer  */
  /* tiles than CUs) combines the partial tiles inside the launch — the last split of a tile to finish adds the    */
  /* others' partials in split order and applies the epilogue — instead of a separate reduce pass over fp32 slabs. */
  /* Needs 2 entries per 128 x 128 output tile. One buffer per stream (like workspace); deterministic. The tickets */
  /* choose only the mechanism: without them (or too few) the same split runs through the reduce pass, and both   */
  /* store bitwise-identical outputs. After a device fault the tickets may be left non-zero (zero them again).    */
  int32_t* tickets; int64_t tickets_len;
  /* ln_wsum != NULL (M <= 128, no ln_gamma): LayerNorm folded into the weights — B holds W[n,k] * gamma[k],  */
  /* ln_wsum[n] = sum_k B[n,k] (fp32, over the stored B values) and bias = b + W . beta, so                    */
  /* C = rstd_m * (A . B^T - mean_m * ln_wsum) + bias equals LN(A) . W^T + b with the row mean / rstd of A  */
  /* (eps = ln_eps) taken inside the launch from the A fragments it already reads; the product runs on raw A  */
  /* (the decode step's ln_1 / ln_2, frozen GPT-2: HF/models/gpt2/modeling_gpt2.py:281,301).                 */
  const float* ln_wsum;
  /* LayerNorm statistics handed from one tile-kernel GEMM to the next (the frozen forward's ln_1 / ln_2 folded     */
  /* into the QKV / c_fc products: HF/models/gpt2/modeling_gpt2.py:281,301; CLIP layer_norm1/2                     */
  /* modeling_clip.py:365-384). ln_stats_out (producer, bf16 C, N % 32 == 0): per row and 32-column group of the   */
  /* stored C values, (mean, M2 = sum of squared deviations) as fp32 pairs [M][N/32][2]. ln_stats_in (consumer,    */
  /* with ln_wsum, bias = b + W.beta, B = W*gamma, ln_eps; K % 128 == 0, K <= 1280, 16-byte aligned): the        */
  /* producer's statistics of A                                                                                      */
  /* [M][K/32][2], combined per row (two-pass: mean of the group means, then M2 + 32 (mean_g - mean)^2) into mean  */
  /* and rstd = 1/sqrt(M2/K + eps), and C = rstd (A.B^T - mean ln_wsum) + bias, then the epilogue. ln_mean_out /   */
  /* ln_rstd_out (optional, consumer): those row statistics (fp32 [M]) for the LayerNorm backward. bf16 inputs,   */
  /* tile kernels only (M > 128 or not), no trans_ab; a split product must be able to combine inside the launch.  */
  float* ln_stats_out; const float* ln_stats_in; float* ln_mean_out; float* ln_rstd_out;
  /* Diagnostic builds only (compiled with -DICAP_STAMPS; ignored otherwise, keep NULL): 8 uint64 per tile-kernel   */
  /* workgroup (blockIdx.x) — phase timestamps (s_memrealtime, 100 MHz) for tools/gemm_stamps.py.                  */
  uint64_t* diag_stamps;
} icap_gemm_args;
/* MX block quantisation (the A / B operands of an ICAP_FP8_MX GEMM): x [R, K] (f32 or bf16, row stride ldx) */
/* -> q [R, K] OCP e4m3fn bytes (row stride ldq % 16 == 0) + the E8M0 scales in icap_gemm_args.a_scale      */
/* layout (icap_mx_scale_bytes(R, K) bytes). Per 32-element block: X = min integer with amax <= 448 * 2^X    */
/* (no element saturates), code X + 127; element = RNE_e4m3(v * 2^-X). K % 128 == 0; 16-byte aligned rows.  */
/* No reference counterpart: the reference computes in fp32 (BASELINE configs[4] asks for the fp8 path);     */
/* GPT-2 large's frozen weights are quantised once, activations before each fp8 product.                    */
size_t icap_mx_scale_bytes(int64_t R, int64_t K);
/* rows_dev: optional device int32 row count (<= R): rows past it are not read (the compacted LM-head rows). */
int icap_quantize_mx(int32_t dtype, int64_t R, int64_t K, const void* x, int64_t ldx, void* q, int64_t ldq,
                     void* scales, const int32_t* rows_dev, void* stream);
/* name of the kernel instantiation icap_gemm launches for these arguments    */
/* (as rocprofv3 prints it, minus the parameter list); NULL on invalid args.   */
const char* icap_gemm_kernel_name(const icap_gemm_args* a);
/* the split-K factor icap_gemm takes for these arguments and whether the splits combine inside the launch   */
/* (tickets) or in a separate reduce pass; ICAP_ERR_ARG on invalid args. Host-only (tests, tools).          */
int icap_gemm_plan_info(const icap_gemm_args* a, int32_t* splits, int32_t* fused);
int icap_gemm(const icap_gemm_args* a, void* stream);
/* Replaces a layer's weight-gradient products of the mapper backward (TORCH/nn/modules/transformer.py:        */
/* 946-950 linear1 / linear2, TORCH/nn/modules/activation.py in_proj / out_proj via src/train.py:145): a group  */
/* of n (1 ... 8) K-outer products a[0 .. n-1] (trans_ab, bf16 A / B, fp32 C, alpha / beta, no epilogue        */
/* operands, no m_dev) in ONE launch, each unsplit on the split-role K-outer kernel (path 11's body): no split-K */
/* slabs, no reduce pass, the group's tiles filling the chip together. Bitwise what icap_gemm gives each with   */
/* split_k = 1 and path 11; products with M or N = 0 are skipped.                                              */
int icap_gemm_group(const icap_gemm_args* a, int32_t n, void* stream);

/* ------------------------------------------------------------------------- */
/* LayerNorm over the last dim D (eps given; GPT-2 ln_1/ln_2/ln_f             */
/* modeling_gpt2.py:252-254,497,620; mapper norm1/norm2 TORCH transformer.py  */
/* :946-950; CLIP pre/post/layer_norm1/2 modeling_clip.py:641-651,365-384).   */
/* y = (x-mean)*rstd*gamma + beta; mean/rstd (fp32 [rows]) saved for backward. */
/* D % 4 == 0, D <= 1024.                                                      */
/* ------------------------------------------------------------------------- */
/* y_rowmap (optional int32 [rows]): row r is stored to y row y_rowmap[r], or  */
/* not at all when it is < 0 (gathers the LM-head target rows).                */
/* rows_dev (optional device int32, <= rows): only rows < *rows_dev are read and written (packed token rows, */
/* icap_caption_pack); the launch stays sized for `rows`, so one captured graph serves every count.          */
int icap_layernorm_fwd(int32_t dtype, int64_t rows, int64_t D, const void* x, int64_t ldx,
                       const float* gamma, const float* beta, float eps, void* y, int64_t ldy,
                       float* mean, float* rstd, const int32_t* y_rowmap, const int32_t* rows_dev,
                       void* stream);
/* dx = LN'(x)^T dy [+ dres];  optional dx_drop = dx * dropmask(p,seed,offset)  */
/* (the residual-dropout backward of the producing layer, fused);             */
/* optional dgamma/dbeta (fp32 [D]: += by default, = when param_overwrite bit 0 */
/* is set — the first micro-batch of a cycle overwrites instead of zeroing     */
/* first) via a caller workspace of icap_layernorm_bwd_workspace_bytes(rows, D) */
/* bytes. param_overwrite bit 1: leave the per-block partials in the workspace */
/* and skip their reduce — the caller reduces them with                        */
/* icap_ln_param_reduce_batch (several LayerNorms in one launch).              */
/* dy_rowmap (optional int32 [rows]): dy of row r is dy row dy_rowmap[r], or 0 */
/* when it is < 0 (scatters the LM-head target-row gradient back).             */
/* rows_dev: as in icap_layernorm_fwd.                                         */
size_t icap_layernorm_bwd_workspace_bytes(int64_t rows, int64_t D);
int icap_layernorm_bwd(int32_t dtype, int64_t rows, int64_t D, const void* x, int64_t ldx,
                       const float* gamma, const float* mean, const float* rstd,
                       const void* dy, int64_t lddy, const void* dres, int64_t lddres,
                       void* dx, int64_t lddx, void* dx_drop, float drop_p, uint64_t seed,
                       uint64_t offset, const uint64_t* seed_ptr, float* dgamma, float* dbeta,
                       void* workspace, const int32_t* dy_rowmap, const int32_t* rows_dev,
                       int32_t param_overwrite, void* stream);
/* The deferred dgamma / dbeta reduces (param_overwrite bit 1 above) of n <= ICAP_LN_PARAM_BATCH_MAX LayerNorm    */
/* backwards in one launch; item: that call's workspace, rows, D, dgamma, dbeta and overwrite (bit 0). Bitwise   */
/* the per-call reduce.                                                                                         */
#define ICAP_LN_PARAM_BATCH_MAX 16
typedef struct icap_ln_param_item {
  const void* workspace; int64_t rows; int64_t D; float* dgamma; float* dbeta; int32_t overwrite;
} icap_ln_param_item;
int icap_ln_param_reduce_batch(int32_t n, const icap_ln_param_item* items, void* stream);

/* ------------------------------------------------------------------------- */
/* Multi-head softmax attention over a fused QKV activation.                  */
/* GPT-2: causal + key padding (HF/integrations/sdpa_attention.py:79-166,     */
/* HF/masking_utils.py:76-80,168-180), attn dropout modeling_gpt2.py:87;      */
/* mapper MHA (TORCH/nn/modules/activation.py, bidirectional, hd 96);         */
/* CLIP (modeling_clip.py:280-335, bidirectional).                            */
/* Row of token (b,s) = b*row_stride_b + s*row_stride_s in qkv/out/dqkv/dout. */
/* q at column h*hd, k at D+h*hd, v at 2D+h*hd (D = H*hd).                     */
/* allowed(q,k) = (!causal || k<=q) && (!key_mask || key_mask[b*S+k]).         */
/* ------------------------------------------------------------------------- */
typedef struct {
  int32_t dtype;
  int32_t B, S, H, hd;
  int64_t row_stride_b, row_stride_s;
  const void* qkv; int64_t ld_qkv;
  void* out; int64_t ld_out;  /* fwd: O (written). bwd: O of the forward (read, optional: with it the   */
                              /* bf16 MFMA backward takes delta = rowsum(dO o O) and needs no transposes) */
  float* lse;               /* [B*H*S] fp32 log-sum-exp of scaled scores, or NULL */
  const int32_t* key_mask;  /* [B*S] or NULL */
  int32_t causal;
  float scale;
  float drop_p; uint64_t seed; uint64_t offset; /* dropout on P, index (b*H+h)*S*S + q*S + k */
  const uint64_t* seed_ptr;
  /* backward only */
  const void* dout; int64_t ld_dout;
  void* dqkv; int64_t ld_dqkv;
  /* packed (unpadded) sequences, both or neither (icap_caption_pack): sequence b has seq_len[b] <= S tokens */
  /* at rows seq_off[b] + s (row_stride_s must be 1; row_stride_b is unused); key_mask is then indexed by    */
  /* that packed row. lse and the dropout index keep the padded [B, H, S(, S)] numbering, so a packed and a   */
  /* padded call draw the same masks for the same (b, h, q, k).                                                */
  const int32_t* seq_off; const int32_t* seq_len;
  /* packed only: 1 = the caller guarantees every seq_len[b] <= 32, so only the pass over short sequences runs   */
  /* (the launch over S > 32 tokens is otherwise split into a short pass and a pass for the longer ones, whose  */
  /* blocks the short sequences exit; a longer sequence under short_only = 1 would be left unwritten). 0 = both. */
  int32_t short_only;
} icap_attn_args;
int icap_attention_fwd(const icap_attn_args* a, void* stream);
int icap_attention_bwd(const icap_attn_args* a, void* stream);

/* Decode-step attention (KV-cached greedy decode; replaces the full          */
/* recompute of src/models.py:395 with an exactly-equivalent causal step).    */
/* cache rows are position-major: row of (b, t) = t*B + b, ld = 3*D (fused qkv).*/
/* The new token is at position `pos`; attends to keys 0..pos.                 */
int icap_attention_decode(int32_t dtype, int32_t B, int32_t H, int32_t hd, int32_t pos,
                          const void* cache, int64_t ld_cache, void* out, int64_t ld_out,
                          float scale, void* stream);
/* Same with KV ancestry (beam search): key t of row b is cache row t*B + anc[t*B + b]       */
/* (anc int32 [pos+1][B]; NULL = the row's own). Replaces the KV-cache reorder of           */
/* HF/generation/utils.py:3476-3488 (Cache.reorder_cache) without moving cache bytes.        */
int icap_attention_decode_anc(int32_t dtype, int32_t B, int32_t H, int32_t hd, int32_t pos,
                              const void* cache, int64_t ld_cache, const int32_t* anc, void* out,
                              int64_t ld_out, float scale, void* stream);

/* ------------------------------------------------------------------------- */
/* Caption/prefix assembly for the GPT-2 input (src/models.py:261,283-317,    */
/* modeling_gpt2.py:571-577,604):                                               */
/*   x[b,t] = (t<P ? prefix[b*prefix_bstride + t*D] : wte[ids[b,t-P]]) + wpe[t]*/
/*   then embd dropout.  key_mask[b,t] = t<P ? 1 : mask[b,t-P] (1 if mask NULL)*/
/*   labels_shift[b*S+t] = t+1<S ? (t+1<P ? -100 : labels[b,t+1-P]) : -100    */
/*   (HF/loss/loss_utils.py:49-71 shift).  S = P + L. ids/mask/labels int64.   */
/* ------------------------------------------------------------------------- */
/* seq_off / seq_len (optional, both or neither; icap_caption_pack): packed rows — token (b,t) goes to row   */
/* seq_off[b] + t and only t < seq_len[b] is written (the dropout index is that row's element index).        */
int icap_gpt2_embed(int32_t dtype, int32_t B, int32_t P, int32_t L, int32_t D,
                    const void* prefix, int64_t prefix_bstride, const void* wte,
                    const void* wpe, const int64_t* ids, void* x, float drop_p,
                    uint64_t seed, uint64_t offset, const uint64_t* seed_ptr,
                    const int32_t* seq_off, const int32_t* seq_len, void* stream);
/* backward of the caption-token gather when GPT-2 is trained (freeze_gpt_weights=False): */
/* dwte[ids[b,t]] += dx[b*(P+L) + P + t]  (fp32 atomics)                                    */
int icap_embedding_scatter_add(int32_t dtype, int32_t B, int32_t P, int32_t L, int32_t D,
                               const void* dx, const int64_t* ids, float* dwte, void* stream);
/* Target compaction (optional, both or neither): row_slot[b*S+t] = index of  */
/* row (b,t) among the rows whose shifted label != -100 (row order), else -1;  */
/* labels_compact[row_slot[i]] = labels_shift[i]. Only those n_valid rows       */
/* reach the loss (loss_utils.py:32-46 ignore_index=-100), so the LM head and  */
/* CE run on them alone; everything they feed back is identical.              */
int icap_caption_prep(int32_t B, int32_t P, int32_t L, const int64_t* mask,
                      const int64_t* labels, int32_t* key_mask, int32_t* labels_shift,
                      int32_t* n_valid, int32_t* row_slot, int32_t* labels_compact, void* stream);
/* Packed (unpadded) token rows for the training step. A position t of caption b feeds the loss only if its  */
/* shifted label is not -100 (loss_utils.py:32-46) or if a later such position attends to it; attention is   */
/* causal (modeling_gpt2.py causal mask), so every position after the last target-feeding one is dead: its   */
/* hidden states reach no loss term and no gradient (padding keys are masked out, labels -100). Only the     */
/* live prefix of each sequence is kept:                                                                     */
/*   seq_len[b] = max(P, 1 + last t with labels_shift[b,t] != -100), seq_off = exclusive scan, m_live = sum;  */
/*   key_mask / labels_shift / row_slot (+ labels_compact, n_valid: as icap_caption_prep) in packed rows;     */
/*   rows in [m_live, B*(P+L)) get key_mask 0, labels_shift -100, row_slot -1.                               */
/* The compacted target rows come out in the same order as icap_caption_prep's, so the LM head / CE see the  */
/* same rows; loss and gradients equal the padded computation's (within the GEMM summation order).          */
int icap_caption_pack(int32_t B, int32_t P, int32_t L, const int64_t* mask, const int64_t* labels,
                      int32_t* seq_off, int32_t* seq_len, int32_t* m_live, int32_t* key_mask,
                      int32_t* labels_shift, int32_t* n_valid, int32_t* row_slot, int32_t* labels_compact,
                      void* stream);
/* dst[b*dst_bstride + t*D + d] = t < seq_len[b] ? src[(seq_off[b] + t)*D + d] : 0, for t < P (the prefix     */
/* rows' gradient of a packed step back to the [B, P, D] layout the mapper backward reads). D % 4 == 0.     */
int icap_rows_unpack(int32_t dtype, int32_t B, int32_t P, int32_t D, const void* src, const int32_t* seq_off,
                     const int32_t* seq_len, void* dst, int64_t dst_bstride, void* stream);

/* ------------------------------------------------------------------------- */
/* Causal-LM cross entropy fused with its backward (HF/loss/loss_utils.py     */
/* :32-46,49-71): per row r with label y != -100 over V classes:               */
/*   loss_r = lse(x_r) - x_r[y];  loss = sum(loss_r)/n_valid                   */
/*   dlogits_r = grad_scale*(softmax(x_r) - onehot(y))/n_valid (0 for ignored  */
/*   rows and for padding columns V..ld). dlogits may alias logits. n_valid is */
/*   read from device memory (written by icap_caption_prep).                   */
/*   rows_dev (optional): only rows r < *rows_dev exist (compacted targets);    */
/*   the others are neither read nor written.                                  */
/* ------------------------------------------------------------------------- */
size_t icap_cross_entropy_workspace_bytes(int64_t rows);
int icap_cross_entropy(int32_t dtype, int64_t rows, int64_t V, const void* logits, int64_t ld,
                       const int32_t* labels, const int32_t* n_valid, float* loss,
                       void* dlogits, float grad_scale, void* workspace, const int32_t* rows_dev,
                       void* stream);

/* ------------------------------------------------------------------------- */
/* Global grad-norm clip + AdamW + linear LR schedule over ONE flat fp32       */
/* parameter buffer (src/train.py:94-103,150-159; TORCH/nn/utils/clip_grad.py */
/* :121-186; TORCH/optim/adam.py:419,457,476,499,545-547;                       */
/* HF/optimization.py:101-107). Step counter and lr live in device memory     */
/* (`state`, 64 bytes, zero-initialised by the caller) so the call is graph-   */
/* capturable. bf16_out (optional) receives the updated params in bf16.        */
/* state layout (float/int64 view): [0]=int64 step (completed steps),         */
/* [2]=f32 last grad norm, [3]=f32 clip coef, [4]=f32 lr used, [5]=f32 step   */
/* size lr/bc1, [6]=f32 sqrt(bc2), [7]=f32 decay factor 1-lr*wd.              */
/* ------------------------------------------------------------------------- */
typedef struct {
  int64_t n;
  float* params; float* grads; float* exp_avg; float* exp_avg_sq;
  void* bf16_out;           /* or NULL */
  void* state;              /* 64-byte device state */
  float lr, beta1, beta2, eps, weight_decay;
  float max_norm;           /* <= 0 disables clipping */
  int64_t num_warmup_steps, num_training_steps;
} icap_adamw_args;
size_t icap_adamw_workspace_bytes(int64_t n);
int icap_adamw_step(const icap_adamw_args* a, void* workspace, void* stream);
/* sum of squares of a flat fp32 buffer -> out[0] (deterministic) */
int icap_sqnorm(int64_t n, const float* x, float* out, void* workspace, void* stream);

/* ------------------------------------------------------------------------- */
/* Layout / reduction helpers used by the backward pass.                      */
/* ------------------------------------------------------------------------- */
/* dst[c*ldd + r] = src[r*lds + c] for r<rows, c<cols; zero for rows<=r<rows_pad */
int icap_transpose(int32_t dtype, int64_t rows, int64_t cols, const void* src, int64_t lds,
                   void* dst, int64_t ldd, int64_t rows_pad, void* stream);
/* Several bf16 transposes in one launch: dst[c*ldd + r] = src[r*lds + c] per item (r < rows, c < cols). Items   */
/* with rows % 64, cols % 8, lds % 8, ldd % 8 == 0 and 16-byte aligned pointers share one launch (up to 32 per     */
/* launch); others fall back to icap_transpose. (The trained mapper's transposed weight copies after each step.)   */
typedef struct {
  const void* src; int64_t lds; void* dst; int64_t ldd; int64_t rows; int64_t cols;
} icap_transpose_item;
int icap_transpose_batch(int32_t n, const icap_transpose_item* items, void* stream);
/* out[n] (+)= sum_m src[m*ld + n]  (bias grads, prefix_const grad); fp32 out */
size_t icap_colsum_workspace_bytes(int64_t M, int64_t N);
int icap_colsum(int32_t dtype, int64_t M, int64_t N, const void* src, int64_t ld, float* out,
                int32_t accumulate, void* workspace, void* stream);
/* Several column sums over the same M rows in two launches (partials + reduce) instead of two each: the trained  */
/* mapper's four bias gradients per layer (src/models.py:100-107 TransformerMapper -> nn.TransformerEncoderLayer    */
/* linear1 / linear2 / in_proj / out_proj biases). Every item needs N % 4 == 0, ld % 4 == 0 and a src aligned to   */
/* 4 elements; at most ICAP_COLSUM_BATCH items. Each out equals what icap_colsum gives for the same item (same     */
/* chunking and summation order: bitwise). Workspace: icap_colsum_workspace_bytes(M, sum of the items' N).          */
#define ICAP_COLSUM_BATCH 16
typedef struct {
  const void* src; int64_t ld; int64_t N; float* out;
} icap_colsum_item;
int icap_colsum_batch(int32_t dtype, int64_t M, int32_t n, const icap_colsum_item* items, int32_t accumulate,
                      void* workspace, void* stream);
/* dst[m, n] = src[m, n] * dropmask(p, seed, offset + m*N + n) (or plain copy) */
int icap_dropout_apply(int32_t dtype, int64_t M, int64_t N, const void* src, int64_t lds,
                       void* dst, int64_t ldd, float drop_p, uint64_t seed, uint64_t offset,
                       const uint64_t* seed_ptr, void* stream);
/* *counter += 1 (device-side dropout seed counter, graph-capturable) */
int icap_counter_increment(uint64_t* counter, void* stream);
/* dtype conversion copy, strided rows: dst = (dst_dtype) src */
int icap_convert(int32_t src_dtype, int32_t dst_dtype, int64_t M, int64_t N, const void* src,
                 int64_t lds, void* dst, int64_t ldd, void* stream);
/* dst[b, r, :] = src[r, :] for b < B (broadcast fp32 rows into a strided dtype tensor):  */
/* mapper prefix_const expand (src/models.py:163-168).                                    */
int icap_broadcast_rows(int32_t dtype, int32_t B, int64_t R, int64_t D, const float* src,
                        void* dst, int64_t dst_bstride, void* stream);

/* ------------------------------------------------------------------------- */
/* CLIP ViT image tower helpers (HF/models/clip/modeling_clip.py:148-219,     */
/* 650-651,751; src/embeddings/clip.py:132-137).                              */
/* ------------------------------------------------------------------------- */
/* patches[(b*G*G + gy*G + gx), c*p*p + ky*p + kx] = pixels[b, c, gy*p+ky, gx*p+kx] (fp32 in); */
/* rows hold round_up(C*p*p, 8) elements, the pad zero (ViT-L/14: 588 -> 592)                 */
int icap_im2col_patches(int32_t dtype, int32_t B, int32_t C, int32_t HW, int32_t patch,
                        const float* pixels, void* patches, void* stream);
/* x[b, 0] = cls + pos[0];  x[b, 1+i] = patch_emb[b*G2 + i] + pos[1+i] */
int icap_vit_embed(int32_t dtype, int32_t B, int32_t G2, int32_t D, const void* patch_emb,
                   const float* cls, const float* pos, void* x, void* stream);
/* Patch embedding + token assembly in one launch, for bf16 towers (round 5; replaces icap_im2col_patches + the
 * patch GEMM + icap_vit_embed / icap_prefix_embed of HF CLIP modeling_clip.py:148-154,209-217, ViT modeling_vit.py,
 * DINOv3 modeling_dinov3_vit.py:75-92; reached through src/embeddings/clip.py:132, vit.py:120, dino.py:166).
 * pixels fp32 [B, C, HW, HW]; w bf16 [N][ldw] = the Conv2d weight flattened in (c, ky, kx) order, columns
 * [C p p, Kp) zero. Rows of out (bf16, ld ldo): out[b S + r] = prefix[r] (+ pos[r]) for r < NP (fp32 prefix [NP, N]:
 * CLS, registers) and out[b S + NP + i] = patch_i(b) . W^T (+ bias) (+ pos[NP + i]), S = NP + (HW / p)^2, patch i
 * in row-major (py, px) order — fp32 sums, rounded once. The GEMM reads the pixels itself (no patch matrix). */
int icap_patch_embed(int32_t B, int32_t C, int32_t HW, int32_t patch, int32_t NP, int32_t N, const float* pixels,
                     const void* w, int64_t ldw, int32_t Kp, const float* bias, const float* pos, const float* prefix,
                     void* out, int64_t ldo, void* stream);
/* DINOv3 token assembly (HF/models/dinov3_vit/modeling_dinov3_vit.py:75-92; BASELINE configs[4], reference
 * src/embeddings/dino.py:166): x[b, t] = prefix[t] (t < NP: CLS, then the register tokens) or
 * patch_emb[b*G2 + t - NP] (t >= NP), plus pos[t] when pos != NULL. prefix fp32 [NP, D], pos fp32 [NP + G2, D]. */
int icap_prefix_embed(int32_t dtype, int32_t B, int32_t G2, int32_t NP, int32_t D, const void* patch_emb,
                      const float* prefix, const float* pos, void* x, void* stream);
/* Rotary position embedding of the patch tokens, in place on the fused QKV activation (DINOv3:
 * modeling_dinov3_vit.py:203-268): for rows t >= NP of each image, q = cols [0, H hd) and k = [H hd, 2 H hd),
 * per head x <- x * cos + rotate_half(x) * sin, rotate_half(x) = (-x[hd/2:], x[:hd/2]); cos / sin fp32
 * [S - NP, hd]. Rows of image b start at b*S; ld_qkv in elements. */
int icap_rope_patches(int32_t dtype, int32_t B, int32_t S, int32_t NP, int32_t H, int32_t hd, void* qkv,
                      int64_t ld_qkv, const float* cos_t, const float* sin_t, void* stream);
/* out[b] = x[b] / ||x[b]||_2 (fp32 out) */
int icap_l2norm_rows(int32_t dtype, int64_t rows, int64_t D, const void* x, int64_t ldx,
                     float* out, int64_t ldo, void* stream);

/* ------------------------------------------------------------------------- */
/* Greedy-decode step helpers (src/models.py:389-469).                        */
/* ------------------------------------------------------------------------- */
/* next[b] = finished[b] ? eos : (forced ? forced[b] : argmax_v(logits[b, :V]))  */
/* (argmax: first max on ties; forced: ids drawn by the top-p sampler);          */
/* finished[b] |= next[b]==eos; tokens[b*ld_tokens + step] = next[b];          */
/* x[b] = wte[next[b]] + wpe[pos] (the next step's input embedding).           */
int icap_greedy_next(int32_t dtype, int32_t B, int64_t V, const void* logits, int64_t ld,
                     int64_t eos, const int64_t* forced, int32_t* finished, int64_t* tokens, int64_t ld_tokens,
                     int32_t step, const void* wte, const void* wpe, int32_t pos, int32_t D,
                     void* x, void* stream);
/* Nucleus sampling of one next token per row (the temperature / top-p branch of   */
/* src/models.py:400-449): l = logits[b] / temperature; keep the */
/* reference's filter set (stable descending sort, cumsum(softmax) > top_p removed */
/* after a shift right by one; top_p >= 1 keeps all); draw by inverse CDF over the */
/* kept tokens in index order with u = hash32(seed', step << 32 | b) / 2^32, where  */
/* seed' = seed + (*seed_ptr) * golden when seed_ptr != NULL. Probabilities are    */
/* 2^31 fixed point (exact integer sums, deterministic). finished[b] != 0 -> eos.  */
/* out: int64 [B]. Needs V <= 65536, temperature > 0.                            */
int icap_topp_sample(int32_t dtype, int32_t B, int64_t V, const void* logits, int64_t ld, float temperature,
                     float top_p, const int32_t* finished, uint64_t seed, const uint64_t* seed_ptr,
                     int32_t step, int64_t eos, int64_t* out, void* stream);
/* ------------------------------------------------------------------------- */
/* Beam search. The reference decodes greedy / top-p  */
/* only (src/models.py:327-477); the definition is transformers' beam search */
/* (GPT2LMHeadModel.generate(num_beams=W, do_sample=False, early_stopping=   */
/* False), HF/generation/utils.py:3208-3540). Decode rows r = b*W + i.        */
/* Per step: icap_beam_rowtop over the R = B*W logits rows, then             */
/* icap_beam_update. icap_beam_init before the first step (after prefill of  */
/* P positions for all R rows), icap_beam_finalize after the last.           */
/* ------------------------------------------------------------------------- */
typedef struct {
  int32_t B, W, V, max_len;          /* captions, beams per caption (<= 8), vocab, token budget     */
  int32_t eos; float length_penalty;
  int32_t K;                         /* row candidates from icap_beam_rowtop: 8 (W <= 4), 16 (W <= 8)*/
  int32_t T;                         /* KV-cache positions (prefix + max_len), <= 1024               */
  const float* top_val; const int32_t* top_idx; const float* top_m; const float* top_ls;
  void* ws;                          /* icap_beam_workspace_bytes(B, W, T, max_len), 16-byte aligned */
  int32_t dtype, D, n_positions;     /* next-step input embedding x[r] = wte[tok] + wpe[pos+1]      */
  const void* wte; const void* wpe; void* x;  /* x [R, D] may be NULL (no next step)             */
} icap_beam_args;
size_t icap_beam_workspace_bytes(int32_t B, int32_t W, int32_t T, int32_t max_len);
/* The workspace carve-up in 4-byte words: word_offsets[0..8] = run_score, run_seq, fin_score,   */
/* fin_len, fin_seq, fin_cnt, done (int32 per caption: 1 once its search is over), anc (int32   */
/* [T, B*W] KV ancestry, the table icap_attention_decode_anc reads), total. Callers that look    */
/* at `done` (early exit) or `anc` take the offsets from here, never from a restated layout.      */
int icap_beam_layout(int32_t B, int32_t W, int32_t T, int32_t max_len, int64_t* word_offsets);
/* running scores (0 for beam 0, -1e9 for the others, :3318-3320), no finished hypotheses, and   */
/* the KV ancestry of the P prefix positions (every row its own).                               */
int icap_beam_init(const icap_beam_args* a, int32_t P, void* stream);
/* per row: top K logits (descending, ties -> lower id) into top_val/top_idx [R, K], the row max */
/* top_m [R] and log(sum(exp(logit - max))) top_ls [R] (log_softmax = (x - m) - ls).             */
int icap_beam_rowtop(int32_t dtype, int64_t R, int64_t V, const void* logits, int64_t ld, int32_t K,
                     float* top_val, int32_t* top_idx, float* top_m, float* top_ls, void* stream);
/* one beam step after the logits of generated-token count `step` (the rows' last computed     */
/* position is `pos`): top 2W candidates of each caption, the next running beams, the finished */
/* merge (score / (step+1)^length_penalty), the early-stop heuristic, histories, the KV        */
/* ancestry and the next input embeddings (HF/generation/utils.py:3077-3206,3008-3053).         */
int icap_beam_update(const icap_beam_args* a, int32_t step, int32_t pos, void* stream);
/* out int64 [B, max_len]: each caption's best finished hypothesis, EOS-padded; out_len [B].    */
int icap_beam_finalize(const icap_beam_args* a, int64_t* out, int32_t* out_len, void* stream);

/* x[(t*B + b)*D + d] = src[b*src_bstride + t*src_tstride + d] + wpe[(pos0+t)*D + d], t < npos */
/* (prefix rows into the position-major decode input, modeling_gpt2.py:571-577).            */
int icap_add_position(int32_t dtype, int32_t B, int32_t npos, int32_t D, const void* src,
                      int64_t src_bstride, int64_t src_tstride, const void* wpe, int32_t pos0,
                      void* x, void* stream);

/* ------------------------------------------------------------------------- */
/* CLIP image preprocessing: the reference's           */
/* CLIPImageProcessor (src/embeddings/clip.py:129 -> HF image_processing_clip:*/
/* shortest-edge PIL-BICUBIC resize, centre crop, x 1/255, (x - mean) / std) */
/* for n decoded RGB uint8 HWC images packed in `pixels`. geo: device int64  */
/* [n][10] = {src_off, in_h, in_w, new_h, new_w, top, left, tmp_off, y_first, */
/* tmp_rows} (icap/ops.py clip_preprocess computes it); tmp: uint8 scratch of */
/* sum(tmp_rows) * crop * 3 bytes; out: fp32 [n][3][crop][crop]. Pillow's    */
/* fixed-point two-pass resampler, bit-exact.                                 */
/* ------------------------------------------------------------------------- */
int icap_clip_preprocess(int32_t n, const uint8_t* pixels, const int64_t* geo, int32_t crop,
                         int32_t max_tmp_rows, uint8_t* tmp, const float* mean, const float* stdv,
                         float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ICAP_H */
