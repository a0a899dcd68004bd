/* lrce_hip.h — C ABI of the MI355X (gfx950) LRCE hot-path library (liblrce_hip.so).
 *
 * Plain pointers and sizes only: every tensor argument is a device pointer owned by the caller
 * (PyTorch's caching allocator in the Python host layer), outputs are written in place, nothing
 * is freed, and every entry point enqueues on the HIP stream passed as `stream` (hipStream_t,
 * NULL = default stream) and returns immediately.  Return value 0 = success; otherwise a
 * LRCE_E_* code, with a message available from lrce_last_error() (thread-local).
 *
 * dtypes: "bf16" = bfloat16 stored as uint16_t, "f32" = IEEE float.  All matrices are row-major
 * with explicit leading dimensions (in elements).
 *
 * The reference (Sejong-VLI/VQA-LRCE-KBS-2023) is pure PyTorch and has no native boundary; each
 * entry point below replaces the ATen kernels the reference's modules launch at the cited
 * file:line (paths relative to the reference root).  SURVEY.md §2.1 lists them.
 */
#ifndef LRCE_HIP_H
#define LRCE_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  LRCE_OK = 0,
  LRCE_E_ARG = 1,     /* bad shape / pointer / flag combination */
  LRCE_E_LAUNCH = 2,  /* hipGetLastError after launch */
  LRCE_E_UNSUPPORTED = 3
};

/* ---------------------------------------------------------------- GEMM (MFMA bf16 -> f32 acc)
 * C[b][m][n] (+)= epilogue( alpha * sum_k A(m,k) * B(n,k) )
 *   A(m,k) = a_kmajor ? A[m*lda + k] : A[k*lda + m]      (a_f32: A is f32, rounded to bf16 on load)
 *   B(n,k) = b_kmajor ? B[n*ldb + k] : B[k*ldb + n]      (bf16, or f32 with b_f32)
 *   a_map (optional int32): gathers A rows — replaces m (a_kmajor) or k (!a_kmajor) by a_map[.]
 *   c_map (optional int32): scatters output rows — row m is written to c_map[m] (also the row of
 *                           the RESID / DGELU aux read); c_map[m] < 0 drops row m (a padded window
 *                           position, cropped by the reference at video_swin_ori.py:292-293).
 * Replaces: nn.Linear forward/backward (addmm/mm) at video_swin_ori.py:46-57,150,152,318;
 * fusionv3.py:154,160; the decoder/BERT linears; conv3d patch-embed as a K=96 GEMM (:458).
 */
enum {
  LRCE_EPI_BIAS = 1,      /* + bias[n] (f32) */
  LRCE_EPI_GELU = 2,      /* y = gelu_erf(y); with AUX_OUT the pre-activation is stored (bf16) */
  LRCE_EPI_DGELU = 4,     /* y *= gelu_erf'(aux[row][n])  (aux bf16 pre-activation) */
  LRCE_EPI_RESID = 8,     /* y += aux[row][n]  (aux f32) */
  LRCE_EPI_OUT_F32 = 16,  /* C is f32 (else bf16) */
  LRCE_EPI_ATOMIC = 32,   /* f32 atomicAdd into C (split-K / gradient accumulation) */
  LRCE_EPI_ACCUM = 64,    /* C(f32) += y, non-atomic */
  LRCE_EPI_AUX_OUT = 128, /* store pre-activation (bf16) into aux_out */
  LRCE_EPI_OUT_BOTH = 256, /* also write a bf16 copy of y into aux_out (f32 C + bf16 shadow) */
  LRCE_EPI_BIAS_GRAD = 512, /* weight-gradient GEMMs (A M-major = dY^T): also bias[m] += sum_k A(m,k)
                              (the nn.Linear bias gradient, with A's row map / row scale applied) */
  LRCE_EPI_AUX_F32 = 2048, /* exact-f32 paths (b_f32): the AUX_OUT pre-activation and the DGELU aux are f32, not bf16
                              (the recurrent decoder's linear1: its GELU derivative sees the exact pre-activation) */
  LRCE_EPI_SLABS = 1024    /* split_k > 1 with a workspace: write the split slices' f32 slabs
                              ws[s][m][n] (alpha applied) and launch NO reduce — a consumer such as
                              lrce_splitk_reduce_ln sums them (C is not written) */
};

typedef struct LrceGemmDesc {
  const void* a;
  const void* b;
  void* c;
  int64_t lda, ldb, ldc;
  int64_t stride_a, stride_b, stride_c; /* batch strides (elements) */
  int32_t m, n, k, batch;
  int32_t a_kmajor, b_kmajor, a_f32;
  int32_t flags;      /* LRCE_EPI_* */
  int32_t split_k;    /* >1 requires LRCE_EPI_ATOMIC */
  const float* bias;
  const void* aux;
  int64_t ld_aux;
  void* aux_out;
  int64_t ld_aux_out;
  const int32_t* a_map;
  const int32_t* c_map;
  float alpha;
  int32_t scale_cols; /* columns [0, scale_cols) are multiplied by scale_val after the bias */
  float scale_val;
  /* DropPath (video_swin_ori.py:243,299): per-sample branch scale.  Epilogue: y *= row_scale[m /
   * rows_per_scale] before the RESID add.  A loader (f32 A only): every A element of logical row r
   * (m if a_kmajor else k, before a_map) is multiplied by a_row_scale[r / a_rows_per_scale]. */
  const float* row_scale;
  int32_t rows_per_scale;
  const float* a_row_scale;
  int32_t a_rows_per_scale;
  /* b_f32 = 1: B is f32 (then A must be f32): exact-f32 MFMA path (v_mfma_f32_16x16x4_f32) for the
   * small-M recurrent-decoder linears.  b_f32 = 2: B is IEEE fp16 (the weights' fp16 shadow, as under
   * the reference's fp16 autocast, agent_oe.py:28), converted exactly to f32 on load, A and the
   * arithmetic f32: half the weight bytes of the latency-bound decoder GEMVs (skinny path only). */
  int32_t b_f32;
  /* Split-K workspace (optional, f32, >= split_k * m * n elements, batch 1, flags = ATOMIC [+ BIAS_GRAD]
   * with no other epilogue): each K slice stores its partial tile with plain vector stores and a
   * second launch adds the slices into C -- no f32 atomics on C (their throughput bounds the
   * weight-gradient GEMMs otherwise). */
  float* workspace;
  int64_t workspace_elems;
  /* nn.Dropout fused into the epilogue (the recurrent decoder's dropouts, fusionv3.py:8-17): after
   * the bias / GELU / dGELU / row scale and before the RESID add, y = keep ? y / (1 - drop_p) : 0 with
   * keep = uniform hash of (drop_seed + device RNG offset, (m * n_cols + n) / drop_group) >= drop_p — the
   * mask lrce_dropout / lrce_dropout_bwd draw for the same contiguous [m][n] tensor.  drop_p = 0: off.
   * Exact-f32 skinny path only (B f32, M <= 64); other paths reject drop_p > 0. */
  float drop_p;
  int32_t drop_group;
  uint64_t drop_seed;
  /* f16 = 1: every 16-bit tensor of the call (A, B, a 16-bit C, aux_out, the DGELU aux) is IEEE
   * fp16 instead of bf16 and the MFMAs are the f16 forms (v_mfma_f32_*_f16): the BERT forward runs
   * in fp16 like the reference's fp16 autocast (agent_oe.py:28), and its backward in fp16 on scaled
   * gradients like the reference's GradScaler (agent_oe.py:40-42).  bf16 x bf16 LDS-DMA path only. */
  int32_t f16;
  /* Non-NULL: alpha is read from this device float instead of `alpha` (the inverse of a gradient
   * scale lrce_grad_scale computed on the GPU).  LDS-DMA and register-staged bf16/fp16 paths. */
  const float* alpha_dev;
  /* Batch stride of `bias` in elements (batch > 1; 0 = the same bias for every batch): BERT's query /
   * key / value linears as one batched launch over their weights and biases in the flat parameter
   * buffers (text.py:11-17 -> HF BertSelfAttention). */
  int64_t stride_bias;
  /* Batch stride of `alpha_dev` in floats (batch > 1; 0 = one alpha for every batch): the deferred BERT
   * weight gradients of all layers as one batched launch, each layer's product scaled by the inverse
   * of that layer's own gradient scale. */
  int64_t stride_alpha;
} LrceGemmDesc;

int lrce_gemm(const LrceGemmDesc* desc, void* stream);
/* One weight gradient of lrce_gemm_grouped: c[m][n] (=|+=) alpha sum_k a[k][m] b[k][n] (16-bit dY M-major
 * with lda >= m, 16-bit X N-major with ldb >= n, f32 dW with ldc >= n) and, with LRCE_EPI_BIAS_GRAD,
 * bias[m] += alpha sum_k a[k][m].  flags = ACCUM (+=) or OUT_F32 (=, a gradient known to be zero)
 * [| BIAS_GRAD: the bias sum is always added].  alpha_dev: alpha read from device memory (a gradient
 * scale computed on the GPU; NULL: the call's alpha).  f16: the 16-bit operands are IEEE fp16 (else
 * bf16).  m, n and the leading dims multiples of 8. */
typedef struct LrceGemmItem {
  const void* a;
  const void* b;
  float* c;
  float* bias;
  const float* alpha_dev;
  int32_t m, n, lda, ldb, ldc, flags, f16;
  /* split > 1: K in `split` slices of k_chunk (a multiple of 64) tokens; slice s stores its partial
   * into c + s * m * ldc and adds its bias partial into bias + s * m (zeroed by the caller): flags
   * must be OUT_F32 [| BIAS_GRAD]; lrce_slab_sum_grouped then sums the slabs in slice order. */
  int32_t split, k_chunk;
} LrceGemmItem;
/* Weight gradients of n linears of any shapes sharing K (the token count) and alpha, as grouped
 * launches (the four linears x blocks of a Swin stage at once, Swin backward, video_swin_ori.py:46-57,
 * 150, 187): each entry's 128 x 128 tiles run one K slice (no split-K slabs or reduce launch), the
 * entries' tiles form one grid.  Up to 80 entries and 8 distinct shapes per launch, one operand
 * format (f16) per launch, and the C / bias / alpha pointers of one launch within 8 GB of each other
 * (more: several launches).  Pointers 16-B aligned (alpha_dev 4-B). */
int lrce_gemm_grouped(const LrceGemmItem* items, int n, int k, float alpha, void* stream);
/* dst (=|+=) sum_s slabs[s * n + i] over s = 0 .. split-1 in that order (deterministic), for a batch of
 * items (a grouped split-K launch's weight / bias slabs).  n % 4 == 0, pointers 16-B aligned. */
typedef struct LrceSlabSum {
  const float* slabs;
  float* dst;
  int64_t n;
  int32_t split, accumulate;
} LrceSlabSum;
int lrce_slab_sum_grouped(const LrceSlabSum* items, int n, void* stream);
/* n same-shape weight gradients (the blocks of a Swin stage): lrce_gemm_grouped with items
 * {a[i], b[i], c[i], bias[i], desc->m, desc->n, desc->lda, desc->ldb, desc->ldc, desc->flags}; desc
 * supplies the shape / leading dims / alpha / flags (ACCUM or OUT_F32 [| BIAS_GRAD]); its pointers,
 * batch, strides and split_k are ignored. */
int lrce_gemm_ptr_batched(const LrceGemmDesc* desc, const void* const* a, const void* const* b, void* const* c,
                          const float* const* bias, int n, void* stream);

/* Exact-f32 skinny linear (b_f32, M <= 64, K-major f32 A, K % 128 == 0, K <= 1024) whose A operand is
 * a LayerNorm input or gradient: the post-norm LayerNorms of the recurrent decoder
 * (nn.TransformerDecoderLayer norm1..3, fusionv3.py:8-17) fold into the GEMM that consumes them.
 *   mode 1: A = x (pre-norm rows); the GEMM consumes y = LN(x) = (x - mean) rstd gamma + beta (eps);
 *           mean / rstd f32 [m] written (optional), y materialised into y_out (optional, f32, ld_y).
 *   mode 2: A = dy (gradient w.r.t. the LN output), x = the pre-norm rows (ld_x), mean / rstd read;
 *           dx = LN backward of dy goes to y_out (optional); the GEMM consumes dropout_bwd(dx)
 *           (mask of lrce_dropout over the [m][k] tensor: drop_p / drop_group / drop_seed, 0 = off),
 *           also written to y2_out (optional); dgamma / dbeta (f32 [k], optional, together) += the
 *           column sums of dy * xhat and dy.
 * The epilogue is lrce_gemm's (bias, GELU, dGELU, fused dropout, residual, f32 / bf16 out). */
typedef struct LrceLnPrologue {
  int32_t mode;
  const float* gamma;
  const float* beta;
  float eps;
  const float* x;
  int64_t ld_x;
  float* mean;
  float* rstd;
  float* y_out;
  int64_t ld_y;
  float* y2_out;
  int64_t ld_y2;
  float* dgamma;
  float* dbeta;
  float drop_p;
  int32_t drop_group;
  uint64_t drop_seed;
} LrceLnPrologue;
int lrce_gemm_ln(const LrceGemmDesc* desc, const LrceLnPrologue* prologue, void* stream);

/* ---------------------------------------------------------------- LayerNorm
 * Row r of the (rows x cols) LN input is the concatenation of nseg segments of cols/nseg
 * channels, segment s read from source row in_map[r*nseg+s] of x (identity if in_map == NULL;
 * a negative index reads zeros = padding before the norm, PatchMerging :328-331).  With nseg == 1 a
 * negative index marks padding AFTER the norm (the block's F.pad of norm1's output, :253-258): the
 * output row is zero, its stats 0, and the backward skips the row (no dx, no dw/db).  Output row r
 * goes to out_map[r] (identity if NULL).
 * Saves per-row mean and rstd (f32) for the backward.  y_bf16_copy (optional): a bf16 copy of y (f32 y
 * for the residual stream + bf16 operand for the next GEMM / weight gradient, one pass).
 * Replaces: nn.LayerNorm at video_swin_ori.py:252,285,339,476-480,684; PatchMerging gather
 * (:333-337, nseg=4); window_partition + torch.roll (:60-72,262) via in_map; embedding.py:22,62;
 * fusionv3.py:48; BERT LayerNorms. */
int lrce_layernorm_fwd(const void* x, int x_f32, const int32_t* in_map, int nseg,
                       const float* w, const float* b, float eps,
                       void* y, int y_f32, uint16_t* y_bf16_copy, const int32_t* out_map,
                       float* mean, float* rstd, int rows, int cols, int copy_f16, void* stream);
/* copy_f16 = 1: the 16-bit copy is IEEE fp16 (the BERT forward operands) instead of bf16. */

/* dy row r (read from dy_map[r] if given), x/mean/rstd as in forward.  dx for segment s is written
 * to row in_map[r*nseg+s] of dx (f32): dx = LN_bwd + (dres ? dres[same row] : 0).  dw/db (f32,
 * may be NULL) are accumulated with atomics.  Optional dx_bf16: a bf16 copy of LN row r's dx,
 * times dx_scale[r / dx_scale_rps] (DropPath of the branch the copy feeds), stored row-major at row
 * dx_bf16_map[r] (e.g. window order) — the A operand of the following weight/input-gradient GEMMs.
 * dx may be NULL when dx_bf16 is given (the bf16 copy is then the only output). */
int lrce_layernorm_bwd(const void* dy, int dy_f32, const int32_t* dy_map,
                       const void* x, int x_f32, const int32_t* in_map, int nseg,
                       const float* mean, const float* rstd, const float* w,
                       float* dx, const float* dres, float* dw, float* db,
                       int rows, int cols, uint16_t* dx_bf16, const int32_t* dx_bf16_map,
                       const float* dx_scale, int dx_scale_rps, float* workspace,
                       int64_t workspace_elems, void* stream);
/* f32 elements of the dw/db partials workspace lrce_layernorm_bwd uses for (rows, cols) (0: one block
 * suffices): with it the weight/bias gradients are a deterministic sum in block order (per-block
 * partials, then a reduce whose last-arriving block per column adds the chunk sums in order) instead
 * of same-address atomics from every block (a NULL or smaller workspace falls back to the atomics). */
int64_t lrce_layernorm_bwd_workspace(int rows, int cols);
/* The output projection + residual + post-norm LayerNorm of a BERT sub-layer (HF BertSelfOutput /
 * BertOutput: LN(resid + dropout(x W^T + b))) from a split-K GEMM's slabs (LRCE_EPI_SLABS): per row
 * s = sum_k ws[k][r] + bias, dropout (the mask of lrce_dropout over [rows][cols]), + resid; s is stored
 * in pre (f32, the LayerNorm backward's input; optional), then y = LN(s) gamma + beta (f32), y16 its
 * 16-bit copy (fp16 when y16_f16, else bf16; optional), mean / rstd.  One wave per row, cols <= 1024,
 * cols % 256 == 0.  Replaces splitk reduce + lrce_layernorm_fwd (two launches and a round trip). */
int lrce_splitk_reduce_ln(const float* ws, int split, int rows, int cols, const float* bias, const float* resid,
                          int64_t ld_res, float p, uint64_t seed, float* pre, const float* gamma, const float* beta,
                          float eps, float* y, uint16_t* y16, int y16_f16, float* mean, float* rstd, void* stream);
/* lrce_layernorm_bwd without its gamma / beta reduction launch: *nb_out = the number of per-block partial
 * rows left in workspace (0: none were needed — a one-block problem, no dw / db, or no workspace — and
 * dw / db are already final).  With nb_out > 0 the caller keeps the workspace and later passes
 * (workspace, nb_out, cols, dw, db) to lrce_layernorm_grad_reduce, which many LayerNorms share: a
 * stage's LayerNorm parameter gradients then cost one launch instead of one per LayerNorm. */
int lrce_layernorm_bwd_deferred(const void* dy, int dy_f32, const int32_t* dy_map, const void* x, int x_f32,
                                const int32_t* in_map, int nseg, const float* mean, const float* rstd, const float* w,
                                float* dx, const float* dres, float* dw, float* db, int rows, int cols,
                                uint16_t* dx_bf16, const int32_t* dx_bf16_map, const float* dx_scale, int dx_scale_rps,
                                float* workspace, int64_t workspace_elems, int* nb_out, void* stream);
/* dw[i][c] += sum_b part_i[b][c], db[i][c] += sum_b part_i[b][cols_i + c] for n deferred LayerNorm
 * backwards (parts[i] / nbs[i] / cols[i] as lrce_layernorm_bwd_deferred left them; dw[i] or db[i] may be
 * NULL): up to 40 per launch, each summed in block order exactly as lrce_layernorm_bwd does (same bits). */
int lrce_layernorm_grad_reduce(const float* const* parts, const int32_t* nbs, const int32_t* cols, float* const* dw,
                               float* const* db, int n, void* stream);

/* ---------------------------------------------------------------- Swin 3D window attention
 * Replaces WindowAttention3D.forward video_swin_ori.py:164-186 (QK^T, relative-position bias,
 * shift mask, softmax, PV) for windows of n in (128, 160] tokens and head_dim 32.
 * qkv: bf16 [n_win*n][3C] window-ordered rows (q columns pre-scaled by head_dim^-0.5*log2(e)),
 * out: bf16 [n_win*n][C], lse: f32 [n_win][nH][160] (log2 domain).
 * bias tiles are built once per layer by lrce_wattn_bias_build from the f32 table
 * (relative_position_bias_table) and the int64 relative_position_index (ld = index_ld), with the
 * shift mask of each window pattern given as per-token region ids region[n_pat][n] (-100 between
 * different regions, video_swin_ori.py:346-359); bias_fwd holds the S^T-oriented tiles (forward),
 * bias_bwd the S-oriented ones (backward).  fwd_f16 / bwd_f16: that set as IEEE fp16 (padded keys
 * -30000) instead of f32 — lrce_wattn_qkv_fwd reads fp16 forward tiles, lrce_wattn_fwd_grouped f32;
 * lrce_wattn_bwd either (bias_f16); a layer's forward and backward should use the same precision. */
int64_t lrce_wattn_bias_elems(int n_pat, int nH);
int lrce_wattn_bias_build(const float* table, const int64_t* index, int index_ld, int n, int nH,
                          const int32_t* region, int n_pat, void* bias_fwd, int fwd_f16, void* bias_bwd,
                          int bwd_f16, void* stream);
/* Forward with windows grouped by mask pattern, GW = 4 windows per group: win_list int32
 * [n_groups*4] (window ids, -1 = empty slot; NULL = identity 0,1,2,...), grp_pat int32 [n_groups]
 * (the group's mask pattern; NULL = pattern 0).  The bias row of a query tile is staged once per
 * group in LDS: build the grouping once per stage geometry (lrce/feature_extractor/video_swin.py). */
int lrce_wattn_fwd_grouped(const uint16_t* qkv, const float* bias_fwd, const int32_t* win_list, const int32_t* grp_pat,
                           int n_groups, uint16_t* out, float* lse, int n_win, int n, int nH, void* stream);
/* Fused QKV projection + window attention forward (WindowAttention3D.forward video_swin_ori.py:158-189
 * including the qkv Linear :150,165): x bf16 [n_win*n][C] (LN1 output in window order), w_qkv bf16
 * [3C][C], b_qkv f32 [3C]; q is scaled by qscale (= head_dim^-0.5 * log2(e)) after the bias.  Writes
 * qkv bf16 [n_win*n][3C] (the backward's input, same layout as above), out and lse as
 * lrce_wattn_fwd_grouped.  bias_fwd16: the fp16 forward tiles (lrce_wattn_bias_build with fwd_f16).
 * win_order int32 [n_win]: the order the windows are visited in (NULL = identity; sorted by mask
 * pattern, so one XCD's workgroups share few bias tiles).  One workgroup per (window, 2 heads);
 * nH % 2 == 0. */
int lrce_wattn_qkv_fwd(const uint16_t* x, const uint16_t* w_qkv, const float* b_qkv, float qscale,
                       const uint16_t* bias_fwd16, const int32_t* win_pat, const int32_t* win_order, uint16_t* qkv,
                       uint16_t* out, float* lse, int n_win, int n, int nH, void* stream);
/* Backward (one kernel): dqkv bf16 [n_win*n][3C] (d/dq, d/dk, d/dv w.r.t. the UNSCALED q).  win_pat
 * int32 [n_win] (the window's mask pattern, NULL = 0).  The window is wd x wh x ww tokens (n = wd*wh*ww,
 * token order (t, h, w)); dbias_part: f32, lrce_wattn_dbias_part_elems(n_win, nH, n_bins) elements with
 * n_bins = (2wd-1)(2wh-1)(2ww-1) <= 1024: per (window, head) the bias-table gradient binned by relative
 * position, reduced by lrce_wattn_dbias (NULL: no bias-table gradient, e.g. a frozen table). */
int64_t lrce_wattn_dbias_part_elems(int n_win, int nH, int n_bins);
int lrce_wattn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse,
                   const void* bias_bwd, int bias_f16, const int32_t* win_pat, uint16_t* dqkv, float* dbias_part,
                   int n_win, int n, int nH, int wh, int ww, void* stream);
/* Bias-table gradient (relative_position_bias_table, f32 [table_rows][nH], accumulated) from
 * lrce_wattn_bwd's bins: bin_row int32 [n_bins] = the table row of each relative-position bin (the
 * relative_position_index entry of any (query, key) pair in that bin; -1 = unused), built once per stage
 * geometry by lrce.kernels.wattn_bin_rows.  Deterministic: windows summed in a fixed order, every table
 * entry written by one thread, no atomics. */
int lrce_wattn_dbias(float* dbias_part, int n_win, int nH, int n_bins, const int32_t* bin_row, float* table_grad,
                     void* stream);
/* lrce_wattn_dbias for n blocks at once (item i: dbias_part[i], n_win[i], nH[i], n_bins[i], bin_row[i],
 * table_grad[i]; up to 24 per pair of launches): the same sums in the same order (same bits), two
 * launches for all of a stage's blocks instead of two per block. */
int lrce_wattn_dbias_batched(float* const* dbias_part, const int32_t* n_win, const int32_t* nH, const int32_t* n_bins,
                             const int32_t* const* bin_row, float* const* table_grad, int n, void* stream);

/* ---------------------------------------------------------------- small multi-head attention
 * Masked SDPA, head_dim 64, for BERT self-attention (text.py:12-17 -> HF BertSelfAttention, L<=64)
 * and the LRCE decoder cross-attention (fusionv3.py:44-49 -> nn.MultiheadAttention, Lq=1).
 * Query row (b, i) at q[(b*Lq + i)*ld_q + h*64].  Keys j < lk1 come from segment 1: row
 * k1[(b/kv1_bdiv)*stride_kv1_b + j*ld_kv1 + h*64]; keys lk1 <= j < lk1+lk2 from segment 2 likewise
 * (e.g. [video tokens of the step ; question tokens] without materialising the concatenation;
 * kv1_bdiv = 5 shares one video memory across the 5 MC choices).  key_mask int32 [B][lk1+lk2]
 * (1 keep / 0 masked, NULL = keep all) = HF's additive -inf padding mask.  drop_p > 0: dropout on
 * the attention probabilities (train mode), mask = hash(seed, ((b*H+h)*Lq+i)*Lk+j) >= drop_p.
 * out bf16 [B*Lq][ld_o], lse f32 [B][H][Lq] (natural log).  Backward: dq f32 written; dk1,dv1,dk2,dv2
 * f32 ACCUMULATED (atomics; caller zeroes), laid out like k1,v1,k2,v2 with their own ld/stride. */
typedef struct LrceMhaDesc {
  const uint16_t* q;
  int64_t ld_q;
  const uint16_t* k1;
  const uint16_t* v1;
  int64_t ld_kv1, stride_kv1_b;
  int32_t kv1_bdiv, lk1;
  const uint16_t* k2;
  const uint16_t* v2;
  int64_t ld_kv2, stride_kv2_b;
  int32_t kv2_bdiv, lk2;
  const int32_t* key_mask;
  uint16_t* out;
  int64_t ld_o;
  float* lse;
  int32_t B, H, Lq, d;
  float scale;
  float drop_p;
  uint64_t seed;
  int32_t f32_io;   /* 1: q, out, dout are f32 (decoder query path); K/V stay bf16 */
  /* backward only */
  const uint16_t* dout;
  float* dq;
  int64_t ld_dq;
  float* dk1;
  float* dv1;
  int64_t ld_dkv1, stride_dkv1_b;
  float* dk2;
  float* dv2;
  int64_t ld_dkv2, stride_dkv2_b;
  /* 1 = q, k, v, out (and, in the backward, dout) are IEEE fp16 (BERT self-attention under the
   * reference's fp16 autocast; the backward's dout a scaled fp16 gradient, its f32 dq / dk / dv carry
   * the same scale); f16 MFMA forms.  Short self-attention path only (Lq = Lk <= 64). */
  int32_t f16;
  /* single-query or short self-attention backward: 1 = the first key segment's dK / dV rows are STORED, not accumulated
   * (every row has one writer in this launch and no earlier contribution: kv1_bdiv == 1 and a memory
   * that is distinct per call, e.g. the video tokens of one recurrent step) — no zero fill, no read. */
  int32_t dkv1_store;
  /* short self-attention backward with dkv1_store: 1 = dq / dk1 / dv1 point to IEEE fp16 buffers (the
   * f32 values rounded once), e.g. the three column blocks of one [rows, 3 * H * d] operand of the
   * fused q/k/v input-gradient GEMM and the deferred weight gradients (BERT, text.py:11-17). */
  int32_t grad16;
} LrceMhaDesc;

int lrce_mha_fwd(const LrceMhaDesc* desc, void* stream);
int lrce_mha_bwd(const LrceMhaDesc* desc, void* stream);

/* ---------------------------------------------------------------- recurrent decoder attention blocks
 * One nn.TransformerDecoderLayer (fusionv3.py:8-17: d_model 768, 12 heads x 64, post-norm, one query
 * token per row) has two attention blocks that factor by head; each is ONE launch of B x 12
 * workgroups (csrc/decoder.hip), replacing three launches of the unfused path (lrce_gemm_ln ->
 * lrce_gemm for the self-attention: v projection -> out_proj; lrce_gemm_ln -> lrce_mha_fwd ->
 * lrce_gemm for the cross-attention: q projection -> attention -> out_proj; and the same three of
 * each backward).  Rows are f32 [B][768] (row stride 768), weights the IEEE fp16 shadow [768][768]
 * (row = output feature), biases / LayerNorm parameters f32.  Dropout (drop_p > 0, train mode) uses
 * the masks of lrce_dropout / lrce_mha_* for the same seeds (seed = the layer's base seed as the
 * unfused path passes it: self-attention head mask `seed`, its out dropout seed + 1; cross-attention
 * probabilities seed + 2, out dropout seed + 3).  slab: f32 workspace of lrce_dec_slab_elems(B)
 * elements; counters: B zero-initialised uint32 (left zero after every launch).  One stream at a time
 * may use a slab / counters pair.  B <= LRCE_DEC_MAX_ROWS. */
#define LRCE_DEC_MAX_ROWS 64
int64_t lrce_dec_slab_elems(int B);
typedef struct LrceDecKv {   /* memory K/V (bf16): key j < lk1 of row b at k1[(b/bdiv1)*stride1 + j*ld1 + h*64],
                                 j >= lk1 at k2[(b/bdiv2)*stride2 + (j-lk1)*ld2 + h*64]; V at K + v_off */
  const uint16_t* k1;
  int64_t stride1, ld1;
  int32_t bdiv1, lk1;
  const uint16_t* k2;
  int64_t stride2, ld2;
  int32_t bdiv2, lk2;
  int64_t v_off;
} LrceDecKv;
/* x1p = x0 + drop(out_proj(drop_head(v_proj(x0)))), x0 = LN(x_in) with (ln_gamma, ln_beta, eps)
 * (the previous layer's norm3; ln_gamma NULL: x0 = x_in) -> x0_out / mean_out / rstd_out;
 * sad = the dropped v projection (the out_proj's input). */
typedef struct LrceDecSa {
  int32_t B;
  const float* x_in;
  const float* ln_gamma;
  const float* ln_beta;
  float eps;
  float* x0_out;
  float* mean_out;
  float* rstd_out;
  const uint16_t* wv;   /* self_attn.in_proj_weight rows 2E..3E */
  const float* bv;
  const uint16_t* wo;   /* self_attn.out_proj.weight */
  const float* bo;
  float* sad;
  float* x1p;
  float drop_p;
  uint64_t seed;
  float* slab;
  uint32_t* counters;
} LrceDecSa;
int lrce_dec_sa_fwd(const LrceDecSa* args, void* stream);
/* x1 = LN1(x1p) -> x1_out, mean_out, rstd_out; q = W_q x1 + b_q -> q_out; ctx = attention(q, memory)
 * -> ctx_out, lse_out [B][12] (natural log); x2p = x1 + drop(out_proj(ctx)).  seed: the layer's seed
 * + 2 (attention probabilities; the out dropout uses seed + 1 of this value). */
typedef struct LrceDecCa {
  int32_t B;
  const float* x1p;
  const float* g1;
  const float* b1;
  float eps;
  float* x1_out;
  float* mean_out;
  float* rstd_out;
  const uint16_t* wq;   /* multihead_attn.in_proj_weight rows 0..E */
  const float* bq;
  LrceDecKv kv;
  float* q_out;
  float* ctx_out;
  float* lse_out;
  const uint16_t* wo;   /* multihead_attn.out_proj.weight */
  const float* bo;
  float* x2p;
  float drop_p;
  uint64_t seed;
  float* slab;
  uint32_t* counters;
} LrceDecCa;
int lrce_dec_ca_fwd(const LrceDecCa* args, void* stream);
/* Backward of the cross-attention block from dx2 = d LN2(x2p): dx2p = LN2 backward (mean2 / rstd2 /
 * g2), dcao = its out-dropout backward -> dcao_out (the out_proj's output gradient); dctx = W_o^T dcao;
 * attention backward -> dq_out, dK / dV of the memory (video rows dk1 (+ dv_off for dV) with their
 * own dstride1 / dld1: STORED when bdiv1 == 1, atomically added otherwise; text rows dk2 accumulated,
 * or stored when dk2_store);
 * dx1_out = dx2p + W_q^T dq.  LayerNorm parameter gradients: lrce_dec_ln_grads. */
typedef struct LrceDecCaBwd {
  int32_t B;
  const float* dx2;
  const float* x2p;
  const float* mean2;
  const float* rstd2;
  const float* g2;
  float* dcao_out;
  const uint16_t* wo;
  LrceDecKv kv;
  const float* q;
  const float* ctx;
  const float* lse;
  float* dq_out;
  float* dk1;
  int64_t dstride1, dld1;
  float* dk2;
  int64_t dstride2, dld2;
  int64_t dv_off;
  const uint16_t* wq;
  float* dx1_out;
  float drop_p;
  uint64_t seed;   /* as lrce_dec_ca_fwd */
  float* slab;
  uint32_t* counters;
  int32_t dk2_store;   /* 1: the text rows' dK / dV are STORED (the first recurrent step of the backward; no zeroed buffer needed), 0: added */
  uint16_t* dk1_bf16;  /* non-NULL (one writer per video row, kv.bdiv1 == 1 only): the video rows' dK / dV go here as bf16, same
                          dstride1 / dld1 / dv_off (the operand of the memory-side GEMMs), and dk1 may be NULL */
} LrceDecCaBwd;
int lrce_dec_ca_bwd(const LrceDecCaBwd* args, void* stream);
/* Backward of the self-attention block from dx1 = d LN1(x1p): dx1p = LN1 backward, dsao = its out-
 * dropout backward -> dsao_out; dsav = head-mask backward of W_o^T dsao -> dsav_out; dx0_out = dx1p +
 * W_v^T dsav. */
typedef struct LrceDecSaBwd {
  int32_t B;
  const float* dx1;
  const float* x1p;
  const float* mean1;
  const float* rstd1;
  const float* g1;
  float* dsao_out;
  const uint16_t* wo;
  float* dsav_out;
  const uint16_t* wv;
  float* dx0_out;
  float drop_p;
  uint64_t seed;   /* as lrce_dec_sa_fwd */
  float* slab;
  uint32_t* counters;
} LrceDecSaBwd;
int lrce_dec_sa_bwd(const LrceDecSaBwd* args, void* stream);
/* LayerNorm parameter gradients over rows [rows][768] of every recurrent step at once (n_ln <= 3
 * LayerNorms): dgamma[c] += sum_r dy (x - mean) rstd, dbeta[c] += sum_r dy, rows in order; one of
 * dgamma[k] / dbeta[k] may be NULL (frozen parameter). */
int lrce_dec_ln_grads(const float* const* dy, const float* const* x, const float* const* mean, const float* const* rstd,
                      float* const* dgamma, float* const* dbeta, int n_ln, int rows, void* stream);
/* ---------------------------------------------------------------- persistent recurrent decoder step
 * FusionTransformer.forward's clip loop body (fusionv3.py:43-49 over the 12 nn.TransformerDecoderLayer of
 * fusionv3.py:8-17): ONE launch per recurrent step and direction (csrc/decoder_step.hip), replacing the
 * 4 + 4 launches per layer of the per-block path above.  12 x R workgroups (R = min(B, 10) row groups)
 * stay resident for all 12 layers and hand rows to each other inside the launch (16-B write-through
 * stores into sentinel-armed buffers, polled with bounded spins: the payload is the flag): per layer, (head h, row b) workgroups run the self-attention
 * block and the cross-attention block (as lrce_dec_sa_fwd / lrce_dec_ca_fwd), and every workgroup takes
 * 32-unit slices of the FFN hidden layer for ALL rows (linear1 -> GELU -> dropout -> its partial of
 * linear2), so each FFN weight is read once per layer-step; the partials are summed by the next layer's
 * (head, row) workgroups, 64 columns each, in slice order (deterministic).  The step tail (norm3 of the
 * last layer, s + x3, fusion_layer_norm, dropout) runs in the same launch.  The backward mirrors it.
 * Saved activations go to an arena laid out by lrce_dec_step_field (f32; element (step, row, col) of
 * field f of layer l at field(f, l) + (step * B + row) * width(f) + col); the layer index n_layers
 * holds the step tail.  Dropout masks and seeds are those of the per-block path: layer (i, l) uses
 * seed + 64 (i n_layers + l) (+ 1 .. + 5 as lrce_dec_*), the tail seed + 7 + 64000 (i + 1). */
#define LRCE_DEC_LAYERS 12
typedef struct LrceDecLayerW {   /* one layer's parameters: 16-bit weights are the fp16 shadow [out][in] */
  const uint16_t* wv; const float* bv;     /* self_attn.in_proj rows 2E..3E */
  const uint16_t* wo; const float* bo;     /* self_attn.out_proj */
  const float* g1; const float* be1;       /* norm1 */
  const uint16_t* wq; const float* bq;     /* multihead_attn.in_proj rows 0..E */
  const uint16_t* woc; const float* boc;   /* multihead_attn.out_proj */
  const float* g2; const float* be2;       /* norm2 */
  const uint16_t* w1; const float* b1;     /* linear1 [3072][768] */
  const uint16_t* w2; const float* b2;     /* linear2 [768][3072] */
  const float* g3; const float* be3;       /* norm3 */
} LrceDecLayerW;
typedef struct LrceDecStep {
  int32_t B, S, step, nmc, lt, n_layers;   /* query rows, steps, this step, rows per video sample, question keys */
  float eps, drop_p;
  uint64_t seed;
  const float* gf; const float* bf;        /* fusion_layer_norm */
  const uint16_t* kv_video; int64_t kv_video_lstride;   /* layer l: [B/nmc*S*150][1536] bf16 (K | V) */
  const uint16_t* kv_text; int64_t kv_text_lstride;     /* layer l: [B*lt][1536] bf16 (NULL when lt == 0) */
  float* acts;                             /* forward arena (written by the forward, read by the backward) */
  float* grads;                            /* backward arena */
  float* s_out;                            /* forward of the last step: the output rows [B][768] */
  const float* ds_in;                      /* backward: gradient of this step's output [B][768] */
  float* ds_out;                           /* backward: gradient of this step's input [B][768] */
  uint16_t* dkv_video16;                   /* backward, nmc == 1: video-row dK|dV stored bf16, layer stride dkv_video_lstride */
  float* dkv_video32;                      /* backward, nmc > 1: f32 (zeroed by the caller), atomically added */
  int64_t dkv_video_lstride;
  float* dkv_text;                         /* backward: [B*lt][1536] f32 per layer, stored at step S-1 then added */
  int64_t dkv_text_lstride;
  float* ws;                               /* lrce_dec_step_ws_elems() f32, every byte 0xFF before the first launch
                                              (the launches keep it so; lrce_dec_step_reset restores it) */
  uint32_t* counters;                      /* lrce_dec_step_counter_words() uint32, zero before the first launch */
  uint32_t* status;                        /* [4] uint32: [0] != 0 after a hand-off timed out (sticky until cleared) */
  LrceDecLayerW layer[LRCE_DEC_LAYERS];
} LrceDecStep;
/* field offsets of the arenas: kind 0 = forward (fields x0 sad x1p x1 q ctx x2p x2 x3p pre gd lse m1 r1 m2 r2 m3
 * r3; the tail block l = n_layers: x0 = tsum, m1 = mean, r1 = rstd), kind 1 = backward (df dgp dcao dq dsao dsav dln1
 * dln2 dln3; tail: df = du, dcao = dt); returns -1 for a bad field.  lrce_dec_step_field(kind, -1, 0, B, S, L) = total. */
int64_t lrce_dec_step_field(int kind, int field, int layer, int B, int S, int n_layers);
int64_t lrce_dec_step_ws_elems(void);
int64_t lrce_dec_step_counter_words(void);
int lrce_dec_step_fwd(const LrceDecStep* args, void* stream);
int lrce_dec_step_bwd(const LrceDecStep* args, void* stream);
/* re-arm the workspace (every byte 0xFF), zero the counter block and the status words (after a timeout:
 * status[0] != 0) */
int lrce_dec_step_reset(float* ws, uint32_t* counters, uint32_t* status, void* stream);
/* Debug: phase timestamps (s_memrealtime, 100 MHz) of the step kernels into buf[((dir * 128 + workgroup) * 16 + layer) * 8 + mark]
 * (dir 0 forward, 1 backward; 2 * 128 * 16 * 8 uint64); NULL turns it off (the default).  tools/decoder_step_bench.py --trace. */
int lrce_dec_step_set_trace(uint64_t* buf);
/* workgroups of one launch for B rows (12 x min(B, 10)) */
int lrce_dec_step_grid(int B);

/* Debug: phase timestamps (s_memrealtime, 100 MHz) of the four fused block kernels (k = sa_fwd, ca_fwd,
 * ca_bwd, sa_bwd) into buf[(k * 1024 + workgroup) * 16 + mark] (device memory, 4 * 1024 * 16 uint64);
 * NULL turns it off (the default).  tools/decoder_trace.py reads it. */
int lrce_dec_set_trace(uint64_t* buf);
/* Debug: phase timestamps (s_memrealtime) of lrce_wattn_bwd into buf[workgroup * 16 + mark] (marks: start,
 * prologue done, steps 0-4 done, stores done, bins written; [10] HW_ID, [11] XCC_ID); NULL turns it off (the
 * default).  Recorded only by a library built with -DLRCE_WATTN_TRACE (tools/wattn_trace.py).  The same
 * buffer also receives lrce_wattn_qkv_fwd's marks (start, GEMM done, epilogue done, qkv stored, attention
 * done, O stored; tools/wattn_trace.py WATTN_FWD=1): trace one kernel per launch. */
int lrce_wattn_set_trace(uint64_t* buf);

/* Debug: phase timestamps of the LDS-DMA GEMM kernel into buf[workgroup * 8 + mark] (marks: start, first K tile
 * landed, K loop done, epilogue stores issued, stores drained; [6] HW_ID, [7] XCC_ID), workgroups of split 0 only;
 * NULL turns it off (the default).  Recorded only by a library built with -DLRCE_GEMM_TRACE
 * (tools/gemm_trace.py). */
int lrce_gemm_set_trace(uint64_t* buf);

/* ---------------------------------------------------------------- elementwise / data movement */
/* Patch-embed input stage: [ImageNet Normalize (video.py:35)] + zero-pad T to a multiple of 2
 * (video_swin_ori.py:472-473) + im2col of the non-overlapping (2,4,4) patches of conv3d (:458,475).
 * Clip n, frame t, channel c lives at clips[n*s_clip + t*s_t + c*s_c] (rows of W floats, H rows):
 * (B,S,T,3,H,W) clips -> s_clip=T*3*H*W, s_t=3*H*W, s_c=H*W; (B,3,T,H,W) -> 3*T*H*W, H*W, T*H*W.
 * patches: bf16 [n_clips*D'*H'*W'][96], rows (n, d, h, w), cols (c, kt, kh, kw). */
int lrce_patch_im2col(const float* clips, int n_clips, int T, int H, int W, int64_t s_clip, int64_t s_t, int64_t s_c,
                      int normalize, uint16_t* patches, void* stream);
/* Clip assembly (e2e_dataset.py:60-116 -> torchvision Resize((h, w)) on PIL + ToTensor): frames is
 * uint8 [n_frames][H][W][3] (decoded RGB); output clip-frame f is frame frame_idx[f] (0 <= idx <
 * n_frames, the caller's multi-scale selection) resampled with Pillow's antialiased BILINEAR filter,
 * bit-exact, and written as f32 [n_out][3][out_h][out_w] in [0, 1]. */
int lrce_frames_resize(const uint8_t* frames, int n_frames, int H, int W, const int32_t* frame_idx, int n_out, int out_h,
                       int out_w, float* out, void* stream);
/* column sums: out[n] += sum_m x[row_map[m]][n] * row_scale[m / rows_per_scale] (x f32 or bf16; map and
 * scale optional): bias gradients (nn.Linear bias, incl. DropPath-scaled branches) */
int lrce_colsum(const void* x, int x_f32, const int32_t* row_map, int64_t ld, int m, int n, const float* row_scale,
                int rows_per_scale, float* out, void* stream);
/* dst[i] = bf16(sum over r < nshard of src[r * len + i]), summed in f32 in rank order (len % 8 == 0,
 * 16-B aligned): the local reduce of the data-parallel gradient exchange (bf16 all-to-all -> this ->
 * bf16 all-gather), replacing the f32 sum of the reference's DDP all-reduce (agent_base.py:76). */
int lrce_sum_shards_bf16(const uint16_t* src, int nshard, int64_t len, uint16_t* dst, void* stream);
/* f32 -> bf16 cast (n elements) */
int lrce_cast_bf16(const float* x, uint16_t* y, int64_t n, void* stream);
/* f32 -> IEEE fp16 cast (n elements): the BERT forward's GEMM operands */
int lrce_cast_f16(const float* x, uint16_t* y, int64_t n, void* stream);
/* IEEE fp16 -> bf16 (n elements): the fp16 activations a BERT layer saved for its backward become
 * the bf16 operands of the backward GEMMs / attention kernel (one pass over the layer's buffer) */
int lrce_cast_f16_bf16(const uint16_t* x, uint16_t* y, int64_t n, void* stream);
/* y[r][:] = bf16(x[r][:] * row_scale[r / rows_per_scale]) for a (rows x cols) f32 matrix (cols % 4 == 0):
 * a DropPath-scaled bf16 copy of a residual-stream gradient, the A operand of the branch's GEMMs. */
int lrce_scale_cast_bf16(const float* x, int64_t rows, int cols, const float* row_scale, int rows_per_scale, uint16_t* y,
                         void* stream);
/* Dropout (nn.Dropout / F.dropout semantics, train mode): y = (res ? res : 0) + x * keep / (1-p),
 * keep = hash(seed, i / group) >= p (group > 1 drops whole groups, e.g. per attention head);
 * p = 0 copies.  Optional bf16 copy of y.  In place allowed.  Backward: dx = dy * keep / (1-p)
 * (the residual's gradient is dy itself). */
int lrce_dropout(const float* x, const float* res, float* y, uint16_t* y_bf16, int64_t n, float p, uint64_t seed,
                 int64_t group, void* stream);
int lrce_dropout_bwd(const float* dy, float* dx, uint16_t* dx_bf16, int64_t n, float p, uint64_t seed, int64_t group,
                     void* stream);  /* dx and/or its bf16 copy dx_bf16 (either may be NULL) */
/* GradScaler for the fp16 backward (the reference's torch.cuda.amp.GradScaler, agent_oe.py:40-42,
 * per tensor instead of per step): scale[0] = S = 2^(7 - floor(log2(max|x|))) (max|x| * S in
 * [128, 256); S = 1 for an all-zero or non-finite x), scale[1] = 1/S.  scale[2..3] are the kernel's
 * arrival words: zero them once when allocating (the kernel leaves them zero).  n % 4 == 0, x 16-B
 * aligned. */
int lrce_grad_scale(const float* x, int64_t n, float* scale, void* stream);
/* Delayed scaling of the BERT backward's fp16 operands (the reference's GradScaler keeps one scale for
 * thousands of steps, agent_oe.py:40-42; here one per tensor, from the previous step): for each of
 * n_slots scale slots [S, 1/S, amax bits, -] with a recorded max (word 2 != 0): S = 2^(7 - floor(log2
 * amax)), 1/S, word 2 cleared; slots without one keep their scale; a non-finite amax (an fp16 operand
 * overflowed) halves S (GradScaler's backoff).  One launch per step. */
int lrce_grad_scale_update(float* scale, int n_slots, void* stream);
/* lrce_layernorm_bwd (identity maps, f32 dy / x, no residual) fused with lrce_dropout_bwd_f16: dx (f32,
 * optional), dx_f16 = fp16(scale[0] * dropout_bwd(dx)) (mask of lrce_dropout over [rows][cols], p / seed
 * + the device RNG offset), max|dx| folded into the slot's word 2 (NaN-sticky); dw / db as
 * lrce_layernorm_bwd (workspace: lrce_layernorm_bwd_workspace).  Replaces BertOutput / BertSelfOutput
 * LayerNorm backward + the fp16 cast of the reference's autocast backward (text.py:11-17). */
int lrce_layernorm_bwd_f16s(const float* dy, const float* x, const float* mean, const float* rstd, const float* w,
                            float* dx, float* dw, float* db, int rows, int cols, uint16_t* dx_f16, float* scale,
                            float p, uint64_t seed, float* workspace, int64_t workspace_elems, void* stream);
/* lrce_layernorm_bwd_f16s with its gamma / beta reduction left to lrce_layernorm_grad_reduce (*nb_out as
 * lrce_layernorm_bwd_deferred): the BERT backward reduces all its LayerNorms in one launch. */
int lrce_layernorm_bwd_f16s_deferred(const float* dy, const float* x, const float* mean, const float* rstd,
                                     const float* w, float* dx, float* dw, float* db, int rows, int cols,
                                     uint16_t* dx_f16, float* scale, float p, uint64_t seed, float* workspace,
                                     int64_t workspace_elems, int* nb_out, void* stream);
/* dx_f16 = fp16(scale[0] * dropout_bwd(dy)) (p = 0: a scaled cast): the fp16 operand of the BERT
 * backward GEMMs from an f32 residual-stream gradient. */
int lrce_dropout_bwd_f16(const float* dy, uint16_t* dx_f16, int64_t n, float p, uint64_t seed, int64_t group,
                         const float* scale, void* stream);
/* Device-side RNG offset for graph replay: every hash-based mask (lrce_dropout*, lrce_mha_* dropout)
 * uses seed + *offset when a device pointer is registered (NULL = 0, the default).  A captured
 * HIP graph bakes the host seeds; advancing *offset (one device add per training step) gives each
 * replay fresh masks while forward and backward of one step still agree. */
int lrce_set_rng_offset(const uint64_t* offset);

/* Fused optimizer step over the flat parameter buffer (agent_base.py:27-44,103-108).  Every tensor
 * starts at a multiple of 1024 elements; chunk_tensor[c] is the tensor id of 1024-element chunk c.
 * lrce_l2norm_multi: sumsq[t] = ||p_t||^2 (zeroed here).  lrce_adamw_step: torch.optim.AdamW update
 * (decoupled weight decay, bias corrections bc1 = 1-beta1^t, bc2 = 1-beta2^t) on the gradient
 * grad_scale * g + reg * p / ||p|| (the L2-regulariser term), tensor_lr[t] per tensor; also writes
 * the bf16 shadow copy of p (p_bf16, optional) used by the next forward.  An element whose gradient
 * term is not finite keeps its parameter and moments; a whole chunk range keeps them when a found-inf
 * flag of skip_slots is set (the reference's GradScaler skips the step on an overflow; here the group
 * whose gradients come from the overflowed fp16 operands, so early per-group updates of the other
 * groups need not wait for BERT's backward). */
int lrce_l2norm_multi(const float* p, const int32_t* chunk_tensor, int n_chunks, float* sumsq, int n_tensors,
                      const int32_t* tensor_chunk_off, float* chunk_sq, void* stream);
int lrce_adamw_step(float* p, const float* g, float* m, float* v, const int32_t* chunk_tensor, const float* tensor_lr,
                    const float* sumsq, uint16_t* p_bf16, int n_chunks, float beta1, float beta2, float eps,
                    float weight_decay, float grad_scale, float reg, float bc1, float bc2, const float* step,
                    float* sumsq_next, uint16_t* p_f16, int64_t f16_lo, int64_t f16_hi, const uint16_t* g_bf16,
                    const int32_t* tensor_chunk_off, float* chunk_sq, int n_tensors, const float* skip_slots,
                    int n_skip_slots, int64_t skip_c0, int64_t skip_c1, void* stream);
/* skip_slots (optional): n_skip_slots (<= 64) gradient-scale slots [S, 1/S, amax, found-inf] of the
 * delayed fp16 backward (lrce_layernorm_bwd_f16s); when any found-inf word is set, chunks [skip_c0,
 * skip_c1) of this call (relative to p) keep their parameters and moments — the step GradScaler would
 * skip, for the parameter group whose gradients those fp16 operands produce (their norms are still
 * written).  step: optional device step count t (bc1/bc2 then computed from it: graph-safe).  sumsq_next:
 * optional zeroed buffer that receives ||p_t||^2 of the UPDATED parameters, i.e. the next step's
 * sumsq without a separate norm pass over the 1.25 GB master copy.  p_f16 (optional): an IEEE fp16
 * shadow of elements [f16_lo, f16_hi) (multiples of 1024; element i at p_f16[i - f16_lo]) — the
 * BERT weights the fp16 forward reads — written in the same pass.  g_bf16 (optional): read the
 * gradient from this bf16 buffer (the all-reduced bf16 gradient buckets) instead of g (g may be NULL).
 * tensor_chunk_off int32 [n_tensors+1] (first chunk of each tensor) + chunk_sq f32 [n_chunks] scratch
 * (both or neither in lrce_l2norm_multi): the per-tensor norms are summed per chunk with plain stores
 * and then per tensor in a fixed order — bitwise reproducible, so data-parallel replicas (whose
 * L2-term gradient reg * p / ||p|| depends on them) stay identical; without them, float atomics.
 * Sub-range updates (p, g, m, v, p_bf16, chunk_tensor, chunk_sq, g_bf16 offset to a chunk range, the
 * f16 range relative to p): chunk_sq without tensor_chunk_off only writes the range's chunk sums;
 * the launch that passes tensor_chunk_off (after all ranges) sums every tensor. */

/* BERT embeddings before their LayerNorm (HF BertEmbeddings): out[r] = word[ids[r]] + pos[r % L] +
 * type[types[r]] (f32 tables, int64 ids), and the scatter-add backward into the three tables. */
int lrce_bert_embed_fwd(const int64_t* ids, const int64_t* types, const float* word, const float* pos, const float* typ,
                        float* out, int rows, int L, int C, void* stream);
int lrce_bert_embed_bwd(const float* dout, const int64_t* ids, const int64_t* types, float* dword, float* dpos, float* dtyp,
                        int rows, int L, int C, int64_t pad_id, void* stream); /* pad_id: word row without grad (-1 none) */
/* LRCE positional embeddings before their LayerNorm (embedding.py:47-63, 17-23). */
int lrce_video_posembed_fwd(const float* x, const float* cls, const float* pos, const float* len, const float* clip, float* out,
                            int B, int S, int Tg, int P, int C, void* stream);
/* Backward: dx (f32) and / or dx_bf16 (either may be NULL, not both) get the token rows, the four
 * tables' gradients are ADDED (f32 atomics) into dcls / dpos / dlen / dclip.  C % 4 == 0. */
int lrce_video_posembed_bwd(const float* dout, float* dx, uint16_t* dx_bf16, float* dcls, float* dpos, float* dlen,
                            float* dclip, int B, int S, int Tg, int P, int C, void* stream);
int lrce_text_posembed_fwd(const float* x, const float* cls, const float* pos, float* out, int B, int L, int C, void* stream);
int lrce_text_posembed_bwd(const float* dout, float* dx, float* dcls, float* dpos, int B, int L, int C, void* stream);

int lrce_version(void);
const char* lrce_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
