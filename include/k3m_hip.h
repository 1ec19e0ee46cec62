/* libk3m_hip — C ABI of the MI355X (gfx950) kernels behind the K3M tri-modal pretraining step.
 *
 * Boundary contract:
 *   - plain device pointers, sizes and a hipStream_t; no torch types;
 *   - the caller (torch's caching allocator) owns every buffer, including saved activations and
 *     workspaces; the library allocates nothing and keeps no state;
 *   - every entry point returns 0 on success, K3M_EINVAL on a bad argument, or -hipError_t of the
 *     launch; no host synchronisation inside (graph-capturable);
 *   - all work is enqueued on the passed stream.
 *
 * Each entry point names the reference code it replaces (file:line in sunzeyeah/K3M).  The
 * reference has no native operator API: its hot path is nn.Module code in
 * vilbert_k3m/vilbert_k3m.py whose ops go to ATen/cuBLAS; these functions are the replacement
 * kernels for those ops, bound from Python by k3m_amd/_lib.py (ctypes).
 */
#ifndef K3M_HIP_H
#define K3M_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define K3M_OK 0
#define K3M_EINVAL 1

enum K3mDType { K3M_F32 = 0, K3M_BF16 = 1 };

/* How fp32-operand GEMMs use the matrix cores (accuracy: k3m_amd/csrc/gemm_x6_tile.h):
 *   K3M_F32_SPLIT_BF16X6 — each fp32 operand split exactly into 3 bf16 planes, 6 bf16 MFMA partial
 *                          products accumulated in fp32 (fp32-level accuracy, 416.7 TF/s roofline);
 *   K3M_F32_MFMA_F32     — v_mfma_f32_32x32x2_f32 (exact f32 fma chain, 157.3 TF/s roofline). */
enum K3mF32Algo { K3M_F32_SPLIT_BF16X6 = 0, K3M_F32_MFMA_F32 = 1 };

enum K3mEpilogue {
  K3M_EPI_NONE = 0,         /* C = alpha*acc + beta*C                                        */
  K3M_EPI_BIAS = 1,         /* C = alpha*(acc + bias) + beta*C                               */
  K3M_EPI_BIAS_GELU = 2,    /* aux = acc + bias; C = gelu(aux)            (BertIntermediate)  */
  K3M_EPI_DGELU = 3,        /* C = acc * gelu'(aux) (+ beta*C)            (its backward)      */
  K3M_EPI_BIAS_SIGMOID = 4  /* C = sigmoid(acc + bias)                    (fusion gate scores)*/
};

/* C[m,n] = op(A)[m,k] . op(B)[k,n] with a fused epilogue.
 *   a_trans = 0: A(i,l) = a[i*lda + l]   (row-major activations, K contiguous)
 *   a_trans = 1: A(i,l) = a[l*lda + i]   (dY^T for weight gradients)
 *   b_trans = 1: B(l,j) = b[j*ldb + l]   (torch Linear weight [n,k]: forward x.W^T)
 *   b_trans = 0: B(l,j) = b[l*ldb + j]   (W for input gradients, X for weight gradients)
 * Replaces every nn.Linear addmm / mm of the step (vilbert_k3m.py: all Linear layers, tied decoder
 * :1838) and their autograd backward GEMMs. */
typedef struct K3mGemm {
  int m, n, k;
  int a_trans, b_trans;
  int epilogue;
  int dtype;             /* operand (A, B) type: K3M_F32, or K3M_BF16 (fp32 accumulation)       */
  int splitk;            /* >1: K split over splitk workgroup slices (epilogue must be NONE);   */
  int c_dtype;           /* C and aux type: K3M_F32 (K3M_F32 operands require it) or K3M_BF16   */
  long long lda, ldb, ldc, ldaux;
  const void* a;
  const void* b;
  void* c;
  const float* bias;
  void* aux;
  float* ws;             /* splitk > 1: fp32 workspace of splitk*m*n floats (deterministic    */
  float alpha, beta;     /* slab reduction, no atomics)                                        */
  int f32_algo;          /* fp32 operands: K3M_F32_SPLIT_BF16X6 (0, default) or K3M_F32_MFMA_F32 */
  long long a_planes;    /* reserved, must be 0 */
  long long b_planes;    /* reserved, must be 0 */
} K3mGemm;
int k3m_gemm(const K3mGemm* g, hipStream_t stream);
/* OR-ed into K3mGemm.epilogue of a split-K GEMM (splitk > 1, epilogue NONE): the kernel writes its fp32
 * slabs (ws[slice][m][n], raw sums) and returns without reducing them — C is untouched.  The caller
 * reduces them later with k3m_slab_reduce_batch (nslab = splitk, cols = m*n, requires ldc == n,
 * alpha == 1; the engine batches these with the LayerNorm / bias slabs of a whole encoder block). */
#define K3M_GEMM_SLABS_ONLY 0x100
/* OR-ed into K3mGemm.epilogue of a K3M_EPI_DGELU GEMM (splitk <= 1, beta == 0): the kernel also writes the
 * column sums of its output C into ws, one fp32 slab per 32-row group (ws[r/32][n], ceil(m/32) slabs of n
 * floats) — the bias gradient of the Linear that C feeds, without re-reading C (replaces k3m_colsum on it).
 * The caller reduces the slabs with k3m_slab_reduce_batch (nslab = ceil(m/32), cols = n). */
#define K3M_GEMM_COLSUM_SLABS 0x200
/* Up to 8 INDEPENDENT problems in one launch (no problem may read another's output).  When all share
 * one kernel template (fp32 operands on the bf16x6 path, same a_trans / b_trans / epilogue, 16-B
 * aligned) they run as one grid of 256x128 tiles — the co-attention blocks' six small GEMMs per
 * step of the wide engine; otherwise each runs through k3m_gemm. */
int k3m_gemm_grouped(const K3mGemm* gs, int count, hipStream_t stream);

/* out[c] (+)= sum_r x[r*ld + c]  — bias gradients (autograd of every Linear bias).
 * ws: >= (256 + 16)*cols floats. */
int k3m_colsum(const void* x, long long ld, int rows, int cols, float* out, int accumulate, float* ws,
               int dtype, hipStream_t stream);
/* k3m_colsum without the reduction: nslab (k3m_colsum_nslab) fp32 slabs of column partials at ws
 * ([nslab][cols]) for k3m_slab_reduce_batch. */
int k3m_colsum_nslab(int rows, int* nslab);
int k3m_colsum_slabs(const void* x, long long ld, int rows, int cols, float* ws, int dtype, hipStream_t stream);
/* Deterministic column-slab reduction of njobs independent jobs (host arrays of njobs entries):
 * out[j][c] = (accumulate[j] ? out[j][c] : 0) + sum_{s < nslab[j]} ws[j][s*cols[j] + c], slabs summed
 * in a fixed order.  Jobs are batched into as few launches as possible (a job whose output repeats an
 * earlier job's output of the same launch starts a new launch, so accumulations keep their order). */
int k3m_slab_reduce_batch(const float* const* ws, float* const* out, const int* nslab, const int* cols,
                          const int* accumulate, int njobs, hipStream_t stream);

/* Post-LN residual block tail (BertSelfOutput/BertOutput/BertBiOutput/BertImageEmbeddings,
 * vilbert_k3m.py:485-489, :528-532, :986-996, :2153-2161, LayerNorm :319-332):
 *   s = dropout_in(x) + res;  y = dropout_out(gamma * (s-mean)*rstd + beta)
 * saves xhat = (s-mean)*rstd and rstd for the backward.  res may be NULL. */
int k3m_ln_fwd(const void* x, const void* res, const float* gamma, const float* beta, void* y, void* xhat,
               float* rstd, int rows, int cols, float eps, float p_in, float p_out, uint64_t seed,
               uint64_t off_in, uint64_t off_out, int dtype, hipStream_t stream);
/* Backward of k3m_ln_fwd.  ds = d(pre-LN sum) is written to dres (or accumulated when
 * accumulate_res), dx = dropout_in'(ds) is written to dx (may alias dres when p_in == 0).
 * dgamma/dbeta are ACCUMULATED (fp32 grad buffer).  dxsum (nullable): the column sums of dx are
 * ACCUMULATED into it — the bias gradient of the Linear that produced x, fused here instead of a
 * separate reduction over dx.  ws: >= 3*(K3M_LN_BWD_SLABS + 16)*cols floats. */
#define K3M_LN_BWD_SLABS 512
int k3m_ln_bwd(const void* dy, const void* xhat, const float* rstd, const float* gamma, void* dres, void* dx,
               float* dgamma, float* dbeta, float* dxsum, int rows, int cols, float p_in, float p_out, uint64_t seed,
               uint64_t off_in, uint64_t off_out, int accumulate_res, float* ws, int dtype, hipStream_t stream);
/* k3m_ln_bwd without the reduction: dres/dx written, the dgamma / dbeta / (want_sum) sum(dx)
 * column partials left as 3 arrays of nslab slabs (array a at ws + a*nslab*cols, nslab from
 * k3m_ln_bwd_nslab) for k3m_slab_reduce_batch. */
int k3m_ln_bwd_nslab(int rows, int* nslab);
int k3m_ln_bwd_slabs(const void* dy, const void* xhat, const float* rstd, const float* gamma, void* dres, void* dx,
                     int rows, int cols, float p_in, float p_out, uint64_t seed, uint64_t off_in, uint64_t off_out,
                     int accumulate_res, int want_sum, float* ws, int dtype, hipStream_t stream);

/* BertEmbeddings (vilbert_k3m.py:361-382): word + position + token-type -> LN -> dropout.
 * The row is written to y0 and, when non-NULL, to y1 and y2 (the same embedding output feeds two
 * encoder passes, vilbert_k3m.py:1703-1743).  ids/tt: int64 [nseq, len]. */
int k3m_embed_fwd(const int64_t* ids, const int64_t* tt, const float* word, const float* pos, const float* type,
                  const float* gamma, const float* beta, void* y0, void* y1, void* y2, void* xhat, float* rstd,
                  int nseq, int len, int hidden, float eps, float p_out, uint64_t seed, uint64_t off,
                  int dtype, hipStream_t stream);
/* Gradient of the lookup: dword[id] += ds (skipping id 0: padding_idx, :343-345), dpos, dtype.
 * ds = d(pre-LN sum) from k3m_ln_bwd. */
int k3m_embed_bwd(const int64_t* ids, const int64_t* tt, const void* ds, float* dword, float* dpos, float* dtype_,
                  int nseq, int len, int hidden, int dtype, hipStream_t stream);

/* Multi-head scaled-dot-product attention with additive key mask, softmax and probability
 * dropout (BertSelfAttention :439-475, BertImageSelfAttention :586-634, BertBiAttention :753-838,
 * BertBiAttention_two_text :882-965).  Row (s, i) of Q starts at q + (s*lq+i)*ldq; head h is
 * columns [h*hd, (h+1)*hd).  kmask: additive float [nseq, lk].  probs: [nseq, nh, lq, lk]
 * (softmax output before dropout), saved for the backward. */
int k3m_attn_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                 const float* kmask, void* ctx, long long ldc, float* probs, int nseq, int lq, int lk, int nh, int hd,
                 float scale, float p_drop, uint64_t seed, uint64_t off, int dtype, hipStream_t stream);
/* Backward (matrix cores): o = the forward context (D_i = dO_i . O_i replaces the per-row
 * sum_j P dP reduction).  hd must be a multiple of 32. */
int k3m_attn_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                 const void* k, long long ldk, const void* v, long long ldv, const float* probs, void* dq, void* dk,
                 void* dv, long long lddq, long long lddk, long long lddv, int nseq, int lq, int lk, int nh, int hd,
                 float scale, float p_drop, uint64_t seed, uint64_t off, int dtype, hipStream_t stream);

/* bf16 attention for the mixed-precision encoder (same semantics as k3m_attn_fwd/bwd; head dim
 * 64, 96 or 128, L <= 128): instead of the [nseq, nh, lq, lk] probabilities the forward saves the row
 * log-sum-exp lse [nseq, nh, lq] and the backward recomputes P from it (kmask is needed again).
 * Every row pointer + ld must allow 16-byte loads (ld % 8 == 0, 16-B aligned base). */
int k3m_flash_attn_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                       const float* kmask, void* ctx, long long ldc, float* lse, int nseq, int lq, int lk, int nh,
                       int hd, float scale, float p_drop, uint64_t seed, uint64_t off, hipStream_t stream);
int k3m_flash_attn_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                       const void* k, long long ldk, const void* v, long long ldv, const float* kmask,
                       const float* lse, void* dq, void* dk, void* dv, long long lddq, long long lddk, long long lddv,
                       int nseq, int lq, int lk, int nh, int hd, float scale, float p_drop, uint64_t seed,
                       uint64_t off, hipStream_t stream);

/* bf16 flash attention for sequences longer than 128, up to max_position_embeddings = 512
 * (config/bert_base_6layer_6conect.json:8; the PV stream of BASELINE configs[4] at 320 tokens, fine-tuning PV 256):
 * same semantics, LSE layout and dropout counters as k3m_flash_attn_fwd / _bwd, any lq, lk in [1, 512], head dim
 * 64, 96 or 128, nothing of size lq x lk in HBM (attention_flash_long.hip).  Replaces the exact-fp32
 * k3m_attn_long_* path of the bf16 encoder (BertSelfAttention :439-475, BertBiAttention :753-838,
 * BertBiAttention_two_text :904-965).  The backward takes a workspace of k3m_flash_attn_long_ws_bytes(...) bytes
 * (16-B aligned): D = rowsum(dO o O) and, when the keys of a head exceed one workgroup, fp32 dQ partials reduced
 * in a fixed order (deterministic); *bytes receives the size.  Rows as in k3m_flash_attn_fwd; dq needs 8-B aligned
 * rows (lddq % 4 == 0). */
int k3m_flash_attn_long_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                            const float* kmask, void* ctx, long long ldc, float* lse, int nseq, int lq, int lk, int nh,
                            int hd, float scale, float p_drop, uint64_t seed, uint64_t off, hipStream_t stream);
int k3m_flash_attn_long_ws_bytes(int nseq, int lq, int lk, int nh, int hd, long long* bytes);
int k3m_flash_attn_long_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                            const void* k, long long ldk, const void* v, long long ldv, const float* kmask,
                            const float* lse, void* dq, void* dk, void* dv, long long lddq, long long lddk,
                            long long lddv, void* ws, long long ws_bytes, int nseq, int lq, int lk, int nh, int hd,
                            float scale, float p_drop, uint64_t seed, uint64_t off, hipStream_t stream);

/* Elementwise: out = g * gelu'(pre) (backward of the MLM/image head transforms :1795-1818). */
int k3m_dgelu(const void* g, const void* pre, void* out, long long n, int dtype, hipStream_t stream);

/* Row gather / scatter-add for the labelled-row heads. idx: int32 [n]. */
int k3m_gather_rows(const void* src, long long lds, const int32_t* idx, int n, int cols, void* dst, long long ldd,
                    int dtype, hipStream_t stream);
int k3m_scatter_add_rows(const void* src, long long lds, const int32_t* idx, int n, int cols, void* dst,
                         long long ldd, int dtype, hipStream_t stream);

/* Compact labelled positions (order preserving, single workgroup, graph-safe): for r in [0,n) with
 * labels[r] >= thresh append, at position count[0] + rank,
 *   idx = (r / inner) * outer + r % inner + base   (row in the sequence buffer),
 *   out_labels = labels[r], src = r, slot = slot_id,
 * then row_scale = 1/appended for the appended rows (mean over the task's labelled rows) and
 * count[0] += appended.  Any of out_labels / src / row_scale / slot may be NULL. */
int k3m_compact_labels_ex(const int64_t* labels, int n, int64_t thresh, int inner, int outer, int base, int slot_id,
                          int32_t* idx, int64_t* out_labels, int32_t* src, float* row_scale, int32_t* slot,
                          int32_t* count, hipStream_t stream);

/* Masked-LM cross-entropy (CrossEntropyLoss(ignore_index=-1), :2255, :2817-2826) over gathered
 * rows: loss_rows[r] = lse - logit[label]; logits are overwritten by row_scale[r]*(softmax-onehot). */
int k3m_ce_fwd_bwd(float* logits, long long ld, const int64_t* labels, const float* row_scale, int rows, int vocab,
                   float* loss_rows, hipStream_t stream);
/* Region KL (KLDivLoss(log_softmax(pred), target), :2753-2760) over gathered rows: loss_rows[r] =
 * sum_c xlogy(t,t) - t*logsoftmax(pred); pred overwritten by scale*(softmax*sum(t) - t). */
int k3m_kl_fwd_bwd(float* logits, long long ld, const float* target, long long ldt, const int32_t* trow,
                   const float* row_scale, int rows, int ncls, float* loss_rows, hipStream_t stream);
/* x[r][c] *= (slot[r] == 0 ? w0 : w1): the shared MLM decoder's gradient rows of the text (slot 0) and PV
 * (slot 1) heads weighted by their losses' upstream gradients (a caller's w_t*mlm_t + w_pv*mlm_pv; the
 * reference sums them with weight 1, train_concap_struc.py:531-533). */
int k3m_scale_rows_by_slot(float* x, long long ld, const int32_t* slot, int rows, int cols, float w0, float w1,
                           hipStream_t stream);
/* out[slot[r]] += loss_rows[r] * row_scale[r] for slots 0..3 (single block). */
int k3m_loss_reduce(const float* loss_rows, const float* row_scale, const int32_t* slot, int rows, float* out,
                    hipStream_t stream);
/* NSP head forward (seq_relationship(dropout(t+pv+v)) + CE, :1881-1887, :2828-2832); forward only
 * (its loss is excluded from the training total, train_concap_struc.py:533). */
int k3m_nsp_loss(const float* pt, const float* ppv, const float* pv, const float* w, const float* b,
                 const int64_t* l0, const int64_t* l1, const int64_t* l2, int batch, int hidden, float* out,
                 hipStream_t stream);

/* Fusion gate, pre_sampling_sequence (vilbert_k3m.py:2331-2374):
 * relu_cat3: c[r, k*D + ch] = relu(x_k[r, ch])                                               */
int k3m_relu_cat3(const void* x0, const void* x1, const void* x2, void* c, int rows, int d, int dtype,
                  hipStream_t stream);
/* gate forward: a = sigmoid scores [rows, 3D]; noise [rows, 3, D] or NULL (then gumbel noise is
 * drawn from (seed, off)); ys = softmax(a + g) over the 3 streams; idx = argmax; out = c[idx]. */
int k3m_gate_fwd(const float* a, const void* c, const float* noise, float* ys, uint8_t* idx, void* out, int rows,
                 int d, uint64_t seed, uint64_t off, int dtype, hipStream_t stream);
/* gate backward (straight-through): dc = onehot*dout; dpre = sigmoid'(a)*softmax'(ys)(dout*c). */
int k3m_gate_bwd(const void* dout, const float* a, const void* c, const float* ys, const uint8_t* idx, void* dc,
                 void* dpre, int rows, int d, int dtype, hipStream_t stream);
/* dx_k (+)= dc[:, kD:(k+1)D] * (c > 0), k = 0..2 (any dx_k may be NULL). */
int k3m_relu_split3_bwd(const void* dc, const void* c, void* dx0, void* dx1, void* dx2, int rows, int d,
                        int accumulate, int dtype, hipStream_t stream);
/* if_pre_sampling == 0: out = (x0+x1+x2)/3 ; backward: dx_k (+)= dout/3 */
int k3m_mean3(const void* x0, const void* x1, const void* x2, void* out, long long n, int dtype, hipStream_t stream);
int k3m_mean3_bwd(const void* dout, void* dx0, void* dx1, void* dx2, long long n, int accumulate, int dtype,
                  hipStream_t stream);
/* out[s, :] (+)= scale * mean(x[s, start:len, :])  (pooled outputs :2405-2409) and backward. */
int k3m_seq_mean(const void* x, int nseq, int len, int start, int d, float scale, float* out, int accumulate,
                 int dtype, hipStream_t stream);
int k3m_seq_mean_bwd(const float* dout, int nseq, int len, int start, int d, float scale, void* dx, int dtype,
                     hipStream_t stream);

/* Structure aggregator + LPM (structure_aggregator, vilbert_k3m.py:2413-2505), vectorised over a
 * padded [B, NPV] triple layout.  X[(i*npv+j), :] = [c_init_i ; p_ij ; v_ij] with p/v the mean of
 * the two endpoint rows of index_p/index_v; nvalid[i] = first j with index_p[i,j,0]==0. */
int k3m_sa_gather(const void* seq, const int64_t* index_p, const int64_t* index_v, const float* c_init, float* X,
                  int32_t* nvalid, int32_t* src, int batch, int len, int npv, int hidden, int dtype,
                  hipStream_t stream);
/* per item: beta_j = w2.leaky_relu(T_j) + b2, att = softmax_j, agg = sum_j att_j T_j
 * (T rows of item src[i]; src[i] = -1 -> agg = c_init[0]). */
int k3m_sa_attn_fwd(const float* T, const int32_t* nvalid, const int32_t* src, const float* w2, const float* b2,
                    const float* c_init, float* att, float* agg, int batch, int npv, int hidden, hipStream_t stream);
int k3m_sa_attn_bwd(const float* dagg, const float* T, const float* att, const int32_t* nvalid,
                    const int32_t* src, const float* w2, float* dT, float* dw2, float* db2, float* dc_init, int batch,
                    int npv, int hidden, hipStream_t stream);
/* LPM margin-ranking loss (:2469-2502); ent_neg [B, NPV, n_ent] / val_neg [B, NPV, n_val] int64 entity /
 * value negative indices (-1 = none; n_ent = num_negative_pv // 2, n_val = num_negative_pv - n_ent,
 * n_ent + n_val <= 16).  loss[0] = mean hinge over every (positive, negative) pair.
 * ws: >= B*NPV*(2*(n_ent + n_val) + 1) + 2 floats.  Backward ACCUMULATES into dc_final [B,H] and the
 * p/v thirds of dX. */
int k3m_lpm_fwd(const float* c_final, const float* X, const int32_t* nvalid, const int64_t* ent_neg,
                const int64_t* val_neg, int batch, int npv, int hidden, int n_ent, int n_val, float margin,
                float* loss, float* ws, hipStream_t stream);
int k3m_lpm_bwd(const float* c_final, const float* X, const int32_t* nvalid, const int64_t* ent_neg,
                const int64_t* val_neg, int batch, int npv, int hidden, int n_ent, int n_val, float margin,
                const float* ws, float* dc_final, float* dX, hipStream_t stream);
/* Device-side draw of the LPM negatives with the reference's semantics (random.sample without
 * replacement of min(#candidates, n_ent) entity indices k != i and min(#candidates, n_val) value
 * indices j' != j, vilbert_k3m.py:2476-2492); unused slots are -1. */
int k3m_lpm_sample(const int32_t* nvalid, int batch, int npv, int n_ent, int n_val, uint64_t seed, uint64_t off,
                   int64_t* ent_neg, int64_t* val_neg, hipStream_t stream);
/* scatter the p / v gradients of dX back to the sequence rows and dX's c_init third into dc_init. */
int k3m_sa_gather_bwd(const float* dX, const int64_t* index_p, const int64_t* index_v, const int32_t* nvalid,
                      void* dseq, float* dc_init, int batch, int len, int npv, int hidden, int dtype,
                      hipStream_t stream);

/* Deterministic mode (K3M_DETERMINISTIC=1 in k3m_amd): the backward kernels above whose sums went through
 * float atomics (order-dependent rounding: two runs of one step differed in the last bits), restated with every sum
 * in a fixed order -- one owning workgroup per destination row, batch-wide sums through per-item partials reduced
 * in item order.  Same arguments; the embedding form takes ws = [len][2][hidden] floats (type_vocab_size 2,
 * config/bert_base_6layer_6conect.json) and the structure-attention form ws = [batch][hidden + 1] floats.
 * hidden <= 1024 (embedding) / 2048 (structure aggregator). */
int k3m_embed_bwd_det(const int64_t* ids, const int64_t* tt, const void* ds, float* dword, float* dpos, float* dtype_,
                      int nseq, int len, int hidden, float* ws, int dtype, hipStream_t stream);
int k3m_sa_attn_bwd_det(const float* dagg, const float* T, const float* att, const int32_t* nvalid,
                        const int32_t* src, const float* w2, float* dT, float* dw2, float* db2, float* dc_init,
                        float* ws, int batch, int npv, int hidden, hipStream_t stream);
int k3m_lpm_bwd_det(const float* c_final, const float* X, const int32_t* nvalid, const int64_t* ent_neg,
                    const int64_t* val_neg, int batch, int npv, int hidden, int n_ent, int n_val, const float* ws,
                    float* dc_final, float* dX, hipStream_t stream);
int k3m_sa_gather_bwd_det(const float* dX, const int64_t* index_p, const int64_t* index_v, const int32_t* nvalid,
                          void* dseq, float* dc_init, int batch, int len, int npv, int hidden, int dtype,
                          hipStream_t stream);

/* pytorch_transformers 1.1.0 AdamW (train_concap_struc.py:436-441) over a contiguous segment of
 * the flat parameter buffer: m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
 * p -= lr*sqrt(1-b2^t)/(1-b1^t) * m/(sqrt(v)+eps); p -= lr*wd*p.  Optionally writes a bf16 copy
 * of the updated parameters (p_bf16 may be NULL).  grad_scale multiplies g (1/world_size).
 * Hyper-parameters are doubles, as the reference's Python floats: every derived scalar
 * (1-beta, the bias-corrected step size, lr*wd) is formed in double and rounded once to fp32. */
int k3m_adamw(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, long long n, double lr, double beta1,
              double beta2, double eps, double wd, int step, float grad_scale, hipStream_t stream);

/* k3m_adamw with options (flags, OR-ed):
 *   K3M_ADAM_ZERO_GRAD — g is zeroed after it is read (optimizer.step(); optimizer.zero_grad(),
 *                        train_concap_struc.py:573-574, in one sweep of the gradient buffer);
 *   K3M_ADAM_APEX      — apex FusedAdam(adam_w_mode) instead, the optimizer of the mixed-precision
 *                        branches (:410-411, :426): p -= lr*((m/bc1)/(sqrt(v/bc2)+eps) + wd*p), with
 *                        bc = 1 unless K3M_ADAM_APEX_BIAS_CORRECTION (the driver passes
 *                        bias_correction=False). */
#define K3M_ADAM_ZERO_GRAD 1
#define K3M_ADAM_APEX 2
#define K3M_ADAM_APEX_BIAS_CORRECTION 4
int k3m_adamw_ex(float* p, float* g, float* m, float* v, uint16_t* p_bf16, long long n, double lr, double beta1,
                 double beta2, double eps, double wd, int step, float grad_scale, int flags, hipStream_t stream);

/* Whole-step hipGraph replay (k3m_amd/graph.py; no reference counterpart — the reference re-issues
 * every launch from Python each step, train_concap_struc.py:466-589).  A captured launch keeps its
 * by-value arguments, so the two per-step values come from device memory:
 *  - k3m_adamw_ex_dev: k3m_adamw_ex whose four derived fp32 scalars (step_size, decay, 1/bc1, 1/bc2)
 *    are read from `scalars` (16-B aligned device memory) when the kernel runs;
 *    k3m_adamw_scalars_n writes, for n (lr[i], wd[i]) pairs, exactly the four values k3m_adamw_ex
 *    would pass for (lr[i], beta1, beta2, wd[i], step, flags) (host memory, out[4*i .. 4*i+3]);
 *  - seeds: a launch whose seed has bit 63 set (K3M_GRAPH_SEED; host seeds are below 2^63) draws
 *    with the 64-bit seed stored at device address (seed & ~K3M_GRAPH_SEED) when it runs (every
 *    dropout / gumbel / sampling kernel of this library). */
#define K3M_GRAPH_SEED (1ull << 63)
int k3m_adamw_ex_dev(float* p, float* g, float* m, float* v, uint16_t* p_bf16, long long n, const float* scalars,
                     double beta1, double beta2, double eps, float grad_scale, int flags, hipStream_t stream);
int k3m_adamw_scalars_n(int n, const double* lr, const double* wd, double beta1, double beta2, int step, int flags,
                        float* out);

/* Attention for sequences longer than 128 (up to 512 keys, d <= 128): the fine-tuning PV text
 * (max_seq_length_pv 256, finetune.py:1275) and SURVEY config 5 (P = 320).  Same arguments,
 * semantics, probability layout and dropout counters as k3m_attn_fwd / k3m_attn_bwd; the backward
 * takes a workspace ds_ws of the probabilities' size (fp32 [nseq*nh*lq*lk]). */
int k3m_attn_long_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                      const float* kmask, void* ctx, long long ldc, float* probs, int nseq, int lq, int lk, int nh,
                      int hd, float scale, float p_drop, uint64_t seed, uint64_t off, int dtype, hipStream_t stream);
int k3m_attn_long_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                      const void* k, long long ldk, const void* v, long long ldv, const float* probs, float* ds_ws,
                      void* dq, void* dk, void* dv, long long lddq, long long lddk, long long lddv, int nseq, int lq,
                      int lk, int nh, int hd, float scale, float p_drop, uint64_t seed, uint64_t off, int dtype,
                      hipStream_t stream);

/* torch.optim.AdamW (decoupled decay applied first, eps added after the bias correction of sqrt(v)):
 * the optimizer of the fine-tuning driver (finetune.py:356-361).  Same arguments as k3m_adamw. */
int k3m_adamw_torch(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, long long n, double lr,
                    double beta1, double beta2, double eps, double wd, int step, float grad_scale, hipStream_t stream);

/* Cast helpers for the mixed-precision path. */
int k3m_cast_f32_bf16(const float* x, uint16_t* y, long long n, hipStream_t stream);
/* y = (accumulate ? y : 0) + alpha * x with a type conversion (fp32 <-> bf16): the boundary between
 * the fp32 heads/fusion and a bf16 encoder, and the bf16 weight shadow.  (Mixed-precision
 * plumbing; the reference's fp16 path is apex amp, train_concap_struc.py:409-432.) */
int k3m_convert(const void* x, int xdtype, void* y, int ydtype, long long n, int accumulate, float alpha,
                hipStream_t stream);
int k3m_add_inplace(void* y, const void* x, long long n, float alpha, int dtype, hipStream_t stream);

/* ---- Item alignment fine-tuning --------------------------------------
 * K3MForItemAlignment.forward (vilbert_k3m.py:3379-3456) heads over the stacked pair embedding
 * e = c_final [2B][H] (item 1 rows, then item 2 rows); forward and backward fused.
 * pair_cat: x[b] = dropout_p([e[b] ; e[B+b]]) [B][2H] (ClassificationHead input, :2177);
 * pair_cat_bwd writes de [2B][H] from dx [B][2H] with the same mask. */
int k3m_align_pair_cat(const float* e, int B, int H, float p, uint64_t seed, uint64_t off, float* x,
                       hipStream_t stream);
int k3m_align_pair_cat_bwd(const float* dx, int B, int H, float p, uint64_t seed, uint64_t off, float* de,
                           hipStream_t stream);
/* "ce": u = classifier.dense(x) [B][H]; logits = out_proj(dropout_p(tanh(u))) (W [2][H], bias [2]),
 * probs = softmax, loss = mean CE with labels (float, truncated to long as labels.to(torch.long)).
 * Writes logits/probs [B][2], dlogits [B][2], loss_rows [B], loss [1], du [B][H]; ACCUMULATES the
 * out_proj gradients into gW / gb. */
int k3m_align_ce_fwd_bwd(const float* u, const float* W, const float* bias, const float* labels, int B, int H,
                         float p, uint64_t seed, uint64_t off, float* logits, float* probs, float* dlogits,
                         float* loss_rows, float* loss, float* du, float* gW, float* gb, hipStream_t stream);
/* "cosine": loss = CosineEmbeddingLoss(margin)(e1, e2, 2*labels-1); probs[b] = (cos(e1_b, e1_b) + 1)/2;
 * de [2B][H] = d loss / d e (written). */
int k3m_align_cosine_fwd_bwd(const float* e, const float* labels, int B, int H, float margin, float* loss,
                             float* probs, float* loss_rows, float* de, hipStream_t stream);

/* ---- Data path ------------------------------------------------------
 * Global-region collation of a batch of region features, fused with mask_region's feature
 * zeroing: replaces the numpy block of ConceptCapLoaderTrain_struc.__iter__
 * (vilbert_k3m/datasets/concept_cap_dataset_struc.py:381-388) and image_feat[i] = 0 (:913-915).
 * feat fp32 [B][R][F] (sample stride ldb floats), zero_feat / masked_label uint8 [B][R] (from
 * k3m_prep_regions, k3m_data.h); out fp32 [B][R+1][F]: row 0 = (float)((double)sum_r feat' / cnt),
 * cnt = #(masked_label == 0) (0 -> 1), rows 1.. = feat' (masked rows zeroed).  Bit-identical to the
 * reference's numpy (row-ordered fp32 sum, double division).  F % 4 == 0, 16-B aligned pointers.
 * Fine-tuning collation (K3MDataLoader.post_process, dataset:265-292): divisor int32 [B] = the raw
 * num_boxes (no 0 -> 1 fix: 0 gives inf / nan as numpy), zero_feat / masked_label may be NULL;
 * divisor NULL selects the pretraining count above. */
int k3m_collate_regions(const float* feat, long long ldb, const uint8_t* zero_feat, const uint8_t* masked_label,
                        const int32_t* divisor, int B, int R, int F, float* out, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
