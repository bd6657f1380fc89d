/*
 * recsys_amd.h - C ABI of librecsys_amd.so, the MI355X (gfx950) kernels behind the
 * two-tower retrieval + contrastive training + DeepFM rerank hot path of
 * DotBlossom/LLM-driven_content-based-feature_recommendation_system.
 *
 * Conventions (every entry point):
 *   - plain device pointers (fp32 row-major unless stated), int64 sizes, no torch types;
 *   - `stream` is a hipStream_t passed as void*; work is enqueued asynchronously, no
 *     host synchronisation, no device allocation inside (callers own every buffer, so a
 *     call can be captured into a hipGraph);
 *   - return 0 on success; non-zero = error code, text via rsx_last_error()
 *     (thread-local; argument errors return 1 before anything is launched);
 *   - "accumulated" outputs are added into and must be zeroed by the caller.
 * Each function names the reference interface it replaces (path:line under the
 * reference tree). The reference is pure Python/PyTorch; these are the kernels under its
 * nn.Module / loss-function surface (see INTEGRATION.md for the ctypes binding).
 */
#ifndef RECSYS_AMD_H
#define RECSYS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- library identity / errors ------------------------------------------------------ */
const char* rsx_last_error(void);
int rsx_abi_version(void);
const char* rsx_target_arch(void);
/* sha256 (first 16 hex digits) of the sources the library was built from (csrc/Makefile: the .hip
 * files sorted by name, rsx_common.h, this header): a caller can tell a stale prebuilt binary. */
const char* rsx_build_hash(void);

/* ---- A2: SASRecUserTower embedding stage --------------------------------------------
 * Replaces tower_code/v1_refine_usertower.py:434-459:
 *   seq_emb = item_proj(pretrained_vecs); seq_emb += E_j(ids_j) * s_g[j] (j = 0..5);
 *   seq_emb += pos_emb(arange(L)); seq_emb = emb_ln(seq_emb); emb_dropout(seq_emb)
 * over T tokens: dense [B, L] (tok_pos NULL => position = token % L) or any packed token
 * list with tok_pos[T] (int64) giving each token's position (L <= 64).
 * base      [T, D] = item_proj output (nullable => 0)
 * ids/tables: ntab (<=6) device pointers, ids int64 [T], tables [rows_j, D]
 * gate      [ntab] device (s_g = sigmoid(seq_gate) * s_mask); a gate that is exactly 0
 *           skips its gather (forward-exact) and reports a zero gate/table gradient
 *           (exact for the reference, whose zero gates come from a constant 0 mask)
 * pos [L, D], ln_w/ln_b [D] (ln_w == NULL => no LayerNorm: out = pre-LN sum, bit-exact
 * with the reference's op order), mean/rstd [T] saved for the backward.
 * D in {64, 128, 256}. Dropout p in [0,1) via counter hash (seed). */
int rsx_seq_embed_fwd(const float* base, const int64_t* const* ids, const float* const* tables, int ntab,
                      const float* gate, const float* pos, const int64_t* tok_pos, const float* ln_w,
                      const float* ln_b, float eps, int64_t T, int64_t L, int64_t D, float p_drop, uint64_t seed,
                      float* out, float* mean, float* rstd, void* stream);

/* Backward of rsx_seq_embed_fwd. dbase [T,D] written; dtables[j], dgate [ntab], dpos [L,D],
 * dln_w/dln_b [D] accumulated (nullable). padding_idx[j]: rows excluded from the table
 * gradient exactly like nn.Embedding(padding_idx=...) (-1 = none). table_rows[j] lets small
 * tables (time buckets) accumulate in LDS. Position, small-table, LN and gate gradients are
 * per-workgroup LDS sums; with a workspace (>= rsx_seq_embed_bwd_workspace_floats floats) they
 * are stored per workgroup and folded in block order by a second kernel (deterministic);
 * workspace NULL flushes them with global float atomics (last bits vary run to run). */
int64_t rsx_seq_embed_bwd_workspace_floats(int64_t T, int64_t L, int64_t D);
int rsx_seq_embed_bwd(const float* base, const int64_t* const* ids, const float* const* tables,
                      const int64_t* table_rows, const int64_t* padding_idx, int ntab, const float* gate,
                      const float* pos, const int64_t* tok_pos, const float* ln_w, const float* mean,
                      const float* rstd, float eps, int64_t T, int64_t L, int64_t D, float p_drop, uint64_t seed,
                      const float* dout, float* dbase, float* const* dtables, float* dgate, float* dpos,
                      float* dln_w, float* dln_b, float* workspace, int64_t ws_floats, void* stream);

/* ---- A3 / A9: masked multi-head self-attention core (L <= 64) -----------------------
 * Replaces the attention inside nn.TransformerEncoderLayer (norm_first, batch_first) at
 * tower_code/v1_refine_usertower.py:343-352,461-466 (causal + key padding) and
 * item_tower.py:169-182,281 (unmasked). Tokens are dense sequences (seg_off NULL: T = B*L)
 * or packed variable-length segments (seg_off [B+1] int32 token offsets, each <= 64 long).
 * qkv [T, 3*H*Dh] = in_proj output; out [T, H*Dh] = pre-out_proj head concat; lse [T, H].
 * key_pad [T] uint8 (1 = pad, nullable). Causal = key position <= query position within
 * the sequence. Training-path semantics: a fully masked query row gets zero probabilities.
 * Dh in {16, 32, 64} (backward: {16, 32}). */
int rsx_mha_fwd(const float* qkv, const uint8_t* key_pad, const int* seg_off, int64_t B, int64_t L, int64_t H,
                int64_t Dh, int causal, float p_drop, uint64_t seed, float* out, float* lse, void* stream);
/* dqkv [T, 3*H*Dh] written. */
int rsx_mha_bwd(const float* qkv, const uint8_t* key_pad, const int* seg_off, const float* out, const float* lse,
                const float* dout, int64_t B, int64_t L, int64_t H, int64_t Dh, int causal, float p_drop,
                uint64_t seed, float* dqkv, void* stream);
/* bf16x3 forms (Dh == 32; the forward also Dh == 64, the item tower's BERT at inference,
 * item_tower.py:264-268; same arguments, masks, dropout stream and lse convention):
 * 16x16 score tiles on v_mfma_f32_16x16x32_bf16 and token sums on v_mfma_f32_16x16x16_bf16
 * with every fp32 operand split hi + lo (~2^-17 relative error per product). The forward of
 * one form may be paired with the backward of the other. */
int rsx_mha_fwd_x3(const float* qkv, const uint8_t* key_pad, const int* seg_off, int64_t B, int64_t L, int64_t H,
                   int64_t Dh, int causal, float p_drop, uint64_t seed, float* out, float* lse, void* stream);
int rsx_mha_bwd_x3(const float* qkv, const uint8_t* key_pad, const int* seg_off, const float* out, const float* lse,
                   const float* dout, int64_t B, int64_t L, int64_t H, int64_t Dh, int causal, float p_drop,
                   uint64_t seed, float* dqkv, void* stream);
/* Fused in-projection + attention forward (replaces nn.TransformerEncoderLayer's
 * self_attn in_proj GEMM followed by the attention core, v1_refine_usertower.py:343-352 ->
 * torch.nn.functional.multi_head_attention_forward): x [T, D] the norm1 output, w [3D, D]
 * in_proj_weight, bias [3D] in_proj_bias (nullable); D = 128 (4 heads of 32), bf16x3. Writes
 * out [T, D] and lse [T, H] as rsx_mha_fwd_x3 does, and qkv [T, 3D] (nullable) for
 * rsx_mha_bwd_x3 and the in_proj weight gradient. */
int rsx_mha_qkv_fwd_x3(const float* x, const float* w, const float* bias, const uint8_t* key_pad, const int* seg_off,
                       int64_t B, int64_t L, int64_t H, int causal, float p_drop, uint64_t seed, float* qkv,
                       float* out, float* lse, void* stream);

/* ---- A6 / A7 / A12: fused in-batch contrastive cross-entropy ------------------------
 * S_ij = <A_i,B_j>/tau - bias_j over an implicit N x M matrix (never materialised),
 * fp32-input MFMA, online log-sum-exp. Row i's label column is i + diag_offset (0 on one
 * GPU; the shard offset when A holds one rank's rows and B the all-gathered columns).
 * flags (supported combinations):
 *   0                 plain InfoNCE, label = diagonal  (duorec unsup v1_refine_usertower.py:588-590,
 *                                                       item_tower.py:1075-1082 per direction)
 *   2 (MASK_K1)       + exclude off-diagonal j with k1_j == k1_i   (shadowed logq loss :520-573)
 *   6 (MASK_K1|K2)    + also k2 (user) keys               (live inbatch_corrected_logq_loss :826-861)
 *   9 (EXCL_DIAG|POS) SupCon term of duorec_loss_refined (:595-625): diagonal excluded,
 *                     positives k1_i == k1_j != 0, loss_i = LSE_i - mean positive logit
 * Keys are int32. D = 128 (row strides lda/ldb >= 128, multiple of 4, 16-B aligned).
 * ws: rsx_nce_workspace_floats(N, M, nsplit_fwd, nsplit_bwd) floats, shared by fwd and bwd.
 * out2 (device, 2 floats) = {sum of row losses over valid rows, number of valid rows};
 * the reference's mean is out2[0] / out2[1] (0 when no row is valid). */
int64_t rsx_nce_workspace_floats(int64_t N, int64_t M, int nsplit_fwd, int nsplit_bwd);
int rsx_nce_fwd(const float* A, const float* B, const float* bias, const int* k1a, const int* k1b, const int* k2a,
                const int* k2b, int64_t N, int64_t M, int64_t lda, int64_t ldb, int64_t diag_offset, float tau,
                int flags, int nsplit, float* ws, float* out2, void* stream);
/* gout = device scalar: gradient of the objective w.r.t. the row-loss SUM out2[0].
 * dA [N,128] / dB [M,128] (nullable; NULL skips that pass) written, or added into when
 * accumulate != 0. Must follow rsx_nce_fwd on the same ws. */
int rsx_nce_bwd(const float* A, const float* B, const float* bias, const int* k1a, const int* k1b, const int* k2a,
                const int* k2b, int64_t N, int64_t M, int64_t lda, int64_t ldb, int64_t diag_offset, float tau,
                int flags, int nsplit_fwd, int nsplit, const float* gout, float* ws, float* dA, float* dB,
                int accumulate, void* stream);

/* bf16x3 form of the two calls above (same flags, objective and outputs; products as
 * hi*hi + hi*lo + lo*hi on the bf16 MFMA, see RSX_NCE_BF16X3 below). The split counts are
 * chosen by the library (enough workgroups for the chip at any N, M); the workspace is
 * rsx_nce_x3_workspace_floats(N, M) floats and carries the hi/lo images between the calls. */
int64_t rsx_nce_x3_workspace_floats(int64_t N, int64_t M);
int rsx_nce_fwd_x3(const float* A, const float* B, const float* bias, const int* k1a, const int* k1b,
                   const int* k2a, const int* k2b, int64_t N, int64_t M, int64_t lda, int64_t ldb,
                   int64_t diag_offset, float tau, int flags, float* ws, float* out2, void* stream);
int rsx_nce_bwd_x3(const float* A, const float* B, const float* bias, const int* k1a, const int* k1b,
                   const int* k2a, const int* k2b, int64_t N, int64_t M, int64_t lda, int64_t ldb,
                   int64_t diag_offset, float tau, int flags, const float* gout, float* ws, float* dA, float* dB,
                   int accumulate, void* stream);

/* Hard-emphasis term of full_batch_hard_emphasis_loss (replaces the reference's dense emphasis tensor,
 * scatter_ and masked cross-entropy over N x N logits, tower_code/v1_refine_usertower.py:762-822): row i's
 * K mined columns top[i*K + r] (int64, from rsx_hnm_mine) get +margin (already divided by tau) on top of
 * the flags-2 objective (k1 = target ids: same-item columns off the label excluded; bias = lambda*logQ).
 * Call rsx_nce_emphasis_fwd after rsx_nce_fwd / rsx_nce_fwd_x3 on the same ws (precision RSX_NCE_FP32 with
 * that call's nsplit_fwd, or RSX_NCE_BF16X3): each row's log-sum-exp and loss are corrected in ws from the
 * K mined logits alone and out2 is recomputed. Then rsx_nce_bwd(_x3) gives the dense gradient and
 * rsx_nce_emphasis_bwd adds the mined entries' extra (e^margin - 1) softmax weight into dA [N,128] / dB [M,128]
 * (nullable; dB by vector atomics: the summation order of a column shared by several rows is not fixed).
 * Mined ids outside [0, M) are skipped. O(N K) work and memory. */
int rsx_nce_emphasis_fwd(const float* A, const float* B, const float* bias, const int* k1a, const int* k1b,
                         const int64_t* top, int64_t N, int64_t M, int64_t K, int64_t lda, int64_t ldb,
                         int64_t diag_offset, float tau, float margin, int precision, int nsplit_fwd, float* ws,
                         float* out2, void* stream);
int rsx_nce_emphasis_bwd(const float* A, const float* B, const float* bias, const int* k1a, const int* k1b,
                         const int64_t* top, int64_t N, int64_t M, int64_t K, int64_t lda, int64_t ldb,
                         int64_t diag_offset, float tau, float margin, int precision, int nsplit_fwd,
                         const float* gout, float* ws, float* dA, float* dB, void* stream);
/* The same without float atomics: the mined entries' weights go to cbuf [N*K] (floats) and one wave per
 * column j adds them into dB from the column-sorted CSR of top (col_ptr [M+1] offsets, col_ent the entry
 * ids i*K + r in column order; ids outside [0, M) left out) -- deterministic for a fixed entry order. */
int rsx_nce_emphasis_bwd_csr(const float* A, const float* B, const float* bias, const int* k1a, const int* k1b,
                             const int64_t* top, int64_t N, int64_t M, int64_t K, int64_t lda, int64_t ldb,
                             int64_t diag_offset, float tau, float margin, int precision, int nsplit_fwd,
                             const int64_t* col_ptr, const int64_t* col_ent, float* cbuf, const float* gout,
                             float* ws, float* dA, float* dB, void* stream);

/* ---- A6 grouped: the live LogQ loss over the batch's DISTINCT targets ------------------
 * Same objective as rsx_nce_fwd flags 6 on columns normalize(item_matrix)[t_j], evaluated
 * over the D distinct targets (B[d] = normalised item uniq[d], bias[d] = logQ*lambda) with
 * exact integer multiplicities w_{i,d} = 1 if d == d(i) else c_d - n_{user(i),d}:
 *   colcnt [D] float  c_d = number of columns with target d
 *   row_col [N] int   d(i), the row's own target column
 *   row_beg/row_end [N] int  range of the row's user's targets in exc_cols (sorted d's)
 *   col_beg/col_end [D] int  range into exc_s/exc_e/exc_n: the user row ranges [s,e) that
 *                            hold target d and their multiplicity n (backward, dB pass only)
 * Rows of one user must be contiguous (flat (b, t) order). FLOPs: N*D instead of N*N.
 * precision: RSX_NCE_FP32 (0) = logits on the fp32-input MFMA (exact fp32 products);
 *            RSX_NCE_BF16X3 (1) = logits as hi*hi + hi*lo + lo*hi of a bf16 hi/lo split
 *            (fp32 accumulate, max |dot error| ~3e-6 on unit vectors), 5.3x fewer MFMA cycles;
 *            the gradient products (dS x rows) use the same split;
 *            RSX_NCE_F16 (2) = in the fused forward and the column pass: logits as the same three
 *            products of an fp16 hi/lo split of x * 2^8 on the fp16 MFMA (~2^-22 relative per term,
 *            tighter than bf16x3), gradient products as ONE fp16 MFMA of the rounded softmax weights
 *            and the rows' fp16 hi image (the reference's autocast(float16) arithmetic for these
 *            products, v1_usertower_train.py:787, with fp32 accumulation; RSX_NCE_F16_GP=2 adds the
 *            lo image); in the column pass the logits take two of the three products (the streamed rows'
 *            lo image dropped: ~2e-5 on unit vectors; RSX_NCE_F16_COLS_S=3 keeps three); elsewhere
 *            (rsx_nce_grouped_fwd, the row pass) as RSX_NCE_BF16X3. */
#define RSX_NCE_FP32 0
#define RSX_NCE_BF16X3 1
#define RSX_NCE_F16 2
/* ws for the grouped pair: >= rsx_nce_grouped_workspace_floats(N, D, nsplit_fwd, 8, precision)
 * (bf16x3 adds the hi/lo bf16 images of A and B; the forward writes B's, the backward's
 * column pass A's). The grouped backward's nsplit is 8. */
int64_t rsx_nce_grouped_workspace_floats(int64_t N, int64_t D, int nsplit_fwd, int nsplit_bwd, int precision);
int rsx_nce_grouped_fwd(const float* A, const float* B, const float* bias, const float* colcnt, const int* row_col,
                        const int* row_beg, const int* row_end, const int* exc_cols, int64_t N, int64_t D,
                        int64_t lda, int64_t ldb, float tau, int precision, int nsplit, float* ws, float* out2,
                        void* stream);
/* Forward fused with the row-side gradient (precision RSX_NCE_BF16X3 or RSX_NCE_F16): same loss as rsx_nce_grouped_fwd
 * (out2, and lse in ws for a later column pass), plus ga [N][128] = d(sum of row losses)/dA
 * per unit upstream gradient, i.e. dA = gout * ga. The row gradient is a softmax-weighted sum
 * of B's rows (an attention output), accumulated in the same sweep over S as the loss, so the
 * backward runs only the column pass (rsx_nce_grouped_bwd with dA = NULL). nsplit in
 * {1, 2, 4, 8}. Replaces the forward of the reference's live loss
 * (tower_code/v1_usertower_train.py:787-845) plus the row half of its autograd backward. */
int rsx_nce_grouped_fwd_grad(const float* A, const float* B, const float* bias, const float* colcnt,
                             const int* row_col, const int* row_beg, const int* row_end, const int* exc_cols,
                             int64_t N, int64_t D, int64_t lda, int64_t ldb, float tau, int precision, int nsplit,
                             float* ws, float* out2, float* ga, void* stream);
/* Measurement hooks (no reference counterpart; bench.py's roofline): while enabled,
 * rsx_nce_grouped_fwd_grad brackets the fused forward kernel's own launch (not the B split or the
 * merge) with two HIP events on its stream; rsx_kernel_events_read waits for them and writes up to
 * max_n durations (ms, launch order), returning how many were recorded (-1 on a HIP error).
 * Enabling clears the list. */
int rsx_kernel_events(int on);
int rsx_kernel_events_read(float* ms, int max_n);
/* The same for the embedding gather (rsx_seq_embed_fwd's kernel, whichever caller issues it: the per-op
 * path or rsx_tower_fwd): rsx_gather_events(1) clears and starts recording; _read waits and writes up to
 * max_n launch times (ms) with each launch's token count. */
int rsx_gather_events(int on);
int rsx_gather_events_read(float* ms, int64_t* tokens, int max_n);
int rsx_nce_grouped_bwd(const float* A, const float* B, const float* bias, const float* colcnt, const int* row_col,
                        const int* row_beg, const int* row_end, const int* exc_cols, const int* col_beg,
                        const int* col_end, const int* exc_s, const int* exc_e, const int* exc_n, int64_t N,
                        int64_t D, int64_t lda, int64_t ldb, float tau, int precision, int nsplit_fwd,
                        int nsplit, const float* gout, float* ws, float* dA, float* dB, int accumulate,
                        void* stream);

/* ---- static-profile embeddings: gated lookups of several tiny tables, concatenated ------
 * out[b, off_j + c] = E_j[ids_j[b]][c] * gate[j]. The backward's dout has B rows, row b from
 * user b % ids_rows (ids hold ids_rows entries: the contrastive step's two dropout views share
 * their users), and gives dE_j (padding_idx rows: 0 when written, untouched when added) and
 * dgate[j], added into (accumulate = 1) or written (0); per-64-row workgroup partials in ws
 * (rsx_static_embed_bwd_workspace_floats) reduced in a fixed order, so the gradients are
 * identical run to run. Replaces the nine nn.Embedding lookups x u_g of
 * tower_code/v1_refine_usertower.py:472-494 (and their sort-based embedding backward).
 * <= 16 tables, <= 256 columns, <= 4096 table floats in total. */
int rsx_static_embed_fwd(const int64_t* const* ids, const float* const* tables, const int64_t* table_rows,
                         const int64_t* dims, int ntab, const float* gate, int64_t B, float* out, int64_t ld_out,
                         void* stream);
int64_t rsx_static_embed_bwd_workspace_floats(int64_t B, int ntab, const int64_t* table_rows, const int64_t* dims);
int rsx_static_embed_bwd(const int64_t* const* ids, const float* const* tables, const int64_t* table_rows,
                         const int64_t* dims, const int64_t* padding_idx, int ntab, const float* gate,
                         const float* dout, int64_t ld_dout, int64_t B, int64_t ids_rows, float* const* dtables,
                         float* dgate, int accumulate, float* ws, int64_t ws_floats, void* stream);

/* ---- LayerNorm fused with the preceding residual add + dropout and a following GELU ----
 * s = x + dropout(res) (res nullable), y = act(LN(s) * w + b), act 0 none / 2 GELU(erf).
 * Replaces norm1/norm2 and the residual adds of the norm_first TransformerEncoderLayer and the
 * output head LayerNorm+GELU (tower_code/v1_refine_usertower.py:40-50, 68-72, 447-510).
 * sum_out (nullable) receives s when res is given; mean/rstd [T] are saved for the backward.
 * Backward: ds_out = LN-backward(dy) + ds_in (ds_in nullable), dres = dropout-backward(ds_out),
 * dw/db via per-block partials (ws >= rsx_ln_bwd_workspace_floats). D in {64, 128, 256}; the
 * forward also takes D in {512, 768, 1024} (the item tower's BERT LayerNorms, item_tower.py:175,
 * inference: rsx_ln_bwd stays at D <= 256). rsx_ln_bwd_workspace_floats returns -1 for a D that
 * rsx_ln_bwd does not accept. */
int rsx_ln_fwd(const float* x, const float* res, float p_drop, uint64_t seed, const float* w, const float* b,
               float eps, int act, int64_t T, int64_t D, float* sum_out, float* y, float* mean, float* rstd,
               void* stream);
/* Backward of the add-only form of rsx_ln_fwd (y = NULL: s = x + dropout_p(res), as after the
 * encoder's last layer, v1_refine_usertower.py:343-352): dres = the forward's keep-mask / (1 - p)
 * applied to ds (flat index row*D + col); dx is ds itself. */
int rsx_dropout_bwd(const float* ds, int64_t T, int64_t D, float p_drop, uint64_t seed, float* dres, void* stream);
int64_t rsx_ln_bwd_workspace_floats(int64_t T, int64_t D);
int rsx_ln_bwd(const float* s, const float* mean, const float* rstd, const float* w, const float* b, int act,
               const float* dy, const float* ds_in, float p_drop, uint64_t seed, int64_t T, int64_t D, float* ds_out,
               float* dres, float* dw, float* db, float* ws, int64_t ws_floats, void* stream);

/* ---- weight gradient of token-level linear layers ---------------------------------------
 * dW[n][k] (+)= sum_t dY[t][n] X[t][k], db[n] (+)= sum_t dY[t][n] (db nullable), fp32 MFMA,
 * split over tokens with a deterministic partial reduction. Replaces autograd's weight-grad
 * GEMM of every per-token nn.Linear in the user tower's step (tower_code/v1_refine_usertower.py
 * :447-510 — item_proj, in_proj/out_proj/linear1/linear2 of both encoder layers, output_proj).
 * N, K multiples of 16; ws >= rsx_linear_wgrad_workspace_floats(T, N, K) floats. */
int64_t rsx_linear_wgrad_workspace_floats(int64_t T, int64_t N, int64_t K);
int rsx_linear_wgrad(const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t T, int64_t N, int64_t K,
                     float* dW, int64_t ldw, float* db, int accumulate, float* ws, int64_t ws_floats, void* stream);
/* Same contract in bf16x3 split precision (hi*hi + hi*lo + lo*hi on the bf16 MFMA, fp32
 * accumulate; db summed in fp32): the default of the training step. */
int rsx_linear_wgrad_x3(const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t T, int64_t N,
                        int64_t K, float* dW, int64_t ldw, float* db, int accumulate, float* ws, int64_t ws_floats,
                        void* stream);

/* ---- forward / input-gradient GEMMs of the token-level linear layers (bf16x3) ------------
 * C[M, N] = epi(A[M, K] . B[N, K]^T + bias): the forward Y = X W^T + b (B = W) and the input
 * gradient dX = dY W (B = W^T) of the same per-token nn.Linear layers as rsx_linear_wgrad,
 * replacing autograd's library GEMMs. epi: 0 bias; 1 z = acc + bias, C = dropout_p(gelu_erf(z))
 * (keep-mask hash(seed, m*N + n)), aux = gelu_erf'(z) (aux may be NULL: inference, e.g. the
 * item tower's BERT intermediate layer, item_tower.py:175); 2 C = acc * keep / (1-p) * aux, its
 * backward (same seed, aux from epi 1). Epilogues 1/2 fuse nn.TransformerEncoderLayer's feed-forward
 * dropout(gelu(linear1(x))) (v1_refine_usertower.py:343-352) into its GEMMs.
 * N % 128 == 0, K % 32 == 0, A/B 16-byte aligned, leading dimensions multiples of 4. */
int rsx_gemm_x3(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int64_t M, int N, int K,
                int epi, float* aux, int64_t ldaux, float p_drop, uint64_t seed, float* C, int64_t ldc, void* stream);
/* The same with a caller workspace for split-K: when the output has fewer 128 x 128 tiles than the device
 * has CUs and K is long (K not 128 / 256 / 384), S K-ranges per tile run as separate workgroups writing
 * partial sums to ws, and one pass adds them in split order and applies epi. ws_floats >=
 * rsx_gemm_x3_split_floats(M, N, K) (0 = no split for this shape; ws may then be null). Deterministic; the
 * summation order over K differs from rsx_gemm_x3's (fp32 rounding level). */
int64_t rsx_gemm_x3_split_floats(int64_t M, int N, int K);
int rsx_gemm_x3_ws(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int64_t M, int N,
                   int K, int epi, float* aux, int64_t ldaux, float p_drop, uint64_t seed, float* C, int64_t ldc,
                   float* ws, int64_t ws_floats, void* stream);
/* C = epi(A . Bt + bias) with Bt [K, N] as stored (row stride ldbt >= N): the input gradient
 * dX = dY . W of the same token linears straight from W [out, in] (K = out, N = in; autograd's
 * dX GEMM of nn.Linear, v1_refine_usertower.py:447-510), no transposed copy of W; epi / aux /
 * p_drop / seed as rsx_gemm_x3 (EPI_DGELU_DROP: the feed-forward's backward through GELU and
 * dropout). K in {128, 256, 384}, N % 128 == 0, A/C 16-byte aligned. */
int rsx_gemm_x3_tn(const float* A, int64_t lda, const float* Bt, int64_t ldbt, const float* bias, int64_t M, int N,
                   int K, int epi, float* aux, int64_t ldaux, float p_drop, uint64_t seed, float* C, int64_t ldc,
                   void* stream);
/* C[m] = A[m] . B^T + bias + R[ridx[m]]: a per-row table added in the epilogue. Replaces
 * output_proj[0](cat(enc_out, profile.expand)) of SASRecUserTower.forward
 * (v1_refine_usertower.py:498-505) over the packed tokens: A = encoder output, B = the token
 * half of output_proj[0].weight (ldb = 256), R = profile half + bias per user, ridx = user of
 * each token. K 128 or 256, N % 128 == 0, every pointer 16-byte aligned. */
int rsx_gemm_x3_rowadd(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int64_t M, int N,
                       int K, const float* R, int64_t ldr, const int64_t* ridx, float* C, int64_t ldc, void* stream);
/* S = X + dropout_p(A . B^T + bias); Y = LayerNorm(S) * ln_w + ln_b; mean / rstd per row.
 * Replaces a norm_first encoder layer's `x = x + dropout(out_proj(attn)); norm2(x)`
 * (v1_refine_usertower.py:343-352, nn.TransformerEncoderLayer._sa_block + norm2) in one
 * weight-stationary GEMM: the add and the LayerNorm run in its epilogue. N = 128, K 128 or 256,
 * every pointer 16-byte aligned; dropout mask = rsx_ln_fwd's (hash(seed, m * N + n)), so
 * rsx_ln_bwd (ds_in, dres) is its backward. ln_w / ln_b nullable (1 / 0). */
int rsx_gemm_x3_addln(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int64_t M, int N,
                      int K, const float* X, int64_t ldx, float p_drop, uint64_t seed, const float* ln_w,
                      const float* ln_b, float eps, float* S, int64_t lds, float* Y, int64_t ldy, float* mean,
                      float* rstd, void* stream);

/* Device-side id range check (no host sync): out[i] = ids[i] if lo <= ids[i] < hi else 0, and
 * *flag = 1 if any id was outside [lo, hi) (untouched otherwise). Replaces the out-of-range
 * failure of nn.Embedding on the item tower's STD ids (item_tower.py:240, vocab ids 0..383,
 * utils/vocab.py:436-441): the caller raises when the flag reaches the host. */
int rsx_ids_check(const int64_t* ids, int64_t n, int64_t lo, int64_t hi, int64_t* out, int* flag, void* stream);

/* ---- A8: the step index on the device ----------------------------------------------------
 * Every data-dependent structure of one contrastive step (train_user_tower_all_time's per-batch
 * flattening, v1_usertower_train.py:794-835, plus the grouped loss's target index) from the
 * batch's [B, L] tensors, with ONE host read (the totals). pm: padding_mask as bytes (1 = pad),
 * tgt / item: target_ids / item_ids int64 [B, L], ids in [0, n_items); L <= 64.
 *   1. rsx_step_index_count   -> tloc [B*L + 1] int32: this rank's loss-row targets (flat
 *      order, -1 padded) and its row count in the last slot
 *   2. (world > 1) the caller all-gathers tloc blocks rank-major into tglob [world][B*L + 1]
 *   3. rsx_step_index_totals  -> totals [8 + world] int64 on the device: T (packed tokens per
 *      view), N (loss rows), D (distinct target columns over tglob), E (distinct (user, target)
 *      pairs), U (distinct item ids among the tokens), C (segment-sum chunks), error flag (ids
 *      out of range), 0, then every rank's row count
 *   4. rsx_step_index_fill(sizes = totals[0..5] read on the host) writes out[0..32]:
 *      0 flat [T] i64, 1 tok_user [T] i64, 2 tok_pos [T] i64, 3 tok_pad [T] u8, 4 seg_off [B+1] i32,
 *      5 seg_off [B+1] i64, 6 valid_tok [N] i64, 7 last_tok [B] i64; the doubled two-view batch:
 *      8 flat [2T], 9 tok_user [2T], 10 tok_pos [2T] i64, 11 tok_pad [2T] u8, 12 seg_off [2B+1]
 *      i32, 13 seg_off [2B+1] i64, 14 tok_ids [6][2T] i64 (seq_ids per token, both views),
 *      15 pretrained rows [2T][128] f32 (nullable; from lookup [n_items][ld_lookup]); the
 *      item-id segment-sum plan: 16 perm [2T], 17 cb [C+1], 18 chunk ids [C], 19 ch_off [U+1],
 *      20 ids [U] (all i64); the grouped-loss index: 21 uniq [D] i64, 22 colcnt [D] f32,
 *      23 row_col, 24 row_beg, 25 row_end, 26 exc_cols [N] i32, 27 exc_s, 28 exc_e, 29 exc_n [E]
 *      i32, 30 col_beg, 31 col_end [D] i32; 32 last_t [B] i32 (the SupCon keys: last targets).
 * ws: rsx_step_index_workspace_bytes(B, L, n_items), the same buffer for all three calls. */
int64_t rsx_step_index_workspace_bytes(int64_t B, int64_t L, int64_t n_items);
int rsx_step_index_count(const uint8_t* pm, const int64_t* tgt, const int64_t* item, int64_t B, int64_t L,
                         int64_t n_items, void* ws, int64_t ws_bytes, int* tloc, void* stream);
int rsx_step_index_totals(const int* tglob, int world, int64_t B, int64_t L, int64_t n_items, void* ws,
                          int64_t ws_bytes, int64_t* totals, void* stream);
int rsx_step_index_fill(const uint8_t* pm, const int64_t* tgt, const int64_t* const* seq_ids, const float* lookup,
                        int64_t ld_lookup, int64_t B, int64_t L, int64_t n_items, const int64_t* sizes, void* ws,
                        int64_t ws_bytes, void* const* out, void* stream);

/* ---- A14: retrieval top-k ------------------------------------------------------------
 * scores = U I^T (fp32 MFMA, never materialised), per query the k best items sorted by
 * (score desc, index asc). Replaces `scores = matmul(user, items.T); topk(k)` at
 * tower_code/v1_usertower_train.py:672-675 and temp_model/ranker_skelet.py:193-196.
 * U [Q, ldu], I [NI, ldi], D = 128, 1 <= k <= 512. ws: rsx_topk_workspace_bytes(Q, NI, k).
 * out_idx = -1 where fewer than k items exist. */
int64_t rsx_topk_workspace_bytes(int64_t Q, int64_t NI, int64_t k);
int rsx_retrieve_topk(const float* U, int64_t ldu, const float* I, int64_t ldi, int64_t Q, int64_t NI, int64_t k,
                      void* ws, float* out_scores, int64_t* out_idx, void* stream);
/* Which exact path a (Q, NI, k) call takes: 0 list kernels, 1 fp32 candidate/threshold path,
 * 2 bf16 single scan + exact fp32 rescoring (large corpora). Every call writes a workspace
 * header: int32 ws[0] = queries path 2 sent to the exact kernels, ws[1] = path id, ws[2] = path
 * 1's whole-batch fallback flag. Path 2 runs the queries in chunks of at most 4096 (workspace
 * bounded in Q). */
int rsx_topk_path(int64_t Q, int64_t NI, int64_t k);
/* Path 2 with a caller-cached corpus image (a static corpus, e.g. the serving item matrix of
 * controller.py:62-124 or evaluate_model's normalised item table, :672): rsx_topk_prepare_corpus
 * writes max ||w||, max ||w - bf16(w)|| and the bf16 image of I into `corpus` (rsx_topk_corpus_bytes(NI) bytes) once;
 * rsx_retrieve_topk_corpus then skips that pass (ws: rsx_topk_workspace_bytes_corpus). I must
 * be the corpus the image was made from (the exact rescoring reads it). */
int64_t rsx_topk_corpus_bytes(int64_t NI);
int rsx_topk_prepare_corpus(const float* I, int64_t ldi, int64_t NI, void* corpus, void* stream);
int64_t rsx_topk_workspace_bytes_corpus(int64_t Q, int64_t NI, int64_t k);
int rsx_retrieve_topk_corpus(const float* U, int64_t ldu, const float* I, int64_t ldi, const void* corpus, int64_t Q,
                             int64_t NI, int64_t k, void* ws, float* out_scores, int64_t* out_idx, void* stream);

/* ---- A16: DeepFM rerank forward ------------------------------------------------------
 * deepctr-torch 0.2.9 DeepFM semantics (absent from the reference tree).
 * rsx_deepfm_embed: x [R, F] int64 per-field ids, V[f] [vocab_f, 16], W[f] [vocab_f] (nullable)
 *   -> emb_out [R, F*16] (concatenated DNN input, nullable) and
 *      lin_out[r] = bias + sum_f W[f][x] + 0.5 * sum_k((sum_f v)^2 - sum_f v^2).
 * rsx_linear_fwd: Y [M, N] = act(X W^T + b), W [N, K] torch Linear layout, N <= 256,
 *   K % 4 == 0, act 0 none / 1 relu / 2 gelu (erf). fp32 MFMA.
 * rsx_linear_dot_fwd: logit[m] = sum_n act(X W^T + b)[m, n] * wo[n] + add[m];
 *   prob = sigmoid(logit) (nullable). */
int rsx_deepfm_embed(const int64_t* x, int64_t R, int F, int E, const float* const* V, const float* const* W,
                     float bias, float* emb_out, float* lin_out, void* stream);
int rsx_linear_fwd(const float* X, int64_t ldx, const float* W, const float* b, int64_t M, int64_t N, int64_t K,
                   int act, float* Y, void* stream);
int rsx_linear_dot_fwd(const float* X, int64_t ldx, const float* W, const float* b, int64_t M, int64_t N, int64_t K,
                       int act, const float* wo, const float* add, float* logit, float* prob, void* stream);

/* rsx_deepfm_fused: the whole forward in one kernel (gather + first-order + FM + the
 *   (256, 128) ReLU DNN on bf16x3 MFMA + final dot + sigmoid); the [R, F*16] DNN input never
 *   reaches HBM. Same arguments as the three calls above with w1 [256, F*16], b1 [256],
 *   w2 [128, 256], b2 [128], wo [128] (torch Linear layouts; dnn_hidden_units = (256, 128),
 *   embed_dim 16). ws: rsx_deepfm_fused_workspace_bytes(F) (per-call bf16 weight images).
 *   Replaces the same deepctr-torch DeepFM forward. */
int64_t rsx_deepfm_fused_workspace_bytes(int F);
int rsx_deepfm_fused(const int64_t* x, int64_t R, int F, const float* const* V, const float* const* W, float bias,
                     const float* w1, const float* b1, const float* w2, const float* b2, const float* wo, void* ws,
                     float* logit, float* prob, void* stream);
/* The two halves of rsx_deepfm_fused, for callers that keep ws across calls (the weight images
 * are a function of w1/w2 only: rebuild them with rsx_deepfm_fused_prep after an update).
 * F in [25, 48] runs the persistent kernel (one workgroup per CU looping over 64-row blocks). */
int rsx_deepfm_fused_prep(int F, const float* w1, const float* w2, void* ws, void* stream);
/* packed: nullable per-field tables from rsx_deepfm_pack, read instead of V/W when
 * rsx_deepfm_fused_uses_packed(F) == 1 (F = 39: deepfm_rows2m_k, 256-row workgroups of eight 32-row
 * waves, 130 KiB of LDS; other F in [25, 48]: the persistent kernel): a field's V row and first-order
 * weight then share one 128-B line, halving the lines fetched per (row, field) on random ids. NULL:
 * V/W are read directly (F = 39: deepfm_rows5_k). */
int rsx_deepfm_fused_run(const int64_t* x, int64_t R, int F, const float* const* V, const float* const* W,
                         const float* const* packed, float bias, const float* b1, const float* b2, const float* wo,
                         const void* ws, float* logit, float* prob, void* stream);
/* packed [vocab][32] = (V [vocab][16] row, W [vocab] (0 if NULL), 15 zeros): one field's table. */
int rsx_deepfm_pack(const float* V, const float* W, int64_t vocab, float* packed, void* stream);
int rsx_deepfm_fused_uses_packed(int F);

/* ---- §8f #3: GDCN reranker batch (utils/data_preprocessing/feature_processor.py:144-195) ----
 * rsx_reranker_batch replaces RerankerDataset.__getitem__ (:156-181) + reranker_collate_fn
 * (:184-191) for a batch of (user row uidx[b], item row iidx[b]) on device tables:
 *   dense [B, 12] = user_scaled[u] (3) | item_scaled[i] (6) | price gap, trend 1w, trend 1m
 *     (cross features in float64 from u_raw [U, 2] = (user_avg_price_log, total_cnt_log) and
 *     i_raw [I, 3] = (avg_item_price_log, velocity_1w, velocity_1m), rounded to fp32 once);
 *   cat [B] = u_cat[u]; target [B] = i_num[i];
 *   seq/mask [B, L]: the last min(len, max_len) ids of the user's CSR sequence (seq_off [U+1],
 *     seq_ids), right-padded with 0; mask = seq != 0. L = the batch maximum of min(len, max_len)
 *     (rsx_reranker_seq_lens gives the per-row lengths). */
int rsx_reranker_seq_lens(const int64_t* uidx, const int64_t* seq_off, int64_t B, int max_len, int64_t* lens,
                          void* stream);
int rsx_reranker_batch(const int64_t* uidx, const int64_t* iidx, int64_t B, const float* u_scaled, const double* u_raw,
                       const int64_t* u_cat, const float* i_scaled, const double* i_raw, const int64_t* i_num,
                       const int64_t* seq_off, const int64_t* seq_ids, int max_len, int64_t L, float* dense,
                       int64_t* cat, int64_t* target, int64_t* seq, int64_t* mask, void* stream);

/* ---- A9: item-tower RE path ------------------------------------------------------------
 * out[t] = LayerNorm((word[ids[t]] + type_row) + pos[tok_pos[t]]) * ln_w + ln_b over packed
 * tokens: BertEmbeddings (word + token type 0 + absolute position, LayerNorm, eval) for the
 * valid tokens of the RE fields only (HybridItemTower.forward, item_tower.py:247-262; their
 * masked mean ignores the padded ones). D in {256, 512, 768, 1024}. */
int rsx_embed3_ln(const float* word, int64_t ld_word, const float* pos, const float* type_row, const float* ln_w,
                  const float* ln_b, float eps, const int64_t* ids, const int64_t* tok_pos, int64_t T, int64_t D,
                  float* out, void* stream);

/* ---- DCN-V2 reranker ------------------------------------------------
 * CrossNet (temp_model/ranker_skelet.py:239-272): x_{l+1} = x_0 * (x_l . k_l + b_l) + x_l for L
 * layers (k_l [D], b_l [D]); writes x_L (x_out, nullable) and/or head_part[b] = x_L . w_head
 * (the cross half of RankingModel.final_head, :313-338). D % 4 == 0, D <= 512, L <= 8. */
int rsx_crossnet(const float* x, int64_t ldx, int64_t B, int D, int L, const float* const* kernels,
                 const float* const* biases, const float* w_head, float* x_out, float* head_part, void* stream);

/* ---- row gather / scatter / L2 normalise ---------------------------------------------
 * out[r] = src[idx[r]] (idx NULL => r), optionally F.normalize'd (eps) with norms saved:
 *   pretrained_lookup[item_ids]            tower_code/v1_usertower_train.py:760
 *   normalize(item_matrix)[target_ids]     v1_usertower_train.py:810-811 + v1_refine_usertower.py:833
 *   F.normalize(x, p=2, dim=-1)            v1_refine_usertower.py:504,584-585; v1_usertower_train.py:807
 * D in {64,128,256}. */
int rsx_gather_rows(const float* src, int64_t ld_src, const int64_t* idx, int64_t n, int64_t D, int normalize,
                    float eps, float* out, float* nrm_out, void* stream);
/* Backward scatter: dst[idx[r]] (op)= g_r where g = dy (or the F.normalize backward of dy
 * given y and norms). mode 0 store, 1 add (unique idx), 2 atomic add (duplicates allowed).
 * Rows whose index equals skip_idx are dropped (nn.Embedding padding_idx), -1 = none. */
int rsx_scatter_rows(const float* dy, const float* y, const float* nrm, const int64_t* idx, int64_t n, int64_t D,
                     int normalize, float eps, int mode, int64_t skip_idx, float* dst, int64_t ld_dst, void* stream);
/* Segmented row sums, the atomic-free scatter-add when the sort by destination is known:
 * dst[rows[u]] (+)= scale[0] * sum_{k in [seg_off[u], seg_off[u+1])} src[perm[k]] (scale
 * nullable = 1; perm nullable = identity; rows nullable = u; rows[u] == skip_row untouched;
 * rows unique). Used for the user tower's item-id embedding gradient
 * (v1_refine_usertower.py:447-459, nn.Embedding backward) with the sort built ahead of the
 * step, and for the per-user profile gradient (the broadcast of :498-505 over each user's
 * contiguous packed tokens); deterministic. */
int rsx_segment_sum_rows(const float* src, int64_t ld_src, const int64_t* perm, const int64_t* seg_off,
                         const int64_t* rows, int64_t nseg, int64_t D, const float* scale, int64_t skip_row,
                         float* dst, int64_t ld_dst, int accumulate, void* stream);

/* The contrastive step's objective from its device loss sums, one launch instead of the
 * scalar tensor ops of train_user_tower_all_time (tower_code/v1_usertower_train.py:814-845):
 * main = s_main * inv_n (s_main nullable: 0), cl = s_un * inv_b + lambda_sup * s_sup / max(cnt, 1)
 * (s_sup nullable), total = main + lambda_cl * cl; total[1] and logs[3] = {total, main, cl} (separate
 * storage: a detached copy for logging / all-reduce). Backward: g3[3] = gradients of g * total w.r.t. s_main, s_un,
 * s_sup (cnt nullable when s_sup was). All device scalars. */
int rsx_loss_combine(const float* s_main, const float* s_un, const float* s_sup, const float* cnt, float inv_n,
                     float inv_b, float lambda_sup, float lambda_cl, float* total, float* logs, void* stream);
int rsx_loss_combine_bwd(const float* g, const float* cnt, float inv_n, float inv_b, float lambda_sup,
                         float lambda_cl, float* g3, void* stream);

/* The user tower's static profile (v1_refine_usertower.py:472-494) as one call per direction:
 *   u_g = sigmoid(static_gate); x = cat(E_j[id_j] * u_g[j] (j < ntab), relu(cont @ Wc^T + bc) * u_g[ntab]);
 *   out = dropout_p(gelu_erf(LayerNorm(x @ Wm^T + bm)))     [U, 128]
 * p[] pointer table (RSX_SP_*; table slots beyond ntab unused): ids int64 [U] and tables
 * [rows_j, dim_j] per table, static_gate [ntab + 1] (raw parameter), cont [U, C], Wc [P, C],
 * bc [P], Wm [128, K], bm [128], ln_w / ln_b [128]. dims[] = {U, ntab, C, P, K, src, rows[ntab],
 * dim[ntab], padding_idx[ntab]} with sum(dim) + P == K <= 128, C == 4, P == 16; the ids and cont
 * hold src rows and output row r reads input row r % src (U % src == 0: the contrastive step's two
 * dropout views share their users' inputs, so they are not duplicated). arena:
 * rsx_static_profile_arena_bytes(U), written by the forward and read by the backward; its first
 * int32 is an error flag the forward sets when an id lies outside [0, rows_j) (nn.Embedding's
 * IndexError: such an id reads row 0 and the backward scatters to row 0, never out of bounds; the
 * caller raises on the flag, ops.py _StaticProfile).
 * Backward: grads[] parallel to p[] (the ids' and cont's slots unused), every gradient WRITTEN
 * (padding rows 0); U > 0; ws: rsx_static_profile_bwd_workspace_bytes(U). Dropout mask
 * hash(seed, row * 128 + col). */
enum {
  RSX_SP_IDS = 0, RSX_SP_TABLES = 16, RSX_SP_GATE = 32, RSX_SP_CONT = 33, RSX_SP_WC = 34, RSX_SP_BC = 35,
  RSX_SP_WM = 36, RSX_SP_BM = 37, RSX_SP_LNW = 38, RSX_SP_LNB = 39, RSX_SP_N = 40
};
int64_t rsx_static_profile_arena_bytes(int64_t U);
int64_t rsx_static_profile_bwd_workspace_bytes(int64_t U);
int rsx_static_profile_fwd(const void* const* p, const int64_t* dims, float eps, float p_drop, uint64_t seed,
                           void* arena, int64_t arena_bytes, float* out, void* stream);
int rsx_static_profile_bwd(const void* const* p, const int64_t* dims, float p_drop, uint64_t seed, const void* arena,
                           const float* dout, float* const* grads, void* ws, int64_t ws_bytes, void* stream);

/* The step's tail: torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm) followed by
 * torch.optim.AdamW.step() (tower_code/v1_usertower_train.py:852-853, :495-496) in two launches.
 * n tensors, each fp32 contiguous with its gradient and both moments (exp_avg, exp_avg_sq);
 * clip[i] != 0 marks the tensors whose gradients form the clipped norm (and are scaled in
 * place by min(max_norm / (norm + 1e-6), 1), as clip_grad_norm_ does); the others (e.g. the item
 * matrix's parameter group) get the unclipped update. Per-tensor hyper-parameters lr,
 * weight_decay, beta1, beta2, eps; the step count AFTER this step's increment is step_dev[i][0]
 * (a device scalar, torch's fused/capturable state) when step_dev and step_dev[i] are non-null,
 * else step[i]. norm_out (device, nullable) receives the total norm. Deterministic: fixed-slot
 * partials reduced in a fixed order. ws: rsx_clip_adamw_workspace_bytes(n, numel, clip). */
int64_t rsx_clip_adamw_workspace_bytes(int n, const int64_t* numel, const int* clip);
int rsx_clip_adamw(int n, float* const* params, float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                   const int64_t* numel, const int* clip, const float* step, const float* const* step_dev,
                   const double* lr, const double* weight_decay, const double* beta1, const double* beta2,
                   const double* eps, float max_norm, void* ws, int64_t ws_bytes, float* norm_out, void* stream);

/* Hard-negative mining: for each row i of u_norm [N,D] against the columns
 * i_norm [N,D] (both already L2-normalised), ignore column j when target_ids[j] ==
 * target_ids[i] or (i_norm[i].i_norm[j] > hnm_threshold and j != i); mining value =
 * (u_norm[i].i_norm[j]) / temperature (-inf when ignored). Writes the k largest per row (value
 * desc, column asc) as top_idx [N,k] int64 with their raw cosines top_cos [N,k], and avail [N]
 * int32 = number of columns not ignored. Two kernels: both products on the fp32 MFMA with the
 * mask applied in registers -> ONE masked N x ld fp32 workspace (ws, 16-B aligned,
 * >= rsx_hnm_workspace_bytes(N)) -> per-row radix select + sort in LDS. Replaces the N x N
 * cos / item_sim / mask tensors and torch.topk of v1_refine_usertower.py:641-669
 * (inbatch_hnm_corrected_loss_with_stats), :705-728 (inbatch_mixed_hnm_loss_with_stats),
 * :776-790 (full_batch_hard_emphasis_loss).
 * D in {64,128}; 1 <= k <= min(N, 4096); N <= rsx_hnm_max_rows() (one row's values live in LDS). */
int rsx_hnm_mine(const float* u_norm, const float* i_norm, const int64_t* target_ids, int64_t N, int64_t D,
                 int64_t k, float hnm_threshold, float temperature, void* ws, size_t ws_bytes, int64_t* top_idx,
                 float* top_cos, int32_t* avail, void* stream);
int64_t rsx_hnm_workspace_bytes(int64_t N);
int64_t rsx_hnm_max_rows(void);

/* ---- A2 + A3 + A4: the user tower's packed-token training program ---------------------
 * SASRecUserTower.forward in training mode over the contrastive step's packed tokens
 * (tower_code/v1_refine_usertower.py:434-510: item_proj, the gated embedding sum + position +
 * emb_ln + dropout, the norm_first TransformerEncoder stack, output_proj[0] over
 * cat(token, profile[user]), LayerNorm + GELU, output_proj[3], F.normalize) and its backward,
 * each as ONE call that launches the same kernels as the per-op entry points above, in the
 * same order with the same arguments (bit-identical results), from the library instead of
 * one host-language call per op. Shapes: d_model 128, 4 heads of 32, feed-forward 256,
 * bf16x3 token linears and attention, L <= 64, 1..8 layers. The static profile rows
 * (:472-494) are an input (computed by the caller, whose autograd takes their gradient).
 *
 * p[] (device pointers, RSX_TW_* order; layer l's 12 parameters at RSX_TW_LAYER0 + 12 l, the
 * output head's 6 after the last layer):
 *   inputs  pretrained rows [T,128], six id arrays int64 [T] (item, time, type, colour,
 *           graphic, section), token positions int64 [T], key-pad flags uint8 [T], user token
 *           offsets int32 / int64 [U+1], token user int64 [T], seq gate [6] (sigmoid(seq_gate)
 *           * s_mask), profile rows [U,128], the item-id gradient plan (perm [T], chunk bounds
 *           [C+1], chunk ids [C], chunk offsets per id [Uq+1], ids [Uq]; ops.sort_segments)
 *   params  item_proj w/b, the six tables, pos_emb, emb_ln w/b; per layer norm1 w/b,
 *           in_proj w/b, out_proj w/b, norm2 w/b, linear1 w/b, linear2 w/b; output_proj[0] w/b,
 *           output_proj[1] w/b, output_proj[3] w/b
 * dims[]  T, U, pos rows (max_len), layers, C, Uq, rows of the six tables, tail B, tail T1
 * tail    (dims[12] = B > 0, round 5) the packed rows are two views of B users each (U = 2B,
 *         T = 2 T1, view 2's token t at row T1 + t) and p[rsx_tower_n_ptrs - 1] holds view 1's
 *         "last" token of each user [B] int64: the last layer past its attention and the output
 *         head run on the R = T1 + B rows the contrastive step reads (all of view 1, then view
 *         2's last row of user b at row T1 + b), `out` is [R,128] and the backward expands their
 *         gradients to every row (the dropped rows' are zero). dims[12] = 0: every row.
 * fargs[] p_drop, emb_ln eps, per layer norm1 eps, norm2 eps, output LayerNorm eps
 * seeds[] 1 + 4 x layers dropout seeds: embedding, then per layer attention, out-projection
 *         add, feed-forward, closing add (the per-op entry points' seed order)
 * arena   saved activations (rsx_tower_arena_bytes), read by the backward; out [T or R,128] (the
 *         backward reads it too: the F.normalize backward).
 * grads[] parallel to p[]: params' gradients written, except the embedding stage's (six
 *         tables, pos_emb, emb_ln w/b) and the seq gate's, which are ACCUMULATED (caller
 *         zeroes); the profile's [U,128] written; the pretrained rows' nullable (written).
 * ws      backward scratch (rsx_tower_bwd_workspace_bytes). */
enum {
  RSX_TW_PV = 0, RSX_TW_IDS = 1, RSX_TW_TOK_POS = 7, RSX_TW_TOK_PAD = 8, RSX_TW_SEG32 = 9, RSX_TW_SEG64 = 10,
  RSX_TW_TOK_USER = 11, RSX_TW_GATE = 12, RSX_TW_PROFILE = 13, RSX_TW_ITEMSEG = 14, RSX_TW_ITEM_PROJ = 19,
  RSX_TW_TABLES = 21, RSX_TW_POS = 27, RSX_TW_EMB_LN = 28, RSX_TW_LAYER0 = 30
};
int64_t rsx_tower_n_ptrs(int layers);
int64_t rsx_tower_arena_bytes(int64_t T, int64_t U, int layers);
int64_t rsx_tower_bwd_workspace_bytes(int64_t T, int64_t U, int64_t L, int layers, int64_t C);
int rsx_tower_fwd(const void* const* p, const int64_t* dims, const float* fargs, const uint64_t* seeds, void* arena,
                  int64_t arena_bytes, float* out, void* stream);
int rsx_tower_bwd(const void* const* p, const int64_t* dims, const float* fargs, const uint64_t* seeds,
                  const void* arena, const float* out, const float* dout, void* const* grads, void* ws,
                  int64_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RECSYS_AMD_H */
