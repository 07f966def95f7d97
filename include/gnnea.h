/*
 * gnnea.h — C-ABI of libgnnea.so, the MI355X (gfx950) hot path of the GNN entity-alignment
 * engine.  This is the drop-in boundary: the reference (HestiaSky/GNN-MTL) has no FFI of its own;
 * its hot path is a handful of PyTorch calls inside its nn.Modules.  Each entry point below states
 * the reference call site it replaces (paths relative to the reference repository root).
 *
 * Rules for every entry point:
 *   - plain pointers + sizes only; all buffers are device-resident, caller-owned (torch-allocated);
 *   - work is enqueued on the caller's HIP stream (`stream` is a hipStream_t, NULL = default);
 *   - no allocation, no host synchronisation, no global state: calls are reentrant and
 *     graph-capturable (gnnea_csr_* query sizes on the host only);
 *   - return 0 on success, a negative GNNEA_E* code for bad arguments, or a positive hipError_t.
 */
#ifndef GNNEA_H
#define GNNEA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNNEA_ABI_VERSION 1

/* status codes (negative); positive values are hipError_t */
#define GNNEA_OK 0
#define GNNEA_EINVAL (-1)      /* bad argument (null pointer, negative size, unsupported combo) */
#define GNNEA_EWORKSPACE (-2)  /* workspace smaller than the matching *_ws_bytes query */
#define GNNEA_EALIGN (-3)      /* pointer / leading-dimension alignment the kernel needs */

/* activation codes fused into epilogues (layers/layers.py:26 `self.act`; config 'act') */
#define GNNEA_ACT_IDENTITY 0
#define GNNEA_ACT_RELU 1
#define GNNEA_ACT_ELU 2
#define GNNEA_ACT_LEAKY_RELU 3 /* negative slope 0.01, F.leaky_relu default */
#define GNNEA_ACT_SIGMOID 4
#define GNNEA_ACT_TANH 5

/* element types */
#define GNNEA_F32 0
#define GNNEA_F64 1
#define GNNEA_BF16 2

int gnnea_abi_version(void);
const char* gnnea_error_string(int code);

/* ------------------------------------------------------------------------------------------ *
 * a1. Adjacency contract: COO -> CSR.
 * Replaces the implicit coalesce inside torch.spmm(adj, hidden) (layers/layers.py:35,64) and
 * adj.coalesce().indices() (layers/att_layers.py:31).  Input is the reference's torch sparse COO
 * (utils/data_utils.py:51-57, 325-336): uncoalesced, int64 (or int32) indices, fp32 values.
 * Output: int32 CSR sorted by (row, col), duplicates summed in input order (explicit zeros kept,
 * as coalesce() keeps them), plus perm[k] = input position of the first duplicate of entry k.
 * The transpose of a CSR is built by calling it again on (col, row) of that CSR.
 * *nnz_out is written on the device (int64); rowptr has n_rows+1 entries.
 * ------------------------------------------------------------------------------------------ */
int64_t gnnea_coo_to_csr_ws_bytes(int64_t nnz, int64_t n_rows, int64_t n_cols);
int gnnea_coo_to_csr(const void* row_idx, const void* col_idx, int index_bytes /*4 or 8*/,
                     const float* val /*nullable: pattern only*/, int64_t nnz, int64_t n_rows,
                     int64_t n_cols, int32_t* rowptr, int32_t* col_out, float* val_out /*nullable*/,
                     int64_t* perm_out /*nullable*/, int64_t* nnz_out, void* ws, int64_t ws_bytes,
                     void* stream);
/* row id of every CSR entry: row_out[e] = r for rowptr[r] <= e < rowptr[r+1] */
int gnnea_csr_expand_rows(const int32_t* rowptr, int32_t n_rows, int64_t nnz, int32_t* row_out,
                          void* stream);
/* inverse permutation: inv[perm[k]] = k (forward CSR position -> transposed position) */
int gnnea_perm_invert(const int64_t* perm, int64_t n, int64_t* inv, void* stream);

/* ------------------------------------------------------------------------------------------ *
 * a2/a3. CSR SpMM  Y = act(A · X)   (layers/layers.py:35 torch.spmm(adj, hidden) + :38 act)
 * Gather model: one wave per destination row, 16-B lanes over the feature row, neighbour
 * (col,val) broadcast by readlane.  X row stride ldx and Y row stride ldy in elements.
 * Fast path needs D % 4 == 0, ldx % 4 == 0, ldy % 4 == 0 and 16-B aligned X, Y.
 * ------------------------------------------------------------------------------------------ */
int gnnea_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                       int32_t n_rows, int32_t D, const float* X, int64_t ldx, float* Y,
                       int64_t ldy, int act, void* stream);
/* Y = act(A · X + beta · Y): partial aggregations over column blocks (the multi-GPU halo
 * overlap sums the locally owned block while the remote rows are in flight). */
int gnnea_spmm_csr_beta_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                            int32_t n_rows, int32_t D, const float* X, int64_t ldx, float beta,
                            float* Y, int64_t ldy, int act, void* stream);

/* Slice-major feature table (replaces the same torch.spmm, layers/layers.py:35, when the gathered
 * matrix exceeds the 256 MB Infinity Cache): the D columns are cut into S = ceil(D/64) slices,
 * element (r, c) at Xs[(c/64)*sstride + r*64 + c%64], sstride >= n*64 floats, Xs 16-B aligned.
 * The aggregation walks the slices in order so each slice's table (256 MB at 1M rows) is what
 * its gathers touch; Y is row-major.  Requires D % 4 == 0, ldy % 4 == 0, 16-B aligned Y, and
 * Xs to hold every row the CSR references.  The fp32 sums are taken in a fixed order that
 * differs from gnnea_spmm_csr_f32's (agreement to fp32 rounding). */
int gnnea_spmm_sliced_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                          int32_t n_rows, int32_t D, const float* Xs, int64_t sstride, float* Y,
                          int64_t ldy, int act, void* stream);
/* bf16 storage (cfg-5): 128-column slices (256 B per slice row), element (r, c) at
 * Xs[(c/128)*sstride + r*128 + c%128], sstride % 128 == 0; fp32 arithmetic, Y bf16 (y_dtype
 * GNNEA_BF16, rounded once) or fp32 (GNNEA_F32); D % 4 == 0, 16-B aligned Xs, 8-B aligned Y. */
int gnnea_spmm_sliced_bf16(const int32_t* rowptr, const int32_t* col, const float* val,
                           int32_t n_rows, int32_t D, const void* Xs, int64_t sstride, void* Y,
                           int64_t ldy, int y_dtype, int act, void* stream);
int gnnea_slice_pack_bf16(const void* X, int64_t ldx, int64_t n, int32_t D, void* Xs,
                          int64_t sstride, void* stream);
/* the same aggregation over 64-column bf16 slices (128 B per row piece, one cfg-5 KG slice =
 * 256 MB, the Infinity Cache's size): the layout of gnnea_slice_pack64_bf16, element (r, c) at
 * Xs[(c/64)*sstride + r*64 + c%64], sstride % 64 == 0, 16-B aligned Xs */
int gnnea_spmm_sliced64_bf16(const int32_t* rowptr, const int32_t* col, const float* val,
                             int32_t n_rows, int32_t D, const void* Xs, int64_t sstride, void* Y,
                             int64_t ldy, int y_dtype, int act, void* stream);
int gnnea_act_bwd_sliced_bf16(const void* dY, int64_t lddy, const void* Y, int64_t ldy,
                              int64_t n, int32_t D, int act, void* Gs, int64_t sstride,
                              void* stream);
/* HighWay layer over a slice-major projection (layers/layers.py:64-76): S = act(A·X) with X the
 * first D columns of the table Xs, g = sigmoid(gate_pre + bias_gate) with gate_pre read from
 * the slice-major table gate_s at column offset goff (the fused layer's ONE projection table
 * Z = x·[W^T | K_g]: gate_s = Xs, goff = D), Y = g*S + (1-g)*resid; resid, Y, S, g row-major. */
int gnnea_spmm_highway_sliced_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                                  int32_t n_rows, int32_t D, const float* Xs, int64_t sstride,
                                  const float* gate_s, int64_t gsstride, int32_t goff,
                                  const float* bias_gate, const float* resid, int64_t ldr,
                                  float* Y, int64_t ldy, float* save_s, float* save_g,
                                  int64_t lds, int act, void* stream);
/* gnnea_highway_bwd_ld_f32 with dS_pre written slice-major (slice stride sstride >= n_rows*64):
 * the input of the transposed sliced aggregation */
int gnnea_highway_bwd_sliced_f32(const float* dY, const float* S, const float* G,
                                 const float* resid, int64_t ld, int64_t n_rows, int32_t D,
                                 float* dS_s, int64_t sstride, float* dgate, int64_t ld_dg,
                                 float* dresid, int64_t ld_dr, int act, void* stream);
/* gnnea_highway_bwd_sliced_f32 without a saved gate: g = sigmoid(gate_pre + bias_gate)
 * recomputed from the slice-major projection table Zs (slice stride zs_stride, gate_pre at
 * column goff: the forward's gate_s / goff), bit-identical to the forward's g, so the forward
 * passes save_g = NULL (autograd of layers/layers.py:64-76; 16-B aligned operands, D % 4 == 0) */
int gnnea_highway_bwd_sliced_zg_f32(const float* dY, const float* S, const float* Zs,
                                    int64_t zs_stride, int32_t goff, const float* bias_gate,
                                    const float* resid, int64_t ld, int64_t n_rows, int32_t D,
                                    float* dS_s, int64_t sstride, float* dgate, int64_t ld_dg,
                                    float* dresid, int64_t ld_dr, int act, void* stream);
/* The fused HighWay layer without S (relu only): the forward stores S's sign instead of S
 * (save_m: [n_rows][ldm] bytes, ldm >= 16 * ceil(D / 64); byte 16 q + l of a row holds bit e =
 * S[row][64 q + 4 l + e] > 0), and the backward takes act' from that mask (act relu; identity
 * needs none: mask may be NULL) and S - resid from the forward's output Y (g (S - resid) =
 * Y - resid): dS_pre = dY g act', dgate = dY (Y - resid)(1 - g), dresid = dY (1 - g). */
int gnnea_spmm_highway_sliced_m_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                                    int32_t n_rows, int32_t D, const float* Xs, int64_t sstride,
                                    const float* gate_s, int64_t gsstride, int32_t goff,
                                    const float* bias_gate, const float* resid, int64_t ldr,
                                    float* Y, int64_t ldy, uint8_t* save_m, int64_t ldm, int act,
                                    void* stream);
int gnnea_highway_bwd_sliced_zgm_f32(const float* dY, const float* Y, const float* Zs,
                                     int64_t zs_stride, int32_t goff, const float* bias_gate,
                                     const float* resid, int64_t ld, int64_t n_rows, int32_t D,
                                     const uint8_t* mask, int64_t ldm, float* dS_s,
                                     int64_t sstride, float* dgate, int64_t ld_dg, float* dresid,
                                     int64_t ld_dr, int act, void* stream);
/* row-major [n, D] (row stride ldx) -> slice-major table (the drop-in path for a row-major
 * hidden that no gnnea GEMM produced) */
int gnnea_slice_pack_f32(const float* X, int64_t ldx, int64_t n, int32_t D, float* Xs,
                         int64_t sstride, void* stream);
/* backward input of the transposed aggregation, written slice-major:  Gs = dY * act'(Y) */
int gnnea_act_bwd_sliced_f32(const float* dY, int64_t lddy, const float* Y, int64_t ldy,
                             int64_t n, int32_t D, int act, float* Gs, int64_t sstride,
                             void* stream);

/* a4. HighWay epilogue (layers/layers.py:64-76):
 *   S = act(A·X);  g = sigmoid(gate_pre + bias_gate);  Y = g*S + (1-g)*resid
 * gate_pre = x·kernel_gate (N x D), bias_gate (D, nullable = 0), resid = x (N x D).
 * save_s / save_g (nullable) receive S and g for the backward pass. */
int gnnea_spmm_highway_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                           int32_t n_rows, int32_t D, const float* X, int64_t ldx,
                           const float* gate_pre, int64_t ldg, const float* bias_gate,
                           const float* resid, int64_t ldr, float* Y, int64_t ldy,
                           float* save_s, float* save_g, int64_t lds, int act, void* stream);

/* Elementwise activation backward through the output:  G = dY * act'(Y)  (n elements). */
int gnnea_act_bwd_f32(const float* dY, const float* Y, float* G, int64_t n, int act, void* stream);

/* The Linear layer's act (layers/layers.py:111-122, MLPDecoder models/decoders.py:57-63),
 * csrc/act.hip.  Y = act(X) over n contiguous elements (Y may be X): the path of a Linear whose
 * GEMM kernel has no fused act epilogue. */
int gnnea_act_fwd_f32(const float* X, float* Y, int64_t n, int act, void* stream);
int gnnea_act_fwd_bf16(const void* X, void* Y, int64_t n, int act, void* stream);
/* The act's backward and the bias gradient in one pass (autograd of act(x·Wᵀ + b),
 * layers/layers.py:121-122):  G = dY * act'(Y) (row-major, ld's in elements; bf16 G rounded
 * once),  db[c] = sum_r G[r][c]  (fp32, summed from the stored G, deterministic: fixed row
 * ranges per workgroup, fp64 fold of their partials).  Workspace: gnnea_act_bwd_colsum_ws_bytes
 * (required).  bf16: dY, Y, G bf16; db fp32. */
int64_t gnnea_act_bwd_colsum_ws_bytes(int64_t n_rows, int32_t D);
int gnnea_act_bwd_colsum_f32(const float* dY, int64_t lddy, const float* Y, int64_t ldy,
                             int64_t n_rows, int32_t D, int act, float* G, int64_t ldg, float* db,
                             void* ws, int64_t ws_bytes, void* stream);
int gnnea_act_bwd_colsum_bf16(const void* dY, int64_t lddy, const void* Y, int64_t ldy,
                              int64_t n_rows, int32_t D, int act, void* G, int64_t ldg, float* db,
                              void* ws, int64_t ws_bytes, void* stream);

/* The non-concatenated GAT layer's head mean (layers/att_layers.py:89-91, torch.mean over the
 * stacked heads), csrc/act.hip.  bwd = 0: Y[i][d] = (sum_h X[i][h dh + d]) / heads (X [n][heads
 * dh], Y [n][dh]; fp32 sum in head order, one rounding); bwd = 1: X is dY [n][dh] and Y receives
 * dX[i][h dh + d] = dY[i][d] / heads.  ld's in elements. */
int gnnea_head_mean_f32(const float* X, int64_t ldx, int64_t n, int32_t heads, int32_t dh,
                        float* Y, int64_t ldy, int bwd, void* stream);
int gnnea_head_mean_bf16(const void* X, int64_t ldx, int64_t n, int32_t heads, int32_t dh,
                         void* Y, int64_t ldy, int bwd, void* stream);

/* HighWay backward, elementwise part (autograd of layers/layers.py:67-76):
 *   dS_pre  = dY * g * act'(S)            (-> SpMM^T gives d hidden)
 *   dgate   = dY * (S - resid) * g*(1-g)  (-> d gate_pre; x-grad via kernel_gate^T)
 *   dresid  = dY * (1 - g)                                                           */
int gnnea_highway_bwd_f32(const float* dY, const float* S, const float* G, const float* resid,
                          int64_t ld, int64_t n_rows, int32_t D, float* dS_pre, float* dgate,
                          float* dresid, int act, void* stream);
/* the same with separate row strides for the outputs (dS_pre, dgate, dresid may be column
 * blocks of wider buffers: the fused HighWay layer writes dgate next to d hidden so that one
 * GEMM [dh | dgate]·[W ; K_gᵀ] gives the whole input gradient) */
int gnnea_highway_bwd_ld_f32(const float* dY, const float* S, const float* G, const float* resid,
                             int64_t ld, int64_t n_rows, int32_t D, float* dS_pre, int64_t ld_ds,
                             float* dgate, int64_t ld_dg, float* dresid, int64_t ld_dr, int act,
                             void* stream);

/* bf16 feature storage (cfg-5; SURVEY.md §8b gnnea_spmm_csr_bf16): X, gate_pre, resid, dY, S, G
 * are bf16 (void*, 2-byte elements), CSR values and bias_gate stay fp32, every product and sum
 * is fp32, outputs are rounded once to bf16 (round-to-nearest-even, as torch) or written fp32
 * (y_dtype GNNEA_F32: gradient partials).  Fast path: D, ldx, ldy % 4 == 0 and 8-B aligned rows
 * (one 8-B load of 4 elements per lane).  beta as gnnea_spmm_csr_beta_f32. */
int gnnea_spmm_csr_bf16(const int32_t* rowptr, const int32_t* col, const float* val,
                        int32_t n_rows, int32_t D, const void* X, int64_t ldx, float beta,
                        void* Y, int64_t ldy, int y_dtype, int act, void* stream);
int gnnea_spmm_highway_bf16(const int32_t* rowptr, const int32_t* col, const float* val,
                            int32_t n_rows, int32_t D, const void* X, int64_t ldx,
                            const void* gate_pre, int64_t ldg, const float* bias_gate,
                            const void* resid, int64_t ldr, void* Y, int64_t ldy, void* save_s,
                            void* save_g, int64_t lds, int act, void* stream);
int gnnea_act_bwd_bf16(const void* dY, const void* Y, void* G, int64_t n, int act, void* stream);
int gnnea_highway_bwd_bf16(const void* dY, const void* S, const void* G, const void* resid,
                           int64_t ld, int64_t n_rows, int32_t D, void* dS_pre, void* dgate,
                           void* dresid, int act, void* stream);
int gnnea_highway_bwd_ld_bf16(const void* dY, const void* S, const void* G, const void* resid,
                              int64_t ld, int64_t n_rows, int32_t D, void* dS_pre, int64_t ld_ds,
                              void* dgate, int64_t ld_dg, void* dresid, int64_t ld_dr, int act,
                              void* stream);

/* ------------------------------------------------------------------------------------------ *
 * a5-a7. Sparse GAT, all heads per edge pass (layers/att_layers.py:29-61, 82-91).
 * H is the head-concatenated projection X·[W_0|...|W_{h-1}] (N x heads*d_head, row stride ldh);
 * s1[i,h] = a_h[:d]·H_i,h ; s2[j,h] = a_h[d:]·H_j,h  (att_layers.py:38-41 factorised per node).
 * score_ij,h = -LeakyReLU_alpha(s1[i,h] + s2[j,h]); the row softmax is computed with the row max
 * subtracted (mathematically identical to the reference's exp without shift, overflow-safe).
 * edge_mask (nullable, nnz x heads) multiplies the numerator only (dropout after the row sum,
 * att_layers.py:51).  Outputs Y = act(h') (ldy), row max m and denominator den (N x heads).
 * Rows without edges produce 0 (the reference raises on them).
 * ------------------------------------------------------------------------------------------ */
int gnnea_gat_scores_f32(const float* H, int64_t ldh, int32_t n_rows, int heads, int d_head,
                         const float* a /*heads x 2*d_head*/, float* s1, float* s2, void* stream);
int gnnea_gat_fwd_f32(const int32_t* rowptr, const int32_t* col, int32_t n_rows, const float* H,
                      int64_t ldh, int heads, int d_head, const float* s1, const float* s2,
                      float alpha, const float* edge_mask, int act, float* Y, int64_t ldy,
                      float* m_out, float* den_out, void* stream);
/* The same forward over a slice-major source table Hs [ceil(D/64)][n_src][64] fp32 (slice
 * stride sstride floats, the gnnea_spmm_sliced_f32 layout): row max / denominator records first
 * (m_out, den_out) and every edge's masked numerator weight (wgt: nnz x heads fp32, by CSR
 * position, workspace), then the aggregation slice by slice (each KG slice a 256-MB table).
 * d_head >= 32, heads <= 8, D % 4 == 0, act identity / relu; Y row-major (ldy % 4 == 0). */
int gnnea_gat_fwd_sliced_f32(const int32_t* rowptr, const int32_t* col, int32_t n_rows,
                             const float* Hs, int64_t sstride, int heads, int d_head,
                             const float* s1, const float* s2, float alpha,
                             const float* edge_mask, int act, float* Y, int64_t ldy,
                             float* m_out, float* den_out, float* wgt, void* stream);
/* The backward over a slice-major G (fp32, d_head >= 32, heads <= 8, D % 4 == 0, D <= 1024):
 *   prep_sliced (dest rows i): G = dY * act'(Y) into Gs ([ceil(D/64)][n_rows][64], sstride
 *                floats per slice) and the records rec (n_rows x heads x 4: s1, m, 1/den, G.h');
 *   src_sliced  (source rows j of A^T, one KG block per call): per-edge weights wT (nnzT x heads,
 *                by A^T position), then slice by slice dH_j = sum_i w_ij G_i (row-major) and the
 *                slice partials of G_i,h . H_j,h in pd (ceil(D/64) x nnzT x 2);
 *   edge_sliced (source rows): dzT (A^T order), ds2, and dH_j += ds2_j (x) a2 when dH != NULL;
 *   dst_sliced  (dest rows): ds1 (dzT through tpos, the A -> A^T position map) and
 *                dH_i += ds1_i (x) a1 (+ ds2_i (x) a2 when ds2 != NULL).
 * Same results as prep / src / dst below up to fp32 summation order (att_layers.py:38-58). */
int gnnea_gat_bwd_prep_sliced_f32(int32_t n_rows, int heads, int d_head, const float* dY,
                                  const float* Y, int64_t ldy, const float* s1, const float* m,
                                  const float* den, int act, float* Gs, int64_t sstride,
                                  float* rec, void* stream);
int gnnea_gat_bwd_src_sliced_f32(const int32_t* rowptrT, const int32_t* colT,
                                 const int64_t* permT, int32_t n_rows, int heads, int d_head,
                                 const float* Hm, int64_t ldh, const float* s2, float alpha,
                                 const float* edge_mask, const float* rec, const float* Gs,
                                 int64_t sstride, float* wT, float* pd, int64_t nnzT, float* dH,
                                 int64_t lddh, void* stream);
int gnnea_gat_bwd_edge_sliced_f32(const int32_t* rowptrT, const int32_t* colT,
                                  const int64_t* permT, int32_t n_rows, int heads, int d_head,
                                  const float* s2, float alpha, const float* edge_mask,
                                  const float* rec, const float* pd, int64_t nnzT,
                                  const float* a, float* dH, int64_t lddh, float* dzT,
                                  float* ds2, void* stream);
int gnnea_gat_bwd_dst_sliced_f32(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows,
                                 int heads, int d_head, const float* dzT, const float* a,
                                 const float* ds2, float* dH, int64_t lddh, float* ds1,
                                 void* stream);
/* bf16 storage (cfg-5) of the same sliced passes: Hs / Gs are 64-column bf16 tables (128 B, one
 * line per gathered row piece; [ceil(D/64)][n][64], sstride elements per slice, so one slice of a
 * 2M-row KG is 256 MB), Y / dY / H / dH row-major bf16 (8-B aligned, ld % 4 == 0); logits, records,
 * weights, partials and dz stay fp32; fp32 arithmetic, each stored bf16 value rounded once per
 * pass (nearest even). */
int gnnea_gat_fwd_sliced_bf16(const int32_t* rowptr, const int32_t* col, int32_t n_rows,
                              const void* Hs, int64_t sstride, int heads, int d_head,
                              const float* s1, const float* s2, float alpha,
                              const float* edge_mask, int act, void* Y, int64_t ldy,
                              float* m_out, float* den_out, float* wgt, void* stream);
int gnnea_gat_bwd_prep_sliced_bf16(int32_t n_rows, int heads, int d_head, const void* dY,
                                   const void* Y, int64_t ldy, const float* s1, const float* m,
                                   const float* den, int act, void* Gs, int64_t sstride,
                                   float* rec, void* stream);
int gnnea_gat_bwd_src_sliced_bf16(const int32_t* rowptrT, const int32_t* colT,
                                  const int64_t* permT, int32_t n_rows, int heads, int d_head,
                                  const void* Hm, int64_t ldh, const float* s2, float alpha,
                                  const float* edge_mask, const float* rec, const void* Gs,
                                  int64_t sstride, float* wT, float* pd, int64_t nnzT, void* dH,
                                  int64_t lddh, void* stream);
int gnnea_gat_bwd_edge_sliced_bf16(const int32_t* rowptrT, const int32_t* colT,
                                   const int64_t* permT, int32_t n_rows, int heads, int d_head,
                                   const float* s2, float alpha, const float* edge_mask,
                                   const float* rec, const float* pd, int64_t nnzT,
                                   const float* a, void* dH, int64_t lddh, float* dzT,
                                   float* ds2, void* stream);
int gnnea_gat_bwd_dst_sliced_bf16(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows,
                                  int heads, int d_head, const float* dzT, const float* a,
                                  const float* ds2, void* dH, int64_t lddh, float* ds1,
                                  void* stream);
/* Slice ranges of the sliced GAT passes, for the staged halo of a row-sharded layer
 * (gnnea/dist_graph.py: slice q is aggregated as soon as its exchange has landed; the backward's
 * source pass per slice, each slice's dH partial reduce-scattered while the next computes).
 *   fwd_sliced_range: slices [s_begin, s_end) of Hs only; stats != 0 first computes m_out,
 *                     den_out and wgt (s_begin == s_end: only that).  Same outputs as
 *                     gnnea_gat_fwd_sliced_* over all slices.
 *   bwd_src_sliced_range: slices [s_begin, s_end); weights != 0 first computes wT.  H and dH
 *                     each row-major (hss / dhss = 64, ldh / lddh >= D) or slice-major 64-column
 *                     tables (ldh / lddh = 64, hss / dhss = the slice stride >= 64 n_rows).
 * Replaces: the halo exchange around att_layers.py:33-58 (reference: one process, no exchange). */
int gnnea_gat_fwd_sliced_range_f32(const int32_t* rowptr, const int32_t* col, int32_t n_rows,
                                   const float* Hs, int64_t sstride, int heads, int d_head,
                                   const float* s1, const float* s2, float alpha,
                                   const float* edge_mask, int act, float* Y, int64_t ldy,
                                   float* m_out, float* den_out, float* wgt, int s_begin,
                                   int s_end, int stats, void* stream);
int gnnea_gat_fwd_sliced_range_bf16(const int32_t* rowptr, const int32_t* col, int32_t n_rows,
                                    const void* Hs, int64_t sstride, int heads, int d_head,
                                    const float* s1, const float* s2, float alpha,
                                    const float* edge_mask, int act, void* Y, int64_t ldy,
                                    float* m_out, float* den_out, float* wgt, int s_begin,
                                    int s_end, int stats, void* stream);
int gnnea_gat_bwd_src_sliced_range_f32(const int32_t* rowptrT, const int32_t* colT,
                                       const int64_t* permT, int32_t n_rows, int heads,
                                       int d_head, const float* Hm, int64_t ldh, int64_t hss,
                                       const float* s2, float alpha, const float* edge_mask,
                                       const float* rec, const float* Gs, int64_t sstride,
                                       float* wT, float* pd, int64_t nnzT, float* dH,
                                       int64_t lddh, int64_t dhss, int s_begin, int s_end,
                                       int weights, void* stream);
int gnnea_gat_bwd_src_sliced_range_bf16(const int32_t* rowptrT, const int32_t* colT,
                                        const int64_t* permT, int32_t n_rows, int heads,
                                        int d_head, const void* Hm, int64_t ldh, int64_t hss,
                                        const float* s2, float alpha, const float* edge_mask,
                                        const float* rec, const void* Gs, int64_t sstride,
                                        float* wT, float* pd, int64_t nnzT, void* dH,
                                        int64_t lddh, int64_t dhss, int s_begin, int s_end,
                                        int weights, void* stream);
/* row-major [n, D] -> the 64-column slice-major GAT table (D % 4 == 0, ldx % 4 == 0, sstride a
 * multiple of 64 and >= 64 n elements) */
int gnnea_slice_pack64_f32(const float* X, int64_t ldx, int64_t n, int32_t D, float* Xs,
                           int64_t sstride, void* stream);
int gnnea_slice_pack64_bf16(const void* X, int64_t ldx, int64_t n, int32_t D, void* Xs,
                            int64_t sstride, void* stream);
/* Backward in one gather sweep over A^T (autograd of att_layers.py:38-58):
 *  prep (rows i):   G_i = dY_i * act'(Y_i) (act: identity / relu, Y = h' there) and the per-node
 *                   record rec[i,h] = {s1, m, 1/den, c = G_i,h . h'_i,h}  (float4 per head);
 *  src  (rows j of A^T; rowptrT/colT/permT from gnnea_coo_to_csr on the transpose):
 *                   dH_j = sum_i alpha_ij*mask*G_i + ds2_j (x) a2,  dz_ij = -LReLU'(z) *
 *                   alpha_ij*(mask*G_i.H_j - c_i) per head, written in A^T order to dzT;
 *  dst  (rows i of A; tpos = inverse of permT): ds1_i = sum_j dz_ij,  dH_i += ds1_i (x) a1.
 * a is [heads][2*d_head] (a_h = [a1 | a2]). */
int gnnea_gat_bwd_prep_f32(int32_t n_rows, int heads, int d_head, const float* dY,
                           const float* Y, int64_t ld, const float* s1, const float* m,
                           const float* den, int act, float* G, float* rec, void* stream);
int gnnea_gat_bwd_src_f32(const int32_t* rowptrT, const int32_t* colT, const int64_t* permT,
                          int32_t n_rows, int heads, int d_head, const float* H, int64_t ldh,
                          const float* s2, float alpha, const float* edge_mask, const float* rec,
                          const float* G, int64_t ldg, const float* a, float* dH, int64_t lddh,
                          float* dzT, float* ds2, void* stream);
int gnnea_gat_bwd_dst_f32(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows, int heads,
                          int d_head, const float* dzT, const float* a, float* dH, int64_t lddh,
                          float* ds1, void* stream);

/* attention-vector gradient pieces (autograd of att_layers.py:38): out[c] = sum_r ds[r, c/d_head]
 * * H[r, c] over the n_rows rows of H (ds: n_rows x heads fp32, ds1 or ds2 of the backward),
 * c < heads*d_head; one streaming pass over H, deterministic two-stage sum.  H rows are read as
 * 16-B granules within their row stride (ldh >= heads*d_head, rows 4-B aligned; the table's
 * last row element by element when its final granule would pass the table's end).
 * Workspace from gnnea_gat_da_ws_bytes. */
int64_t gnnea_gat_da_ws_bytes(int64_t n_rows, int32_t D);
int gnnea_gat_da_f32(const float* H, int64_t ldh, int64_t n_rows, int heads, int d_head,
                     const float* ds, float* out, void* ws, int64_t ws_bytes, void* stream);
int gnnea_gat_da_bf16(const void* H, int64_t ldh, int64_t n_rows, int heads, int d_head,
                      const float* ds, float* out, void* ws, int64_t ws_bytes, void* stream);
/* both pieces of one layer in ONE pass over H when they weight the same rows (the whole-graph
 * backward: ds1 and ds2 are both n_rows x heads): out1 from ds1, out2 from ds2 */
int gnnea_gat_da2_f32(const float* H, int64_t ldh, int64_t n_rows, int heads, int d_head,
                      const float* ds1, const float* ds2, float* out1, float* out2, void* ws,
                      int64_t ws_bytes, void* stream);
int gnnea_gat_da2_bf16(const void* H, int64_t ldh, int64_t n_rows, int heads, int d_head,
                       const float* ds1, const float* ds2, float* out1, float* out2, void* ws,
                       int64_t ws_bytes, void* stream);
/* column sums out[c] = sum_r X[r, c], c < D (the bias gradients, autograd of nn.Linear's bias,
 * layers/layers.py:32): the same streaming pass with unit weights, fp32 sums; workspace from
 * gnnea_gat_da_ws_bytes(n_rows, D); X rows 4-B aligned */
int gnnea_colsum_f32(const float* X, int64_t ldx, int64_t n_rows, int32_t D, float* out,
                     void* ws, int64_t ws_bytes, void* stream);
int gnnea_colsum_bf16(const void* X, int64_t ldx, int64_t n_rows, int32_t D, float* out,
                      void* ws, int64_t ws_bytes, void* stream);

/* bf16 feature storage (cfg-5): H, Y, dY, G, dH are bf16 (void*, row strides % 4 == 0, 8-B
 * aligned); s1, s2, m, den, rec, dzT, ds1, ds2, a and edge_mask stay fp32; arithmetic is fp32 and
 * every bf16 output is rounded once (nearest even). */
int gnnea_gat_scores_bf16(const void* H, int64_t ldh, int32_t n_rows, int heads, int d_head,
                          const float* a, float* s1, float* s2, void* stream);
int gnnea_gat_fwd_bf16(const int32_t* rowptr, const int32_t* col, int32_t n_rows, const void* H,
                       int64_t ldh, int heads, int d_head, const float* s1, const float* s2,
                       float alpha, const float* edge_mask, int act, void* Y, int64_t ldy,
                       float* m, float* den, void* stream);
int gnnea_gat_bwd_prep_bf16(int32_t n_rows, int heads, int d_head, const void* dY, const void* Y,
                            int64_t ld, const float* s1, const float* m, const float* den,
                            int act, void* G, float* rec, void* stream);
int gnnea_gat_bwd_src_bf16(const int32_t* rowptrT, const int32_t* colT, const int64_t* permT,
                           int32_t n_rows, int heads, int d_head, const void* H, int64_t ldh,
                           const float* s2, float alpha, const float* edge_mask, const float* rec,
                           const void* G, int64_t ldg, const float* a, void* dH, int64_t lddh,
                           float* dzT, float* ds2, void* stream);
/* gnnea_gat_bwd_src_bf16 for a G of g_rows rows: the in-neighbours' G rows are read as one
 * 16-B window per lane (the head-grouped run of <= 6 elements; the window may run into the next
 * row, so G's last row is read element-wise) -- one load instruction per edge. */
int gnnea_gat_bwd_src_rows_bf16(const int32_t* rowptrT, const int32_t* colT,
                                const int64_t* permT, int32_t n_rows, int heads, int d_head,
                                const void* H, int64_t ldh, const float* s2, float alpha,
                                const float* edge_mask, const float* rec, const void* G,
                                int64_t ldg, int64_t g_rows, const float* a, void* dH,
                                int64_t lddh, float* dzT, float* ds2, void* stream);
int gnnea_gat_bwd_dst_bf16(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows, int heads,
                           int d_head, const float* dzT, const float* a, void* dH, int64_t lddh,
                           float* ds1, void* stream);

/* ------------------------------------------------------------------------------------------ *
 * Dense projection (nn.Linear at layers/layers.py:32,61,93; torch.mm at att_layers.py:33;
 * torch.spmm(x, kernel_gate) at layers.py:69).  f32-in / f32-accumulate MFMA
 * (v_mfma_f32_32x32x2_f32): bit-for-bit an fmaf chain in k order.
 *   C[M,N] = op(A)[M,K] · op(B)[K,N] (+ bias[N]) (+ beta*C) ; op = transpose when trans_* != 0.
 * Row-major, leading dimensions in elements.  Products whose output tiles cannot fill the chip
 * but have a long K (weight gradients: K = number of nodes) split K over workgroups into fp32
 * slabs in `ws` (gnnea_gemm_ws_bytes) reduced in fixed order — deterministic; ws may be NULL.
 * ------------------------------------------------------------------------------------------ */
int64_t gnnea_gemm_ws_bytes(int64_t M, int64_t N, int64_t K);
int gnnea_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                   int64_t lda, const float* B, int64_t ldb, const float* bias, float beta,
                   float* C, int64_t ldc, void* ws, int64_t ws_bytes, void* stream);

/* fp32 GEMM on the bf16 MFMA: each operand element split exactly into three bf16 terms
 * (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m)), the six products of order <= 2 summed
 * in fp32 (error at fp32 rounding level: the dropped terms are below 2^-24 relative); 6/16 of
 * the f32 MFMA time.  Arguments and layouts as gnnea_gemm_f32 / _sliced_f32; workspace from
 * gnnea_gemm_x3_ws_bytes (op(B) split once into three bf16 planes + split-K slabs; required).
 * trans_a = 1 with trans_b = 0 is the weight-gradient form dW = Aᵀ·B (A [K][M], B [K][N], both
 * tall): both operands are split on the fly, split-K over the long K, workspace from
 * gnnea_gemm_x3t_ws_bytes (slabs only).  trans_a = trans_b = 1 runs on the f32 MFMA kernel.
 * Tall projections (trans_a = 0, M >= 65536, K in (288, 320] or (576, 608]) run on the fp16
 * MFMA instead: two fp16 pieces per element (hi = f16(x s), lo = f16(x s - hi)), every row of A
 * and column of op(B) scaled by a power of two s into fp16's range, three products (hi·lo,
 * lo·hi, hi·hi; the dropped lo·lo and lo's rounding each <= 2^-22 |a||b|), the inverse scales
 * applied exactly in the epilogue (csrc/gemm_x3w.hip k_gemm_f16x2_ring). */
int64_t gnnea_gemm_x3_ws_bytes(int64_t M, int64_t N, int64_t K);
int64_t gnnea_gemm_x3t_ws_bytes(int64_t M, int64_t N, int64_t K);
int gnnea_gemm_x3_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                      int64_t lda, const float* B, int64_t ldb, const float* bias, float beta,
                      float* C, int64_t ldc, void* ws, int64_t ws_bytes, void* stream);
int gnnea_gemm_x3_sliced_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                             const float* A, int64_t lda, const float* B, int64_t ldb,
                             const float* bias, float beta, float* Cs, int64_t sstride, void* ws,
                             int64_t ws_bytes, void* stream);
/* C = act(A·op(B) + bias), beta = 0 (nn.Linear + its act, layers/layers.py:121-122): relu is
 * applied in the epilogue of the weight-resident ring kernel (K in (288, 320], tall M), every
 * other case runs the product and then the act in place.  Workspace as gnnea_gemm_x3_f32. */
int gnnea_gemm_x3_act_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                          const float* A, int64_t lda, const float* B, int64_t ldb,
                          const float* bias, int act, float* C, int64_t ldc, void* ws,
                          int64_t ws_bytes, void* stream);
/* C row-major AND a slice-major copy C2s (element (r, c) at C2s[(c/64)*sstride2 + r*64 + c%64]):
 * the second store rides the GEMM epilogue (the GAT projection: row-major for the backward,
 * slice-major for gnnea_gat_fwd_sliced_f32).  Workspace from gnnea_gemm_x3_ws_bytes. */
int gnnea_gemm_x3_dual_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                           const float* A, int64_t lda, const float* B, int64_t ldb,
                           const float* bias, float beta, float* C, int64_t ldc, float* C2s,
                           int64_t sstride2, void* ws, int64_t ws_bytes, void* stream);
/* the same GEMM writing C slice-major (the layout gnnea_spmm_sliced_f32 gathers from):
 * element (r, c) of the M x N product at Cs[(c/64)*sstride + r*64 + c%64], sstride >= M*64.
 * The projection x W^T of a GCN layer writes its hidden this way at no extra cost. */
int gnnea_gemm_sliced_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                          const float* A, int64_t lda, const float* B, int64_t ldb,
                          const float* bias, float beta, float* Cs, int64_t sstride, void* ws,
                          int64_t ws_bytes, void* stream);

/* fp64 GEMM on the f64 matrix cores (v_mfma_f64_16x16x4_f64) for the GW / FGW outer loops
 * (SinkhornOT/cderivation.py:146-188: C1 · T · C2ᵀ and the constC products):
 *   D[M,N] = alpha · op(A)[M,K] · op(B)[K,N] + beta · E[M,N]   (E nullable, may alias D)
 * Row-major, leading dimensions in elements, caller's stream, no workspace.
 * Replaces torch.matmul at cderivation.py:150-151,161. */
int gnnea_gemm_f64(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const double* A,
                   int64_t lda, const double* B, int64_t ldb, double alpha, const double* E,
                   int64_t lde, double beta, double* D, int64_t ldd, void* stream);

/* bf16 operands (cfg-5 storage), v_mfma_f32_32x32x16_bf16: A, B bf16 (void*), fp32 accumulate,
 * bias fp32 (nullable), C bf16 (c_dtype GNNEA_BF16, rounded once, nearest even) or fp32
 * (GNNEA_F32).  Workspace (split-K slabs) from gnnea_gemm_bf16_ws_bytes; NULL = no split.
 * Fast path: lda, ldb and the operands' contiguous extents % 4 == 0, 8-B aligned A, B. */
int64_t gnnea_gemm_bf16_ws_bytes(int64_t M, int64_t N, int64_t K);
int gnnea_gemm_bf16(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const void* A,
                    int64_t lda, const void* B, int64_t ldb, const float* bias, float beta,
                    void* C, int64_t ldc, int c_dtype, void* ws, int64_t ws_bytes, void* stream);
/* C = act(A·op(B) + bias), beta = 0 (the bf16 Linear + its act, layers/layers.py:121-122):
 * relu in the weight-resident kernel's epilogue (K in (288, 320], tall M), otherwise the product
 * then the act in place.  Workspace as gnnea_gemm_bf16. */
int gnnea_gemm_bf16_act(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const void* A,
                        int64_t lda, const void* B, int64_t ldb, const float* bias, int act,
                        void* C, int64_t ldc, int c_dtype, void* ws, int64_t ws_bytes,
                        void* stream);
/* The backward of a relu Linear through the product that consumed its output Y (MLPDecoder,
 * models/decoders.py; replaces torch's dY·W then threshold_backward(·, Y, 0) and the bias
 * gradient's sum(0) of layers/layers.py:121-122 under autograd): G = bf16(A·op(B)) * relu'(Y),
 * bit-identical to gnnea_gemm_bf16 + gnnea_act_bwd_colsum_bf16's G (the bias gradient: a
 * gnnea_colsum_bf16 pass over G).  A, B, Y, G bf16 row-major.  Only where the weight-resident
 * kernel runs (gnnea_gemm_bf16_dmask_applies: K in (288, 320], M >= 65536, 128 < N <= 4096,
 * N % 4 == 0, 8-B aligned Y / G with ld % 4 == 0), else GNNEA_EINVAL.  Workspace:
 * gnnea_gemm_bf16_dmask_ws_bytes. */
int gnnea_gemm_bf16_dmask_applies(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldy,
                                  int64_t ldg);
int64_t gnnea_gemm_bf16_dmask_ws_bytes(int64_t N, int64_t K);
int gnnea_gemm_bf16_dmask(int trans_b, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                          const void* B, int64_t ldb, const void* Y, int64_t ldy, void* G,
                          int64_t ldg, void* ws, int64_t ws_bytes, void* stream);
/* The forward of that relu Linear keeping 1 bit per element for the backward: C = relu(A·op(B) +
 * bias) bf16 (bit-identical to gnnea_gemm_bf16_act's relu) and its sign bits Mo (byte
 * 20 t + 4 u + g of a row: columns 160 t + 32 u + 8 g + 0..7, bit e set where that column's
 * stored value > 0; ldm >= gnnea_gemm_bf16_mask_ld(N), % 4 == 0); gnnea_gemm_bf16_dmask_bits is
 * gnnea_gemm_bf16_dmask reading them instead of Y.  Same applicability and workspace as
 * gnnea_gemm_bf16_dmask. */
int64_t gnnea_gemm_bf16_mask_ld(int64_t N);
int gnnea_gemm_bf16_relu_mask(int trans_b, int64_t M, int64_t N, int64_t K, const void* A,
                              int64_t lda, const void* B, int64_t ldb, const float* bias, void* C,
                              int64_t ldc, void* Mo, int64_t ldm, void* ws, int64_t ws_bytes,
                              void* stream);
int gnnea_gemm_bf16_dmask_bits(int trans_b, int64_t M, int64_t N, int64_t K, const void* A,
                               int64_t lda, const void* B, int64_t ldb, const void* Mi, int64_t ldm,
                               void* G, int64_t ldg, void* ws, int64_t ws_bytes, void* stream);
/* The fp32 forms of the relu Linear's sign bits (the f16x2 weight-resident ring, K in (288, 320],
 * N <= 336, tall M: gnnea_gemm_f32_mask_applies; workspace gnnea_gemm_f32_mask_ws_bytes):
 * gnnea_gemm_f32_relu_mask = gnnea_gemm_x3_act_f32 with relu, bit for bit, plus the bits (byte
 * 16 t + 2 j + h of a row: columns 112 t + 16 j + 8 h + 0..7; ldm >= gnnea_gemm_f32_mask_ld(N),
 * % 16 == 0, 16-B aligned); gnnea_gemm_f32_dmask_bits = the product times relu'(y) from them
 * (= gnnea_gemm_x3_f32 then gnnea_act_bwd_colsum_f32's G, bit for bit). */
int gnnea_gemm_f32_mask_applies(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldc);
int64_t gnnea_gemm_f32_mask_ld(int64_t N);
int64_t gnnea_gemm_f32_mask_ws_bytes(int64_t N);
int gnnea_gemm_f32_relu_mask(int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                             int64_t lda, const float* B, int64_t ldb, const float* bias, float* C,
                             int64_t ldc, void* Mo, int64_t ldm, void* ws, int64_t ws_bytes,
                             void* stream);
int gnnea_gemm_f32_dmask_bits(int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                              int64_t lda, const float* B, int64_t ldb, const void* Mi,
                              int64_t ldm, float* G, int64_t ldg, void* ws, int64_t ws_bytes,
                              void* stream);
/* A layer's weight AND bias gradients in one pass over its output gradient: C = Aᵀ·B (A [K][M]
 * = dh row-major, B [K][N] = x; the gnnea_gemm_x3_f32 trans_a product, same kernel, same values)
 * and db = column sums of A (fp32 [M]) from a ones column in the kernel's B-tile padding
 * (N % 160 != 0, M, N <= 320, K >= 128: gnnea_gemm_x3_ta_db_applies; workspace
 * gnnea_gemm_x3_ta_db_ws_bytes).  Replaces the separate gnnea_colsum_f32 pass (the bias
 * gradient of layers/layers.py:32,61 under autograd). */
int gnnea_gemm_x3_ta_db_applies(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
int64_t gnnea_gemm_x3_ta_db_ws_bytes(int64_t M, int64_t N, int64_t K);
int gnnea_gemm_x3_ta_db_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                            const float* B, int64_t ldb, float* C, int64_t ldc, float* db,
                            void* ws, int64_t ws_bytes, void* stream);
/* The same for bf16 operands (gnnea_gemm_bf16's trans_a product; C bf16 or fp32 by c_dtype; the
 * workspace of gnnea_gemm_x3_ta_db_ws_bytes). */
int gnnea_gemm_bf16_ta_db_applies(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
int gnnea_gemm_bf16_ta_db(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                          const void* B, int64_t ldb, void* C, int64_t ldc, int c_dtype, float* db,
                          void* ws, int64_t ws_bytes, void* stream);
/* The GCN layer's relu with 1 bit per element kept for the backward (fp32, the slice-major
 * path): gnnea_spmm_sliced_m_f32 = gnnea_spmm_sliced_f32 with act relu, also writing the sign
 * bits of Y (save_m [n_rows][ldm] bytes, ldm >= D / 4: byte q holds elements 4 q .. 4 q + 3, bit
 * e set where Y > 0); gnnea_act_bwd_sliced_bits_f32 = gnnea_act_bwd_sliced_f32 (relu) reading
 * them instead of Y (the same G, bit for bit). */
int gnnea_spmm_sliced_m_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                            int32_t n_rows, int32_t D, const float* Xs, int64_t sstride, float* Y,
                            int64_t ldy, uint8_t* save_m, int64_t ldm, void* stream);
int gnnea_act_bwd_sliced_bits_f32(const float* dY, int64_t lddy, const uint8_t* M, int64_t ldm,
                                  int64_t n, int32_t D, float* Gs, int64_t sstride, void* stream);
/* the bf16 GEMM writing C slice-major (bf16, 128-column slices):
 * element (r, c) at Cs[(c/128)*sstride + r*128 + c%128], sstride % 128 == 0, >= M*128 */
int gnnea_gemm_sliced_bf16(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                           const void* A, int64_t lda, const void* B, int64_t ldb,
                           const float* bias, float beta, void* Cs, int64_t sstride, void* ws,
                           int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------ *
 * a9-a12. Sinkhorn solvers in the reference's scaling form, fp64 arithmetic.
 *   GNNEA_SK_KNOPP : utils/ot_loss.py:5-76 sinkhorn(a, b, M, reg, numItermax, stopThr)
 *   GNNEA_SK_STAB  : SinkhornOT/sinkhorn_loss.py:159-220 sinkhorn_iteration
 *   GNNEA_SK_GEN   : SinkhornOT/sinkhorn_loss.py:223-288 gsinkhorn_iteration
 *   GNNEA_SK_RELAX : SinkhornOT/sinkhorn_loss.py:291-356 forward_relax_sinkhorn_iteration
 * The cost may be stored fp32 (widened exactly, as the reference's .type(torch.DoubleTensor)) or
 * fp64.  Default path: the fp64 kernel matrix K (I*J*8 bytes) lives in `ws`, built once (KNOPP) or
 * at every absorption (STAB family), one sweep over it per iteration.  variant 1 (or J > 16384):
 * log-domain passes with online log-sum-exp, nothing I*J-sized kept.  The host drives the data-dependent loop with
 * gnnea_sinkhorn_iterate() batches and reads the status block (first GNNEA_SK_STATUS_BYTES of ws)
 * between batches.  Kernels of an iteration after the stop condition are no-ops, so
 * over-enqueueing is harmless.
 * ------------------------------------------------------------------------------------------ */
#define GNNEA_SK_KNOPP 0
#define GNNEA_SK_STAB 1
#define GNNEA_SK_GEN 2
#define GNNEA_SK_RELAX 3

/* status block (int64 words at the start of ws) */
#define GNNEA_SK_ST_DONE 0       /* 1 once the loop has stopped */
#define GNNEA_SK_ST_ITERS 1      /* reference's final iteration counter (cpt / ii) */
#define GNNEA_SK_ST_REASON 2     /* 0 running/max-iter, 1 tolerance, 2 numerical-error break */
#define GNNEA_SK_ST_SLOT 3       /* ping-pong slot holding the final scalings */
#define GNNEA_SK_ST_TIMEOUT 16   /* nonzero: a wait between the workgroups of the on-chip KNOPP
                                    kernel timed out (the loop was stopped; results invalid) */
#define GNNEA_SK_STATUS_BYTES 256
/* double words (indices into the block viewed as doubles) */
#define GNNEA_SK_SD_ERR 8        /* KNOPP: last err = ||v * (K^T u) - b|| */
#define GNNEA_SK_SD_TPREV 9      /* STAB family: transport at the previous check */
#define GNNEA_SK_SD_LOSS 10      /* KNOPP: sum P * M */
#define GNNEA_SK_SD_TOL 11       /* the stop threshold (set by init) */
#define GNNEA_SK_SD_TNEW 12      /* STAB family: transport at the last check */

typedef struct gnnea_sinkhorn {
  int mode;         /* GNNEA_SK_* */
  int c_dtype;      /* GNNEA_F32 or GNNEA_F64 */
  int I, J;         /* cost is I x J */
  int64_t ldc;      /* row stride of C in elements */
  const void* C;    /* cost matrix (M for KNOPP) */
  const double* a;  /* I: source weights (a / mu) */
  const double* b;  /* J: target weights (b / nu) */
  double eps;       /* reg (KNOPP) or epsilon */
  double p;         /* lambda/(lambda+eps) for GEN / RELAX; ignored otherwise */
  double tol;       /* stopThr (KNOPP) or tol */
  int max_iter;     /* numItermax / numIterMax */
  int iters_run;    /* iterations enqueued so far (read by gnnea_sinkhorn_finish) */
  int variant;      /* 0: scaling form with the fp64 K resident in ws (J <= 16384; KNOPP on
                          chip where the blocks fit the CUs);
                       1: log-domain passes recomputing every term from C (no I*J state, any J;
                          used automatically above J = 16384; KNOPP: the fused sweep, one pass
                          over C per iteration, for J <= 16384 fp32 / 8192 fp64 C);
                       GNNEA_SK_AUTO (3, the Python default): KNOPP on chip where it fits, else
                          the fused log-domain sweep, else variant 0 / 1 as above; the STAB
                          family as variant 0 (sharded KNOPP: as variant 0) */
  int flags;        /* bit set: GNNEA_SK_NO_ONCHIP: never take the on-chip KNOPP path (the host's
                       retry after an inter-workgroup wait timed out; A/B measurements);
                       GNNEA_SK_TWO_PASS: KNOPP log domain as the two-pass form instead of the
                       fused sweep (the parity tests compare the two);
                       GNNEA_SK_DEBUG_SPIN: the on-chip kernel's inter-workgroup waits get a
                       zero time budget, so it times out (tests of the timeout path) */
  void* ws;         /* device workspace of gnnea_sinkhorn_ws_bytes(I, J) bytes */
} gnnea_sinkhorn;

#define GNNEA_SK_NO_ONCHIP 1
#define GNNEA_SK_TWO_PASS 2
#define GNNEA_SK_DEBUG_SPIN 4
#define GNNEA_SK_AUTO 3

int64_t gnnea_sinkhorn_ws_bytes(int I, int J);
int gnnea_sinkhorn_init(const gnnea_sinkhorn* prob, void* stream);
/* enqueue iterations [first, first+count) (count >= 1) */
int gnnea_sinkhorn_iterate(const gnnea_sinkhorn* prob, int first, int count, void* stream);
/* plan (I x J, plan_dtype, row stride ldp, nullable): KNOPP: P = diag(u) K diag(v);
 * others: the last K = clamp(exp((u+v-C)/eps), 0, 1e30).  Also writes row sums (I) and column
 * sums (J) of the plan into row_sum/col_sum (nullable, fp64) and the scalars into the status
 * block. */
int gnnea_sinkhorn_finish(const gnnea_sinkhorn* prob, void* plan, int plan_dtype, int64_t ldp,
                          double* row_sum, double* col_sum, void* stream);
/* which device path gnnea_sinkhorn_* take for this problem on the current device (host-side
 * query, no launch): GNNEA_SK_PATH_SWEEP -- the scaling form streaming the resident fp64 K
 * (k_sk_sweep); GNNEA_SK_PATH_ONCHIP -- KNOPP with K held in registers + LDS by one persistent
 * launch per batch (k_sk_res: I x J fits P x Q <= #CUs blocks of 144 x 256); GNNEA_SK_PATH_LOG --
 * the log-domain passes (variant 1 or J > 16384).  GNNEA_SK_RESIDENT=0 in the environment
 * disables the on-chip path (A/B measurements).  Negative on an invalid problem. */
#define GNNEA_SK_PATH_SWEEP 0
#define GNNEA_SK_PATH_ONCHIP 1
#define GNNEA_SK_PATH_LOG 2
int gnnea_sinkhorn_path(const gnnea_sinkhorn* prob);

/* §8e. KNOPP (utils/ot_loss.py:5-76) with the cost rows sharded over W ranks (rank r holds a
 * contiguous block of rows, rank order = row order).  `prob` is the rank's own problem: I = its
 * rows, C = its cost rows, a = its rows' source weights, b = all J target weights, mode KNOPP.
 * Per iteration it (host loop, every rank):
 *   gnnea_sinkhorn_shard_colpart(prob, it, pair)      pair: gnnea_sinkhorn_shard_pair_len doubles
 *   <all-gather the W pair rows into pairs [W][pair_len], rank order>
 *   gnnea_sinkhorn_shard_step(prob, it, pairs, W)     g, stop decisions, its row pass
 * Every rank takes the same decisions from the same gathered data; the status block (ws) is
 * read as for gnnea_sinkhorn_iterate.  After the loop (iters_run = iterations enqueued):
 *   gnnea_sinkhorn_shard_flag(prob, flag)  -> all-gather the W flags ->
 *   gnnea_sinkhorn_shard_close(prob, flags, W)        settles the last iteration's u check
 *   gnnea_sinkhorn_shard_finish(...)                  its plan rows / row sums, loss_part[1] =
 *                                                     its sum P.M, col_part[J] = its column sums
 * The caller sums loss_part and col_part over the ranks. */
int64_t gnnea_sinkhorn_shard_ws_bytes(int I_local, int J);
/* doubles per rank of the gathered row ("pair"): J + 2 for the scaling form (variant 0,
 * J <= 16384: fp64 K of the rank's rows resident, column sums gathered) or 2J + 2 for the
 * log-domain form (variant 1 or wider J: (max, sum-exp) pairs); the flag sits at index J resp. 2J */
int gnnea_sinkhorn_shard_pair_len(const gnnea_sinkhorn* prob);
int gnnea_sinkhorn_shard_init(const gnnea_sinkhorn* prob, int I_global, void* stream);
int gnnea_sinkhorn_shard_colpart(const gnnea_sinkhorn* prob, int it, double* pair, void* stream);
int gnnea_sinkhorn_shard_step(const gnnea_sinkhorn* prob, int it, const double* pairs, int W,
                              void* stream);
int gnnea_sinkhorn_shard_flag(const gnnea_sinkhorn* prob, double* flag, void* stream);
int gnnea_sinkhorn_shard_close(const gnnea_sinkhorn* prob, const double* flags, int W,
                               void* stream);
int gnnea_sinkhorn_shard_finish(const gnnea_sinkhorn* prob, void* plan, int plan_dtype,
                                int64_t ldp, double* row_sum, double* loss_part, double* col_part,
                                void* stream);

/* ------------------------------------------------------------------------------------------ *
 * §8f #1. L1 (cityblock) distance search.  scipy.spatial.distance.cdist(.., 'cityblock') as
 * used by BaseModel.get_neg (models/models_ea.py:19-30), get_hits (utils/eval_utils.py:71-98)
 * and UEAModel.generate_pairs (models/models_ea.py:143-167).  fp32 rows, fp64 sums of
 * |q_d - x_d| in d order: bit-identical to scipy's fp64 distances.  Row-major, ld in elements.
 * ------------------------------------------------------------------------------------------ */
/* keys[q*ldk + x] = (float) L1(Q[q], X[x])   (nq x nx; monotone rounding of the exact value) */
int gnnea_l1_keys_f32(const float* Q, int64_t ldq, int32_t nq, const float* X, int64_t ldx,
                      int32_t nx, int32_t D, float* keys, int64_t ldk, void* stream);
/* out[j] = sum_d |X[a[j]][d] - X[b[j]][d]| in fp64, j < n (row indices int64, in range: the
 * caller checks).  The per-term partial distances of the column-sharded EA margin loss: every
 * rank sums its column block, one all-reduce of the n partials gives the distances
 * (models/models_ea.py:103-123 over a row-sharded embedding, gnnea/dist_loss.py). */
int gnnea_l1_terms_f32(const float* X, int64_t ldx, int32_t D, int64_t n, const int64_t* a,
                       const int64_t* b, double* out, void* stream);
/* Bandwidth anchors of the bench (csrc/ubench.hip; measurement aids, no reference call):
 *   gnnea_ub_copy:   dst = src, bytes % 16 == 0, 16-B aligned, `blocks` workgroups of 256 striding;
 *                    flags: GNNEA_UB_NT nontemporal loads / stores, GNNEA_UB_DEEP 8 (not 4)
 *                    16-B accesses in flight per lane, GNNEA_UB_READ_ONLY loads only (dst gets one
 *                    word per thread, blocks * 1 KB <= bytes);
 *   gnnea_ub_gather: reads the rows idx[0..n) of a row-major table (row_bytes % 8 == 0, <= 2 KB)
 *                    as 8-B chunks (mode 0), or in the access shapes of the bf16 GAT passes
 *                    (mode GNNEA_UB_GAT_*), writes one value per 64 rows to out[(n + 63) / 64]. */
#define GNNEA_UB_NT 1
#define GNNEA_UB_DEEP 2
#define GNNEA_UB_READ_ONLY 4
int gnnea_ub_copy(const void* src, void* dst, int64_t bytes, int32_t blocks, int32_t flags,
                  void* stream);
#define GNNEA_UB_GAT_WIN12 1 /* 600-B rows, a 12-B window per lane (the bf16 GAT passes) */
#define GNNEA_UB_GAT_V16 2   /* rows padded to a multiple of 16 B, 16 B per lane */
int gnnea_ub_gather(const void* table, int64_t row_bytes, const int32_t* idx, int64_t n,
                    float* out, int32_t mode, void* stream);
/* out[i] = L1(A[i], B[i]) in fp64 (the diagonal of cdist(A, B)) */
int gnnea_l1_pairs_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int32_t n,
                       int32_t D, double* out, void* stream);
/* rank[q] = #{x : L1(Q[q],X[x]) < diag[q]} + #{x < q : L1(Q[q],X[x]) == diag[q]}: the position of
 * x = q in a stable argsort of row q (get_hits' rank_index).  rank is zeroed by the call. */
int gnnea_l1_rank_f32(const float* Q, int64_t ldq, int32_t nq, const float* X, int64_t ldx,
                      int32_t nx, int32_t D, const double* diag, int32_t* rank, void* stream);
/* The same count over one block of the candidates, X = candidates [x_off, x_off + nx): rank[q]
 * = #{x : d < diag[q] or (d == diag[q] and x_off + x < q)} (no nq <= nx requirement).  The
 * row-sharded get_hits (gnnea/dist_search.py) sums the blocks' counts over the ranks; replaces the
 * same utils/eval_utils.py:71-98 argsort position as gnnea_l1_rank_f32. */
int gnnea_l1_rank_range_f32(const float* Q, int64_t ldq, int32_t nq, const float* X, int64_t ldx,
                            int32_t nx, int32_t D, const double* diag, int32_t x_off, int32_t* rank,
                            void* stream);
/* Per row q of keys (from gnnea_l1_keys_f32 of the same Q, X): the K smallest exact distances
 * ordered by (distance, index), entries [skip, K) written to out_idx / out_dist (nullable) rows
 * of stride ldo.  get_neg: K = k+1, skip = 1.  K <= 512.  *overflow (nullable) counts rows where
 * more than 1024 - K candidates shared the K-th fp32 key (selection then keeps the lowest
 * indices of that key). */
int gnnea_topk_rows_f32(const float* keys, int64_t ldk, int32_t nq, int32_t nx, int32_t K,
                        const float* Q, int64_t ldq, const float* X, int64_t ldx, int32_t D,
                        int32_t skip, int64_t* out_idx, double* out_dist, int32_t ldo,
                        int32_t* overflow, void* stream);

/* ------------------------------------------------------------------------------------------ *
 * §8f #2. Entity-alignment margin loss (EAModel.get_loss, models/models_ea.py:103-123; the same
 * body in UEAModel.get_loss :169-183).  out [N, D] fp32 rows of stride ld; left/right [t] pair
 * rows; neg_* [t*k] negative-pair rows (int64).  Terms j in [0, M), M = 2tk + t: side-1
 * negatives, side-2 negatives, then the pairs.
 * Forward: A[t] = |out[left]-out[right]|_1, h[2tk] = relu(A_i + 1 - |out[neg_l]-out[neg_r]|_1)
 * (loss = sum(h) / (2tk), summed by the caller) and the integer multipliers m[M] the backward
 * needs (-[h>0] per negative, number of active terms per pair).
 * Backward: grad (N x ldg, caller-zeroed) += scale * grad_loss[0] *
 *   sum over the incidence of each row r of m_j * sgn(out[r] - out[other end of term j]).
 * The incidence CSR (inc_rowptr, inc_ent) is gnnea_coo_to_csr of
 *   rows = [nl1 | nl2 | left | nr1 | nr2 | right]  (2M entries),  cols = 0 .. 2M-1
 * (entry p < M: row is term p's first end; p >= M: term p-M's second end).  Its rows are cut
 * into work items {row, beg, end, slot} (int32 x 4, entries [beg, end) of inc_ent, at most a
 * few hundred each): slot = -1 for a row with one item (written to grad directly), else a
 * distinct scratch slot (scratch: n_slots x D floats); long rows are listed in long_rows with
 * their slots long_ptr[w] .. long_ptr[w+1]-1 in order, and summed by a second kernel.  All of it
 * depends on the index arrays only (built once per negative set).  scale = 1 / (2tk).  D <= 1024.
 * ------------------------------------------------------------------------------------------ */
int gnnea_margin_fwd_f32(const float* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                         const int64_t* left, const int64_t* right, const int64_t* neg_left,
                         const int64_t* neg_right, const int64_t* neg2_left,
                         const int64_t* neg2_right, float* A, float* h, float* m, void* stream);
int gnnea_margin_bwd_f32(const float* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                         const int64_t* left, const int64_t* right, const int64_t* neg_left,
                         const int64_t* neg_right, const int64_t* neg2_left,
                         const int64_t* neg2_right, const float* m, const int32_t* inc_ent,
                         const int32_t* items, int32_t n_items, const int32_t* long_rows,
                         const int32_t* long_ptr, int32_t n_long, float* scratch,
                         const float* grad_loss, float scale, float* grad, int64_t ldg,
                         void* stream);

/* Sign-code variant (D % 4 == 0, ld % 4 == 0, out 16-B aligned): the forward also writes, per
 * term j, codes[j*sb + q] for q < ceil(D/4): 2 bits per column of columns 4q..4q+3, the 2-bit
 * two's complement of sgn(out[a] - out[b]) (01: +1, 11: -1, 00: equal; a/b the term's
 * first/second end); sb >= D/4.
 * The backward then reads those codes instead of the rows (no out / index arguments): the same
 * sum with the same multipliers in the same order, bit-identical to gnnea_margin_bwd_f32. */
int gnnea_margin_fwd_code_f32(const float* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                              const int64_t* left, const int64_t* right, const int64_t* neg_left,
                              const int64_t* neg_right, const int64_t* neg2_left,
                              const int64_t* neg2_right, float* A, float* h, float* m,
                              void* codes, int64_t sb, void* stream);
int gnnea_margin_bwd_code_f32(int32_t D, int32_t t, int32_t k, const float* m, const void* codes,
                              int64_t sb, const int32_t* inc_ent, const int32_t* items,
                              int32_t n_items, const int32_t* long_rows, const int32_t* long_ptr,
                              int32_t n_long, float* scratch, const float* grad_loss, float scale,
                              float* grad, int64_t ldg, void* stream);
/* The same two calls over bf16 rows (cfg-5 storage; the reference model converted with
 * .bfloat16()): out is bf16 [N][ld], the rows widened exactly to fp32, every sum as in the _f32
 * calls on the fp32 copy of the rows; grad is bf16 [N][ldg], each value rounded once (nearest
 * even) from the fp32 gradient -- bit-identical to the _f32 calls on out.float() followed by a
 * cast of their gradient.  out 8-B aligned, ld % 4 == 0. */
int gnnea_margin_fwd_code_bf16(const void* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                               const int64_t* left, const int64_t* right,
                               const int64_t* neg_left, const int64_t* neg_right,
                               const int64_t* neg2_left, const int64_t* neg2_right, float* A,
                               float* h, float* m, void* codes, int64_t sb, void* stream);
int gnnea_margin_bwd_code_bf16(int32_t D, int32_t t, int32_t k, const float* m, const void* codes,
                               int64_t sb, const int32_t* inc_ent, const int32_t* items,
                               int32_t n_items, const int32_t* long_rows, const int32_t* long_ptr,
                               int32_t n_long, float* scratch, const float* grad_loss,
                               float scale, void* grad, int64_t ldg, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GNNEA_H */
