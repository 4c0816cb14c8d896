/*
 * ppgat.h -- C ABI of the MI355X-native GAT message-passing library (libppgat.so).
 *
 * This is the drop-in boundary beneath the reference's GAT layer call site
 *     x = conv(x, edge_index)          scripts/train_gat_pyg.py:86-87
 *     x = gat(x, edge_index)           scripts/train_gat_custom.py:113-114
 * i.e. torch_geometric.nn.GATConv(hidden, hidden, heads=H, dropout=p,
 * add_self_loops=False, concat=False)  (scripts/train_gat_pyg.py:77) and
 * SimpleGATLayer.forward               (scripts/train_gat_custom.py:75-93).
 *
 * Conventions
 *  - every pointer is DEVICE memory allocated by the caller (the library never
 *    allocates or frees device memory; workspace sizes are queried first);
 *  - float tensors are fp32, row-major, contiguous; node rows are [N, H, C];
 *  - indices are int32 after preprocessing (edge_index stays int64 on input);
 *  - work is enqueued on `stream` (a hipStream_t passed as void*); no host sync
 *    except where a function says so;
 *  - return 0 on success, nonzero on error; ppgat_last_error() gives a
 *    thread-local message.  Unsupported shapes return PPGAT_ERR_UNSUPPORTED.
 *
 * Semantics (mode):
 *  PPGAT_MODE_PYG    : e = leaky_relu(s_src[j] + s_dst[i], slope);
 *                      alpha = exp(e - max_i) / (sum exp(e - max_i) + 1e-16);
 *                      out_i = mean_h sum_j alpha * h_j + bias    (PyG GATConv, concat=False)
 *  PPGAT_MODE_CUSTOM : e = clamp(leaky_relu(z, 0.2), -10, 10); alpha = exp(e) / (sum exp(e) + 1e-9);
 *                      out_i = sum_j alpha * h_j        (SimpleGATLayer, heads must be 1, bias NULL)
 *  Dropout on alpha (training) uses a counter-based hash of (seed, original edge id, head):
 *  keep iff u(seed, eid, head) >= p, kept values scaled by 1/(1-p).  The same mask is
 *  regenerated in the backward pass and restated bit-for-bit in oracle/gat_oracle.py.
 */
#ifndef PPGAT_H
#define PPGAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPGAT_OK 0
#define PPGAT_ERR_INVALID 1
#define PPGAT_ERR_UNSUPPORTED 2
#define PPGAT_ERR_HIP 3

#define PPGAT_MODE_PYG 0
#define PPGAT_MODE_CUSTOM 1

/* Library identification: 2 = ppgat_schedule carries n_long_items (schedule counts int32[4]);
 * 3 = ppgat_fwd / ppgat_bwd / ppgat_bwd_edges carry seed_used, ppgat_adam_step_device takes one
 * step pointer per tensor. */
int ppgat_version(void);
const char* ppgat_last_error(void);

/* Channels per head the fused kernels are instantiated for (C in {4,8,...,256}). */
int ppgat_supported_channels(int channels);

/* ---- graph preprocessing ------------------------------------------------
 * Replaces: the COO edge_index consumed by GATConv.propagate / index_add_
 * (scripts/train_gat_pyg.py:139-147 builds it; train_gat_custom.py:78,86-92 uses it).
 * Builds, from edge_index int64 [2,E] (row 0 = src, row 1 = dst):
 *   CSR by destination : rowptr[N+1], col[E] (= src), csr_eid[E] (original column id)
 *   CSC by source      : colptr[N+1], row[E] (= dst), csc_eid[E], csc2csr[E] (CSR slot of each CSC edge)
 * In-segment order is the original column order (stable), so results are deterministic.
 * bad_count (device int32[1]) receives the number of out-of-range indices (0 = valid).
 */
int ppgat_csr_workspace_bytes(int64_t n_nodes, int64_t n_edges, size_t* bytes);
int ppgat_csr_build(const int64_t* edge_index, int64_t n_edges, int64_t n_nodes,
                    int32_t* rowptr, int32_t* col, int32_t* csr_eid,
                    int32_t* colptr, int32_t* row, int32_t* csc_eid, int32_t* csc2csr,
                    int32_t* bad_count, void* workspace, size_t workspace_bytes, void* stream);

/* ---- work schedule -------------------------------------------------------
 * Cuts the rows of a CSR/CSC (ptr[N+1]) into work items of at most max_edges edges for
 * the fused kernels: rows with deg > max_edges ("hubs") become ceil(deg/max_edges)
 * pieces listed first (hubs in row order, pieces merged deterministically afterwards),
 * then every other row as one item in descending-degree order (longest work first).
 * Capacities: items <= ppgat_schedule_capacity(), hub_row <= N, hub_ptr <= N+1.
 * counts (device int32[4]) receives {n_hubs, n_hub_items, n_items, n_long_rows}, n_long_rows
 * = rows that are not hubs and have more than PPGAT_SHORT_ITEM_EDGES edges; the caller
 * reads it once (a one-time host sync per static graph) to fill a ppgat_schedule, with
 * n_long_items = n_hub_items + n_long_rows.
 */
#define PPGAT_SHORT_ITEM_EDGES 16
typedef struct ppgat_schedule {
  const int32_t* item_row;  /* [n_items] row (dst for CSR, src for CSC) */
  const int32_t* item_beg;  /* [n_items] first edge slot */
  const int32_t* item_end;  /* [n_items] one past the last edge slot */
  int64_t n_items;
  int64_t n_hub_items;      /* items [0, n_hub_items) are hub pieces */
  const int32_t* hub_row;   /* [n_hubs] */
  const int32_t* hub_ptr;   /* [n_hubs+1] piece (= item) ranges per hub */
  int64_t n_hubs;
  int64_t n_long_items;     /* items [0, n_long_items) have > PPGAT_SHORT_ITEM_EDGES edges; the
                               rest (descending degree) are run four per wavefront (heads = 1).
                               -1: unknown (every item takes the one-per-wavefront path) */
} ppgat_schedule;

int64_t ppgat_schedule_capacity(int64_t n_nodes, int64_t n_edges, int32_t max_edges);
int ppgat_schedule_workspace_bytes(int64_t n_nodes, size_t* bytes);
int ppgat_schedule_build(const int32_t* ptr, int64_t n_nodes, int64_t n_edges, int32_t max_edges,
                         int32_t* item_row, int32_t* item_beg, int32_t* item_end,
                         int32_t* hub_row, int32_t* hub_ptr, int32_t* counts,
                         void* workspace, size_t workspace_bytes, void* stream);

/* ---- per-node attention terms -------------------------------------------
 * Replaces: PyG alpha_src = (x * att_src).sum(-1), alpha_dst likewise (GATConv.forward);
 *           custom (h[src]*a_src).sum(-1) / (h[dst]*a_dst).sum(-1) (train_gat_custom.py:79),
 *           hoisted from edges to nodes.
 * h [N,H,C], att_src/att_dst [H,C] -> s_src/s_dst [N,H].
 */
int ppgat_node_scores(const float* h, const float* att_src, const float* att_dst,
                      int64_t n_nodes, int heads, int channels,
                      float* s_src, float* s_dst, void* stream);

/* ---- fused forward -------------------------------------------------------
 * Replaces: GATConv edge_update + softmax + dropout + propagate/SumAggregation + head mean + bias
 *           (train_gat_pyg.py:77,87 -> PyG), and train_gat_custom.py:78-93.
 * dst_sched: schedule over the CSR by destination (rowptr).  Writes out [N,C], the
 * per-(node,head) softmax state m [N,H] and inv_l = 1/(l+eps) [N,H] (saved for the
 * backward), and agg [N,H,C] (per-head aggregate) when agg != NULL (required for heads > 1
 * training).  workspace: hub-piece partials, ppgat_fwd_workspace_bytes().
 * seed_used (device uint64[1], nullable; written when dropout_p > 0): the effective mask seed
 * (seed folded with the dropout epoch at the time the forward runs).  Passing it to the
 * backward below makes the backward regenerate exactly the forward's mask even if the epoch
 * advances in between (ppgat_dropout_advance from another replayed graph, a recompute).
 */
int ppgat_fwd_workspace_bytes(int64_t n_hub_items, int heads, int channels, size_t* bytes);
int ppgat_fwd(const ppgat_schedule* dst_sched, const int32_t* col, const int32_t* csr_eid,
              int64_t n_nodes, int64_t n_edges, int heads, int channels,
              const float* h, const float* s_src, const float* s_dst, const float* bias,
              int mode, float negative_slope, float dropout_p, uint64_t seed, uint64_t* seed_used,
              float* out, float* m, float* inv_l, float* agg,
              void* workspace, size_t workspace_bytes, void* stream);

/* ---- fused backward ------------------------------------------------------
 * Replaces: autograd of the ops above (index_put_ accumulate, mul backward, scatter
 *           backward; 34%+25%+11.5% of the reference CPU step).
 * src_sched: schedule over the CSC by source (colptr).  Given grad_out [N,C] returns
 * grad_h [N,H,C] (message term plus the attention-logit terms ds_src (x) att_src +
 * ds_dst (x) att_dst), grad_att_src/grad_att_dst [H,C] and, when grad_bias != NULL,
 * grad_bias [C] = column sums of grad_out.  Atomic-free and
 * deterministic (segment-owned sums in a fixed order).  agg may be NULL when heads == 1
 * (out - bias is used).  seed_used: the forward's ppgat_fwd seed_used (nullable: then seed is
 * folded with the current dropout epoch).
 */
int ppgat_bwd_workspace_bytes(int64_t n_nodes, int64_t n_edges, int64_t n_hub_items, int heads, int channels,
                              size_t* bytes);
int ppgat_bwd(const ppgat_schedule* src_sched, const int32_t* rowptr, const int32_t* row,
              const int32_t* csc_eid, const int32_t* csc2csr,
              int64_t n_nodes, int64_t n_edges, int heads, int channels,
              const float* h, const float* s_src, const float* s_dst,
              const float* att_src, const float* att_dst, const float* bias,
              const float* out, const float* agg, const float* m, const float* inv_l,
              const float* grad_out,
              int mode, float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used,
              float* grad_h, float* grad_att_src, float* grad_att_dst, float* grad_bias,
              void* workspace, size_t workspace_bytes, void* stream);

/* ---- backward, staged (multi-GPU: collectives go between the stages) ----------
 * ppgat_bwd == prologue -> edges -> epilogue on one device.  Row-sharded:
 *  prologue over the rank's own destination rows -> nstate (all-gathered with grad_out),
 *  edges over the rank's own SOURCE rows (CSC slice; `row` indexes the gathered dst space,
 *  dz_slot gives each edge's position in a [world x max-local-edges] dz buffer that is then
 *  reduce-scattered), epilogue over the own destination rows with the local dz.
 *  dz_slot == NULL: each edge's dz goes to its own CSC position (read back through
 *  ppgat_bwd_dst_sum_csc); csc2csr as dz_slot gives the CSR-order layout of ppgat_bwd_dst_sum.
 *  nstate: [N_dst, H] float4 {s_dst, m, inv_l, D}.  grad_bias (nullable) needs bias_part
 *  [ppgat_bwd_partial_rows(n) * C]; epilogue part: [ppgat_bwd_partial_rows(n) * 2*H*C].
 */
int64_t ppgat_bwd_partial_rows(int64_t n_nodes);
int ppgat_bwd_prologue(const float* grad_out, const float* out, const float* agg, const float* bias,
                       const float* s_dst, const float* m, const float* inv_l, int64_t n_nodes, int heads,
                       int channels, int mode, float* nstate, float* grad_bias, float* bias_part, void* stream);
int ppgat_bwd_edges(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                    const int32_t* dz_slot, int64_t n_edges, int heads, int channels, const float* h,
                    const float* s_src, const float* nstate, const float* grad_out, int mode, float negative_slope,
                    float dropout_p, uint64_t seed, const uint64_t* seed_used, float* grad_h, int64_t ld_grad_h,
                    float* ds_src,
                    int64_t ld_ds_src, float* dz, void* workspace, size_t workspace_bytes, void* stream);
/* ds_dst[i*ld + h] = sum of dz over the CSR segment of destination i, walked with the
 * forward (destination) schedule so hub rows are split; workspace >= n_hub_items*heads*4
 * bytes (hub partials, added in piece order: deterministic).  With
 * grad_h and ds_src/ds_dst written side by side into one [N, ld] buffer
 * D = [dh_msg | ds_src | ds_dst], the projection gradients follow from two GEMMs with
 * W_aug = [W; A_src; A_dst] (A_src[h] = sum_c att_src[h,c] W[h*C+c, :]):
 *   dx = D W_aug,   D^T x = [dh_msg^T x ; ds_src^T x ; ds_dst^T x]  (ppgat_gemm_tn with V),
 *   dW = dh_msg^T x + att_src (x) (ds_src^T x) + att_dst (x) (ds_dst^T x),
 *   datt_src[h] = W_h (ds_src^T x)[h],  datt_dst[h] = W_h (ds_dst^T x)[h]. */
int ppgat_bwd_dst_sum(const ppgat_schedule* fwd_sched, int64_t n_nodes, int heads, const float* dz, float* ds_dst,
                      int64_t ld_ds_dst, void* workspace, size_t workspace_bytes, void* stream);
/* Same sums with dz in CSC (source) order -- the layout ppgat_bwd_edges writes when dz_slot is
 * NULL (contiguous per-edge stores instead of a 4-B scatter per edge): CSR slot k of a
 * destination reads dz[csr2csc[k]], csr2csc = the inverse of ppgat_csr_build's csc2csr
 * (ppgat_invert_index).  Same summation order, so the result equals ppgat_bwd_dst_sum's on the
 * CSR-order layout bit for bit. */
int ppgat_bwd_dst_sum_csc(const ppgat_schedule* fwd_sched, int64_t n_nodes, int64_t n_edges, int heads,
                          const float* dz, const int32_t* csr2csc, float* ds_dst, int64_t ld_ds_dst,
                          void* workspace, size_t workspace_bytes, void* stream);
/* inverse[index[k]] = k for a permutation index of [0, n) (int32). */
int ppgat_invert_index(const int32_t* index, int64_t n, int32_t* inverse, void* stream);
int ppgat_bwd_epilogue(const int32_t* rowptr, int64_t n_nodes, int heads, int channels, const float* h,
                       const float* att_src, const float* att_dst, const float* ds_src, const float* dz,
                       float* grad_h, float* grad_att_src, float* grad_att_dst, float* part, void* stream);

/* ---- loss of the training step ---------------------------------------------
 * Replaces: pos = (U[u]*I[i]).sum(-1); neg = (U[u]*I[j]).sum(-1); BPR
 *           -log(sigmoid(pos-neg)+1e-8).mean() (loss_kind 0) or BCE-with-logits over
 *           [pos; neg] with labels [1; 0] (loss_kind 1)  -- scripts/train_gat_pyg.py:313-322,
 *           and its autograd (gather backward = index_put_ accumulate).
 * Z [n_rows, C]; node id v (users [0, n_users), items n_users + i) lives in row v, or in
 * row row_map[v] when row_map != NULL (int32 [n_users + n_items]; the row-sharded path keeps
 * the gathered Z in a padded per-rank layout).  A user whose row_map entry is -1 is not held
 * by this caller: its triples contribute nothing (loss 0, no gradient), while the mean still
 * divides by S -- the row-sharded loss evaluates the triples of its own users only and
 * the ranks' losses add up to the reference's.  u, i, j int64 [S].
 * Forward writes the scalar mean loss and coef [S, 2] (dloss/dpos, dloss/dneg); the
 * backward writes the full grad_Z [N, C] (zero rows included) = grad_loss * sum of the
 * per-triple contributions, deterministically (sorted contributions, ordered sums).
 * Indices outside their range are clamped and counted into bad_count (device int32[1],
 * nullable; zeroed by the call) so the caller can raise without a host sync here.
 */
int ppgat_bpr_workspace_bytes(int64_t n_rows, int64_t n_samples, int channels, size_t* bytes);
int ppgat_bpr_fwd(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                  int channels, const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples,
                  int loss_kind, float* loss, float* coef, int32_t* bad_count, void* workspace,
                  size_t workspace_bytes, void* stream);
int ppgat_bpr_bwd(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                  int channels, const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples,
                  const float* coef, const float* grad_loss, float* grad_Z,
                  void* workspace, size_t workspace_bytes, void* stream);
/* ppgat_bpr_bwd in two calls: the part that depends on the triples only (their destination
 * rows, sorted; the touched-row marks) and the rest.  The first may run on another stream while
 * the model computes Z (train_gat_pyg.py:313-322 samples the triples before the forward); the
 * second must be stream-ordered after it and after ppgat_bpr_fwd, on the same workspace, with
 * the same sizes, row_map and u, i, j.  Same result as ppgat_bpr_bwd, bit for bit. */
int ppgat_bpr_bwd_prepare(int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map, int channels,
                          const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples,
                          void* workspace, size_t workspace_bytes, void* stream);
int ppgat_bpr_bwd_prepared(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                           int channels, const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples,
                           const float* coef, const float* grad_loss, float* grad_Z,
                           void* workspace, size_t workspace_bytes, void* stream);
/* ppgat_bpr_bwd (row_map NULL, after ppgat_bpr_fwd on the same workspace) that also does the
 * backward prologue of the GAT layer whose output Z is (heads = 1; the last conv of
 * train_gat_pyg.py:86-87 feeding the loss of :313-322) -- ppgat_bwd_prologue's outputs for that
 * layer from grad_Z while its rows are on chip, instead of a second pass over grad_Z and Z:
 *   prev_nstate[r] = {prev_s_dst[r], prev_m[r], prev_inv_l[r], prev_gscale <dZ_r, Z_r - prev_bias>}
 *   prev_grad_bias = sum_r dZ_r                    (prev_bias / prev_grad_bias nullable)
 * Z_r is loaded with the row's last contributions, so the dot adds no round trip.  grad_Z bit
 * for bit that of ppgat_bpr_bwd; deterministic. */
int ppgat_bpr_bwd_producer(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, int channels,
                           const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples, const float* coef,
                           const float* grad_loss, float* grad_Z, const float* prev_bias, const float* prev_s_dst,
                           const float* prev_m, const float* prev_inv_l, float prev_gscale, float* prev_nstate,
                           float* prev_grad_bias, void* workspace, size_t workspace_bytes, void* stream);

/* ---- projection weight gradient ----------------------------------------------
 * Replaces: the weight (and bias) gradient of torch.nn.Linear in GATConv.lin /
 *           SimpleGATLayer.lin (train_gat_custom.py:66,77) and PyGGAT.item_proj
 *           (train_gat_pyg.py:74,81): out[M,K] = A[N,M]^T B[N,K]; colsum[M] = sum_n A[n,:]
 *           when colsum != NULL; vout[nv, K] = V[N, nv]^T B when nv > 0 (nv <= 16).
 *           Row strides lda/ldb/ldv (floats; lda, ldb multiples of 4).  fp32 in, fp32 MFMA
 *           (exact fp32 FMA), N split over workgroups with an ordered reduction of the
 *           partials (deterministic).
 */
int ppgat_gemm_tn_workspace_bytes(int64_t n, int m, int k, int nv, size_t* bytes);
int ppgat_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t n, int m, int k, float* out,
                  float* colsum, const float* V, int64_t ldv, int nv, float* vout,
                  void* workspace, size_t workspace_bytes, void* stream);

/* Same as ppgat_gemm_tn with B given as two row segments: rows [0, split) from b0 (ldb0),
 * rows [split, n) from b1 (row - split, ldb1) -- x = cat(user_emb, item_proj(feats))
 * (train_gat_pyg.py:79-82) without materialising the concatenation. */
int ppgat_gemm_tn_seg(const float* A, int64_t lda, const float* b0, int64_t ldb0, const float* b1, int64_t ldb1,
                      int64_t split, int64_t n, int m, int k, float* out, float* colsum, const float* V, int64_t ldv,
                      int nv, float* vout, void* workspace, size_t workspace_bytes, void* stream);

/* ---- fused projection (matrix cores) ------------------------------------------------
 * Replaces: h = GATConv.lin(x) (PyG Linear, no bias; train_gat_pyg.py:77) /
 *           SimpleGATLayer.lin (train_gat_custom.py:66,77) followed by the node attention
 *           terms (alpha_src/alpha_dst; custom :79), and PyGGAT.item_proj (train_gat_pyg.py:74,81):
 *   y[r, :] = x_r W^T (+ bias),   x_r = x0[r] for r < split, x1[r - split] otherwise
 *   s_src[r] = y[r] . att_src,  s_dst[r] = y[r] . att_dst   when att_src != NULL (heads = 1)
 * W [out_cols, k] row-major (ldw); k <= 128 and k % 4 == 0; out_cols == 128.  Row strides in
 * floats, multiples of 4, 16-byte aligned rows.  fp32 MFMA (exact fp32 FMA chains). */
int ppgat_project_supported(int k, int out_cols);
int ppgat_project(const float* x0, int64_t ldx0, const float* x1, int64_t ldx1, int64_t split, int64_t n, int k,
                  const float* w, int64_t ldw, int out_cols, const float* bias, const float* att_src,
                  const float* att_dst, float* y, int64_t ldy, float* s_src, float* s_dst, void* stream);
/* Input gradient of the layer (heads = 1), from the message gradient D [n, k] (ldd) and the
 * node logit gradients S [n, 2] = {ds_src, ds_dst} (lds) of ppgat_bwd_edges +
 * ppgat_bwd_dst_sum:
 *   dx = D W + ds_src (x) (att_src W) + ds_dst (x) (att_dst W)
 * W [k, out_cols] row-major = lin.weight; k <= 128, out_cols == 128. */
int ppgat_project_bwd_input(const float* D, int64_t ldd, int64_t n, int k, const float* w, int64_t ldw, int out_cols,
                            const float* att_src, const float* att_dst, const float* S, int64_t lds, float* dx,
                            int64_t lddx, void* stream);
/* The heads = 1 layer's input gradient AND its weight-gradient products in one pass over D and
 * x (replaces, with the two calls above: the autograd of GATConv.lin / SimpleGATLayer.lin,
 * train_gat_pyg.py:77, train_gat_custom.py:77, for the x rows and the weight):
 *   dx = D W + ds_src (x) (att_src W) + ds_dst (x) (att_dst W)    (dx nullable: skipped)
 *   G  = D^T x [k, k],   GV = [ds_src^T x ; ds_dst^T x] [2, k]     (for ppgat_weight_grads)
 * x rows [0, split) from x0, [split, n) from x1 (x1 nullable).  Supported when k == 128 and
 * the split-bf16 GEMM family is on (ppgat_project_bwd_fused_supported); deterministic. */
int ppgat_project_bwd_fused_supported(int k);
int ppgat_project_bwd_fused_workspace_bytes(int64_t n, size_t* bytes);
int ppgat_project_bwd_fused(const float* D, int64_t ldd, const float* S, int64_t lds, const float* x0, int64_t ldx0,
                            const float* x1, int64_t ldx1, int64_t split, int64_t n, int k, const float* w,
                            int64_t ldw, const float* att_src, const float* att_dst, float* dx, int64_t lddx,
                            float* G, float* GV, void* workspace, size_t workspace_bytes, void* stream);
/* ppgat_project_bwd_fused (dx required) that also does the backward prologue of the layer that
 * produced x, when x IS that layer's output (heads = 1, no op in between: the stacked convs of
 * train_gat_pyg.py:86-87) and dx is its whole grad_out -- ppgat_bwd_prologue's outputs for that
 * layer, from dx while it is still on chip instead of a second pass over dx and x:
 *   prev_nstate[r] = {prev_s_dst[r], prev_m[r], prev_inv_l[r], prev_gscale <dx_r, x_r - prev_bias>}
 *   prev_grad_bias = sum_r dx_r                       (prev_bias / prev_grad_bias nullable)
 * Same dx, G, GV as ppgat_project_bwd_fused, bit for bit; deterministic. */
int ppgat_project_bwd_fused_producer(const float* D, int64_t ldd, const float* S, int64_t lds, const float* x0,
                                     int64_t ldx0, const float* x1, int64_t ldx1, int64_t split, int64_t n, int k,
                                     const float* w, int64_t ldw, const float* att_src, const float* att_dst,
                                     float* dx, int64_t lddx, float* G, float* GV, const float* prev_bias,
                                     const float* prev_s_dst, const float* prev_m, const float* prev_inv_l,
                                     float prev_gscale, float* prev_nstate, float* prev_grad_bias, void* workspace,
                                     size_t workspace_bytes, void* stream);
/* Weight and attention-vector gradients from G = dh_msg^T x [H*C, K] and
 * GV = [ds_src^T x ; ds_dst^T x] [2H, K] (ppgat_gemm_tn with V):
 *   dW = G + att_src (x) GV[:H] + att_dst (x) GV[H:],  datt_src[h] = W_h GV[h],  datt_dst[h] = W_h GV[H + h]. */
int ppgat_weight_grads(const float* G, const float* GV, const float* w, const float* att_src, const float* att_dst,
                       int heads, int channels, int in_channels, float* dW, float* datt_src, float* datt_dst,
                       void* stream);

/* ---- optimizer -------------------------------------------------------------------------
 * Replaces: torch.optim.Adam(model.parameters(), lr, weight_decay) .step()
 * (train_gat_pyg.py:299,323) for fp32 dense tensors, amsgrad=False, maximize=False:
 *   g += wd * p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2   ((1 - b) rounded from double);
 *   p -= step_size * m / (sqrt(v) / bias_correction2_sqrt + eps)
 * with step_size = lr / (1 - b1^t), bias_correction2_sqrt = sqrt(1 - b2^t) per tensor
 * (host arrays).  count <= ppgat_adam_max_tensors() tensors in one launch. */
int ppgat_adam_max_tensors(void);
int ppgat_adam_step(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                    float* const* exp_avg_sq, const int64_t* numel, const float* step_size,
                    const float* bias_correction2_sqrt, double beta1, double beta2, float eps, float weight_decay,
                    void* stream);
/* Graph-capturable variant: tensor k's step count t is read on the device from *step[k] (one
 * float per parameter, as torch.optim.Adam(capturable=True) keeps it; the caller increments
 * them on the same stream before the launch), step_size = lr / (1 - beta1^t)
 * and bias_correction2_sqrt = sqrt(1 - beta2^t) are formed in double in the kernel and
 * rounded once -- the values the host path passes.  Same replacement as ppgat_adam_step
 * (torch.optim.Adam(capturable=True) semantics); one launch per <= max_tensors tensors. */
int ppgat_adam_step_device(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                           float* const* exp_avg_sq, const int64_t* numel, const float* const* step, double lr,
                           double beta1,
                           double beta2, float eps, float weight_decay, void* stream);

/* ---- replicated-item partition: cross-rank merge of item destination rows -----------------
 * Replaces: nothing one-to-one -- in the reference every destination's softmax sees all of
 * its in-edges (PyG softmax over edge_index, train_gat_pyg.py:77); with users sharded over
 * ranks and the item rows replicated (dist.py), an item's in-edges are split over the ranks,
 * so each rank's ppgat_fwd output for item rows is merged exactly (PyG mode, eps 1e-16):
 *   phase 0: mx[i,h] = m[i,h] if row i has local in-edges else -inf      -> all_reduce(MAX, mx)
 *   phase 1: pack = [c * a | c], c = (1/inv_l - eps) * exp(m - mx) (0 for rows without local
 *            in-edges), a = agg (heads > 1) or out - bias (heads = 1)     -> all_reduce(SUM, pack)
 *   phase 2: agg = pack_a / (pack_c + eps), out = mean_h agg + bias, inv_l = 1/(pack_c + eps),
 *            m = pack_c > 0 ? mx : 0   (in place on the item rows)
 * item_rowptr: the local CSR rowptr at the first item row (n_items + 1 entries); out/agg/m/inv_l
 * point at the first item row; pack holds n_items*heads*(channels + 1) floats ([a] then [c]). */
int ppgat_rep_merge(int phase, const int32_t* item_rowptr, int64_t n_items, int heads, int channels, float* out,
                    float* agg, const float* bias, float* m, float* inv_l, float* mx, float* pack, void* stream);

/* ---- row-sharded partition: halo exchange rows ------------------------------------------
 * Replaces: nothing one-to-one -- the reference is one process on one GPU; with nodes
 * row-sharded over ranks (dist.py ExchangePlan) every layer all_to_all's the rows the peers'
 * edges read, and the backward returns their gradients to the owner.
 *   ppgat_rows_gather:     dst[r, :] = src[idx[r], :]      (pack the all_to_all send buffer)
 *   ppgat_rows_return_add: dst[o, :] += sum_{k = ret_ptr[o]}^{ret_ptr[o+1]-1} ret[ret_pos[k], :]
 *                          (returned halo gradients, added in peer order: deterministic)
 * Rows of `cols` floats with row strides ld_* (floats). */
int ppgat_rows_gather(const float* src, int64_t ld_src, const int64_t* idx, int64_t n_rows, int cols, float* dst,
                      int64_t ld_dst, void* stream);
int ppgat_rows_return_add(float* dst, int64_t ld_dst, const float* ret, int64_t ld_ret, const int32_t* ret_ptr,
                          const int32_t* ret_pos, int64_t n_rows, int cols, void* stream);

/* ---- dropout epoch (hipGraph replays) ------------------------------------------------------
 * Every dropout mask of ppgat_fwd / ppgat_bwd_edges uses seed' = seed + epoch * 0xD1B54A32D192ED03
 * (mod 2^64), epoch a device-side counter (0 at load: seeds are used as passed).  A training
 * step captured once in a hipGraph bakes its host seeds in; enqueueing ppgat_dropout_advance
 * at the top of the captured step gives every replay fresh masks (the reference draws new
 * F.dropout masks per call, train_gat_pyg.py:77 attn dropout).  Stream-ordered.
 * Replaces: nothing in the reference (eager PyTorch draws from its generator each call). */
int ppgat_dropout_advance(void* stream);
int ppgat_dropout_set_epoch(uint64_t epoch, void* stream);

/* ---- I-I kNN graph (config 3's second relation) ------------------------------------
 * Replaces: the per-item selection loop of graphs/build_ii_knn.py:76-99 (self excluded as
 * -inf, argpartition top-k, sorted descending, kept where sim >= min_similarity).  S is a
 * block of the cosine-similarity matrix: rows = query items q0 .. q0 + rows - 1, columns =
 * all n_cols items (row stride ld floats).  Writes, per row, the k best (item, similarity)
 * sorted by similarity descending with ties by smaller item index (out_idx / out_sim
 * [rows, k]; -1 / -inf where fewer than k items exist) and out_cnt[row] = how many of them
 * reach min_sim (a prefix).  k <= ppgat_knn_max_k().  Deterministic. */
int ppgat_knn_max_k(void);
int ppgat_knn_topk(const float* S, int64_t ld, int64_t rows, int64_t n_cols, int64_t q0, int k, float min_sim,
                   int32_t* out_idx, float* out_sim, int32_t* out_cnt, void* stream);

/* ---- BPR triple sampler ---------------------------------------------------------------
 * Replaces: sample_bpr_epoch, scripts/train_gat_pyg.py:179-190 (Python loop per epoch):
 *   u uniform over users with >= 1 train item; i uniform over the positions of u's train
 *   list (random.choice); j uniform over [0, n_items), redrawn while j is one of u's items.
 * Same distribution, a counter-based stream instead of Python's Mersenne twister: every
 * draw hashes (seed, t0 + s, draw number), so a triple does not depend on how the S
 * triples are split over calls (oracle/sampler_oracle.py restates the stream bit for bit).
 * prepare (once per graph): user_ptr [n_users+1] int64 CSR over user_items [nnz] int32 item
 * ids (any order within a user) -> items_sorted [nnz] (each user's items ascending),
 * eligible [n_users] (ids of users with items, ascending) and *n_eligible (device int64).
 * sample: u, i, j [S] int64; *bad (device) = 1 if no user has items, 2 if some user's
 * negative was not found in 1024 draws (the user holds ~all items; the reference loops). */
int ppgat_bpr_sampler_workspace_bytes(int64_t n_users, int64_t nnz, size_t* bytes);
int ppgat_bpr_sampler_prepare(const int64_t* user_ptr, const int32_t* user_items, int64_t n_users, int64_t nnz,
                              int32_t* items_sorted, int32_t* eligible, int64_t* n_eligible, void* workspace,
                              size_t workspace_bytes, void* stream);
int ppgat_bpr_sample(const int64_t* user_ptr, const int32_t* items_sorted, const int32_t* eligible,
                     const int64_t* n_eligible, int64_t n_items, int64_t n_triples, uint64_t seed, int64_t t0,
                     int64_t* u, int64_t* i, int64_t* j, int32_t* bad, void* stream);

/* ---- sampled-evaluation candidates ---------------------------------------------------
 * Replaces: the candidate draw of eval_sampled, scripts/train_gat_pyg.py:157-167 (a Python
 *   loop over ~192k users: np.random.randint(0, n_items) redrawn while the item is in the
 *   user's train set or is the held-out positive, eval_neg_k times per user).
 * cands [n_eval, n_neg + 1] int64: column 0 = pos[b], column 1 + k = the first draw d of the
 * counter-based stream (seed, t = b * n_neg + k, d) outside u's train items (items_sorted /
 * user_ptr of ppgat_bpr_sampler_prepare) and != pos[b] (oracle/sampler_oracle.py restates it);
 * *bad = 2 if some negative was not found in 1024 draws. */
int ppgat_eval_sample(const int64_t* user_ptr, const int32_t* items_sorted, const int64_t* users, const int64_t* pos,
                      int64_t n_eval, int64_t n_neg, int64_t n_items, uint64_t seed, int64_t* cands, int32_t* bad,
                      void* stream);

/* ---- sampled ranking (evaluation) ------------------------------------------------
 * Replaces: the per-user loop of eval_sampled, scripts/train_gat_pyg.py:160-175:
 *   scores = I[cands[b]] @ U[users[b]];  rank[b] = #(scores[1:] > scores[0]) + 1
 * cands [n_eval, n_cand] int64 item ids (column 0 = the held-out positive); Z rows as in
 * ppgat_bpr_fwd (row_map nullable).
 */
int ppgat_sampled_rank(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                       int channels, const int64_t* users, const int64_t* cands, int64_t n_eval, int64_t n_cand,
                       int32_t* rank, void* stream);

/* ---- serving top-K ------------------------------------------------------------------
 * Replaces: RecommenderRuntime.top_k_for_user_items, serving/runtime.py:56-76 (numpy):
 *   user_vec = mean(item_vecs[history]); scores = item_vecs @ user_vec; scores[history] = -1e9;
 *   the k best, descending.
 * Batched over n_users (<= 256) histories given as CSR (hist_ptr [n_users + 1] int64 into
 * hist_items; max_hist = the longest history).  The mean adds the history rows in order and
 * divides by the count (numpy's float32 mean over axis 0); ties between equal scores go to
 * the smaller item index (a total order).  out_idx/out_score [n_users, k]. */
int ppgat_serve_topk_workspace_bytes(int64_t n_items, int channels, int n_users, size_t* bytes);
int ppgat_serve_topk(const float* item_vecs, int64_t n_items, int channels, const int64_t* hist_ptr,
                     const int64_t* hist_items, int64_t max_hist, int n_users, int k, int32_t* out_idx,
                     float* out_score, void* workspace, size_t workspace_bytes, void* stream);

/* ---- fusion MLP inference on the matrix cores (north star's MFMA target) ----------
 * Replaces: FusionMLP.forward + the normalisation and the per-row image copy loop of the
 *           inference pass, embeddings/fuse_modal.py:18-36,227-241:
 *   out = normalize?(relu([txt | img_row] W1^T + b1) W2^T + b2)   (norm: y / (||y|| + 1e-8))
 * img_row = img[img_index[b]] when img_index != NULL and img_index[b] >= 0, img_fallback
 * (the mean image embedding) when img_index[b] < 0, img[b] when img_index == NULL.
 * z1 (nullable) receives the pre-activation [n, hidden] for a training backward.
 * fp32 MFMA (exact fp32 FMA chains).  hidden_dim must be 256, output_dim 128, text_dim and
 * img_dim multiples of 32 (the reference's 384 + 512 -> 256 -> 128).
 */
int ppgat_fusion_fwd(const float* txt, const float* img, const int32_t* img_index, const float* img_fallback,
                     int64_t n, int text_dim, int img_dim, const float* w1, const float* b1, int hidden_dim,
                     const float* w2, const float* b2, int output_dim, int normalize, float* out, float* z1,
                     void* stream);
/* The same with a caller workspace (ppgat_fusion_fwd_workspace_bytes, 16-byte aligned): W1 and
 * W2 are split into their bf16 images once per call and the kernel stages them straight into
 * LDS (8 waves per workgroup share each staged chunk); bitwise the results of
 * ppgat_fusion_fwd. */
int ppgat_fusion_fwd_workspace_bytes(int text_dim, int img_dim, int hidden_dim, int output_dim, size_t* bytes);
int ppgat_fusion_fwd_ws(const float* txt, const float* img, const int32_t* img_index, const float* img_fallback,
                        int64_t n, int text_dim, int img_dim, const float* w1, const float* b1, int hidden_dim,
                        const float* w2, const float* b2, int output_dim, int normalize, float* out, float* z1,
                        void* workspace, size_t workspace_bytes, void* stream);

/* ---- fusion MLP training: InfoNCE loss and backward, ReLU + dropout -----------------------
 * Replaces: contrastive_fusion_loss + its autograd backward, embeddings/fuse_modal.py:39-72
 *           (called by the training loop :179-214), and the ReLU/Dropout(0.1) of FusionMLP.mlp
 *           (:27-29) in train mode.  The Linear layers around them run on ppgat_gemm_nn /
 *           ppgat_gemm_tn_big / ppgat_colsum.
 * ppgat_infonce: F = fused, T = txt_proj(txt), I = img_proj(img), each [B, D] (D = 128,
 *   B <= 4096).  Fn, Tn, In = rows / max(||row||, 1e-12) (F.normalize); S_t = Fn Tn^T / tau,
 *   S_i = Fn In^T / tau; loss_t = mean_b CE(S_t[b], b), loss_i likewise.
 *   loss[3] = {(loss_t + loss_i) / 2, loss_t, loss_i} (device); dF, dT, dI = d loss / d(F, T, I).
 *   Fixed-order reductions (deterministic).  Workspace queried first.
 * ppgat_relu_dropout: backward 0: a = relu(z) * mask; backward 1: a <- a * mask * [z > 0] in place
 *   (a holds dL/da on entry).  mask = 0 with probability p, else 1 / (1 - p), from a counter hash
 *   of (seed, element index) -- the same draw forward and backward; p = 0 is plain ReLU. */
int ppgat_infonce_workspace_bytes(int64_t batch, int dim, size_t* bytes);
int ppgat_infonce(const float* fused, const float* txt_p, const float* img_p, int64_t batch, int dim, float tau,
                  float* loss, float* d_fused, float* d_txt_p, float* d_img_p, void* workspace, size_t workspace_bytes,
                  void* stream);
int ppgat_relu_dropout(const float* z, int64_t n, float p, uint64_t seed, int backward, float* a, void* stream);

/* ---- fp32 matrix-core GEMMs (v_mfma_f32_32x32x2_f32, exact fp32 FMA chains) ---------------
 * Replaces: the hipBLAS/cuBLAS GEMMs of torch.nn.Linear in GATConv.lin at shapes past the fused
 *           128-column projection (config 5: lin 256 -> 1024, train_gat_pyg.py:77) and of
 *           PyGGAT.item_proj (train_gat_pyg.py:74,81), and their weight gradients.
 * ppgat_gemm_nn:  y[m, n] = alpha x[m, k] B + bias  with B[k][j] = b[k * ldb + j] (b_layout 0)
 *                 or b[j * ldb + k] (b_layout 1: x W^T with W = b [n, k]); k % 32 == 0,
 *                 n % 128 == 0; bias nullable.
 * ppgat_gemm_tn_big: out[ma, nb] = a[m, ma]^T b[m, nb] over m rows, ma and nb multiples of 128;
 *                 row splits summed in split order (deterministic); workspace queried first.
 * ppgat_colsum:   out[c] = sum_i y[i, c] (c in {128, 256}), fixed order. */
int ppgat_gemm_nn_supported(int64_t m, int k, int n, int b_layout);
int ppgat_gemm_nn(const float* x, int64_t ldx, int64_t m, int k, const float* b, int64_t ldb, int b_layout, int n,
                  float alpha, const float* bias, float* y, int64_t ldy, void* stream);
/* ppgat_gemm_nn_ws: the same product; with few output tiles (small m, e.g. a 512-row batch)
 *   and a long reduction it splits k over workgroups into the workspace and sums the splits in
 *   order (deterministic); workspace_bytes() returns 0 when no split is taken. */
int ppgat_gemm_nn_workspace_bytes(int64_t m, int k, int n, size_t* bytes);
int ppgat_gemm_nn_ws(const float* x, int64_t ldx, int64_t m, int k, const float* b, int64_t ldb, int b_layout, int n,
                     float alpha, const float* bias, float* y, int64_t ldy, void* workspace, size_t workspace_bytes,
                     void* stream);
/* ppgat_gemm_nn_rank: y = alpha x b + bias + s a (s [m, nv] with row stride lds, a [nv, n] with
 *   row stride lda, nv <= 16, the terms added in v order after alpha and bias: the bits of
 *   ppgat_gemm_nn_ws followed by ppgat_rows_rank_update).  On the fp16 two-term large-m path
 *   with nv <= 8 the rank terms are added in the GEMM's epilogue (no second pass over y) --
 *   the multi-head backward's dx = acc W / H + S A_att (ppgat_xgat_bwd_edges_g).  Same
 *   workspace as ppgat_gemm_nn_ws. */
int ppgat_gemm_nn_rank(const float* x, int64_t ldx, int64_t m, int k, const float* b, int64_t ldb, int b_layout, int n,
                       float alpha, const float* bias, const float* s, int64_t lds, int nv, const float* a,
                       int64_t lda, float* y, int64_t ldy, void* workspace, size_t workspace_bytes, void* stream);
int ppgat_gemm_tn_big_workspace_bytes(int64_t m, int ma, int nb, size_t* bytes);
int ppgat_gemm_tn_big(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma, int nb, float* out,
                      void* workspace, size_t workspace_bytes, void* stream);
/* ppgat_gemm_tn_big_bounded: the same product, with the caller's upper bound of |b| per column
 *   (b_bound_bits[j % bound_period] as IEEE bits, times bound_scale >= 1) in place of the
 *   column-max pass over b that the fp16 two-term kernel otherwise makes -- e.g. the multi-head
 *   layer's G = g^T agg with |agg^h_i[k]| <= max_j |x_j[k]| / (1 - p) (train_gat_pyg.py:77 backward).
 *   The fp16 split's error is relative to the bound, not to b's own column maxima: a column
 *   whose bound is 2^k above its true maximum loses about k bits (22 - k significant bits per
 *   product), so the bound should be tight -- for agg, the column maxima over the rows that are
 *   the SOURCE of an edge (ppgat_colmax_abs_sources), not over all rows of x.  The fp32 / bf16
 *   families ignore it.
 * ppgat_colmax_abs: out_bits[c] = IEEE bits of max_i |x[i, c]| (order-free: deterministic).
 * ppgat_colmax_abs_sources: the same over the rows i with src_ptr[i + 1] > src_ptr[i] (src_ptr:
 *   the CSC pointers [n + 1] of the edge list; rows with no out-edge never enter an aggregate). */
int ppgat_gemm_tn_big_bounded(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma, int nb,
                              const unsigned* b_bound_bits, int bound_period, float bound_scale, float* out,
                              void* workspace, size_t workspace_bytes, void* stream);
/* ppgat_gemm_tn_big_bounds: both bounds the caller's (either nullable: that operand's column-max
 *   pass instead).  a_bound_bits[i] bounds |a[r, i]| over the rows r whose b row is NOT all zero
 *   (e.g. g over the destinations that have an in-edge, from ppgat_xgat_bwd_edges_gd_colmax, for
 *   G = g^T agg: agg_r = 0 without in-edges); the other rows' a values are clamped to the fp16
 *   range in the split, so they add 0 as they must.  b_bound_bits as in _bounded. */
int ppgat_gemm_tn_big_bounds(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma, int nb,
                             const unsigned* a_bound_bits, const unsigned* b_bound_bits, int bound_period,
                             float bound_scale, float* out, void* workspace, size_t workspace_bytes, void* stream);
/* ppgat_gemm_tn_big_colsum: ppgat_gemm_tn_big_bounds (either bound nullable) that also writes
 *   colsum_out[i] = sum_r a[r, i] (the bias gradient beside a weight gradient: Linear.bias,
 *   GATConv.bias) -- on the fp16 TN kernel from the rows its staging threads already hold (no
 *   second pass over a), in a fixed order: deterministic.  Replaces the reference's separate
 *   autograd sum for the bias (torch.nn.Linear / PyG GATConv bias, train_gat_pyg.py:75-77). */
int ppgat_gemm_tn_big_colsum(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma, int nb,
                             const unsigned* a_bound_bits, const unsigned* b_bound_bits, int bound_period,
                             float bound_scale, float* out, float* colsum_out, void* workspace,
                             size_t workspace_bytes, void* stream);
int ppgat_colmax_abs(const float* x, int64_t ldx, int64_t n, int c, unsigned* out_bits, void* stream);
int ppgat_colmax_abs_sources(const float* x, int64_t ldx, int64_t n, int c, const int32_t* src_ptr,
                             unsigned* out_bits, void* stream);
int ppgat_colsum_workspace_bytes(int64_t n, int c, size_t* bytes);
int ppgat_colsum(const float* y, int64_t ldy, int64_t n, int c, float* out, void* workspace, size_t workspace_bytes,
                 void* stream);

/* ---- multi-head layer, aggregate-then-transform ----------------------------------------------
 * Replaces: GATConv(C_in, C, heads=H, concat=False) forward and backward (train_gat_pyg.py:77,
 *           SURVEY.md Appendix A) when H*C > C_in -- config 5 (C_in = C = 256, H = 4).  The
 *           message is linear in x_j, so the edge pass gathers x_j (C_in floats) once per edge
 *           for all heads instead of h_j (H*C floats):
 *   att_proj [2, H, C_in]: A_v[h] = W_h^T att_v[h]                      (ppgat_xgat_weights)
 *   w_xform [H*C_in, C]: w_xform[h*C_in + k][c] = W[h*C + c][k];  w_grad [C, H*C_in] = w_xform^T / H
 *   s_src[n][h] = x_n . A_src[h] (n < n_rows), s_dst likewise (n < n_dst)   (ppgat_xgat_scores)
 *   agg[i][h] = sum_{j->i} alpha_ij^h x_j, m, inv_l [n_dst, H]  (ppgat_xgat_fwd; CSR over the
 *     destination rows; x rows indexed by col may extend past n_dst: the halo rows of dist.py)
 *   out = agg w_xform / H + bias                                          (ppgat_gemm_nn)
 * Backward with g = dL/dout: gt = g w_grad [n_dst, H*C_in] (ppgat_gemm_nn); nstate[i][h] =
 * {s_dst, m, inv_l, gt_i^h . agg_i^h} (prologue); one pass by source over the CSC
 * (ppgat_xgat_bwd_edges): dx_j = sum_k sum_h beta gt_i^h + sum_h ds_src_j^h A_src[h],
 * S[j][h] = ds_src, dz at each edge's CSR slot; S[i][H + h] = ds_dst by ppgat_bwd_dst_sum;
 * dx_i += sum_h ds_dst_i^h A_dst[h] (epilogue); GV = S^T x [2H, C_in] (ppgat_gemm_tn),
 * G = g^T agg [C, H*C_in] (ppgat_gemm_tn_big); dW, datt (ppgat_xgat_weight_grads):
 *   dW[h*C + c][k] = G[c][h*C_in + k] / H + att_src[h][c] GV[h][k] + att_dst[h][c] GV[H+h][k],
 *   datt_v[h][c] = sum_k W[h*C + c][k] GV[v*H + h][k].
 * Supported: C_in = 256, H in {2, 4}, C % 128 == 0 (ppgat_xgat_supported).  Dropout as ppgat_fwd
 * (seed_used required when dropout_p > 0: the forward writes it, the backward reads it). */
int ppgat_xgat_supported(int in_channels, int heads, int channels);
int ppgat_xgat_weights(const float* w, const float* att_src, const float* att_dst, int heads, int channels,
                       int in_channels, float* att_proj, float* w_xform, float* w_grad, void* stream);
int ppgat_xgat_scores(const float* x, int64_t ldx, int64_t n_rows, int64_t n_dst, int in_channels, int heads,
                      const float* att_proj, float* s_src, float* s_dst, void* stream);
int ppgat_xgat_fwd_workspace_bytes(int64_t n_hub_items, int heads, int in_channels, size_t* bytes);
int ppgat_xgat_fwd(const ppgat_schedule* dst_sched, const int32_t* col, const int32_t* csr_eid, int64_t n_dst,
                   int64_t n_edges, int in_channels, int heads, const float* x, int64_t ldx, const float* s_src,
                   const float* s_dst, float negative_slope, float dropout_p, uint64_t seed, uint64_t* seed_used,
                   float* agg, float* m, float* inv_l, void* workspace, size_t workspace_bytes, void* stream);
/* ppgat_xgat_fwd that also merges into x_colmax_bits[k] (caller-initialised, e.g. zeros; 16-byte
 * aligned) the IEEE bits of max |x_j[k]| over the rows it gathers -- every source of an edge,
 * the rows ppgat_colmax_abs_sources covers -- by atomic max (order-free: deterministic).  The
 * bound of |agg| the weight gradient's fp16 split needs, without a pass over x. */
int ppgat_xgat_fwd_colmax(const ppgat_schedule* dst_sched, const int32_t* col, const int32_t* csr_eid, int64_t n_dst,
                          int64_t n_edges, int in_channels, int heads, const float* x, int64_t ldx, const float* s_src,
                          const float* s_dst, float negative_slope, float dropout_p, uint64_t seed,
                          uint64_t* seed_used, float* agg, float* m, float* inv_l, unsigned* x_colmax_bits,
                          void* workspace, size_t workspace_bytes, void* stream);
int ppgat_xgat_bwd_prologue(const float* gt, const float* agg, const float* s_dst, const float* m, const float* inv_l,
                            int64_t n_dst, int in_channels, int heads, float* nstate, void* stream);
int ppgat_xgat_bwd_workspace_bytes(int64_t n_hub_items, int in_channels, size_t* bytes);
int ppgat_xgat_bwd_edges(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                         const int32_t* dz_slot, int64_t n_edges, int in_channels, int heads, const float* x,
                         int64_t ldx, const float* s_src, const float* nstate, const float* gt, const float* att_proj,
                         float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used, float* dx,
                         int64_t lddx, float* S, int64_t lds, float* dz, void* workspace, size_t workspace_bytes,
                         void* stream);
/* The same backward edge pass gathering g_i (C floats per edge) instead of gt_i (H * C_in):
 *   dalpha^h_ij = g_i . hs^h_j with hs^h_j = W_h x_j / heads (caller's GEMM, [n_src, H, C]),
 *   acc[j][h] = sum_k beta^h g_i [n_src, H, C]; dx = acc W / heads (caller's GEMM, W = lin.weight
 *   [H*C, C_in]) + the attention terms of S (ppgat_gemm_nn_rank).  dz, S[:, :H] as
 *   ppgat_xgat_bwd_edges.  Channels C == 256, heads 2 or 4. */
int ppgat_xgat_bwd_g_workspace_bytes(int64_t n_hub_items, int channels, int heads, size_t* bytes);
int ppgat_xgat_bwd_edges_g(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                           const int32_t* dz_slot, int64_t n_edges, int channels, int heads, const float* hs,
                           const float* s_src, const float* nstate, const float* g, int64_t ldg, float negative_slope,
                           float dropout_p, uint64_t seed, const uint64_t* seed_used, float* acc, float* S, int64_t lds,
                           float* dz, void* workspace, size_t workspace_bytes, void* stream);
/* Deferred D (the default multi-head backward: no gt GEMM, no gt.agg prologue).  The prologue's
 * D^h_i = gt^h_i . agg^h_i equals sum_j beta^h_ij dalpha^h_ij with dalpha = g_i . hs^h_j, so:
 *   ppgat_xgat_nstate: nstate[i][h] = {s_dst, m, inv_l, D or 0 (D NULL)}, D [n_dst, heads];
 *   ppgat_xgat_bwd_edges_gd: ppgat_xgat_bwd_edges_g's pass with dalpha and pdalpha = beta dalpha
 *     stored per edge and head (at dz_slot, as dz) instead of dz and ds_src; acc as _g;
 *   D = the destination sum of pdalpha (ppgat_bwd_dst_sum_csc / ppgat_bwd_dst_sum, heads H);
 *   ppgat_xgat_bwd_dz: dz = alpha e'(z) (dm dalpha - D_i) in place over dalpha (by source over
 *     the CSC; nstate with D) and S[j][h] = ds_src_j = sum of the source's dz (fixed order);
 *   ds_dst = the destination sum of dz, as before.  Heads 2 or 4. */
int ppgat_xgat_bwd_edges_gd(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                            const int32_t* dz_slot, int64_t n_edges, int channels, int heads, const float* hs,
                            const float* s_src, const float* nstate, const float* g, int64_t ldg,
                            float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used,
                            float* acc, float* dalpha, float* pdalpha, void* workspace, size_t workspace_bytes,
                            void* stream);
/* ppgat_xgat_bwd_edges_gd that also merges into g_colmax_bits[c] the bits of max |g_i[c]| over the
 * rows it gathers (every destination of an edge), as ppgat_xgat_fwd_colmax: the A bound of
 * ppgat_gemm_tn_big_bounds for G = g^T agg. */
int ppgat_xgat_bwd_edges_gd_colmax(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                                   const int32_t* dz_slot, int64_t n_edges, int channels, int heads, const float* hs,
                                   const float* s_src, const float* nstate, const float* g, int64_t ldg,
                                   float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used,
                                   float* acc, float* dalpha, float* pdalpha, unsigned* g_colmax_bits,
                                   void* workspace, size_t workspace_bytes, void* stream);
int ppgat_xgat_nstate(const float* s_dst, const float* m, const float* inv_l, const float* D, int64_t n_dst, int heads,
                      float* nstate, void* stream);
/* Halo partition (dist.py): set the D component of every row of an nstate table whose other three
 * came by exchange -- nstate[i][h].w = D[i * heads + h] for i < n_rows.  Replaces dist.py:
 * `ntab.x.view(R, H, 4)[:, :, 3].copy_(Dtab.x)` (no reference counterpart: the reference has no
 * sharded backward). */
int ppgat_xgat_nstate_set_d(float* nstate, const float* D, int64_t n_rows, int heads, void* stream);
int ppgat_xgat_bwd_dz_workspace_bytes(int64_t n_hub_items, int heads, size_t* bytes);
int ppgat_xgat_bwd_dz(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                      const int32_t* dz_slot, int64_t n_edges, int heads, const float* s_src, const float* nstate,
                      float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used, float* dz,
                      float* S, int64_t lds, void* workspace, size_t workspace_bytes, void* stream);
int ppgat_xgat_bwd_epilogue(const float* S, int64_t lds, const float* att_proj, int64_t n_dst, int in_channels,
                            int heads, float* dx, int64_t lddx, void* stream);
int ppgat_xgat_weight_grads(const float* G, const float* GV, const float* w, const float* att_src,
                            const float* att_dst, int heads, int channels, int in_channels, float* dW, float* datt_src,
                            float* datt_dst, void* stream);

/* ---- multi-head layer, transform-then-aggregate (H*C <= C_in, or the replicated partition) ----
 * Replaces: the input-gradient terms of GATConv's attention logits (PyG, train_gat_pyg.py:77;
 *   SURVEY.md Appendix B): dx = D W + ds_src A_src + ds_dst A_dst, with D W on ppgat_gemm_nn.
 * ppgat_att_proj: att_proj [2, H, C_in] = [W_h^T att_src[h]; W_h^T att_dst[h]] for any shape
 *   (W [H*C, C_in] row-major, att [H, C]).
 * ppgat_rows_rank_update: dx[i][k] += sum_{v < nv} S[i][v] A[v][k] (v ascending) over n_rows
 *   rows, nv <= 16, k % 4 == 0, 16-byte aligned A / dx rows.  Deterministic. */
int ppgat_att_proj(const float* w, const float* att_src, const float* att_dst, int heads, int channels,
                   int in_channels, float* att_proj, void* stream);
int ppgat_rows_rank_update(const float* S, int64_t lds, int nv, const float* A, int64_t lda, int64_t n_rows, int k,
                           float* dx, int64_t lddx, void* stream);

/* ---- validation / debug build -----------------------------------------------------------
 * ppgat_check_index_range: *n_bad = number of entries of idx (int32 when elem_bytes == 4,
 *   int64 when 8) outside [lo, hi); synchronises the stream (a validation tool, not for use
 *   inside a captured graph).  Used by the Python layer to validate graph views and exchange
 *   plans when the library is a debug build.
 * ppgat_debug_build: 1 for libppgat_debug.so (make debug: -O1 -g -DPPGAT_DEBUG=1), whose entry
 *   points validate the index inputs whose bounds they know (BPR triples, eval users and
 *   candidates, serving histories) and synchronise after their kernels, so an asynchronous
 *   fault is reported by the entry point that launched it; 0 for libppgat.so. */
int ppgat_debug_build(void);
int ppgat_check_index_range(const void* idx, int elem_bytes, int64_t n, int64_t lo, int64_t hi, int64_t* n_bad,
                            void* stream);

/* ---- measurement ------------------------------------------------------------------------
 * ppgat_stream_copy: dst[0 .. n_bytes) = src[...], a float4 streaming copy (16 B per lane,
 *   non-temporal loads and stores, one pass): the achievable-HBM yardstick bench.py reports
 *   beside the 8 TB/s spec peak (the guide's measured float4 copy: 6.29 TB/s; this one 6.58 on
 *   1 GiB, profiles/r06/x3_copy_lab.log).  n_bytes and both pointers must be multiples of 16. */
int ppgat_stream_copy(const void* src, void* dst, int64_t n_bytes, void* stream);

/* ---- in-process kernel timing (HIP events on the launch stream) --------- */
#define PPGAT_K_CSR 0
#define PPGAT_K_SCORES 1
#define PPGAT_K_FWD 2
#define PPGAT_K_BWD_PRO 3
#define PPGAT_K_BWD_SRC 4
#define PPGAT_K_BWD_EPI 5
#define PPGAT_K_BWD_RED 6
#define PPGAT_K_SCHED 7
#define PPGAT_K_GEMM_TN 8
#define PPGAT_K_FUSION 9
#define PPGAT_K_PROJ 10
#define PPGAT_K_ADAM 11
#define PPGAT_K_SAMPLE 12
#define PPGAT_K_INFONCE 13
#define PPGAT_K_PROJ_BWD 14
#define PPGAT_K_COUNT 15
int ppgat_profile_enable(int on);
int ppgat_profile_reset(void);
/* Synchronises the recorded events; total milliseconds and launch count of kernel k. */
int ppgat_profile_read(int kernel, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* PPGAT_H */
