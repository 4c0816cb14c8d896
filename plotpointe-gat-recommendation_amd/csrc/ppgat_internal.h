// Internal declarations shared by the kernel, graph and ABI translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace ppgat {

constexpr int kModePyg = 0;
constexpr int kModeCustom = 1;
constexpr int kMaxHeads = 8;
#ifndef PPGAT_EPI_BLOCKS
#define PPGAT_EPI_BLOCKS 1024
#endif
constexpr int64_t kEpiMaxBlocks = PPGAT_EPI_BLOCKS;
constexpr int kShortItemEdges = 16;  // include/ppgat.h PPGAT_SHORT_ITEM_EDGES

// host-side view of a work schedule (see include/ppgat.h ppgat_schedule)
struct ItemsArg {
  const int32_t* row;
  const int32_t* beg;
  const int32_t* end;
  int64_t n_items;
  int64_t n_hub_items;
  int64_t n_long_items;  // -1: unknown (no four-per-wave short-item path)
};

hipError_t launch_stream_copy(const void* src, void* dst, int64_t n_bytes, hipStream_t st);
hipError_t launch_scores(const float* h, const float* as, const float* ad, int64_t n, int heads, int C, float* ss,
                         float* sd, hipStream_t st);
hipError_t launch_fwd(const ItemsArg& it, const int32_t* col, const int32_t* eid, int heads, int C,
                      const float* h, const float* ss, const float* sd, const float* bias, int mode, float slope,
                      float eps, float p, uint64_t seed, uint64_t* seed_out, float* out, float* m, float* invl,
                      float* agg, float* partial, const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs,
                      hipStream_t st);
hipError_t launch_bwd_pro(const float* go, const float* out, const float* agg, const float* bias, const float* sd,
                          const float* m, const float* invl, int64_t n, int heads, int C, float gscale,
                          float* nstate, float* bias_part, int64_t blocks, hipStream_t st);
hipError_t launch_bwd_src(const ItemsArg& it, const int32_t* row, const int32_t* csc_eid, const int32_t* csc2csr,
                          int heads, int C, const float* h, const float* ss, const float* nstate, const float* go,
                          int mode, float slope, float gscale, float p, uint64_t seed, const uint64_t* seed_in,
                          float* dh, int64_t ld_dh,
                          float* ds_src, int64_t ld_ds, float* dz, float* partial, const int32_t* hub_row,
                          const int32_t* hub_ptr, int64_t n_hubs, hipStream_t st);
hipError_t launch_dst_sum(const ItemsArg& it, int heads, const float* dz, const int32_t* csr2csc, float* ds_dst,
                          int64_t ld, float* partial, const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs,
                          hipStream_t st);
hipError_t launch_invert_index(const int32_t* p, int64_t n, int32_t* inv, hipStream_t st);
int64_t epi_blocks(int64_t n);
hipError_t launch_bwd_epi(const int32_t* rowptr, int64_t n, int heads, int C, const float* h, const float* as,
                          const float* ad, const float* ds_src, const float* dz, float* dh, float* partial,
                          int64_t blocks, hipStream_t st);
hipError_t launch_col_reduce(const float* partial, int64_t rows, int cols, int split, float* out_a, float* out_b,
                             hipStream_t st);

// graph preprocessing (ppgat_graph.hip)
size_t csr_workspace_bytes(int64_t n_nodes, int64_t n_edges);
hipError_t csr_build(const int64_t* edge_index, int64_t E, int64_t N, int32_t* rowptr, int32_t* col, int32_t* csr_eid,
                     int32_t* colptr, int32_t* row, int32_t* csc_eid, int32_t* csc2csr, int32_t* bad,
                     void* ws, size_t ws_bytes, hipStream_t st);
int64_t schedule_capacity(int64_t n_nodes, int64_t n_edges, int32_t max_edges);
size_t schedule_workspace_bytes(int64_t n_nodes);
hipError_t schedule_build(const int32_t* ptr, int64_t N, int32_t T, int32_t* item_row, int32_t* item_beg,
                          int32_t* item_end, int32_t* hub_row, int32_t* hub_ptr, int32_t* counts, void* ws,
                          size_t ws_bytes, hipStream_t st);

// training-step kernels (ppgat_train.hip)
bool bpr_channels_ok(int C);
// the backward prologue of the layer that produced Z (heads = 1), fused into the loss backward
struct BprProducer {
  const float* bias;  // nullable
  const float* s_dst;
  const float* m;
  const float* inv_l;
  float gscale;
  float* nstate;      // [n_rows, 4]
  float* grad_bias;   // nullable: [C]
};
size_t bpr_workspace_bytes(int64_t N, int64_t S, int C);
hipError_t bpr_fwd(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map, int C,
                   const int64_t* u, const int64_t* i, const int64_t* j, int64_t S, int kind, float* loss,
                   float* coef, int32_t* bad, void* ws, hipStream_t st);
hipError_t bpr_bwd(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map, int C,
                   const int64_t* u, const int64_t* i, const int64_t* j, int64_t S, const float* coef,
                   const float* grad_loss, float* dZ, void* ws, size_t ws_bytes, hipStream_t st,
                   const BprProducer* prod = nullptr);
hipError_t bpr_bwd_prepare(int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map, int C,
                           const int64_t* u, const int64_t* i, const int64_t* j, int64_t S, void* ws,
                           size_t ws_bytes, hipStream_t st);
hipError_t bpr_bwd_finish(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                          int C, const int64_t* u, const int64_t* i, const int64_t* j, int64_t S, const float* coef,
                          const float* grad_loss, float* dZ, void* ws, size_t ws_bytes, hipStream_t st,
                          const BprProducer* prod = nullptr);
size_t gemm_tn_workspace_bytes(int64_t N, int M, int K, int nv);
hipError_t gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t N, int M, int K, float* out,
                   float* colsum, const float* V, int64_t ldv, int nv, float* vout, void* ws, hipStream_t st);

// projection GEMMs, weight gradients, optimizer (ppgat_gemm.hip)
bool proj_shape_ok(int K, int ncols);
hipError_t proj_fwd(const float* x0, int64_t ldx0, const float* x1, int64_t ldx1, int64_t split, int64_t n, int K,
                    const float* W, int64_t ldw, const float* bias, const float* att_src, const float* att_dst,
                    float* y, int64_t ldy, float* s_src, float* s_dst, hipStream_t st);
hipError_t proj_dx(const float* D, int64_t ldd, int64_t n, int K, const float* W, int64_t ldw, const float* att_src,
                   const float* att_dst, const float* S, int64_t lds, float* y, int64_t ldy, hipStream_t st);
bool tn128_shape_ok(int M, int K, int nv, const float* V, int64_t ldv);
size_t tn128_workspace_bytes(int64_t N);
hipError_t tn128(const float* A, int64_t lda, const float* B, int64_t ldb, const float* B1, int64_t ldb1, int64_t split,
                 int64_t N, int M, int K, float* out, float* colsum, const float* V, int64_t ldv, int nv, float* vout,
                 void* ws, hipStream_t st);
hipError_t wgrad_assemble(const float* G, const float* GV, const float* W, const float* att_src, const float* att_dst,
                          int heads, int C, int K, float* dW, float* datt_src, float* datt_dst, hipStream_t st);
bool dxw_ok(int hc, int k);
size_t dxw_workspace_bytes(int64_t n);
// the backward prologue of the layer that produced x (heads = 1), fused into k_dxw's epilogue
struct DxwProducer {
  const float* bias;  // nullable
  const float* s_dst;
  const float* m;
  const float* inv_l;
  float gscale;
  float* nstate;      // [n, 4]
  float* grad_bias;   // nullable: [128]
};
hipError_t dxw(const float* D, int64_t ldd, const float* S, int64_t lds, const float* x0, int64_t ldx0, const float* x1,
               int64_t ldx1, int64_t split, int64_t n, const float* W, int64_t ldw, const float* att_src,
               const float* att_dst, float* dx, int64_t lddx, float* G, float* GV, void* ws, hipStream_t st,
               const DxwProducer* prod = nullptr);
int adam_max_tensors();
hipError_t dropout_epoch(int set, uint64_t value, hipStream_t st);
// replicated-item merge (ppgat_dist.hip): phase 0 max, 1 pack, 2 finish
hipError_t rep_merge(int phase, const int32_t* rowptr, int64_t n, int heads, int C, float eps, float* out, float* agg,
                     const float* bias, float* m, float* invl, float* mx, float* pack_a, float* pack_c,
                     hipStream_t st);
// halo exchange rows (ppgat_dist.hip)
hipError_t rows_gather(const float* src, int64_t lds, const int64_t* idx, int64_t n, int cols, float* dst,
                       int64_t ldd, hipStream_t st);
hipError_t rows_return_add(float* dst, int64_t ldd, const float* ret, int64_t ldr, const int32_t* ptr,
                           const int32_t* pos, int64_t n, int cols, hipStream_t st);
hipError_t adam_step(int count, float* const* p, const float* const* g, float* const* m, float* const* v,
                     const int64_t* n, const float* step_size, const float* bc2_sqrt, double beta1, double beta2,
                     float eps, float wd, const float* const* tstep, double lr, hipStream_t st);

// I-I kNN neighbour selection (ppgat_knn.hip)
int knn_max_k();
hipError_t knn_topk(const float* S, int64_t ld, int64_t rows, int64_t n_cols, int64_t q0, int k, float min_sim,
                    int32_t* out_idx, float* out_sim, int32_t* out_cnt, hipStream_t st);

// BPR triple sampler (ppgat_sample.hip)
size_t bpr_sampler_workspace_bytes(int64_t n_users, int64_t nnz);
hipError_t bpr_sampler_prepare(const int64_t* ptr, const int32_t* items, int64_t n_users, int64_t nnz,
                               int32_t* items_sorted, int32_t* eligible, int64_t* n_eligible, void* ws,
                               size_t ws_bytes, hipStream_t st);
hipError_t bpr_sample(const int64_t* ptr, const int32_t* items_sorted, const int32_t* eligible,
                      const int64_t* n_eligible, int64_t n_items, int64_t S, uint64_t seed, int64_t t0, int64_t* u,
                      int64_t* i, int64_t* j, int32_t* bad, hipStream_t st);

hipError_t eval_sample(const int64_t* ptr, const int32_t* items_sorted, const int64_t* users, const int64_t* pos,
                       int64_t n_eval, int64_t n_neg, int64_t n_items, uint64_t seed, int64_t* cands, int32_t* bad,
                       hipStream_t st);

// evaluation (ppgat_eval.hip)
hipError_t serve_topk(const float* iv, int64_t n_items, int C, const int64_t* hptr, const int64_t* hist,
                      int64_t max_hist, int B, int k, float* U, float* scores, int32_t* out_idx, float* out_score,
                      hipStream_t st);
hipError_t sampled_rank(const float* Z, int64_t n_users, int64_t n_items, const int32_t* row_map, int C,
                        const int64_t* users, const int64_t* cands, int64_t B, int64_t K1, int32_t* rank,
                        hipStream_t st);

// fusion MLP (ppgat_fusion.hip)
bool fusion_shape_ok(int Dt, int Di, int h1, int d_out);
size_t fusion_workspace_bytes(int Dt, int Di);
hipError_t fusion_fwd(const float* txt, const float* img, const int32_t* img_index, const float* img_fallback,
                      int64_t B, int Dt, int Di, const float* W1, const float* b1, const float* W2, const float* b2,
                      int normalize, float* out, float* z1_out, hipStream_t st,
                      void* ws = nullptr);

// index-range validation (ppgat_debug.hip)
hipError_t count_out_of_range(const void* idx, int elem_bytes, int64_t n, int64_t lo, int64_t hi, int64_t* n_bad,
                              hipStream_t st);

// fusion MLP training: InfoNCE loss + backward, ReLU/dropout (ppgat_infonce.hip)
bool infonce_shape_ok(int64_t B, int D);
size_t infonce_workspace_bytes(int64_t B);
hipError_t infonce(const float* F, const float* T, const float* I, int64_t B, float tau, float* loss, float* dF,
                   float* dT, float* dI, void* ws, hipStream_t st);
hipError_t relu_dropout(const float* z, int64_t n, float p, uint64_t seed, int backward, float* a, hipStream_t st);

// aggregate-then-transform multi-head layer and fp32 MFMA GEMMs (ppgat_xform.hip)
hipError_t seed_snapshot(uint64_t seed, uint64_t* out, hipStream_t st);
bool gemm_nn_shape_ok(int64_t M, int K, int N, int bmode);
// split-bf16 matrix-core GEMMs on (default) or the fp32 MFMA kernels (PPGAT_GEMM=fp32)
bool gemm_split_enabled();
hipError_t gemm_nn(const float* X, int64_t ldx, int64_t M, int K, const float* B, int64_t ldb, int bmode, int N,
                   float alpha, const float* bias, float* Y, int64_t ldy, hipStream_t st,
                   void* ws = nullptr, const float* rS = nullptr, int64_t ldrs = 0, int nv = 0,
                   const float* rA = nullptr, int64_t ldra = 0);
size_t gemm_nn_workspace_bytes(int64_t M, int K, int N);
// the split bf16 images of a GEMM's B operand per (32 nt columns, 32-deep k chunk), once per call
hipError_t nnx_presplit(const float* B, int64_t ldb, int bmode, int K, int N, int nt, uint16_t* img, hipStream_t st);
size_t nnx_image_bytes(int K, int N, int nt);
// the fp16 two-term family (PPGAT_GEMM_F16=0 turns it off): pre-split images + column exponents
bool gemm_f16_enabled();
size_t nnh_image_bytes(int K, int N, int nt);
hipError_t nnh_presplit(const float* B, int64_t ldb, int bmode, int K, int N, int nt, uint16_t* img, int* ecol,
                        hipStream_t st);
// A [2H, K] = [W_h^T att_src[h]; W_h^T att_dst[h]] (any shape) and dx += S A (rank nv <= 16)
hipError_t att_proj(const float* W, const float* att_src, const float* att_dst, int H, int C, int K, float* A,
                    hipStream_t st);
hipError_t rank_update(const float* S, int64_t lds, int nv, const float* A, int64_t lda, int64_t n, int K, float* dx,
                       int64_t lddx, hipStream_t st);
bool gemm_tn_big_shape_ok(int Ma, int Nb);
size_t gemm_tn_big_workspace_bytes(int64_t M, int Ma, int Nb);
hipError_t gemm_tn_big(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int Ma, int Nb, float* out,
                       void* ws, hipStream_t st, const unsigned* b_bound = nullptr, int b_period = 0,
                       float b_scale = 1.f, const unsigned* a_bound = nullptr, float* colsum_out = nullptr);
hipError_t colmax_abs(const float* X, int64_t ldx, int64_t M, int C, unsigned* out, hipStream_t st,
                      const int32_t* src_ptr = nullptr);
bool xgat_shape_ok(int K, int H, int C);
hipError_t xgat_weights(const float* W, const float* att_src, const float* att_dst, int H, int C, int K, float* A,
                        float* Wt, float* Wg, hipStream_t st);
hipError_t xgat_scores(const float* x, int64_t ldx, int64_t n_rows, int64_t n_dst, int K, int H, const float* A,
                       float* s_src, float* s_dst, hipStream_t st);
hipError_t xgat_fwd(const ItemsArg& it, const int32_t* col, const int32_t* eid, const float* x, int64_t ldx, int K,
                    int H, const float* s_src, const float* s_dst, float slope, float p, uint64_t seed,
                    const uint64_t* seed_in, float* agg, float* m, float* invl, float* partial,
                    const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs, hipStream_t st,
                    unsigned* xmax = nullptr);
hipError_t xgat_bwd_pro(const float* gt, const float* agg, const float* s_dst, const float* m, const float* invl,
                        int64_t n, int K, int H, float* nstate, hipStream_t st);
hipError_t xgat_bwd_edges(const ItemsArg& it, const int32_t* row, const int32_t* csc_eid, const int32_t* csc2csr,
                          const float* x, int64_t ldx, int K, int H, const float* s_src, const float* nstate,
                          const float* gt, const float* A_src, float slope, float p, uint64_t seed,
                          const uint64_t* seed_in, float* dx, int64_t lddx, float* S, int64_t lds, float* dz,
                          float* partial, const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs,
                          hipStream_t st);
hipError_t xgat_bwd_edges_g(const ItemsArg& it, const int32_t* row, const int32_t* csc_eid, const int32_t* csc2csr,
                            const float* hs, int C, int H, const float* s_src, const float* nstate, const float* g,
                            int64_t ldg, float slope, float p, uint64_t seed, const uint64_t* seed_in, float* acc,
                            float* S, int64_t lds, float* dz, float* partial, const int32_t* hub_row,
                            const int32_t* hub_ptr, int64_t n_hubs, hipStream_t st, float* pz = nullptr,
                            unsigned* gmax = nullptr);
int nnh_pipeline_variant();  // the fp16 NN main loop: 1 k_gemm_nnh, 2 k_gemm_nnh2, 3 k_gemm_nnh3 (PPGAT_NNH2)
hipError_t xgat_nstate_set_d(float* nstate, const float* D, int64_t n, int H, hipStream_t st);
hipError_t xgat_nstate(const float* s_dst, const float* m, const float* invl, const float* D, int64_t n, int H,
                       float* nstate, hipStream_t st);
hipError_t xgat_bwd_dz(const ItemsArg& it, const int32_t* row, const int32_t* csc_eid, const int32_t* csc2csr, int H,
                       const float* s_src, const float* nstate, float slope, float p, uint64_t seed,
                       const uint64_t* seed_in, float* dz, float* S, int64_t lds, float* partial,
                       const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs, hipStream_t st);
hipError_t xgat_bwd_epi(const float* S, int64_t lds, const float* A_dst, int64_t n, int K, int H, float* dx,
                        int64_t lddx, hipStream_t st);
hipError_t xgat_wgrad(const float* G, const float* GV, const float* W, const float* att_src, const float* att_dst,
                      int H, int C, int K, float* dW, float* datt_src, float* datt_dst, hipStream_t st);
int64_t colsum_blocks(int64_t n);
hipError_t colsum(const float* Y, int64_t ldy, int64_t n, int C, float* out, float* part, hipStream_t st);

}  // namespace ppgat
