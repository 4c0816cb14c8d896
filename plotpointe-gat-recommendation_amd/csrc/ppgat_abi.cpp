// ppgat_abi.cpp -- extern "C" entry points declared in include/ppgat.h.
//
// Argument validation, workspace carving, dispatch to the HIP launchers, thread-local
// error strings, and optional per-kernel HIP-event timing on the launch stream.
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ppgat.h"
#include "ppgat_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  return fail(PPGAT_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

bool channels_ok(int c) {
  return c == 4 || c == 8 || c == 16 || c == 32 || c == 64 || c == 128 || c == 256;
}

// ---- profiling: HIP events recorded on the launch stream around each kernel ----
struct Profiler {
  std::mutex mu;
  bool on = false;
  std::vector<hipEvent_t> pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending[PPGAT_K_COUNT];
  double total_ms[PPGAT_K_COUNT] = {};
  int64_t launches[PPGAT_K_COUNT] = {};

  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  void drain(int k) {
    for (auto& pr : pending[k]) {
      float ms = 0.f;
      if (hipEventSynchronize(pr.second) == hipSuccess && hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
        total_ms[k] += ms;
        launches[k] += 1;
      }
      pool.push_back(pr.first);
      pool.push_back(pr.second);
    }
    pending[k].clear();
  }
};
Profiler g_prof;

struct Timed {
  int k;
  hipStream_t st;
  hipEvent_t a = nullptr;
  Timed(int kid, hipStream_t s) : k(kid), st(s) {
    if (!g_prof.on) return;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    a = g_prof.get();
    if (a) (void)hipEventRecord(a, st);
  }
  ~Timed() {
#if PPGAT_DEBUG
    // debug build: an asynchronous fault surfaces at the entry point that launched it
    (void)hipStreamSynchronize(st);
#endif
    if (!a) return;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    hipEvent_t b = g_prof.get();
    if (!b) return;
    (void)hipEventRecord(b, st);
    g_prof.pending[k].push_back({a, b});
  }
};

#ifndef PPGAT_DEBUG
#define PPGAT_DEBUG 0
#endif

// debug build: index inputs with known bounds are validated before any launch
int debug_range(const void* idx, int elem_bytes, int64_t n, int64_t lo, int64_t hi, const char* who, hipStream_t st) {
  if (!PPGAT_DEBUG || n <= 0 || idx == nullptr) return 0;
  int64_t bad = 0;
  hipError_t e = ppgat::count_out_of_range(idx, elem_bytes, n, lo, hi, &bad, st);
  if (e != hipSuccess) return hip_fail(e, who);
  if (bad)
    return fail(PPGAT_ERR_INVALID, std::string(who) + ": " + std::to_string(bad) + " of " + std::to_string(n) +
                                       " indices outside [" + std::to_string(lo) + ", " + std::to_string(hi) + ")");
  return 0;
}

}  // namespace

extern "C" {

int ppgat_version(void) { return 3; }

int ppgat_debug_build(void) { return PPGAT_DEBUG ? 1 : 0; }

int ppgat_check_index_range(const void* idx, int elem_bytes, int64_t n, int64_t lo, int64_t hi, int64_t* n_bad,
                            void* stream) {
  if (!n_bad || n < 0 || (elem_bytes != 4 && elem_bytes != 8) || (n > 0 && !idx))
    return fail(PPGAT_ERR_INVALID, "check_index_range: bad arguments (elem_bytes 4 or 8)");
  hipError_t e = ppgat::count_out_of_range(idx, elem_bytes, n, lo, hi, n_bad, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "check_index_range");
  return PPGAT_OK;
}

const char* ppgat_last_error(void) { return g_err.c_str(); }

int ppgat_supported_channels(int channels) { return channels_ok(channels) ? 1 : 0; }

int ppgat_csr_workspace_bytes(int64_t n_nodes, int64_t n_edges, size_t* bytes) {
  if (!bytes || n_nodes < 0 || n_edges < 0) return fail(PPGAT_ERR_INVALID, "csr_workspace_bytes: bad arguments");
  *bytes = ppgat::csr_workspace_bytes(n_nodes, n_edges);
  return PPGAT_OK;
}

int ppgat_csr_build(const int64_t* edge_index, int64_t n_edges, int64_t n_nodes, int32_t* rowptr, int32_t* col,
                    int32_t* csr_eid, int32_t* colptr, int32_t* row, int32_t* csc_eid, int32_t* csc2csr,
                    int32_t* bad_count, void* workspace, size_t workspace_bytes, void* stream) {
  if (n_edges < 0 || n_nodes < 0) return fail(PPGAT_ERR_INVALID, "csr_build: negative size");
  if (n_edges >= (int64_t)1 << 31 || n_nodes >= (int64_t)1 << 31)
    return fail(PPGAT_ERR_UNSUPPORTED, "csr_build: N and E must be < 2^31 (int32 CSR indices)");
  if (!rowptr || !colptr || !bad_count || (n_edges > 0 && (!edge_index || !col || !csr_eid || !row || !csc_eid ||
                                                            !csc2csr)))
    return fail(PPGAT_ERR_INVALID, "csr_build: null pointer");
  if (workspace_bytes < ppgat::csr_workspace_bytes(n_nodes, n_edges) || !workspace)
    return fail(PPGAT_ERR_INVALID, "csr_build: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_CSR, st);
  hipError_t e = ppgat::csr_build(edge_index, n_edges, n_nodes, rowptr, col, csr_eid, colptr, row, csc_eid, csc2csr,
                                  bad_count, workspace, workspace_bytes, st);
  if (e != hipSuccess) return hip_fail(e, "csr_build");
  return PPGAT_OK;
}

int64_t ppgat_schedule_capacity(int64_t n_nodes, int64_t n_edges, int32_t max_edges) {
  if (n_nodes < 0 || n_edges < 0 || max_edges < 1) return -1;
  return ppgat::schedule_capacity(n_nodes, n_edges, max_edges);
}

int ppgat_schedule_workspace_bytes(int64_t n_nodes, size_t* bytes) {
  if (!bytes || n_nodes < 0) return fail(PPGAT_ERR_INVALID, "schedule_workspace_bytes: bad arguments");
  *bytes = ppgat::schedule_workspace_bytes(n_nodes);
  return PPGAT_OK;
}

int ppgat_schedule_build(const int32_t* ptr, int64_t n_nodes, int64_t n_edges, int32_t max_edges, int32_t* item_row,
                         int32_t* item_beg, int32_t* item_end, int32_t* hub_row, int32_t* hub_ptr, int32_t* counts,
                         void* workspace, size_t workspace_bytes, void* stream) {
  if (n_nodes < 0 || n_edges < 0 || max_edges < 1 || max_edges >= (1 << 20) - 2)
    return fail(PPGAT_ERR_INVALID, "schedule_build: bad sizes (1 <= max_edges < 2^20-2)");
  if (!ptr || !hub_ptr || !counts || (n_nodes > 0 && (!item_row || !item_beg || !item_end || !hub_row)))
    return fail(PPGAT_ERR_INVALID, "schedule_build: null pointer");
  if (!workspace || workspace_bytes < ppgat::schedule_workspace_bytes(n_nodes))
    return fail(PPGAT_ERR_INVALID, "schedule_build: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_SCHED, st);
  hipError_t e = ppgat::schedule_build(ptr, n_nodes, max_edges, item_row, item_beg, item_end, hub_row, hub_ptr,
                                       counts, workspace, workspace_bytes, st);
  if (e != hipSuccess) return hip_fail(e, "schedule_build");
  return PPGAT_OK;
}

static_assert(ppgat::kShortItemEdges == PPGAT_SHORT_ITEM_EDGES, "short-item bound");

static int check_sched(const ppgat_schedule* s, int64_t n_nodes, const char* who) {
  if (!s) return fail(PPGAT_ERR_INVALID, std::string(who) + ": null schedule");
  if (s->n_items < 0 || s->n_hub_items < 0 || s->n_hubs < 0 || s->n_hub_items > s->n_items ||
      s->n_items < n_nodes - s->n_hubs ||
      (s->n_long_items != -1 && (s->n_long_items < s->n_hub_items || s->n_long_items > s->n_items)))
    return fail(PPGAT_ERR_INVALID, std::string(who) + ": inconsistent schedule counts");
  if (s->n_items > 0 && (!s->item_row || !s->item_beg || !s->item_end))
    return fail(PPGAT_ERR_INVALID, std::string(who) + ": null schedule arrays");
  if (s->n_hubs > 0 && (!s->hub_row || !s->hub_ptr))
    return fail(PPGAT_ERR_INVALID, std::string(who) + ": null hub arrays");
  return PPGAT_OK;
}

int ppgat_node_scores(const float* h, const float* att_src, const float* att_dst, int64_t n_nodes, int heads,
                      int channels, float* s_src, float* s_dst, void* stream) {
  if (!channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "node_scores: unsupported channels");
  if (heads < 1 || n_nodes < 0) return fail(PPGAT_ERR_INVALID, "node_scores: bad sizes");
  if (n_nodes > 0 && (!h || !att_src || !att_dst || !s_src || !s_dst))
    return fail(PPGAT_ERR_INVALID, "node_scores: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_SCORES, st);
  hipError_t e = ppgat::launch_scores(h, att_src, att_dst, n_nodes, heads, channels, s_src, s_dst, st);
  if (e != hipSuccess) return hip_fail(e, "node_scores");
  return PPGAT_OK;
}

static int check_mode(int mode, int heads, const float* bias, float p) {
  if (mode != PPGAT_MODE_PYG && mode != PPGAT_MODE_CUSTOM) return fail(PPGAT_ERR_INVALID, "unknown mode");
  if (mode == PPGAT_MODE_CUSTOM && (heads != 1 || bias != nullptr))
    return fail(PPGAT_ERR_INVALID, "custom mode requires heads == 1 and no bias");
  if (!(p >= 0.f && p < 1.f)) return fail(PPGAT_ERR_INVALID, "dropout p must be in [0, 1)");
  if (heads > ppgat::kMaxHeads) return fail(PPGAT_ERR_UNSUPPORTED, "heads > 8 not supported");
  return PPGAT_OK;
}

static size_t partial_bytes(int64_t n_hub_items, int heads, int channels) {
  return align_up((size_t)(n_hub_items > 0 ? n_hub_items : 1) * heads * (channels + 4) * 4);
}

int ppgat_fwd_workspace_bytes(int64_t n_hub_items, int heads, int channels, size_t* bytes) {
  if (!bytes || n_hub_items < 0 || heads < 1 || channels < 1)
    return fail(PPGAT_ERR_INVALID, "fwd_workspace_bytes: bad arguments");
  *bytes = partial_bytes(n_hub_items, heads, channels);
  return PPGAT_OK;
}

int ppgat_fwd(const ppgat_schedule* sched, const int32_t* col, const int32_t* csr_eid, int64_t n_nodes,
              int64_t n_edges, int heads, int channels, const float* h, const float* s_src, const float* s_dst,
              const float* bias, int mode, float negative_slope, float dropout_p, uint64_t seed, uint64_t* seed_used,
              float* out, float* m, float* inv_l, float* agg, void* workspace, size_t workspace_bytes, void* stream) {
  if (!channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "fwd: unsupported channels");
  if (heads < 1 || n_nodes < 0 || n_edges < 0) return fail(PPGAT_ERR_INVALID, "fwd: bad sizes");
  if (int rc = check_mode(mode, heads, bias, dropout_p)) return rc;
  if (int rc = check_sched(sched, n_nodes, "fwd")) return rc;
  if (n_nodes > 0 && (!h || !s_src || !s_dst || !out || !m || !inv_l))
    return fail(PPGAT_ERR_INVALID, "fwd: null pointer");
  if (n_edges > 0 && !col) return fail(PPGAT_ERR_INVALID, "fwd: null col");
  if (dropout_p > 0.f && n_edges > 0 && !csr_eid) return fail(PPGAT_ERR_INVALID, "fwd: dropout needs csr_eid");
  if (sched->n_hub_items > 0 && (!workspace || workspace_bytes < partial_bytes(sched->n_hub_items, heads, channels)))
    return fail(PPGAT_ERR_INVALID, "fwd: workspace too small");
  const float eps = mode == PPGAT_MODE_PYG ? 1e-16f : 1e-9f;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const ppgat::ItemsArg it{sched->item_row, sched->item_beg, sched->item_end, sched->n_items, sched->n_hub_items,
                           sched->n_long_items};
  Timed t(PPGAT_K_FWD, st);
  hipError_t e = ppgat::launch_fwd(it, col, csr_eid, heads, channels, h, s_src, s_dst, bias, mode, negative_slope,
                                   eps, dropout_p, seed, dropout_p > 0.f ? seed_used : nullptr, out, m, inv_l, agg,
                                   static_cast<float*>(workspace),
                                   sched->hub_row, sched->hub_ptr, sched->n_hubs, st);
  if (e != hipSuccess) return hip_fail(e, "fwd");
  return PPGAT_OK;
}

// ---- backward, staged ---------------------------------------------------------------
int64_t ppgat_bwd_partial_rows(int64_t n_nodes) { return n_nodes < 0 ? -1 : ppgat::epi_blocks(n_nodes); }

int ppgat_bwd_prologue(const float* grad_out, const float* out, const float* agg, const float* bias,
                       const float* s_dst, const float* m, const float* inv_l, int64_t n_nodes, int heads,
                       int channels, int mode, float* nstate, float* grad_bias, float* bias_part, void* stream) {
  if (!channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "bwd_prologue: unsupported channels");
  if (heads < 1 || heads > ppgat::kMaxHeads || n_nodes < 0) return fail(PPGAT_ERR_INVALID, "bwd_prologue: bad sizes");
  if (mode != PPGAT_MODE_PYG && mode != PPGAT_MODE_CUSTOM) return fail(PPGAT_ERR_INVALID, "unknown mode");
  if (heads > 1 && agg == nullptr) return fail(PPGAT_ERR_INVALID, "bwd_prologue: heads > 1 needs the saved agg");
  if (n_nodes > 0 && (!grad_out || !out || !s_dst || !m || !inv_l || !nstate))
    return fail(PPGAT_ERR_INVALID, "bwd_prologue: null pointer");
  if (grad_bias && !bias_part) return fail(PPGAT_ERR_INVALID, "bwd_prologue: grad_bias needs bias_part");
  const float gscale = mode == PPGAT_MODE_PYG ? 1.f / (float)heads : 1.f;
  const int64_t blocks = ppgat::epi_blocks(n_nodes);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e;
  {
    Timed t(PPGAT_K_BWD_PRO, st);
    e = ppgat::launch_bwd_pro(grad_out, out, agg, heads == 1 ? bias : nullptr, s_dst, m, inv_l, n_nodes, heads,
                              channels, gscale, nstate, grad_bias ? bias_part : nullptr, blocks, st);
    if (e == hipSuccess && grad_bias)
      e = ppgat::launch_col_reduce(bias_part, blocks, channels, channels, grad_bias, nullptr, st);
  }
  if (e != hipSuccess) return hip_fail(e, "bwd_prologue");
  return PPGAT_OK;
}

int ppgat_bwd_edges(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                    const int32_t* dz_slot, int64_t n_edges, int heads, int channels, const float* h,
                    const float* s_src, const float* nstate, const float* grad_out, int mode, float negative_slope,
                    float dropout_p, uint64_t seed, const uint64_t* seed_used, float* grad_h, int64_t ld_grad_h,
                    float* ds_src, int64_t ld_ds_src, float* dz, void* workspace, size_t workspace_bytes,
                    void* stream) {
  if (ld_grad_h < (int64_t)heads * channels || (ld_grad_h % 4) || ld_ds_src < heads)
    return fail(PPGAT_ERR_INVALID, "bwd_edges: bad leading dimensions (ld_grad_h >= H*C, multiple of 4)");
  if (!channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "bwd_edges: unsupported channels");
  if (heads < 1 || heads > ppgat::kMaxHeads || n_edges < 0) return fail(PPGAT_ERR_INVALID, "bwd_edges: bad sizes");
  if (mode != PPGAT_MODE_PYG && mode != PPGAT_MODE_CUSTOM) return fail(PPGAT_ERR_INVALID, "unknown mode");
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(PPGAT_ERR_INVALID, "dropout p must be in [0, 1)");
  if (int rc = check_sched(src_sched, 0, "bwd_edges")) return rc;
  if (src_sched->n_items > 0 && (!h || !s_src || !grad_h || !ds_src))
    return fail(PPGAT_ERR_INVALID, "bwd_edges: null pointer");
  if (n_edges > 0 && (!row || !nstate || !grad_out || !dz))  // dz_slot NULL: dz in CSC order
    return fail(PPGAT_ERR_INVALID, "bwd_edges: null edge pointer");
  if (dropout_p > 0.f && n_edges > 0 && !csc_eid) return fail(PPGAT_ERR_INVALID, "bwd_edges: dropout needs csc_eid");
  if (src_sched->n_hub_items > 0 &&
      (!workspace || workspace_bytes < partial_bytes(src_sched->n_hub_items, heads, channels)))
    return fail(PPGAT_ERR_INVALID, "bwd_edges: workspace too small");
  const float gscale = mode == PPGAT_MODE_PYG ? 1.f / (float)heads : 1.f;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const ppgat::ItemsArg it{src_sched->item_row, src_sched->item_beg, src_sched->item_end, src_sched->n_items,
                           src_sched->n_hub_items, src_sched->n_long_items};
  hipError_t e;
  {
    Timed t(PPGAT_K_BWD_SRC, st);
    e = ppgat::launch_bwd_src(it, row, csc_eid, dz_slot, heads, channels, h, s_src, nstate, grad_out, mode,
                              negative_slope, gscale, dropout_p, seed, seed_used, grad_h, ld_grad_h, ds_src,
                              ld_ds_src, dz,
                              static_cast<float*>(workspace), src_sched->hub_row, src_sched->hub_ptr,
                              src_sched->n_hubs, st);
  }
  if (e != hipSuccess) return hip_fail(e, "bwd_edges");
  return PPGAT_OK;
}

static int bwd_dst_sum_impl(const ppgat_schedule* fwd_sched, int64_t n_nodes, int heads, const float* dz,
                            const int32_t* csr2csc, float* ds_dst, int64_t ld_ds_dst, void* workspace,
                            size_t workspace_bytes, void* stream) {
  if (n_nodes < 0 || heads < 1 || ld_ds_dst < heads) return fail(PPGAT_ERR_INVALID, "bwd_dst_sum: bad sizes");
  if (int rc = check_sched(fwd_sched, n_nodes, "bwd_dst_sum")) return rc;
  if (n_nodes > 0 && !ds_dst) return fail(PPGAT_ERR_INVALID, "bwd_dst_sum: null pointer");
  const size_t need = (size_t)fwd_sched->n_hub_items * heads * sizeof(float);
  if (need > 0 && (!workspace || workspace_bytes < need))
    return fail(PPGAT_ERR_INVALID, "bwd_dst_sum: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_BWD_EPI, st);
  const ppgat::ItemsArg it{fwd_sched->item_row, fwd_sched->item_beg, fwd_sched->item_end, fwd_sched->n_items,
                           fwd_sched->n_hub_items, fwd_sched->n_long_items};
  hipError_t e = ppgat::launch_dst_sum(it, heads, dz, csr2csc, ds_dst, ld_ds_dst, static_cast<float*>(workspace),
                                       fwd_sched->hub_row, fwd_sched->hub_ptr, fwd_sched->n_hubs, st);
  if (e != hipSuccess) return hip_fail(e, "bwd_dst_sum");
  return PPGAT_OK;
}

int ppgat_bwd_dst_sum(const ppgat_schedule* fwd_sched, int64_t n_nodes, int heads, const float* dz, float* ds_dst,
                      int64_t ld_ds_dst, void* workspace, size_t workspace_bytes, void* stream) {
  return bwd_dst_sum_impl(fwd_sched, n_nodes, heads, dz, nullptr, ds_dst, ld_ds_dst, workspace, workspace_bytes,
                          stream);
}

int ppgat_bwd_dst_sum_csc(const ppgat_schedule* fwd_sched, int64_t n_nodes, int64_t n_edges, int heads,
                          const float* dz, const int32_t* csr2csc, float* ds_dst, int64_t ld_ds_dst, void* workspace,
                          size_t workspace_bytes, void* stream) {
  if (n_edges > 0 && !csr2csc) return fail(PPGAT_ERR_INVALID, "bwd_dst_sum_csc: null csr2csc");
  if (int rc = debug_range(csr2csc, 4, n_edges, 0, n_edges, "bwd_dst_sum_csc: csr2csc",
                           static_cast<hipStream_t>(stream)))
    return rc;
  return bwd_dst_sum_impl(fwd_sched, n_nodes, heads, dz, csr2csc, ds_dst, ld_ds_dst, workspace, workspace_bytes,
                          stream);
}

int ppgat_stream_copy(const void* src, void* dst, int64_t n_bytes, void* stream) {
  if (n_bytes < 0 || n_bytes % 16 || (n_bytes > 0 && (!src || !dst)) ||
      reinterpret_cast<uintptr_t>(src) % 16 || reinterpret_cast<uintptr_t>(dst) % 16)
    return fail(PPGAT_ERR_INVALID, "stream_copy: pointers and size must be non-null multiples of 16");
  hipError_t e = ppgat::launch_stream_copy(src, dst, n_bytes, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "stream_copy");
  return PPGAT_OK;
}

int ppgat_invert_index(const int32_t* index, int64_t n, int32_t* inverse, void* stream) {
  if (n < 0 || (n > 0 && (!index || !inverse))) return fail(PPGAT_ERR_INVALID, "invert_index: bad arguments");
  if (int rc = debug_range(index, 4, n, 0, n, "invert_index: index", static_cast<hipStream_t>(stream))) return rc;
  hipError_t e = ppgat::launch_invert_index(index, n, inverse, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "invert_index");
  return PPGAT_OK;
}

int ppgat_bwd_epilogue(const int32_t* rowptr, int64_t n_nodes, int heads, int channels, const float* h,
                       const float* att_src, const float* att_dst, const float* ds_src, const float* dz,
                       float* grad_h, float* grad_att_src, float* grad_att_dst, float* part, void* stream) {
  if (!channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "bwd_epilogue: unsupported channels");
  if (heads < 1 || heads > ppgat::kMaxHeads || n_nodes < 0) return fail(PPGAT_ERR_INVALID, "bwd_epilogue: bad sizes");
  if (!att_src || !att_dst || !grad_att_src || !grad_att_dst || !part)
    return fail(PPGAT_ERR_INVALID, "bwd_epilogue: null pointer");
  if (n_nodes > 0 && (!rowptr || !h || !ds_src || !grad_h)) return fail(PPGAT_ERR_INVALID, "bwd_epilogue: null pointer");
  const int64_t blocks = ppgat::epi_blocks(n_nodes);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e;
  {
    Timed t(PPGAT_K_BWD_EPI, st);
    e = ppgat::launch_bwd_epi(rowptr, n_nodes, heads, channels, h, att_src, att_dst, ds_src, dz, grad_h, part, blocks,
                              st);
  }
  if (e != hipSuccess) return hip_fail(e, "bwd_epilogue");
  {
    Timed t(PPGAT_K_BWD_RED, st);
    e = ppgat::launch_col_reduce(part, blocks, 2 * heads * channels, heads * channels, grad_att_src, grad_att_dst,
                                 st);
  }
  if (e != hipSuccess) return hip_fail(e, "bwd_reduce");
  return PPGAT_OK;
}

// ---- backward, composed (single device): nstate | ds_src | dz | partials | hub partial ----
int ppgat_bwd_workspace_bytes(int64_t n_nodes, int64_t n_edges, int64_t n_hub_items, int heads, int channels,
                              size_t* bytes) {
  if (!bytes || n_nodes < 0 || n_edges < 0 || n_hub_items < 0 || heads < 1 || channels < 1)
    return fail(PPGAT_ERR_INVALID, "bwd_workspace_bytes: bad arguments");
  const size_t ns = align_up((size_t)n_nodes * heads * 16 + 16);
  const size_t nh = align_up((size_t)n_nodes * heads * 4 + 4);
  const size_t eh = align_up((size_t)n_edges * heads * 4 + 4);
  const size_t part = align_up((size_t)ppgat::epi_blocks(n_nodes) * (2 * heads + 1) * channels * 4);
  *bytes = ns + nh + eh + part + partial_bytes(n_hub_items, heads, channels);
  return PPGAT_OK;
}

int ppgat_bwd(const ppgat_schedule* sched, const int32_t* rowptr, const int32_t* row, const int32_t* csc_eid,
              const int32_t* csc2csr, int64_t n_nodes, int64_t n_edges, int heads, int channels, const float* h,
              const float* s_src, const float* s_dst, const float* att_src, const float* att_dst, const float* bias,
              const float* out, const float* agg, const float* m, const float* inv_l, const float* grad_out, int mode,
              float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used, float* grad_h,
              float* grad_att_src, float* grad_att_dst, float* grad_bias, void* workspace, size_t workspace_bytes,
              void* stream) {
  if (!channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "bwd: unsupported channels");
  if (heads < 1 || n_nodes < 0 || n_edges < 0) return fail(PPGAT_ERR_INVALID, "bwd: bad sizes");
  if (int rc = check_mode(mode, heads, bias, dropout_p)) return rc;
  if (int rc = check_sched(sched, n_nodes, "bwd")) return rc;
  size_t need = 0;
  ppgat_bwd_workspace_bytes(n_nodes, n_edges, sched->n_hub_items, heads, channels, &need);
  if (!workspace || workspace_bytes < need) return fail(PPGAT_ERR_INVALID, "bwd: workspace too small");
  const size_t ns = align_up((size_t)n_nodes * heads * 16 + 16);
  const size_t nh = align_up((size_t)n_nodes * heads * 4 + 4);
  const size_t eh = align_up((size_t)n_edges * heads * 4 + 4);
  const int64_t blocks = ppgat::epi_blocks(n_nodes);
  const size_t part = align_up((size_t)blocks * (2 * heads + 1) * channels * 4);
  char* p = static_cast<char*>(workspace);
  float* nstate = reinterpret_cast<float*>(p);
  float* ds_src = reinterpret_cast<float*>(p + ns);
  float* dz = reinterpret_cast<float*>(p + ns + nh);
  float* bpart = reinterpret_cast<float*>(p + ns + nh + eh);
  float* hpart = reinterpret_cast<float*>(p + ns + nh + eh + part);
  float* bias_part = bpart + (size_t)blocks * 2 * heads * channels;
  if (int rc = ppgat_bwd_prologue(grad_out, out, agg, bias, s_dst, m, inv_l, n_nodes, heads, channels, mode, nstate,
                                  grad_bias, bias_part, stream))
    return rc;
  if (int rc = ppgat_bwd_edges(sched, row, csc_eid, csc2csr, n_edges, heads, channels, h, s_src, nstate, grad_out,
                               mode, negative_slope, dropout_p, seed, seed_used, grad_h, (int64_t)heads * channels,
                               ds_src,
                               heads, dz, hpart, partial_bytes(sched->n_hub_items, heads, channels), stream))
    return rc;
  return ppgat_bwd_epilogue(rowptr, n_nodes, heads, channels, h, att_src, att_dst, ds_src, dz, grad_h, grad_att_src,
                            grad_att_dst, bpart, stream);
}

// ---- training-step kernels ----
int ppgat_bpr_workspace_bytes(int64_t n_rows, int64_t n_samples, int channels, size_t* bytes) {
  if (!bytes || n_rows < 0 || n_samples < 0) return fail(PPGAT_ERR_INVALID, "bpr_workspace_bytes: bad arguments");
  if (!ppgat::bpr_channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "bpr: channels must be 32/64/128/256");
  *bytes = ppgat::bpr_workspace_bytes(n_rows, n_samples, channels);
  return PPGAT_OK;
}

static int check_bpr(int64_t n_users, int64_t n_items, int channels, int64_t S, const void* Z, const void* u,
                     const void* i, const void* j, const char* who) {
  if (!ppgat::bpr_channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, std::string(who) + ": channels");
  if (n_users < 1 || n_items < 1 || S < 0) return fail(PPGAT_ERR_INVALID, std::string(who) + ": bad sizes");
  if (n_users + n_items >= ((int64_t)1 << 31) || 4 * S >= ((int64_t)1 << 31))
    return fail(PPGAT_ERR_UNSUPPORTED, std::string(who) + ": sizes exceed int32 indexing");
  if (!Z || (S > 0 && (!u || !i || !j))) return fail(PPGAT_ERR_INVALID, std::string(who) + ": null pointer");
  return PPGAT_OK;
}

int ppgat_bpr_fwd(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                  int channels, const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples, int loss_kind,
                  float* loss, float* coef, int32_t* bad_count, void* workspace, size_t workspace_bytes,
                  void* stream) {
  if (int rc = check_bpr(n_users, n_items, channels, n_samples, Z, u, i, j, "bpr_fwd")) return rc;
  {
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (int rc = debug_range(u, 8, n_samples, 0, n_users, "bpr_fwd: u", st)) return rc;
    if (int rc = debug_range(i, 8, n_samples, 0, n_items, "bpr_fwd: i", st)) return rc;
    if (int rc = debug_range(j, 8, n_samples, 0, n_items, "bpr_fwd: j", st)) return rc;
  }
  if (row_map == nullptr ? n_rows != n_users + n_items : n_rows < 1)
    return fail(PPGAT_ERR_INVALID, "bpr_fwd: n_rows must be n_users + n_items without a row_map");
  if (loss_kind != 0 && loss_kind != 1) return fail(PPGAT_ERR_INVALID, "bpr_fwd: loss_kind must be 0 (bpr) or 1 (bce)");
  if (!loss || (n_samples > 0 && !coef)) return fail(PPGAT_ERR_INVALID, "bpr_fwd: null output");
  if (!workspace || workspace_bytes < ppgat::bpr_workspace_bytes(n_rows, n_samples, channels))
    return fail(PPGAT_ERR_INVALID, "bpr_fwd: workspace too small");
  hipError_t e = ppgat::bpr_fwd(Z, n_rows, n_users, n_items, row_map, channels, u, i, j, n_samples, loss_kind, loss, coef,
                                bad_count, workspace, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "bpr_fwd");
  return PPGAT_OK;
}

int ppgat_bpr_bwd(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                  int channels, const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples,
                  const float* coef, const float* grad_loss, float* grad_Z, void* workspace, size_t workspace_bytes,
                  void* stream) {
  if (int rc = check_bpr(n_users, n_items, channels, n_samples, Z, u, i, j, "bpr_bwd")) return rc;
  if (row_map == nullptr ? n_rows != n_users + n_items : n_rows < 1)
    return fail(PPGAT_ERR_INVALID, "bpr_bwd: n_rows must be n_users + n_items without a row_map");
  if (!grad_Z || !grad_loss || (n_samples > 0 && !coef)) return fail(PPGAT_ERR_INVALID, "bpr_bwd: null pointer");
  if (!workspace || workspace_bytes < ppgat::bpr_workspace_bytes(n_rows, n_samples, channels))
    return fail(PPGAT_ERR_INVALID, "bpr_bwd: workspace too small");
  hipError_t e = ppgat::bpr_bwd(Z, n_rows, n_users, n_items, row_map, channels, u, i, j, n_samples, coef, grad_loss,
                                grad_Z, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "bpr_bwd");
  return PPGAT_OK;
}

int ppgat_bpr_bwd_prepare(int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map, int channels,
                          const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples, void* workspace,
                          size_t workspace_bytes, void* stream) {
  const float dummy = 0.f;  // check_bpr wants a Z; the prepare never reads one
  if (int rc = check_bpr(n_users, n_items, channels, n_samples, &dummy, u, i, j, "bpr_bwd_prepare")) return rc;
  if (row_map == nullptr ? n_rows != n_users + n_items : n_rows < 1)
    return fail(PPGAT_ERR_INVALID, "bpr_bwd_prepare: n_rows must be n_users + n_items without a row_map");
  if (!workspace || workspace_bytes < ppgat::bpr_workspace_bytes(n_rows, n_samples, channels))
    return fail(PPGAT_ERR_INVALID, "bpr_bwd_prepare: workspace too small");
  hipError_t e = ppgat::bpr_bwd_prepare(n_rows, n_users, n_items, row_map, channels, u, i, j, n_samples, workspace,
                                        workspace_bytes, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "bpr_bwd_prepare");
  return PPGAT_OK;
}

int ppgat_bpr_bwd_prepared(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                           int channels, const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples,
                           const float* coef, const float* grad_loss, float* grad_Z, void* workspace,
                           size_t workspace_bytes, void* stream) {
  if (int rc = check_bpr(n_users, n_items, channels, n_samples, Z, u, i, j, "bpr_bwd_prepared")) return rc;
  if (row_map == nullptr ? n_rows != n_users + n_items : n_rows < 1)
    return fail(PPGAT_ERR_INVALID, "bpr_bwd_prepared: n_rows must be n_users + n_items without a row_map");
  if (!grad_Z || !grad_loss || (n_samples > 0 && !coef)) return fail(PPGAT_ERR_INVALID, "bpr_bwd_prepared: null pointer");
  if (!workspace || workspace_bytes < ppgat::bpr_workspace_bytes(n_rows, n_samples, channels))
    return fail(PPGAT_ERR_INVALID, "bpr_bwd_prepared: workspace too small");
  hipError_t e = ppgat::bpr_bwd_finish(Z, n_rows, n_users, n_items, row_map, channels, u, i, j, n_samples, coef,
                                       grad_loss, grad_Z, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "bpr_bwd_prepared");
  return PPGAT_OK;
}

int ppgat_bpr_bwd_producer(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, int channels,
                           const int64_t* u, const int64_t* i, const int64_t* j, int64_t n_samples, const float* coef,
                           const float* grad_loss, float* grad_Z, const float* prev_bias, const float* prev_s_dst,
                           const float* prev_m, const float* prev_inv_l, float prev_gscale, float* prev_nstate,
                           float* prev_grad_bias, void* workspace, size_t workspace_bytes, void* stream) {
  if (int rc = check_bpr(n_users, n_items, channels, n_samples, Z, u, i, j, "bpr_bwd_producer")) return rc;
  if (n_rows != n_users + n_items) return fail(PPGAT_ERR_INVALID, "bpr_bwd_producer: n_rows must be n_users + n_items");
  if (!grad_Z || !grad_loss || (n_samples > 0 && !coef)) return fail(PPGAT_ERR_INVALID, "bpr_bwd_producer: null pointer");
  if (!prev_s_dst || !prev_m || !prev_inv_l || !prev_nstate)
    return fail(PPGAT_ERR_INVALID, "bpr_bwd_producer: the producer's state is required");
  if ((reinterpret_cast<uintptr_t>(prev_nstate) | reinterpret_cast<uintptr_t>(prev_bias)) % 16)
    return fail(PPGAT_ERR_UNSUPPORTED, "bpr_bwd_producer: nstate / bias 16-byte aligned");
  if (!workspace || workspace_bytes < ppgat::bpr_workspace_bytes(n_rows, n_samples, channels))
    return fail(PPGAT_ERR_INVALID, "bpr_bwd_producer: workspace too small");
  const ppgat::BprProducer prod{prev_bias, prev_s_dst, prev_m, prev_inv_l, prev_gscale, prev_nstate, prev_grad_bias};
  hipError_t e = ppgat::bpr_bwd(Z, n_rows, n_users, n_items, nullptr, channels, u, i, j, n_samples, coef, grad_loss,
                                grad_Z, workspace, workspace_bytes, static_cast<hipStream_t>(stream), &prod);
  if (e != hipSuccess) return hip_fail(e, "bpr_bwd_producer");
  return PPGAT_OK;
}

// workspace covers both GEMM variants (the choice also depends on V's alignment)
static size_t tn_ws(int64_t n, int m, int k, int nv) {
  const size_t a = ppgat::tn128_workspace_bytes(n), b = ppgat::gemm_tn_workspace_bytes(n, m, k, nv);
  return (m <= 128 && k <= 128 && nv <= 2) ? (a > b ? a : b) : b;
}

int ppgat_gemm_tn_workspace_bytes(int64_t n, int m, int k, int nv, size_t* bytes) {
  if (!bytes || n < 0 || m < 1 || k < 1 || nv < 0) return fail(PPGAT_ERR_INVALID, "gemm_tn_workspace_bytes: bad arguments");
  *bytes = tn_ws(n, m, k, nv);
  return PPGAT_OK;
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) % 16) == 0; }

int ppgat_gemm_tn_seg(const float* A, int64_t lda, const float* b0, int64_t ldb0, const float* b1, int64_t ldb1,
                      int64_t split, int64_t n, int m, int k, float* out, float* colsum, const float* V, int64_t ldv,
                      int nv, float* vout, void* workspace, size_t workspace_bytes, void* stream) {
  if (n < 0 || m < 1 || k < 1 || nv < 0 || nv > 16) return fail(PPGAT_ERR_INVALID, "gemm_tn: bad sizes (nv <= 16)");
  if (split < 0 || split > n) return fail(PPGAT_ERR_INVALID, "gemm_tn: split outside [0, n]");
  if (lda < m || ldb0 < k || (b1 && ldb1 < k) || (nv > 0 && ldv < nv))
    return fail(PPGAT_ERR_INVALID, "gemm_tn: bad leading dimension");
  // the skinny kernel reads A (and V) by scalars: only B's rows need 16-byte alignment there;
  // it takes every m <= 16 product, with or without the extras (path-independent bits)
  const bool skinny = m <= 16 && nv <= 16 && !(b1 && split < n) && (k % 4) == 0 && k <= 1024;
  if ((!skinny && ((lda % 4) || !al16(A))) || (ldb0 % 4) || (b1 && (ldb1 % 4)) || !al16(b0) || (b1 && !al16(b1)))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_tn: A/B rows must be 16-byte aligned");
  if (!out || (n > 0 && (!A || !b0)) || (nv > 0 && (!V || !vout)))
    return fail(PPGAT_ERR_INVALID, "gemm_tn: null pointer");
  if (!workspace || workspace_bytes < tn_ws(n, m, k, nv))
    return fail(PPGAT_ERR_INVALID, "gemm_tn: workspace too small");
  // the register-accumulator kernel pays a fixed per-wave ramp/epilogue: below ~1e5 rows the
  // LDS-staged split-N kernel is faster (item_proj's 63k rows: 30 vs 46 us)
  // skinny A (m <= 16, plain A^T B): the VALU kernel of ppgat::gemm_tn, not a padded MFMA tile
  const bool fast = !skinny && ppgat::tn128_shape_ok(m, k, nv, V, ldv) && (n >= 100000 || (b1 && split < n));
  if (!fast && b1 && split < n) return fail(PPGAT_ERR_UNSUPPORTED, "gemm_tn: segmented B needs m, k <= 128, nv <= 2");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_GEMM_TN, st);
  hipError_t e = fast ? ppgat::tn128(A, lda, b0, ldb0, b1, ldb1, b1 ? split : n, n, m, k, out, colsum,
                                     nv > 0 ? V : nullptr, ldv, nv, vout, workspace, st)
                      : ppgat::gemm_tn(A, lda, b0, ldb0, n, m, k, out, colsum, nv > 0 ? V : nullptr, ldv, nv, vout,
                                       workspace, st);
  if (e != hipSuccess) return hip_fail(e, "gemm_tn");
  return PPGAT_OK;
}

int ppgat_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t n, int m, int k, float* out,
                  float* colsum, const float* V, int64_t ldv, int nv, float* vout, void* workspace,
                  size_t workspace_bytes, void* stream) {
  return ppgat_gemm_tn_seg(A, lda, B, ldb, nullptr, 0, n, n, m, k, out, colsum, V, ldv, nv, vout, workspace,
                           workspace_bytes, stream);
}

int ppgat_project_supported(int k, int out_cols) { return ppgat::proj_shape_ok(k, out_cols) ? 1 : 0; }

int ppgat_project(const float* x0, int64_t ldx0, const float* x1, int64_t ldx1, int64_t split, int64_t n, int k,
                  const float* w, int64_t ldw, int out_cols, const float* bias, const float* att_src,
                  const float* att_dst, float* y, int64_t ldy, float* s_src, float* s_dst, void* stream) {
  if (!ppgat::proj_shape_ok(k, out_cols)) return fail(PPGAT_ERR_UNSUPPORTED, "project: needs k <= 128, k % 4 == 0, out_cols == 128");
  if (n < 0 || split < 0 || split > n) return fail(PPGAT_ERR_INVALID, "project: bad sizes");
  if (ldx0 < k || (x1 && ldx1 < k) || ldw < k || ldy < out_cols || (ldx0 % 4) || (x1 && (ldx1 % 4)) || (ldw % 4))
    return fail(PPGAT_ERR_INVALID, "project: bad leading dimension (>= width, multiple of 4)");
  if (n > 0 && (!x0 || !w || !y || (att_src && (!att_dst || !s_src || !s_dst))))
    return fail(PPGAT_ERR_INVALID, "project: null pointer");
  if (!al16(x0) || (x1 && !al16(x1)) || !al16(w)) return fail(PPGAT_ERR_UNSUPPORTED, "project: rows must be 16-byte aligned");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_PROJ, st);
  hipError_t e = ppgat::proj_fwd(x0, ldx0, x1, ldx1, x1 ? split : n, n, k, w, ldw, bias, att_src, att_dst, y, ldy,
                                 s_src, s_dst, st);
  if (e != hipSuccess) return hip_fail(e, "project");
  return PPGAT_OK;
}

int ppgat_project_bwd_input(const float* D, int64_t ldd, int64_t n, int k, const float* w, int64_t ldw, int out_cols,
                            const float* att_src, const float* att_dst, const float* S, int64_t lds, float* dx,
                            int64_t lddx, void* stream) {
  if (!ppgat::proj_shape_ok(k, out_cols)) return fail(PPGAT_ERR_UNSUPPORTED, "project_bwd_input: needs k <= 128, k % 4 == 0, out_cols == 128");
  if (n < 0) return fail(PPGAT_ERR_INVALID, "project_bwd_input: bad sizes");
  if (ldd < k || (ldd % 4) || ldw < out_cols || lddx < out_cols || lds < 2 || (lds % 2))
    return fail(PPGAT_ERR_INVALID, "project_bwd_input: bad leading dimension (ldd >= k and % 4, lds >= 2 and even)");
  if (n > 0 && (!D || !w || !att_src || !att_dst || !S || !dx)) return fail(PPGAT_ERR_INVALID, "project_bwd_input: null pointer");
  if (!al16(D) || (reinterpret_cast<uintptr_t>(S) % 8)) return fail(PPGAT_ERR_UNSUPPORTED, "project_bwd_input: D rows 16-byte, S rows 8-byte aligned");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_PROJ, st);
  hipError_t e = ppgat::proj_dx(D, ldd, n, k, w, ldw, att_src, att_dst, S, lds, dx, lddx, st);
  if (e != hipSuccess) return hip_fail(e, "project_bwd_input");
  return PPGAT_OK;
}

int ppgat_project_bwd_fused_supported(int k) { return ppgat::dxw_ok(k, k) ? 1 : 0; }

int ppgat_project_bwd_fused_workspace_bytes(int64_t n, size_t* bytes) {
  if (n < 0 || !bytes) return fail(PPGAT_ERR_INVALID, "project_bwd_fused_workspace_bytes: bad arguments");
  *bytes = ppgat::dxw_workspace_bytes(n);
  return PPGAT_OK;
}

static int project_bwd_fused_impl(const float* D, int64_t ldd, const float* S, int64_t lds, const float* x0,
                                  int64_t ldx0, const float* x1, int64_t ldx1, int64_t split, int64_t n, int k,
                                  const float* w, int64_t ldw, const float* att_src, const float* att_dst, float* dx,
                                  int64_t lddx, float* G, float* GV, const ppgat::DxwProducer* prod, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  if (!ppgat::dxw_ok(k, k)) return fail(PPGAT_ERR_UNSUPPORTED, "project_bwd_fused: needs k == 128 and the split GEMMs");
  if (n < 0 || split < 0 || split > n) return fail(PPGAT_ERR_INVALID, "project_bwd_fused: bad sizes");
  if (ldd < k || (ldd % 4) || ldx0 < k || (ldx0 % 4) || (x1 && (ldx1 < k || (ldx1 % 4))) || ldw < k ||
      (dx && (lddx < k || (lddx % 4))) || lds < 2 || (lds % 2))
    return fail(PPGAT_ERR_INVALID, "project_bwd_fused: bad leading dimension (>= k and % 4; lds >= 2 and even)");
  if (!G || !GV || (n > 0 && (!D || !S || !x0 || !w || !att_src || !att_dst)))
    return fail(PPGAT_ERR_INVALID, "project_bwd_fused: null pointer");
  if (!al16(D) || !al16(x0) || (x1 && !al16(x1)) || (dx && !al16(dx)) || (reinterpret_cast<uintptr_t>(S) % 8))
    return fail(PPGAT_ERR_UNSUPPORTED, "project_bwd_fused: D/x/dx rows 16-byte, S rows 8-byte aligned");
  if (!workspace || workspace_bytes < ppgat::dxw_workspace_bytes(n))
    return fail(PPGAT_ERR_INVALID, "project_bwd_fused: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_PROJ_BWD, st);
  hipError_t e = ppgat::dxw(D, ldd, S, lds, x0, ldx0, x1, ldx1, x1 ? split : n, n, w, ldw, att_src, att_dst, dx, lddx,
                            G, GV, workspace, st, prod);
  if (e != hipSuccess) return hip_fail(e, "project_bwd_fused");
  return PPGAT_OK;
}

int ppgat_project_bwd_fused(const float* D, int64_t ldd, const float* S, int64_t lds, const float* x0, int64_t ldx0,
                            const float* x1, int64_t ldx1, int64_t split, int64_t n, int k, const float* w,
                            int64_t ldw, const float* att_src, const float* att_dst, float* dx, int64_t lddx,
                            float* G, float* GV, void* workspace, size_t workspace_bytes, void* stream) {
  return project_bwd_fused_impl(D, ldd, S, lds, x0, ldx0, x1, ldx1, split, n, k, w, ldw, att_src, att_dst, dx, lddx, G,
                                GV, nullptr, workspace, workspace_bytes, stream);
}

int ppgat_project_bwd_fused_producer(const float* D, int64_t ldd, const float* S, int64_t lds, const float* x0,
                                     int64_t ldx0, const float* x1, int64_t ldx1, int64_t split, int64_t n, int k,
                                     const float* w, int64_t ldw, const float* att_src, const float* att_dst,
                                     float* dx, int64_t lddx, float* G, float* GV, const float* prev_bias,
                                     const float* prev_s_dst, const float* prev_m, const float* prev_inv_l,
                                     float prev_gscale, float* prev_nstate, float* prev_grad_bias, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  if (n > 0 && (!dx || !prev_s_dst || !prev_m || !prev_inv_l || !prev_nstate))
    return fail(PPGAT_ERR_INVALID, "project_bwd_fused_producer: dx and the producer's state are required");
  if ((prev_nstate && !al16(prev_nstate)) || (prev_bias && !al16(prev_bias)) || (prev_grad_bias && !al16(prev_grad_bias)))
    return fail(PPGAT_ERR_UNSUPPORTED, "project_bwd_fused_producer: nstate / bias 16-byte aligned");
  const ppgat::DxwProducer prod{prev_bias, prev_s_dst, prev_m, prev_inv_l, prev_gscale, prev_nstate, prev_grad_bias};
  return project_bwd_fused_impl(D, ldd, S, lds, x0, ldx0, x1, ldx1, split, n, k, w, ldw, att_src, att_dst, dx, lddx, G,
                                GV, &prod, workspace, workspace_bytes, stream);
}

int ppgat_weight_grads(const float* G, const float* GV, const float* w, const float* att_src, const float* att_dst,
                       int heads, int channels, int in_channels, float* dW, float* datt_src, float* datt_dst,
                       void* stream) {
  if (heads < 1 || channels < 1 || in_channels < 1) return fail(PPGAT_ERR_INVALID, "weight_grads: bad sizes");
  if (!G || !GV || !w || !att_src || !att_dst || !dW || !datt_src || !datt_dst)
    return fail(PPGAT_ERR_INVALID, "weight_grads: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_GEMM_TN, st);
  hipError_t e = ppgat::wgrad_assemble(G, GV, w, att_src, att_dst, heads, channels, in_channels, dW, datt_src,
                                       datt_dst, st);
  if (e != hipSuccess) return hip_fail(e, "weight_grads");
  return PPGAT_OK;
}

int ppgat_adam_max_tensors(void) { return ppgat::adam_max_tensors(); }

int ppgat_adam_step(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                    float* const* exp_avg_sq, const int64_t* numel, const float* step_size,
                    const float* bias_correction2_sqrt, double beta1, double beta2, float eps, float weight_decay,
                    void* stream) {
  if (count < 0 || count > ppgat::adam_max_tensors()) return fail(PPGAT_ERR_INVALID, "adam_step: bad tensor count");
  if (count > 0 && (!params || !grads || !exp_avg || !exp_avg_sq || !numel || !step_size || !bias_correction2_sqrt))
    return fail(PPGAT_ERR_INVALID, "adam_step: null pointer");
  for (int t = 0; t < count; ++t) {
    if (numel[t] < 0) return fail(PPGAT_ERR_INVALID, "adam_step: negative numel");
    if (numel[t] > 0 && (!params[t] || !grads[t] || !exp_avg[t] || !exp_avg_sq[t]))
      return fail(PPGAT_ERR_INVALID, "adam_step: null tensor");
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_ADAM, st);
  hipError_t e = ppgat::adam_step(count, params, grads, exp_avg, exp_avg_sq, numel, step_size, bias_correction2_sqrt,
                                  beta1, beta2, eps, weight_decay, nullptr, 0.0, st);
  if (e != hipSuccess) return hip_fail(e, "adam_step");
  return PPGAT_OK;
}

int ppgat_adam_step_device(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                           float* const* exp_avg_sq, const int64_t* numel, const float* const* step, double lr,
                           double beta1,
                           double beta2, float eps, float weight_decay, void* stream) {
  if (count < 0 || count > ppgat::adam_max_tensors())
    return fail(PPGAT_ERR_INVALID, "adam_step_device: bad tensor count");
  if (count > 0 && (!params || !grads || !exp_avg || !exp_avg_sq || !numel || !step))
    return fail(PPGAT_ERR_INVALID, "adam_step_device: null pointer");
  for (int t = 0; t < count; ++t) {
    if (numel[t] < 0) return fail(PPGAT_ERR_INVALID, "adam_step_device: negative numel");
    if (!step[t]) return fail(PPGAT_ERR_INVALID, "adam_step_device: null step pointer");
    if (numel[t] > 0 && (!params[t] || !grads[t] || !exp_avg[t] || !exp_avg_sq[t]))
      return fail(PPGAT_ERR_INVALID, "adam_step_device: null tensor");
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_ADAM, st);
  hipError_t e = ppgat::adam_step(count, params, grads, exp_avg, exp_avg_sq, numel, nullptr, nullptr, beta1, beta2,
                                  eps, weight_decay, step, lr, st);
  if (e != hipSuccess) return hip_fail(e, "adam_step_device");
  return PPGAT_OK;
}

int ppgat_rep_merge(int phase, const int32_t* item_rowptr, int64_t n_items, int heads, int channels, float* out,
                    float* agg, const float* bias, float* m, float* inv_l, float* mx, float* pack, void* stream) {
  if (phase < 0 || phase > 2) return fail(PPGAT_ERR_INVALID, "rep_merge: phase must be 0, 1 or 2");
  if (n_items < 0 || heads < 1 || heads > ppgat::kMaxHeads || channels < 4 || channels % 4 != 0)
    return fail(PPGAT_ERR_INVALID, "rep_merge: bad sizes");
  if (n_items > 0 && (!item_rowptr || !out || !m || !inv_l || !mx || !pack))
    return fail(PPGAT_ERR_INVALID, "rep_merge: null pointer");
  if (n_items > 0 && heads > 1 && !agg) return fail(PPGAT_ERR_INVALID, "rep_merge: heads > 1 needs agg");
  if (heads == 1) agg = nullptr;
  float* pack_c = pack + n_items * heads * channels;
  hipError_t e = ppgat::rep_merge(phase, item_rowptr, n_items, heads, channels, 1e-16f, out, agg, bias, m, inv_l, mx,
                                  pack, pack_c, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "rep_merge");
  return PPGAT_OK;
}

int ppgat_rows_gather(const float* src, int64_t ld_src, const int64_t* idx, int64_t n_rows, int cols, float* dst,
                      int64_t ld_dst, void* stream) {
  if (n_rows < 0 || cols < 0 || ld_src < cols || ld_dst < cols) return fail(PPGAT_ERR_INVALID, "rows_gather: bad sizes");
  if (n_rows > 0 && cols > 0 && (!src || !idx || !dst)) return fail(PPGAT_ERR_INVALID, "rows_gather: null pointer");
  hipError_t e = ppgat::rows_gather(src, ld_src, idx, n_rows, cols, dst, ld_dst, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "rows_gather");
  return PPGAT_OK;
}

int ppgat_rows_return_add(float* dst, int64_t ld_dst, const float* ret, int64_t ld_ret, const int32_t* ret_ptr,
                          const int32_t* ret_pos, int64_t n_rows, int cols, void* stream) {
  if (n_rows < 0 || cols < 0 || ld_dst < cols || ld_ret < cols)
    return fail(PPGAT_ERR_INVALID, "rows_return_add: bad sizes");
  if (n_rows > 0 && cols > 0 && (!dst || !ret_ptr || (!ret && ret_pos)))
    return fail(PPGAT_ERR_INVALID, "rows_return_add: null pointer");
  hipError_t e = ppgat::rows_return_add(dst, ld_dst, ret, ld_ret, ret_ptr, ret_pos, n_rows, cols,
                                        static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "rows_return_add");
  return PPGAT_OK;
}

int ppgat_dropout_advance(void* stream) {
  hipError_t e = ppgat::dropout_epoch(0, 0, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "dropout_advance");
  return PPGAT_OK;
}

int ppgat_dropout_set_epoch(uint64_t epoch, void* stream) {
  hipError_t e = ppgat::dropout_epoch(1, epoch, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "dropout_set_epoch");
  return PPGAT_OK;
}

int ppgat_knn_max_k(void) { return ppgat::knn_max_k(); }

int ppgat_knn_topk(const float* S, int64_t ld, int64_t rows, int64_t n_cols, int64_t q0, int k, float min_sim,
                   int32_t* out_idx, float* out_sim, int32_t* out_cnt, void* stream) {
  if (k < 1 || k > ppgat::knn_max_k()) return fail(PPGAT_ERR_UNSUPPORTED, "knn_topk: k must be in [1, 64]");
  if (rows < 0 || n_cols < 1 || ld < n_cols || q0 < 0) return fail(PPGAT_ERR_INVALID, "knn_topk: bad sizes");
  if (n_cols > INT32_MAX) return fail(PPGAT_ERR_UNSUPPORTED, "knn_topk: item ids must fit int32");
  if (rows > 0 && (!S || !out_idx || !out_sim || !out_cnt)) return fail(PPGAT_ERR_INVALID, "knn_topk: null pointer");
  hipError_t e = ppgat::knn_topk(S, ld, rows, n_cols, q0, k, min_sim, out_idx, out_sim, out_cnt,
                                 static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "knn_topk");
  return PPGAT_OK;
}

int ppgat_bpr_sampler_workspace_bytes(int64_t n_users, int64_t nnz, size_t* bytes) {
  if (!bytes || n_users < 0 || nnz < 0) return fail(PPGAT_ERR_INVALID, "bpr_sampler_workspace_bytes: bad arguments");
  if (n_users > INT32_MAX || nnz > UINT32_MAX)
    return fail(PPGAT_ERR_UNSUPPORTED, "bpr_sampler: users must fit int32 and nnz uint32");
  *bytes = ppgat::bpr_sampler_workspace_bytes(n_users, nnz);
  return PPGAT_OK;
}

int ppgat_bpr_sampler_prepare(const int64_t* user_ptr, const int32_t* user_items, int64_t n_users, int64_t nnz,
                              int32_t* items_sorted, int32_t* eligible, int64_t* n_eligible, void* workspace,
                              size_t workspace_bytes, void* stream) {
  if (n_users < 0 || nnz < 0) return fail(PPGAT_ERR_INVALID, "bpr_sampler_prepare: bad sizes");
  if (n_users > INT32_MAX || nnz > UINT32_MAX)
    return fail(PPGAT_ERR_UNSUPPORTED, "bpr_sampler: users must fit int32 and nnz uint32");
  if (!user_ptr || !n_eligible || (n_users > 0 && (!eligible || !workspace)) || (nnz > 0 && (!user_items || !items_sorted)))
    return fail(PPGAT_ERR_INVALID, "bpr_sampler_prepare: null pointer");
  if (workspace_bytes < ppgat::bpr_sampler_workspace_bytes(n_users, nnz))
    return fail(PPGAT_ERR_INVALID, "bpr_sampler_prepare: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_SAMPLE, st);
  hipError_t e = ppgat::bpr_sampler_prepare(user_ptr, user_items, n_users, nnz, items_sorted, eligible, n_eligible,
                                            workspace, workspace_bytes, st);
  if (e != hipSuccess) return hip_fail(e, "bpr_sampler_prepare");
  return PPGAT_OK;
}

int ppgat_bpr_sample(const int64_t* user_ptr, const int32_t* items_sorted, const int32_t* eligible,
                     const int64_t* n_eligible, int64_t n_items, int64_t n_triples, uint64_t seed, int64_t t0,
                     int64_t* u, int64_t* i, int64_t* j, int32_t* bad, void* stream) {
  if (n_items < 0 || n_items > INT32_MAX || n_triples < 0 || t0 < 0)
    return fail(PPGAT_ERR_INVALID, "bpr_sample: bad sizes");
  if (!bad || (n_triples > 0 && (!user_ptr || !eligible || !n_eligible || !u || !i || !j)))
    return fail(PPGAT_ERR_INVALID, "bpr_sample: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_SAMPLE, st);
  hipError_t e = ppgat::bpr_sample(user_ptr, items_sorted, eligible, n_eligible, n_items, n_triples, seed, t0, u, i,
                                   j, bad, st);
  if (e != hipSuccess) return hip_fail(e, "bpr_sample");
  return PPGAT_OK;
}

int ppgat_eval_sample(const int64_t* user_ptr, const int32_t* items_sorted, const int64_t* users, const int64_t* pos,
                      int64_t n_eval, int64_t n_neg, int64_t n_items, uint64_t seed, int64_t* cands, int32_t* bad,
                      void* stream) {
  if (n_eval < 0 || n_neg < 0 || n_items < 1 || n_items > INT32_MAX) return fail(PPGAT_ERR_INVALID, "eval_sample: sizes");
  if (!bad || (n_eval > 0 && (!user_ptr || !users || !pos || !cands))) return fail(PPGAT_ERR_INVALID, "eval_sample: null");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_SAMPLE, st);
  hipError_t e = ppgat::eval_sample(user_ptr, items_sorted, users, pos, n_eval, n_neg, n_items, seed, cands, bad, st);
  if (e != hipSuccess) return hip_fail(e, "eval_sample");
  return PPGAT_OK;
}

int ppgat_sampled_rank(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                       int channels, const int64_t* users, const int64_t* cands, int64_t n_eval, int64_t n_cand,
                       int32_t* rank, void* stream) {
  if (!ppgat::bpr_channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "sampled_rank: channels");
  if (n_users < 1 || n_items < 1 || n_eval < 0 || n_cand < 1) return fail(PPGAT_ERR_INVALID, "sampled_rank: sizes");
  if (row_map == nullptr && n_rows != n_users + n_items)
    return fail(PPGAT_ERR_INVALID, "sampled_rank: n_rows must be n_users + n_items without a row_map");
  if (!Z || (n_eval > 0 && (!users || !cands || !rank))) return fail(PPGAT_ERR_INVALID, "sampled_rank: null pointer");
  if (int rc = debug_range(users, 8, n_eval, 0, n_users, "sampled_rank: users", static_cast<hipStream_t>(stream)))
    return rc;
  if (int rc = debug_range(cands, 8, n_eval * n_cand, 0, n_items, "sampled_rank: cands", static_cast<hipStream_t>(stream)))
    return rc;
  hipError_t e = ppgat::sampled_rank(Z, n_users, n_items, row_map, channels, users, cands, n_eval, n_cand, rank,
                                     static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "sampled_rank");
  return PPGAT_OK;
}

int ppgat_serve_topk_workspace_bytes(int64_t n_items, int channels, int n_users, size_t* bytes) {
  if (!bytes || n_items < 1 || n_users < 0) return fail(PPGAT_ERR_INVALID, "serve_topk_workspace_bytes: bad sizes");
  if (channels != 64 && channels != 128 && channels != 256) return fail(PPGAT_ERR_UNSUPPORTED, "serve_topk: channels");
  *bytes = align_up((size_t)n_users * channels * 4) + align_up((size_t)n_users * n_items * 4);
  return PPGAT_OK;
}

int ppgat_serve_topk(const float* item_vecs, int64_t n_items, int channels, const int64_t* hist_ptr,
                     const int64_t* hist_items, int64_t max_hist, int n_users, int k, int32_t* out_idx,
                     float* out_score, void* workspace, size_t workspace_bytes, void* stream) {
  if (channels != 64 && channels != 128 && channels != 256) return fail(PPGAT_ERR_UNSUPPORTED, "serve_topk: channels");
  if (k < 1 || k > ppgat::knn_max_k() || k > n_items) return fail(PPGAT_ERR_UNSUPPORTED, "serve_topk: 1 <= k <= 64");
  if (n_items < 1 || n_items > INT32_MAX || n_users < 0 || n_users > 256 || max_hist < 0)
    return fail(PPGAT_ERR_INVALID, "serve_topk: bad sizes (n_users <= 256 per call)");
  if (n_users > 0 && (!item_vecs || !hist_ptr || !out_idx || !out_score || (max_hist > 0 && !hist_items)))
    return fail(PPGAT_ERR_INVALID, "serve_topk: null pointer");
  size_t need = 0;
  ppgat_serve_topk_workspace_bytes(n_items, channels, n_users, &need);
  if (!workspace || workspace_bytes < need) return fail(PPGAT_ERR_INVALID, "serve_topk: workspace too small");
  if (n_users > 0 && max_hist > 0) {
    int64_t n_hist = 0;  // the CSR's last offset
    if (PPGAT_DEBUG) {
      if (hipMemcpy(&n_hist, hist_ptr + n_users, sizeof(n_hist), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(PPGAT_ERR_HIP, "serve_topk: reading hist_ptr");
    }
    if (int rc = debug_range(hist_items, 8, n_hist, 0, n_items, "serve_topk: hist_items", static_cast<hipStream_t>(stream)))
      return rc;
  }
  float* U = static_cast<float*>(workspace);
  float* scores = reinterpret_cast<float*>(static_cast<char*>(workspace) + align_up((size_t)n_users * channels * 4));
  hipError_t e = ppgat::serve_topk(item_vecs, n_items, channels, hist_ptr, hist_items, max_hist, n_users, k, U, scores,
                                   out_idx, out_score, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "serve_topk");
  return PPGAT_OK;
}

static int fusion_check(const float* txt, const float* img, const int32_t* img_index, const float* img_fallback,
                        int64_t n, int text_dim, int img_dim, const float* w1, const float* b1, int hidden_dim,
                        const float* w2, const float* b2, int output_dim, float* out) {
  if (!ppgat::fusion_shape_ok(text_dim, img_dim, hidden_dim, output_dim))
    return fail(PPGAT_ERR_UNSUPPORTED, "fusion_fwd: needs hidden 256, output 128, text/img dims % 32 == 0");
  if (n < 0) return fail(PPGAT_ERR_INVALID, "fusion_fwd: n < 0");
  if (n > 0 && (!w1 || !b1 || !w2 || !b2 || !out || (text_dim > 0 && !txt) ||
                (img_dim > 0 && !img && !img_fallback)))
    return fail(PPGAT_ERR_INVALID, "fusion_fwd: null pointer");
  if (img_dim > 0 && img_index != nullptr && !img_fallback)
    return fail(PPGAT_ERR_INVALID, "fusion_fwd: img_index needs img_fallback for rows without an image");
  return PPGAT_OK;
}

int ppgat_fusion_fwd(const float* txt, const float* img, const int32_t* img_index, const float* img_fallback,
                     int64_t n, int text_dim, int img_dim, const float* w1, const float* b1, int hidden_dim,
                     const float* w2, const float* b2, int output_dim, int normalize, float* out, float* z1,
                     void* stream) {
  const int rc = fusion_check(txt, img, img_index, img_fallback, n, text_dim, img_dim, w1, b1, hidden_dim, w2, b2,
                              output_dim, out);
  if (rc != PPGAT_OK) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_FUSION, st);
  hipError_t e = ppgat::fusion_fwd(txt, img, img_index, img_fallback, n, text_dim, img_dim, w1, b1, w2, b2, normalize,
                                   out, z1, st);
  if (e != hipSuccess) return hip_fail(e, "fusion_fwd");
  return PPGAT_OK;
}

int ppgat_fusion_fwd_workspace_bytes(int text_dim, int img_dim, int hidden_dim, int output_dim, size_t* bytes) {
  if (!bytes || !ppgat::fusion_shape_ok(text_dim, img_dim, hidden_dim, output_dim))
    return fail(PPGAT_ERR_UNSUPPORTED, "fusion_fwd_workspace_bytes: needs hidden 256, output 128, dims % 32 == 0");
  *bytes = ppgat::fusion_workspace_bytes(text_dim, img_dim);
  return PPGAT_OK;
}

int ppgat_fusion_fwd_ws(const float* txt, const float* img, const int32_t* img_index, const float* img_fallback,
                        int64_t n, int text_dim, int img_dim, const float* w1, const float* b1, int hidden_dim,
                        const float* w2, const float* b2, int output_dim, int normalize, float* out, float* z1,
                        void* workspace, size_t workspace_bytes, void* stream) {
  const int rc = fusion_check(txt, img, img_index, img_fallback, n, text_dim, img_dim, w1, b1, hidden_dim, w2, b2,
                              output_dim, out);
  if (rc != PPGAT_OK) return rc;
  if (n > 0 && (!workspace || workspace_bytes < ppgat::fusion_workspace_bytes(text_dim, img_dim) ||
                (reinterpret_cast<uintptr_t>(workspace) & 15)))
    return fail(PPGAT_ERR_INVALID, "fusion_fwd_ws: workspace too small or not 16-byte aligned");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_FUSION, st);
  hipError_t e = ppgat::fusion_fwd(txt, img, img_index, img_fallback, n, text_dim, img_dim, w1, b1, w2, b2, normalize,
                                   out, z1, st, workspace);
  if (e != hipSuccess) return hip_fail(e, "fusion_fwd_ws");
  return PPGAT_OK;
}

int ppgat_infonce_workspace_bytes(int64_t batch, int dim, size_t* bytes) {
  if (!bytes || !ppgat::infonce_shape_ok(batch, dim))
    return fail(PPGAT_ERR_UNSUPPORTED, "infonce: needs dim 128 and 1 <= batch <= 4096");
  *bytes = ppgat::infonce_workspace_bytes(batch);
  return PPGAT_OK;
}

int ppgat_infonce(const float* fused, const float* txt_p, const float* img_p, int64_t batch, int dim, float tau,
                  float* loss, float* d_fused, float* d_txt_p, float* d_img_p, void* workspace, size_t workspace_bytes,
                  void* stream) {
  if (!ppgat::infonce_shape_ok(batch, dim))
    return fail(PPGAT_ERR_UNSUPPORTED, "infonce: needs dim 128 and 1 <= batch <= 4096");
  if (!(tau > 0.f)) return fail(PPGAT_ERR_INVALID, "infonce: tau must be > 0");
  if (!fused || !txt_p || !img_p || !loss || !d_fused || !d_txt_p || !d_img_p)
    return fail(PPGAT_ERR_INVALID, "infonce: null pointer");
  if (!al16(fused) || !al16(txt_p) || !al16(img_p) || !al16(d_fused) || !al16(d_txt_p) || !al16(d_img_p))
    return fail(PPGAT_ERR_UNSUPPORTED, "infonce: 16-byte aligned rows");
  if (!workspace || workspace_bytes < ppgat::infonce_workspace_bytes(batch))
    return fail(PPGAT_ERR_INVALID, "infonce: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_INFONCE, st);
  hipError_t e = ppgat::infonce(fused, txt_p, img_p, batch, tau, loss, d_fused, d_txt_p, d_img_p, workspace, st);
  if (e != hipSuccess) return hip_fail(e, "infonce");
  return PPGAT_OK;
}

int ppgat_relu_dropout(const float* z, int64_t n, float p, uint64_t seed, int backward, float* a, void* stream) {
  if (n < 0 || !(p >= 0.f && p < 1.f) || (backward != 0 && backward != 1))
    return fail(PPGAT_ERR_INVALID, "relu_dropout: n >= 0, 0 <= p < 1, backward 0 or 1");
  if (n > 0 && (!z || !a)) return fail(PPGAT_ERR_INVALID, "relu_dropout: null pointer");
  hipError_t e = ppgat::relu_dropout(z, n, p, seed, backward, a, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "relu_dropout");
  return PPGAT_OK;
}

// ---- fp32 matrix-core GEMMs and the aggregate-then-transform multi-head layer ----------
int ppgat_gemm_nn_supported(int64_t m, int k, int n, int b_layout) {
  return ppgat::gemm_nn_shape_ok(m, k, n, b_layout) ? 1 : 0;
}

int ppgat_gemm_nn(const float* x, int64_t ldx, int64_t m, int k, const float* b, int64_t ldb, int b_layout, int n,
                  float alpha, const float* bias, float* y, int64_t ldy, void* stream) {
  if (!ppgat::gemm_nn_shape_ok(m, k, n, b_layout))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_nn: needs k % 32 == 0, n % 128 == 0, b_layout 0 or 1");
  if (ldx < k || (ldx % 4) || ldy < n || (b_layout == 0 ? ldb < n : ldb < k) || (ldb % 4))
    return fail(PPGAT_ERR_INVALID, "gemm_nn: bad leading dimension (>= width, multiple of 4)");
  if (m > 0 && (!x || !b || !y)) return fail(PPGAT_ERR_INVALID, "gemm_nn: null pointer");
  if (!al16(x) || !al16(b)) return fail(PPGAT_ERR_UNSUPPORTED, "gemm_nn: 16-byte aligned rows");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_PROJ, st);
  hipError_t e = ppgat::gemm_nn(x, ldx, m, k, b, ldb, b_layout, n, alpha, bias, y, ldy, st);
  if (e != hipSuccess) return hip_fail(e, "gemm_nn");
  return PPGAT_OK;
}

int ppgat_gemm_nn_workspace_bytes(int64_t m, int k, int n, size_t* bytes) {
  if (!bytes || !ppgat::gemm_nn_shape_ok(m, k, n, 0))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_nn_workspace_bytes: needs k % 32 == 0, n % 128 == 0");
  *bytes = ppgat::gemm_nn_workspace_bytes(m, k, n);
  return PPGAT_OK;
}

int ppgat_gemm_nn_ws(const float* x, int64_t ldx, int64_t m, int k, const float* b, int64_t ldb, int b_layout, int n,
                     float alpha, const float* bias, float* y, int64_t ldy, void* workspace, size_t workspace_bytes,
                     void* stream) {
  if (!ppgat::gemm_nn_shape_ok(m, k, n, b_layout))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_nn: needs k % 32 == 0, n % 128 == 0, b_layout 0 or 1");
  if (ldx < k || (ldx % 4) || ldy < n || (ldy % 4) || (b_layout == 0 ? ldb < n : ldb < k) || (ldb % 4))
    return fail(PPGAT_ERR_INVALID, "gemm_nn: bad leading dimension (>= width, multiple of 4)");
  if (m > 0 && (!x || !b || !y)) return fail(PPGAT_ERR_INVALID, "gemm_nn: null pointer");
  if (!al16(x) || !al16(b) || !al16(y)) return fail(PPGAT_ERR_UNSUPPORTED, "gemm_nn: 16-byte aligned rows");
  const size_t need = ppgat::gemm_nn_workspace_bytes(m, k, n);
  if (need > 0 && (!workspace || workspace_bytes < need))
    return fail(PPGAT_ERR_INVALID, "gemm_nn_ws: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_PROJ, st);
  hipError_t e = ppgat::gemm_nn(x, ldx, m, k, b, ldb, b_layout, n, alpha, bias, y, ldy, st, need > 0 ? workspace : nullptr);
  if (e != hipSuccess) return hip_fail(e, "gemm_nn_ws");
  return PPGAT_OK;
}

int ppgat_gemm_nn_rank(const float* x, int64_t ldx, int64_t m, int k, const float* b, int64_t ldb, int b_layout, int n,
                       float alpha, const float* bias, const float* s, int64_t lds, int nv, const float* a,
                       int64_t lda, float* y, int64_t ldy, void* workspace, size_t workspace_bytes, void* stream) {
  if (!ppgat::gemm_nn_shape_ok(m, k, n, b_layout))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_nn_rank: needs k % 32 == 0, n % 128 == 0, b_layout 0 or 1");
  if (ldx < k || (ldx % 4) || ldy < n || (ldy % 4) || (b_layout == 0 ? ldb < n : ldb < k) || (ldb % 4))
    return fail(PPGAT_ERR_INVALID, "gemm_nn_rank: bad leading dimension (>= width, multiple of 4)");
  if (nv < 0 || nv > 16 || (nv > 0 && (lds < nv || lda < n || (lda % 4))))
    return fail(PPGAT_ERR_INVALID, "gemm_nn_rank: nv <= 16, lds >= nv, lda >= n and a multiple of 4");
  if (m > 0 && (!x || !b || !y || (nv > 0 && (!s || !a)))) return fail(PPGAT_ERR_INVALID, "gemm_nn_rank: null pointer");
  if (!al16(x) || !al16(b) || !al16(y) || (a && !al16(a)))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_nn_rank: 16-byte aligned rows");
  const size_t need = ppgat::gemm_nn_workspace_bytes(m, k, n);
  if (need > 0 && (!workspace || workspace_bytes < need))
    return fail(PPGAT_ERR_INVALID, "gemm_nn_rank: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_PROJ, st);
  hipError_t e = ppgat::gemm_nn(x, ldx, m, k, b, ldb, b_layout, n, alpha, bias, y, ldy, st,
                                need > 0 ? workspace : nullptr, s, lds, nv, a, lda);
  if (e != hipSuccess) return hip_fail(e, "gemm_nn_rank");
  return PPGAT_OK;
}

int ppgat_gemm_tn_big_workspace_bytes(int64_t m, int ma, int nb, size_t* bytes) {
  if (!bytes || m < 0 || !ppgat::gemm_tn_big_shape_ok(ma, nb))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_tn_big: needs ma, nb multiples of 128");
  *bytes = ppgat::gemm_tn_big_workspace_bytes(m, ma, nb);
  return PPGAT_OK;
}

int ppgat_gemm_tn_big(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma, int nb, float* out,
                      void* workspace, size_t workspace_bytes, void* stream) {
  if (m < 0 || !ppgat::gemm_tn_big_shape_ok(ma, nb))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_tn_big: needs ma, nb multiples of 128");
  if (lda < ma || ldb < nb || (lda % 4) || (ldb % 4)) return fail(PPGAT_ERR_INVALID, "gemm_tn_big: bad leading dimension");
  if (!out || (m > 0 && (!a || !b))) return fail(PPGAT_ERR_INVALID, "gemm_tn_big: null pointer");
  if (!al16(a) || !al16(b)) return fail(PPGAT_ERR_UNSUPPORTED, "gemm_tn_big: 16-byte aligned rows");
  if (!workspace || workspace_bytes < ppgat::gemm_tn_big_workspace_bytes(m, ma, nb))
    return fail(PPGAT_ERR_INVALID, "gemm_tn_big: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_GEMM_TN, st);
  hipError_t e = ppgat::gemm_tn_big(a, lda, b, ldb, m, ma, nb, out, workspace, st);
  if (e != hipSuccess) return hip_fail(e, "gemm_tn_big");
  return PPGAT_OK;
}

static int gemm_tn_big_bounds_impl(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma,
                                   int nb, const unsigned* a_bound_bits, const unsigned* b_bound_bits,
                                   int bound_period, float bound_scale, float* out, void* workspace,
                                   size_t workspace_bytes, void* stream, float* colsum_out = nullptr) {
  if (m < 0 || !ppgat::gemm_tn_big_shape_ok(ma, nb))
    return fail(PPGAT_ERR_UNSUPPORTED, "gemm_tn_big_bounded: needs ma, nb multiples of 128");
  if (lda < ma || ldb < nb || (lda % 4) || (ldb % 4))
    return fail(PPGAT_ERR_INVALID, "gemm_tn_big_bounded: bad leading dimension");
  if (!out || (m > 0 && (!a || !b))) return fail(PPGAT_ERR_INVALID, "gemm_tn_big_bounded: null pointer");
  if (b_bound_bits && (bound_period < 1 || nb % bound_period || !(bound_scale >= 1.f) || !(bound_scale < 3.4e38f)))
    return fail(PPGAT_ERR_INVALID, "gemm_tn_big_bounded: period must divide nb, scale >= 1 and finite");
  if (!al16(a) || !al16(b)) return fail(PPGAT_ERR_UNSUPPORTED, "gemm_tn_big_bounded: 16-byte aligned rows");
  if (!workspace || workspace_bytes < ppgat::gemm_tn_big_workspace_bytes(m, ma, nb))
    return fail(PPGAT_ERR_INVALID, "gemm_tn_big_bounded: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_GEMM_TN, st);
  hipError_t e = ppgat::gemm_tn_big(a, lda, b, ldb, m, ma, nb, out, workspace, st, b_bound_bits, bound_period,
                                    bound_scale, a_bound_bits, colsum_out);
  if (e != hipSuccess) return hip_fail(e, "gemm_tn_big_bounded");
  return PPGAT_OK;
}

int ppgat_gemm_tn_big_bounded(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma, int nb,
                              const unsigned* b_bound_bits, int bound_period, float bound_scale, float* out,
                              void* workspace, size_t workspace_bytes, void* stream) {
  if (!b_bound_bits) return fail(PPGAT_ERR_INVALID, "gemm_tn_big_bounded: null pointer");
  return gemm_tn_big_bounds_impl(a, lda, b, ldb, m, ma, nb, nullptr, b_bound_bits, bound_period, bound_scale, out,
                                 workspace, workspace_bytes, stream);
}

int ppgat_gemm_tn_big_bounds(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma, int nb,
                             const unsigned* a_bound_bits, const unsigned* b_bound_bits, int bound_period,
                             float bound_scale, float* out, void* workspace, size_t workspace_bytes, void* stream) {
  return gemm_tn_big_bounds_impl(a, lda, b, ldb, m, ma, nb, a_bound_bits, b_bound_bits, bound_period, bound_scale, out,
                                 workspace, workspace_bytes, stream);
}

int ppgat_gemm_tn_big_colsum(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t m, int ma, int nb,
                             const unsigned* a_bound_bits, const unsigned* b_bound_bits, int bound_period,
                             float bound_scale, float* out, float* colsum_out, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (!colsum_out) return fail(PPGAT_ERR_INVALID, "gemm_tn_big_colsum: null pointer");
  return gemm_tn_big_bounds_impl(a, lda, b, ldb, m, ma, nb, a_bound_bits, b_bound_bits, bound_period, bound_scale, out,
                                 workspace, workspace_bytes, stream, colsum_out);
}

int ppgat_colmax_abs(const float* x, int64_t ldx, int64_t n, int c, unsigned* out_bits, void* stream) {
  if (n < 0 || c < 4 || (c % 4) || ldx < c || (ldx % 4)) return fail(PPGAT_ERR_INVALID, "colmax_abs: bad sizes");
  if (!out_bits || (n > 0 && !x)) return fail(PPGAT_ERR_INVALID, "colmax_abs: null pointer");
  if (!al16(x)) return fail(PPGAT_ERR_UNSUPPORTED, "colmax_abs: 16-byte aligned rows");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_GEMM_TN, st);
  hipError_t e = ppgat::colmax_abs(x, ldx, n, c, out_bits, st);
  if (e != hipSuccess) return hip_fail(e, "colmax_abs");
  return PPGAT_OK;
}

int ppgat_colmax_abs_sources(const float* x, int64_t ldx, int64_t n, int c, const int32_t* src_ptr,
                             unsigned* out_bits, void* stream) {
  if (n < 0 || c < 4 || (c % 4) || ldx < c || (ldx % 4)) return fail(PPGAT_ERR_INVALID, "colmax_abs_sources: bad sizes");
  if (!out_bits || (n > 0 && (!x || !src_ptr))) return fail(PPGAT_ERR_INVALID, "colmax_abs_sources: null pointer");
  if (!al16(x)) return fail(PPGAT_ERR_UNSUPPORTED, "colmax_abs_sources: 16-byte aligned rows");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_GEMM_TN, st);
  hipError_t e = ppgat::colmax_abs(x, ldx, n, c, out_bits, st, src_ptr);
  if (e != hipSuccess) return hip_fail(e, "colmax_abs_sources");
  return PPGAT_OK;
}

int ppgat_colsum_workspace_bytes(int64_t n, int c, size_t* bytes) {
  if (!bytes || n < 0 || (c != 128 && c != 256)) return fail(PPGAT_ERR_UNSUPPORTED, "colsum: c must be 128 or 256");
  *bytes = align_up((size_t)ppgat::colsum_blocks(n) * c * 4);
  return PPGAT_OK;
}

int ppgat_colsum(const float* y, int64_t ldy, int64_t n, int c, float* out, void* workspace, size_t workspace_bytes,
                 void* stream) {
  if (n < 0 || (c != 128 && c != 256) || ldy < c || (ldy % 4)) return fail(PPGAT_ERR_INVALID, "colsum: bad sizes");
  if (!out || (n > 0 && !y)) return fail(PPGAT_ERR_INVALID, "colsum: null pointer");
  if (!workspace || workspace_bytes < (size_t)ppgat::colsum_blocks(n) * c * 4)
    return fail(PPGAT_ERR_INVALID, "colsum: workspace too small");
  hipError_t e = ppgat::colsum(y, ldy, n, c, out, static_cast<float*>(workspace), static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "colsum");
  return PPGAT_OK;
}

int ppgat_xgat_supported(int in_channels, int heads, int channels) {
  return ppgat::xgat_shape_ok(in_channels, heads, channels) ? 1 : 0;
}

int ppgat_xgat_weights(const float* w, const float* att_src, const float* att_dst, int heads, int channels,
                       int in_channels, float* att_proj, float* w_xform, float* w_grad, void* stream) {
  if (!ppgat::xgat_shape_ok(in_channels, heads, channels)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat: shape");
  if (!w || (att_proj && (!att_src || !att_dst))) return fail(PPGAT_ERR_INVALID, "xgat_weights: null pointer");
  hipError_t e = ppgat::xgat_weights(w, att_src, att_dst, heads, channels, in_channels, att_proj, w_xform, w_grad,
                                     static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "xgat_weights");
  return PPGAT_OK;
}

int ppgat_xgat_scores(const float* x, int64_t ldx, int64_t n_rows, int64_t n_dst, int in_channels, int heads,
                      const float* att_proj, float* s_src, float* s_dst, void* stream) {
  if (in_channels != 256 || (heads != 2 && heads != 4)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_scores: shape");
  if (n_rows < 0 || n_dst < 0 || n_dst > n_rows || ldx < in_channels || (ldx % 4))
    return fail(PPGAT_ERR_INVALID, "xgat_scores: bad sizes");
  if (n_rows > 0 && (!x || !att_proj || !s_src || (n_dst > 0 && !s_dst)))
    return fail(PPGAT_ERR_INVALID, "xgat_scores: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_SCORES, st);
  hipError_t e = ppgat::xgat_scores(x, ldx, n_rows, n_dst, in_channels, heads, att_proj, s_src, s_dst, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_scores");
  return PPGAT_OK;
}

int ppgat_xgat_fwd_workspace_bytes(int64_t n_hub_items, int heads, int in_channels, size_t* bytes) {
  if (!bytes || n_hub_items < 0 || heads < 1 || in_channels < 1) return fail(PPGAT_ERR_INVALID, "xgat_fwd_ws: bad args");
  *bytes = partial_bytes(n_hub_items, heads, in_channels);
  return PPGAT_OK;
}

static int xgat_fwd_impl(const ppgat_schedule* dst_sched, const int32_t* col, const int32_t* csr_eid, int64_t n_dst,
                   int64_t n_edges, int in_channels, int heads, const float* x, int64_t ldx, const float* s_src,
                   const float* s_dst, float negative_slope, float dropout_p, uint64_t seed, uint64_t* seed_used,
                   float* agg, float* m, float* inv_l, void* workspace, size_t workspace_bytes, void* stream,
                   unsigned* x_colmax_bits) {
  if (in_channels != 256 || (heads != 2 && heads != 4)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_fwd: shape");
  if (n_dst < 0 || n_edges < 0 || ldx < in_channels || (ldx % 4)) return fail(PPGAT_ERR_INVALID, "xgat_fwd: bad sizes");
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(PPGAT_ERR_INVALID, "dropout p must be in [0, 1)");
  if (int rc = check_sched(dst_sched, n_dst, "xgat_fwd")) return rc;
  if (n_dst > 0 && (!x || !s_src || !s_dst || !agg || !m || !inv_l)) return fail(PPGAT_ERR_INVALID, "xgat_fwd: null pointer");
  if (n_edges > 0 && !col) return fail(PPGAT_ERR_INVALID, "xgat_fwd: null col");
  if (dropout_p > 0.f && (!seed_used || (n_edges > 0 && !csr_eid)))
    return fail(PPGAT_ERR_INVALID, "xgat_fwd: dropout needs seed_used and csr_eid");
  if (dst_sched->n_hub_items > 0 &&
      (!workspace || workspace_bytes < partial_bytes(dst_sched->n_hub_items, heads, in_channels)))
    return fail(PPGAT_ERR_INVALID, "xgat_fwd: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const ppgat::ItemsArg it{dst_sched->item_row, dst_sched->item_beg, dst_sched->item_end, dst_sched->n_items,
                           dst_sched->n_hub_items, dst_sched->n_long_items};
  Timed t(PPGAT_K_FWD, st);
  hipError_t e = hipSuccess;
  if (dropout_p > 0.f) e = ppgat::seed_snapshot(seed, seed_used, st);
  if (e == hipSuccess)
    e = ppgat::xgat_fwd(it, col, csr_eid, x, ldx, in_channels, heads, s_src, s_dst, negative_slope, dropout_p, seed,
                        seed_used, agg, m, inv_l, static_cast<float*>(workspace), dst_sched->hub_row,
                        dst_sched->hub_ptr, dst_sched->n_hubs, st, x_colmax_bits);
  if (e != hipSuccess) return hip_fail(e, "xgat_fwd");
  return PPGAT_OK;
}

int ppgat_xgat_fwd(const ppgat_schedule* dst_sched, const int32_t* col, const int32_t* csr_eid, int64_t n_dst,
                   int64_t n_edges, int in_channels, int heads, const float* x, int64_t ldx, const float* s_src,
                   const float* s_dst, float negative_slope, float dropout_p, uint64_t seed, uint64_t* seed_used,
                   float* agg, float* m, float* inv_l, void* workspace, size_t workspace_bytes, void* stream) {
  return xgat_fwd_impl(dst_sched, col, csr_eid, n_dst, n_edges, in_channels, heads, x, ldx, s_src, s_dst,
                       negative_slope, dropout_p, seed, seed_used, agg, m, inv_l, workspace, workspace_bytes, stream,
                       nullptr);
}

int ppgat_xgat_fwd_colmax(const ppgat_schedule* dst_sched, const int32_t* col, const int32_t* csr_eid, int64_t n_dst,
                          int64_t n_edges, int in_channels, int heads, const float* x, int64_t ldx, const float* s_src,
                          const float* s_dst, float negative_slope, float dropout_p, uint64_t seed,
                          uint64_t* seed_used, float* agg, float* m, float* inv_l, unsigned* x_colmax_bits,
                          void* workspace, size_t workspace_bytes, void* stream) {
  if (!x_colmax_bits || (reinterpret_cast<uintptr_t>(x_colmax_bits) % 16))
    return fail(PPGAT_ERR_INVALID, "xgat_fwd_colmax: x_colmax_bits [in_channels], 16-byte aligned");
  return xgat_fwd_impl(dst_sched, col, csr_eid, n_dst, n_edges, in_channels, heads, x, ldx, s_src, s_dst,
                       negative_slope, dropout_p, seed, seed_used, agg, m, inv_l, workspace, workspace_bytes, stream,
                       x_colmax_bits);
}

int ppgat_xgat_bwd_prologue(const float* gt, const float* agg, const float* s_dst, const float* m, const float* inv_l,
                            int64_t n_dst, int in_channels, int heads, float* nstate, void* stream) {
  if (in_channels != 256 || (heads != 2 && heads != 4)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_prologue: shape");
  if (n_dst < 0) return fail(PPGAT_ERR_INVALID, "xgat_bwd_prologue: bad sizes");
  if (n_dst > 0 && (!gt || !agg || !s_dst || !m || !inv_l || !nstate))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_prologue: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_BWD_PRO, st);
  hipError_t e = ppgat::xgat_bwd_pro(gt, agg, s_dst, m, inv_l, n_dst, in_channels, heads, nstate, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_bwd_prologue");
  return PPGAT_OK;
}

int ppgat_xgat_bwd_workspace_bytes(int64_t n_hub_items, int in_channels, size_t* bytes) {
  if (!bytes || n_hub_items < 0 || in_channels < 1) return fail(PPGAT_ERR_INVALID, "xgat_bwd_ws: bad args");
  *bytes = partial_bytes(n_hub_items, 1, in_channels);
  return PPGAT_OK;
}

int ppgat_xgat_bwd_edges(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                         const int32_t* dz_slot, int64_t n_edges, int in_channels, int heads, const float* x,
                         int64_t ldx, const float* s_src, const float* nstate, const float* gt, const float* att_proj,
                         float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used, float* dx,
                         int64_t lddx, float* S, int64_t lds, float* dz, void* workspace, size_t workspace_bytes,
                         void* stream) {
  if (in_channels != 256 || (heads != 2 && heads != 4)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_edges: shape");
  if (n_edges < 0 || ldx < in_channels || (ldx % 4) || lddx < in_channels || (lddx % 4) || lds < 2 * heads)
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges: bad sizes / leading dimensions");
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(PPGAT_ERR_INVALID, "dropout p must be in [0, 1)");
  if (int rc = check_sched(src_sched, 0, "xgat_bwd_edges")) return rc;
  if (src_sched->n_items > 0 && (!x || !s_src || !att_proj || !dx || !S))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges: null pointer");
  if (n_edges > 0 && (!row || !nstate || !gt || !dz))  // dz_slot NULL: dz in CSC order
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges: null edge pointer");
  if (dropout_p > 0.f && (!seed_used || (n_edges > 0 && !csc_eid)))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges: dropout needs seed_used and csc_eid");
  if (src_sched->n_hub_items > 0 &&
      (!workspace || workspace_bytes < partial_bytes(src_sched->n_hub_items, 1, in_channels)))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const ppgat::ItemsArg it{src_sched->item_row, src_sched->item_beg, src_sched->item_end, src_sched->n_items,
                           src_sched->n_hub_items, src_sched->n_long_items};
  Timed t(PPGAT_K_BWD_SRC, st);
  hipError_t e = ppgat::xgat_bwd_edges(it, row, csc_eid, dz_slot, x, ldx, in_channels, heads, s_src, nstate, gt,
                                       att_proj, negative_slope, dropout_p, seed, seed_used, dx, lddx, S, lds, dz,
                                       static_cast<float*>(workspace), src_sched->hub_row, src_sched->hub_ptr,
                                       src_sched->n_hubs, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_bwd_edges");
  return PPGAT_OK;
}

int ppgat_xgat_bwd_g_workspace_bytes(int64_t n_hub_items, int channels, int heads, size_t* bytes) {
  if (!bytes || n_hub_items < 0 || channels != 256 || (heads != 2 && heads != 4))
    return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_g_workspace_bytes: channels 256, heads 2 or 4");
  *bytes = partial_bytes(n_hub_items, heads, channels);
  return PPGAT_OK;
}

int ppgat_xgat_bwd_edges_g(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                           const int32_t* dz_slot, int64_t n_edges, int channels, int heads, const float* hs,
                           const float* s_src, const float* nstate, const float* g, int64_t ldg, float negative_slope,
                           float dropout_p, uint64_t seed, const uint64_t* seed_used, float* acc, float* S, int64_t lds,
                           float* dz, void* workspace, size_t workspace_bytes, void* stream) {
  if (channels != 256 || (heads != 2 && heads != 4)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_edges_g: shape");
  if (n_edges < 0 || ldg < channels || (ldg % 4) || lds < 2 * heads)
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_g: bad sizes / leading dimensions");
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(PPGAT_ERR_INVALID, "dropout p must be in [0, 1)");
  if (int rc = check_sched(src_sched, 0, "xgat_bwd_edges_g")) return rc;
  if (src_sched->n_items > 0 && (!hs || !s_src || !acc || !S)) return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_g: null pointer");
  if (n_edges > 0 && (!row || !nstate || !g || !dz)) return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_g: null edge pointer");
  if (dropout_p > 0.f && (!seed_used || (n_edges > 0 && !csc_eid)))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_g: dropout needs seed_used and csc_eid");
  if (src_sched->n_hub_items > 0 && (!workspace || workspace_bytes < partial_bytes(src_sched->n_hub_items, heads, channels)))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_g: workspace too small");
  if (!al16(hs) || !al16(g) || !al16(acc)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_edges_g: 16-byte aligned rows");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const ppgat::ItemsArg it{src_sched->item_row, src_sched->item_beg, src_sched->item_end, src_sched->n_items,
                           src_sched->n_hub_items, src_sched->n_long_items};
  Timed t(PPGAT_K_BWD_SRC, st);
  hipError_t e = ppgat::xgat_bwd_edges_g(it, row, csc_eid, dz_slot, hs, channels, heads, s_src, nstate, g, ldg,
                                         negative_slope, dropout_p, seed, seed_used, acc, S, lds, dz,
                                         static_cast<float*>(workspace), src_sched->hub_row, src_sched->hub_ptr,
                                         src_sched->n_hubs, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_bwd_edges_g");
  return PPGAT_OK;
}

static int xgat_bwd_edges_gd_impl(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                            const int32_t* dz_slot, int64_t n_edges, int channels, int heads, const float* hs,
                            const float* s_src, const float* nstate, const float* g, int64_t ldg,
                            float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used,
                            float* acc, float* dalpha, float* pdalpha, void* workspace, size_t workspace_bytes,
                            void* stream, unsigned* g_colmax_bits) {
  if (channels != 256 || (heads != 2 && heads != 4)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_edges_gd: shape");
  if (n_edges < 0 || ldg < channels || (ldg % 4)) return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_gd: bad sizes");
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(PPGAT_ERR_INVALID, "dropout p must be in [0, 1)");
  if (int rc = check_sched(src_sched, 0, "xgat_bwd_edges_gd")) return rc;
  if (src_sched->n_items > 0 && (!hs || !s_src || !acc)) return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_gd: null pointer");
  if (n_edges > 0 && (!row || !nstate || !g || !dalpha || !pdalpha))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_gd: null edge pointer");
  if (dropout_p > 0.f && (!seed_used || (n_edges > 0 && !csc_eid)))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_gd: dropout needs seed_used and csc_eid");
  if (src_sched->n_hub_items > 0 && (!workspace || workspace_bytes < partial_bytes(src_sched->n_hub_items, heads, channels)))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_gd: workspace too small");
  if (!al16(hs) || !al16(g) || !al16(acc)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_edges_gd: 16-byte aligned rows");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const ppgat::ItemsArg it{src_sched->item_row, src_sched->item_beg, src_sched->item_end, src_sched->n_items,
                           src_sched->n_hub_items, src_sched->n_long_items};
  Timed t(PPGAT_K_BWD_SRC, st);
  hipError_t e = ppgat::xgat_bwd_edges_g(it, row, csc_eid, dz_slot, hs, channels, heads, s_src, nstate, g, ldg,
                                         negative_slope, dropout_p, seed, seed_used, acc, nullptr, 0, dalpha,
                                         static_cast<float*>(workspace), src_sched->hub_row, src_sched->hub_ptr,
                                         src_sched->n_hubs, st, pdalpha, g_colmax_bits);
  if (e != hipSuccess) return hip_fail(e, "xgat_bwd_edges_gd");
  return PPGAT_OK;
}

int ppgat_xgat_bwd_edges_gd(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                            const int32_t* dz_slot, int64_t n_edges, int channels, int heads, const float* hs,
                            const float* s_src, const float* nstate, const float* g, int64_t ldg,
                            float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used,
                            float* acc, float* dalpha, float* pdalpha, void* workspace, size_t workspace_bytes,
                            void* stream) {
  return xgat_bwd_edges_gd_impl(src_sched, row, csc_eid, dz_slot, n_edges, channels, heads, hs, s_src, nstate, g, ldg,
                                negative_slope, dropout_p, seed, seed_used, acc, dalpha, pdalpha, workspace,
                                workspace_bytes, stream, nullptr);
}

int ppgat_xgat_bwd_edges_gd_colmax(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                                   const int32_t* dz_slot, int64_t n_edges, int channels, int heads, const float* hs,
                                   const float* s_src, const float* nstate, const float* g, int64_t ldg,
                                   float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used,
                                   float* acc, float* dalpha, float* pdalpha, unsigned* g_colmax_bits,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  if (!g_colmax_bits || (reinterpret_cast<uintptr_t>(g_colmax_bits) % 16))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_edges_gd_colmax: g_colmax_bits [channels], 16-byte aligned");
  return xgat_bwd_edges_gd_impl(src_sched, row, csc_eid, dz_slot, n_edges, channels, heads, hs, s_src, nstate, g, ldg,
                                negative_slope, dropout_p, seed, seed_used, acc, dalpha, pdalpha, workspace,
                                workspace_bytes, stream, g_colmax_bits);
}

int ppgat_xgat_nstate(const float* s_dst, const float* m, const float* inv_l, const float* D, int64_t n_dst, int heads,
                      float* nstate, void* stream) {
  if (n_dst < 0 || heads < 1) return fail(PPGAT_ERR_INVALID, "xgat_nstate: bad sizes");
  if (n_dst > 0 && (!s_dst || !m || !inv_l || !nstate)) return fail(PPGAT_ERR_INVALID, "xgat_nstate: null pointer");
  if (!al16(nstate)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_nstate: 16-byte aligned nstate");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_BWD_PRO, st);
  hipError_t e = ppgat::xgat_nstate(s_dst, m, inv_l, D, n_dst, heads, nstate, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_nstate");
  return PPGAT_OK;
}

int ppgat_xgat_nstate_set_d(float* nstate, const float* D, int64_t n_rows, int heads, void* stream) {
  if (n_rows < 0 || heads < 1) return fail(PPGAT_ERR_INVALID, "xgat_nstate_set_d: bad sizes");
  if (n_rows > 0 && (!nstate || !D)) return fail(PPGAT_ERR_INVALID, "xgat_nstate_set_d: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_BWD_PRO, st);
  hipError_t e = ppgat::xgat_nstate_set_d(nstate, D, n_rows, heads, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_nstate_set_d");
  return PPGAT_OK;
}

int ppgat_xgat_bwd_dz_workspace_bytes(int64_t n_hub_items, int heads, size_t* bytes) {
  if (!bytes || n_hub_items < 0 || heads < 1) return fail(PPGAT_ERR_INVALID, "xgat_bwd_dz_workspace_bytes: bad sizes");
  *bytes = (size_t)n_hub_items * heads * sizeof(float);
  return PPGAT_OK;
}

int ppgat_xgat_bwd_dz(const ppgat_schedule* src_sched, const int32_t* row, const int32_t* csc_eid,
                      const int32_t* dz_slot, int64_t n_edges, int heads, const float* s_src, const float* nstate,
                      float negative_slope, float dropout_p, uint64_t seed, const uint64_t* seed_used, float* dz,
                      float* S, int64_t lds, void* workspace, size_t workspace_bytes, void* stream) {
  if (heads != 2 && heads != 4) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_dz: heads 2 or 4");
  if (n_edges < 0 || lds < heads) return fail(PPGAT_ERR_INVALID, "xgat_bwd_dz: bad sizes / leading dimension");
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(PPGAT_ERR_INVALID, "dropout p must be in [0, 1)");
  if (int rc = check_sched(src_sched, 0, "xgat_bwd_dz")) return rc;
  if (src_sched->n_items > 0 && (!s_src || !S)) return fail(PPGAT_ERR_INVALID, "xgat_bwd_dz: null pointer");
  if (n_edges > 0 && (!row || !nstate || !dz)) return fail(PPGAT_ERR_INVALID, "xgat_bwd_dz: null edge pointer");
  if (dropout_p > 0.f && (!seed_used || (n_edges > 0 && !csc_eid)))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_dz: dropout needs seed_used and csc_eid");
  if (src_sched->n_hub_items > 0 && (!workspace || workspace_bytes < (size_t)src_sched->n_hub_items * heads * 4))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_dz: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const ppgat::ItemsArg it{src_sched->item_row, src_sched->item_beg, src_sched->item_end, src_sched->n_items,
                           src_sched->n_hub_items, src_sched->n_long_items};
  Timed t(PPGAT_K_BWD_EPI, st);
  hipError_t e = ppgat::xgat_bwd_dz(it, row, csc_eid, dz_slot, heads, s_src, nstate, negative_slope, dropout_p, seed,
                                    seed_used, dz, S, lds, static_cast<float*>(workspace), src_sched->hub_row,
                                    src_sched->hub_ptr, src_sched->n_hubs, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_bwd_dz");
  return PPGAT_OK;
}

int ppgat_xgat_bwd_epilogue(const float* S, int64_t lds, const float* att_proj, int64_t n_dst, int in_channels,
                            int heads, float* dx, int64_t lddx, void* stream) {
  if (in_channels != 256 || (heads != 2 && heads != 4)) return fail(PPGAT_ERR_UNSUPPORTED, "xgat_bwd_epilogue: shape");
  if (n_dst < 0 || lds < 2 * heads || lddx < in_channels || (lddx % 4))
    return fail(PPGAT_ERR_INVALID, "xgat_bwd_epilogue: bad sizes");
  if (n_dst > 0 && (!S || !att_proj || !dx)) return fail(PPGAT_ERR_INVALID, "xgat_bwd_epilogue: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_BWD_EPI, st);
  hipError_t e = ppgat::xgat_bwd_epi(S, lds, att_proj + (size_t)heads * in_channels, n_dst, in_channels, heads, dx,
                                     lddx, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_bwd_epilogue");
  return PPGAT_OK;
}

int ppgat_xgat_weight_grads(const float* G, const float* GV, const float* w, const float* att_src,
                            const float* att_dst, int heads, int channels, int in_channels, float* dW, float* datt_src,
                            float* datt_dst, void* stream) {
  if (heads < 1 || channels < 1 || in_channels < 1) return fail(PPGAT_ERR_INVALID, "xgat_weight_grads: bad sizes");
  if (!G || !GV || !w || !att_src || !att_dst || !dW || !datt_src || !datt_dst)
    return fail(PPGAT_ERR_INVALID, "xgat_weight_grads: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_GEMM_TN, st);
  hipError_t e = ppgat::xgat_wgrad(G, GV, w, att_src, att_dst, heads, channels, in_channels, dW, datt_src, datt_dst, st);
  if (e != hipSuccess) return hip_fail(e, "xgat_weight_grads");
  return PPGAT_OK;
}

int ppgat_att_proj(const float* w, const float* att_src, const float* att_dst, int heads, int channels,
                   int in_channels, float* att_proj, void* stream) {
  if (heads < 1 || channels < 1 || in_channels < 1) return fail(PPGAT_ERR_INVALID, "att_proj: bad sizes");
  if (!w || !att_src || !att_dst || !att_proj) return fail(PPGAT_ERR_INVALID, "att_proj: null pointer");
  hipError_t e = ppgat::att_proj(w, att_src, att_dst, heads, channels, in_channels, att_proj,
                                 static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "att_proj");
  return PPGAT_OK;
}

int ppgat_rows_rank_update(const float* S, int64_t lds, int nv, const float* A, int64_t lda, int64_t n_rows, int k,
                           float* dx, int64_t lddx, void* stream) {
  if (n_rows < 0 || nv < 0 || nv > 16 || k < 4 || (k % 4)) return fail(PPGAT_ERR_INVALID, "rows_rank_update: bad sizes");
  if (lds < nv || lda < k || (lda % 4) || lddx < k || (lddx % 4))
    return fail(PPGAT_ERR_INVALID, "rows_rank_update: bad leading dimension");
  if (n_rows > 0 && nv > 0 && (!S || !A || !dx)) return fail(PPGAT_ERR_INVALID, "rows_rank_update: null pointer");
  if ((A && !al16(A)) || (dx && !al16(dx))) return fail(PPGAT_ERR_UNSUPPORTED, "rows_rank_update: 16-byte aligned rows");
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_PROJ, st);
  hipError_t e = ppgat::rank_update(S, lds, nv, A, lda, n_rows, k, dx, lddx, st);
  if (e != hipSuccess) return hip_fail(e, "rows_rank_update");
  return PPGAT_OK;
}

int ppgat_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(g_prof.mu);
  g_prof.on = on != 0;
  return PPGAT_OK;
}

int ppgat_profile_reset(void) {
  std::lock_guard<std::mutex> lk(g_prof.mu);
  for (int k = 0; k < PPGAT_K_COUNT; ++k) {
    g_prof.drain(k);
    g_prof.total_ms[k] = 0.0;
    g_prof.launches[k] = 0;
  }
  return PPGAT_OK;
}

int ppgat_profile_read(int kernel, double* total_ms, int64_t* launches) {
  if (kernel < 0 || kernel >= PPGAT_K_COUNT || !total_ms || !launches)
    return fail(PPGAT_ERR_INVALID, "profile_read: bad arguments");
  std::lock_guard<std::mutex> lk(g_prof.mu);
  g_prof.drain(kernel);
  *total_ms = g_prof.total_ms[kernel];
  *launches = g_prof.launches[kernel];
  return PPGAT_OK;
}

}  // extern "C"
