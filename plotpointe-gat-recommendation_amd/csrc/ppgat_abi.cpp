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
    if (!a) return;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    hipEvent_t b = g_prof.get();
    if (!b) return;
    (void)hipEventRecord(b, st);
    g_prof.pending[k].push_back({a, b});
  }
};

}  // namespace

extern "C" {

int ppgat_version(void) { return 1; }

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

int ppgat_fwd(const int32_t* rowptr, const int32_t* col, const int32_t* csr_eid, int64_t n_nodes, int64_t n_edges,
              int heads, int channels, const float* h, const float* s_src, const float* s_dst, const float* bias,
              int mode, float negative_slope, float dropout_p, uint64_t seed, float* out, float* m, float* inv_l,
              float* agg, void* stream) {
  if (!channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "fwd: unsupported channels");
  if (heads < 1 || n_nodes < 0 || n_edges < 0) return fail(PPGAT_ERR_INVALID, "fwd: bad sizes");
  if (int rc = check_mode(mode, heads, bias, dropout_p)) return rc;
  if (n_nodes > 0 && (!rowptr || !h || !s_src || !s_dst || !out || !m || !inv_l))
    return fail(PPGAT_ERR_INVALID, "fwd: null pointer");
  if (n_edges > 0 && !col) return fail(PPGAT_ERR_INVALID, "fwd: null col");
  if (dropout_p > 0.f && n_edges > 0 && !csr_eid) return fail(PPGAT_ERR_INVALID, "fwd: dropout needs csr_eid");
  const float eps = mode == PPGAT_MODE_PYG ? 1e-16f : 1e-9f;
  hipStream_t st = static_cast<hipStream_t>(stream);
  Timed t(PPGAT_K_FWD, st);
  hipError_t e = ppgat::launch_fwd(rowptr, col, csr_eid, n_nodes, heads, channels, h, s_src, s_dst, bias, mode,
                                   negative_slope, eps, dropout_p, seed, out, m, inv_l, agg, st);
  if (e != hipSuccess) return hip_fail(e, "fwd");
  return PPGAT_OK;
}

// workspace: D [N*H] | ds_src [N*H] | dz [E*H] | partial [waves*2*H*C]
int ppgat_bwd_workspace_bytes(int64_t n_nodes, int64_t n_edges, int heads, int channels, size_t* bytes) {
  if (!bytes || n_nodes < 0 || n_edges < 0 || heads < 1 || channels < 1)
    return fail(PPGAT_ERR_INVALID, "bwd_workspace_bytes: bad arguments");
  const size_t nh = align_up((size_t)n_nodes * heads * 4 + 4);
  const size_t eh = align_up((size_t)n_edges * heads * 4 + 4);
  const size_t part = align_up((size_t)ppgat::epi_waves(n_nodes) * 2 * heads * channels * 4);
  *bytes = 2 * nh + eh + part;
  return PPGAT_OK;
}

int ppgat_bwd(const int32_t* rowptr, const int32_t* colptr, const int32_t* row, const int32_t* csc_eid,
              const int32_t* csc2csr, int64_t n_nodes, int64_t n_edges, int heads, int channels, const float* h,
              const float* s_src, const float* s_dst, const float* att_src, const float* att_dst, const float* bias,
              const float* out, const float* agg, const float* m, const float* inv_l, const float* grad_out, int mode,
              float negative_slope, float dropout_p, uint64_t seed, float* grad_h, float* grad_att_src,
              float* grad_att_dst, void* workspace, size_t workspace_bytes, void* stream) {
  if (!channels_ok(channels)) return fail(PPGAT_ERR_UNSUPPORTED, "bwd: unsupported channels");
  if (heads < 1 || n_nodes < 0 || n_edges < 0) return fail(PPGAT_ERR_INVALID, "bwd: bad sizes");
  if (int rc = check_mode(mode, heads, bias, dropout_p)) return rc;
  if (heads > 1 && agg == nullptr) return fail(PPGAT_ERR_INVALID, "bwd: heads > 1 needs the saved agg");
  if (!grad_att_src || !grad_att_dst || !att_src || !att_dst)
    return fail(PPGAT_ERR_INVALID, "bwd: null attention pointer");
  if (n_nodes > 0 && (!rowptr || !colptr || !h || !s_src || !s_dst || !out || !m || !inv_l || !grad_out || !grad_h))
    return fail(PPGAT_ERR_INVALID, "bwd: null pointer");
  if (n_edges > 0 && (!row || !csc2csr)) return fail(PPGAT_ERR_INVALID, "bwd: null CSC pointer");
  if (dropout_p > 0.f && n_edges > 0 && !csc_eid) return fail(PPGAT_ERR_INVALID, "bwd: dropout needs csc_eid");
  size_t need = 0;
  ppgat_bwd_workspace_bytes(n_nodes, n_edges, heads, channels, &need);
  if (!workspace || workspace_bytes < need) return fail(PPGAT_ERR_INVALID, "bwd: workspace too small");
  const size_t nh = align_up((size_t)n_nodes * heads * 4 + 4);
  const size_t eh = align_up((size_t)n_edges * heads * 4 + 4);
  char* p = static_cast<char*>(workspace);
  float* D = reinterpret_cast<float*>(p);
  float* ds_src = reinterpret_cast<float*>(p + nh);
  float* dz = reinterpret_cast<float*>(p + 2 * nh);
  float* partial = reinterpret_cast<float*>(p + 2 * nh + eh);
  const float gscale = mode == PPGAT_MODE_PYG ? 1.f / (float)heads : 1.f;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e;
  {
    Timed t(PPGAT_K_BWD_PRO, st);
    e = ppgat::launch_bwd_pro(grad_out, out, agg, heads == 1 ? bias : nullptr, n_nodes, heads, channels, gscale, D,
                              st);
  }
  if (e != hipSuccess) return hip_fail(e, "bwd_prologue");
  {
    Timed t(PPGAT_K_BWD_SRC, st);
    e = ppgat::launch_bwd_src(colptr, row, csc_eid, csc2csr, n_nodes, heads, channels, h, s_src, s_dst, m, inv_l, D,
                              grad_out, mode, negative_slope, gscale, dropout_p, seed, grad_h, ds_src, dz, st);
  }
  if (e != hipSuccess) return hip_fail(e, "bwd_src");
  const int64_t waves = ppgat::epi_waves(n_nodes);
  {
    Timed t(PPGAT_K_BWD_EPI, st);
    e = ppgat::launch_bwd_epi(rowptr, n_nodes, heads, channels, h, att_src, att_dst, ds_src, dz, grad_h, partial,
                              waves, st);
  }
  if (e != hipSuccess) return hip_fail(e, "bwd_epilogue");
  {
    Timed t(PPGAT_K_BWD_RED, st);
    e = ppgat::launch_bwd_red(partial, waves, heads * channels, grad_att_src, grad_att_dst, st);
  }
  if (e != hipSuccess) return hip_fail(e, "bwd_reduce");
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
