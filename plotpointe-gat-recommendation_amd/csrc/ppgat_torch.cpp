// ppgat_torch.cpp -- the GAT layer's device ops registered with the PyTorch dispatcher
// (TORCH_LIBRARY(ppgat)), so they appear as torch.ops.ppgat.* to torch.compile, TorchScript
// and C++ callers ("ops registered via TORCH_LIBRARY from a HIP .so, with a
// thin extern "C" ABI for ctypes").  Every op is a thin adapter onto the C ABI of
// include/ppgat.h (libppgat.so): shape/dtype/device checks with TORCH_CHECK (-> Python
// RuntimeError naming the argument), outputs allocated through the caching allocator,
// work enqueued on the current HIP stream.  No arithmetic lives here.
//
//   csr_build      -> edge_index [2, E] int64 -> CSR by dst / CSC by src      (ppgat_csr_build)
//   schedule_build -> work items over a row pointer                          (ppgat_schedule_build)
//   node_scores    -> s_src, s_dst                                            (ppgat_node_scores)
//   gat_fwd        -> fused softmax-aggregate: out, m, inv_l, agg, seed_used (ppgat_fwd)
//   gat_bwd        -> atomic-free backward: grad_h, datt_src, datt_dst, dbias (ppgat_bwd)
// Replaces: torch_geometric.nn.GATConv's propagate / softmax (train_gat_pyg.py:77) and
// SimpleGATLayer.forward (train_gat_custom.py:75-93) at the op level.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>

#include <string>
#include <tuple>
#include <vector>

#include "../../include/ppgat.h"

namespace {

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == PPGAT_OK, what, " failed (code ", rc, "): ", ppgat_last_error());
}

void* stream_of(const at::Tensor& t) {
  return static_cast<void*>(c10::hip::getCurrentHIPStream(t.device().index()).stream());
}

void check_dev(const at::Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), name, ": ppgat runs on ROCm devices only (got ", t.device(), "); there is no CPU path");
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected ", dt, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": must be contiguous");
}

const void* optr(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

ppgat_schedule make_sched(const at::Tensor& item_row, const at::Tensor& item_beg, const at::Tensor& item_end,
                          const at::Tensor& hub_row, const at::Tensor& hub_ptr, c10::IntArrayRef counts) {
  TORCH_CHECK(counts.size() == 4, "schedule counts: [n_items, n_hub_items, n_hubs, n_long_items]");
  for (const at::Tensor* t : {&item_row, &item_beg, &item_end, &hub_row, &hub_ptr}) check_dev(*t, "schedule", at::kInt);
  ppgat_schedule s{};
  s.item_row = item_row.data_ptr<int32_t>();
  s.item_beg = item_beg.data_ptr<int32_t>();
  s.item_end = item_end.data_ptr<int32_t>();
  s.n_items = counts[0];
  s.n_hub_items = counts[1];
  s.hub_row = hub_row.data_ptr<int32_t>();
  s.hub_ptr = hub_ptr.data_ptr<int32_t>();
  s.n_hubs = counts[2];
  s.n_long_items = counts[3];
  return s;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> csr_build(
    const at::Tensor& edge_index, int64_t n_nodes) {
  check_dev(edge_index, "edge_index", at::kLong);
  TORCH_CHECK(edge_index.dim() == 2 && edge_index.size(0) == 2, "edge_index must be [2, E]");
  const int64_t E = edge_index.size(1), N = n_nodes;
  auto i32 = edge_index.options().dtype(at::kInt);
  at::Tensor rowptr = at::empty({N + 1}, i32), colptr = at::empty({N + 1}, i32);
  at::Tensor col = at::empty({std::max<int64_t>(E, 1)}, i32), csr_eid = at::empty_like(col), row = at::empty_like(col);
  at::Tensor csc_eid = at::empty_like(col), csc2csr = at::empty_like(col), bad = at::empty({1}, i32);
  size_t nbytes = 0;
  check_rc(ppgat_csr_workspace_bytes(N, E, &nbytes), "csr_workspace_bytes");
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(nbytes, 1)}, edge_index.options().dtype(at::kByte));
  check_rc(ppgat_csr_build(edge_index.data_ptr<int64_t>(), E, N, rowptr.data_ptr<int32_t>(), col.data_ptr<int32_t>(),
                           csr_eid.data_ptr<int32_t>(), colptr.data_ptr<int32_t>(), row.data_ptr<int32_t>(),
                           csc_eid.data_ptr<int32_t>(), csc2csr.data_ptr<int32_t>(), bad.data_ptr<int32_t>(),
                           ws.data_ptr(), nbytes, stream_of(edge_index)),
           "csr_build");
  const int nbad = bad.item<int32_t>();  // one sync per static graph
  TORCH_CHECK(nbad == 0, "edge_index has ", nbad, " entries outside [0, ", N, ")");
  return {rowptr, col.narrow(0, 0, E), csr_eid.narrow(0, 0, E), colptr, row.narrow(0, 0, E), csc_eid.narrow(0, 0, E),
          csc2csr.narrow(0, 0, E)};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> schedule_build(
    const at::Tensor& ptr, int64_t n_edges, int64_t max_edges) {
  check_dev(ptr, "ptr", at::kInt);
  const int64_t N = ptr.numel() - 1;
  const int64_t cap = ppgat_schedule_capacity(N, n_edges, (int32_t)max_edges);
  TORCH_CHECK(cap >= 0, "schedule_capacity: bad arguments");
  auto i32 = ptr.options();
  at::Tensor item_row = at::empty({std::max<int64_t>(cap, 1)}, i32), item_beg = at::empty_like(item_row);
  at::Tensor item_end = at::empty_like(item_row), hub_row = at::empty({std::max<int64_t>(N, 1)}, i32);
  at::Tensor hub_ptr = at::empty({N + 1}, i32), counts = at::empty({4}, i32);
  size_t nbytes = 0;
  check_rc(ppgat_schedule_workspace_bytes(N, &nbytes), "schedule_workspace_bytes");
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(nbytes, 1)}, ptr.options().dtype(at::kByte));
  check_rc(ppgat_schedule_build(ptr.data_ptr<int32_t>(), N, n_edges, (int32_t)max_edges, item_row.data_ptr<int32_t>(),
                                item_beg.data_ptr<int32_t>(), item_end.data_ptr<int32_t>(), hub_row.data_ptr<int32_t>(),
                                hub_ptr.data_ptr<int32_t>(), counts.data_ptr<int32_t>(), ws.data_ptr(), nbytes,
                                stream_of(ptr)),
           "schedule_build");
  return {item_row, item_beg, item_end, hub_row, hub_ptr, counts};
}

std::tuple<at::Tensor, at::Tensor> node_scores(const at::Tensor& h, const at::Tensor& att_src,
                                               const at::Tensor& att_dst, int64_t heads, int64_t channels) {
  check_dev(h, "h", at::kFloat);
  check_dev(att_src, "att_src", at::kFloat);
  check_dev(att_dst, "att_dst", at::kFloat);
  const int64_t N = h.size(0);
  TORCH_CHECK(h.numel() == N * heads * channels, "h must be [N, heads * channels]");
  at::Tensor s_src = at::empty({N, heads}, h.options()), s_dst = at::empty({N, heads}, h.options());
  check_rc(ppgat_node_scores(h.data_ptr<float>(), att_src.data_ptr<float>(), att_dst.data_ptr<float>(), N, (int)heads,
                             (int)channels, s_src.data_ptr<float>(), s_dst.data_ptr<float>(), stream_of(h)),
           "node_scores");
  return {s_src, s_dst};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> gat_fwd(
    const at::Tensor& h, const at::Tensor& s_src, const at::Tensor& s_dst, const c10::optional<at::Tensor>& bias,
    const at::Tensor& col, const at::Tensor& csr_eid, const at::Tensor& item_row, const at::Tensor& item_beg,
    const at::Tensor& item_end, const at::Tensor& hub_row, const at::Tensor& hub_ptr, c10::IntArrayRef sched,
    int64_t heads, int64_t channels, int64_t mode, double slope, double dropout_p, int64_t seed, bool want_agg) {
  check_dev(h, "h", at::kFloat);
  check_dev(s_src, "s_src", at::kFloat);
  check_dev(s_dst, "s_dst", at::kFloat);
  check_dev(col, "col", at::kInt);
  check_dev(csr_eid, "csr_eid", at::kInt);
  if (bias.has_value()) check_dev(*bias, "bias", at::kFloat);
  const int64_t N = s_dst.size(0), E = col.numel();
  ppgat_schedule s = make_sched(item_row, item_beg, item_end, hub_row, hub_ptr, sched);
  at::Tensor out = at::empty({N, channels}, h.options()), m = at::empty({N, heads}, h.options());
  at::Tensor inv_l = at::empty({N, heads}, h.options());
  at::Tensor agg = want_agg ? at::empty({N, heads, channels}, h.options()) : at::empty({0}, h.options());
  at::Tensor seed_used = at::empty({1}, h.options().dtype(at::kLong));
  size_t nbytes = 0;
  check_rc(ppgat_fwd_workspace_bytes(s.n_hub_items, (int)heads, (int)channels, &nbytes), "fwd_workspace_bytes");
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(nbytes, 1)}, h.options().dtype(at::kByte));
  check_rc(ppgat_fwd(&s, E ? col.data_ptr<int32_t>() : nullptr, E ? csr_eid.data_ptr<int32_t>() : nullptr, N, E,
                     (int)heads, (int)channels, h.data_ptr<float>(), s_src.data_ptr<float>(), s_dst.data_ptr<float>(),
                     static_cast<const float*>(optr(bias)), (int)mode, (float)slope, (float)dropout_p, (uint64_t)seed,
                     reinterpret_cast<uint64_t*>(seed_used.data_ptr<int64_t>()), out.data_ptr<float>(),
                     m.data_ptr<float>(), inv_l.data_ptr<float>(), want_agg ? agg.data_ptr<float>() : nullptr,
                     ws.data_ptr(), nbytes, stream_of(h)),
           "gat_fwd");
  return {out, m, inv_l, agg, seed_used};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> gat_bwd(
    const at::Tensor& h, const at::Tensor& s_src, const at::Tensor& s_dst, const at::Tensor& att_src,
    const at::Tensor& att_dst, const c10::optional<at::Tensor>& bias, const at::Tensor& out,
    const c10::optional<at::Tensor>& agg, const at::Tensor& m, const at::Tensor& inv_l, const at::Tensor& grad_out,
    const at::Tensor& rowptr, const at::Tensor& row, const at::Tensor& csc_eid, const at::Tensor& csc2csr,
    const at::Tensor& item_row, const at::Tensor& item_beg, const at::Tensor& item_end, const at::Tensor& hub_row,
    const at::Tensor& hub_ptr, c10::IntArrayRef sched, int64_t heads, int64_t channels, int64_t mode, double slope,
    double dropout_p, int64_t seed, const c10::optional<at::Tensor>& seed_used, bool want_bias_grad) {
  for (auto* t : {&h, &s_src, &s_dst, &att_src, &att_dst, &out, &m, &inv_l, &grad_out}) check_dev(*t, "gat_bwd", at::kFloat);
  for (auto* t : {&rowptr, &row, &csc_eid, &csc2csr}) check_dev(*t, "gat_bwd graph", at::kInt);
  const int64_t N = h.size(0), E = row.numel();
  ppgat_schedule s = make_sched(item_row, item_beg, item_end, hub_row, hub_ptr, sched);
  at::Tensor grad_h = at::empty({N, heads * channels}, h.options());
  at::Tensor datt_src = at::empty({heads, channels}, h.options()), datt_dst = at::empty({heads, channels}, h.options());
  at::Tensor dbias = want_bias_grad ? at::empty({channels}, h.options()) : at::empty({0}, h.options());
  size_t nbytes = 0;
  check_rc(ppgat_bwd_workspace_bytes(N, E, s.n_hub_items, (int)heads, (int)channels, &nbytes), "bwd_workspace_bytes");
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(nbytes, 1)}, h.options().dtype(at::kByte));
  const float* aggp = (agg.has_value() && agg->numel() > 0) ? agg->data_ptr<float>() : nullptr;
  check_rc(ppgat_bwd(&s, rowptr.data_ptr<int32_t>(), E ? row.data_ptr<int32_t>() : nullptr,
                     E ? csc_eid.data_ptr<int32_t>() : nullptr, E ? csc2csr.data_ptr<int32_t>() : nullptr, N, E,
                     (int)heads, (int)channels, h.data_ptr<float>(), s_src.data_ptr<float>(), s_dst.data_ptr<float>(),
                     att_src.data_ptr<float>(), att_dst.data_ptr<float>(), static_cast<const float*>(optr(bias)),
                     out.data_ptr<float>(), aggp, m.data_ptr<float>(), inv_l.data_ptr<float>(),
                     grad_out.data_ptr<float>(), (int)mode, (float)slope, (float)dropout_p, (uint64_t)seed,
                     seed_used.has_value() ? reinterpret_cast<const uint64_t*>(seed_used->data_ptr<int64_t>()) : nullptr,
                     grad_h.data_ptr<float>(), datt_src.data_ptr<float>(), datt_dst.data_ptr<float>(),
                     want_bias_grad ? dbias.data_ptr<float>() : nullptr, ws.data_ptr(), nbytes, stream_of(h)),
           "gat_bwd");
  return {grad_h, datt_src, datt_dst, dbias};
}

}  // namespace

TORCH_LIBRARY(ppgat, m) {
  m.def("csr_build(Tensor edge_index, int n_nodes) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("schedule_build(Tensor ptr, int n_edges, int max_edges=256) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("node_scores(Tensor h, Tensor att_src, Tensor att_dst, int heads, int channels) -> (Tensor, Tensor)");
  m.def(
      "gat_fwd(Tensor h, Tensor s_src, Tensor s_dst, Tensor? bias, Tensor col, Tensor csr_eid, Tensor item_row, "
      "Tensor item_beg, Tensor item_end, Tensor hub_row, Tensor hub_ptr, int[] sched, int heads, int channels, "
      "int mode, float slope, float dropout_p, int seed, bool want_agg) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "gat_bwd(Tensor h, Tensor s_src, Tensor s_dst, Tensor att_src, Tensor att_dst, Tensor? bias, Tensor out, "
      "Tensor? agg, Tensor m, Tensor inv_l, Tensor grad_out, Tensor rowptr, Tensor row, Tensor csc_eid, "
      "Tensor csc2csr, Tensor item_row, Tensor item_beg, Tensor item_end, Tensor hub_row, Tensor hub_ptr, "
      "int[] sched, int heads, int channels, int mode, float slope, float dropout_p, int seed, Tensor? seed_used, "
      "bool want_bias_grad) -> (Tensor, Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(ppgat, CUDA, m) {
  m.impl("csr_build", &csr_build);
  m.impl("schedule_build", &schedule_build);
  m.impl("node_scores", &node_scores);
  m.impl("gat_fwd", &gat_fwd);
  m.impl("gat_bwd", &gat_bwd);
}
