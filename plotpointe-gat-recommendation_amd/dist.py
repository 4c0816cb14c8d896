"""Row-sharded multi-GPU GAT: one process per GPU, RCCL over xGMI.

Partition.  The node ids are cut into segments (default: one, [0, N); the recommender
uses two, users [0, n_users) and items [n_users, N)) and every segment into `world`
contiguous ranges balanced by in-degree + out-degree + a per-node constant, so each rank
holds a slice of every segment.  A rank's block is its segment slices, each padded to
that segment's largest slice, R rows in all; per-node tensors are [R, ...] per rank and
[world*R, ...] gathered ("padded space"; node n of segment s owned by rank r lives at row
r*R + off_s + n - lo_s(r)).  The graph is static: the global
CSR/CSC in padded space is built once on every rank (device radix sort) and each rank
keeps slices of it:
  forward : CSR rows of its own destinations (col indexes the gathered padded space)
  backward: CSC rows of its own sources with their full out-edge lists (row indexes the
            gathered padded space); each edge's logit gradient goes to its slot in a
            [world, E_max] buffer laid out by destination owner and CSR slot.

Per layer.
  forward : local lin -> node scores -> all_gather(h, s_src) -> fused kernel on own rows
  backward: prologue on own rows -> all_gather(grad_out, nstate) -> edge pass on own
            sources (complete dh for them: no reverse exchange) -> reduce_scatter(dz)
            (every slot is written by exactly one rank, so the sum is exact) -> epilogue
            on own rows.
Loss: with the (users, items) segments a rank evaluates the triples of its own users
against an all_gather of the item rows only (n_items x C instead of N x C), and the
item-row gradients return by reduce_scatter; with one segment, all_gather of Z and a
contiguous share of the triples.  Dense parameters (lin, att, bias, item_proj) are
replicated and all-reduced once per step; user-embedding rows are owner-held.
On a locality-free graph the halo is ~all nodes, so all_gather is the natural collective
here (a per-peer all-to-all index list would carry the same rows).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


# ---------------------------------------------------------------------------
# communication
# ---------------------------------------------------------------------------
class Comm:
    """Row collectives on [R, ...] shards.  NCCL(=RCCL) runs on device tensors directly;
    gloo (CPU tests, or device tensors staged through the host when several ranks share
    one GPU in a test) uses list all_gather and all_reduce+slice for reduce_scatter."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        # active: run the collectives (world > 1, or PPGAT_COMM_ALWAYS=1 to rehearse the RCCL
        # calls -- e.g. their hipGraph capture -- on a single-GPU box)
        self.active = self.world > 1 or os.environ.get("PPGAT_COMM_ALWAYS") == "1"

    def _host(self, t):
        return self.backend == "gloo" and t.is_cuda

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        t = t.contiguous()
        if not self.active:
            return t
        if self.backend == "gloo":
            src = t.cpu() if t.is_cuda else t
            parts = [torch.empty_like(src) for _ in range(self.world)]
            dist.all_gather(parts, src, group=self.group)
            return torch.cat(parts, 0).to(t.device)
        out = torch.empty((self.world * t.size(0),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        t = t.contiguous()
        if not self.active:
            return t
        R = t.size(0) // self.world
        if self.backend == "gloo":
            src = t.cpu() if t.is_cuda else t.clone()
            dist.all_reduce(src, group=self.group)
            return src[self.rank * R:(self.rank + 1) * R].contiguous().to(t.device)
        out = torch.empty((R,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, t, group=self.group)
        return out

    def all_reduce_(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        if not self.active:
            return t
        if self._host(t):
            h = t.cpu()
            dist.all_reduce(h, op=op, group=self.group)
            t.copy_(h)
            return t
        dist.all_reduce(t, op=op, group=self.group)
        return t


class _AllGatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, comm):
        ctx.comm = comm
        return comm.all_gather_rows(t)

    @staticmethod
    def backward(ctx, g):
        return ctx.comm.reduce_scatter_rows(g), None


def all_gather_rows(t, comm):
    return _AllGatherRows.apply(t, comm)


# ---------------------------------------------------------------------------
# partition and the per-rank graph views
# ---------------------------------------------------------------------------
def partition_bounds(weights: np.ndarray, world: int) -> np.ndarray:
    """Contiguous ranges [b_r, b_{r+1}) with ~equal sum of weights."""
    n = len(weights)
    cum = np.concatenate([[0], np.cumsum(weights, dtype=np.float64)])
    targets = cum[-1] * np.arange(1, world) / world
    inner = np.searchsorted(cum, targets, side="left")
    b = np.concatenate([[0], np.clip(inner, 0, n), [n]]).astype(np.int64)
    return np.maximum.accumulate(b)


@dataclass
class LocalView:
    """Slices of the padded-space CSR/CSC a rank runs the stages on."""
    n_rows: int                 # R
    rowptr: torch.Tensor        # [R+1] rebased, CSR of own destination rows
    col: torch.Tensor           # [E_fwd] padded source ids
    csr_eid: torch.Tensor       # [E_fwd] original column ids (dropout hash key)
    n_fwd_edges: int
    colptr: torch.Tensor        # [R+1] rebased, CSC of own source rows
    row: torch.Tensor           # [E_bwd] padded destination ids
    csc_eid: torch.Tensor       # [E_bwd]
    dz_slot: torch.Tensor       # [E_bwd] position in the [world * E_max] dz buffer
    n_bwd_edges: int
    fwd_sched: object = None
    bwd_sched: object = None


@dataclass
class DistGraph:
    world: int
    rank: int
    n_nodes: int
    n_edges: int
    bounds: np.ndarray          # segment 0's range bounds (the only segment by default)
    R: int
    row_map: torch.Tensor       # [N] int32, node id -> padded row
    e_max: int
    view: LocalView
    seg_bounds: list = None     # per segment: [world + 1] range bounds (node ids)
    seg_R: list = None          # per segment: padded rows per rank
    seg_off: list = None        # per segment: row offset inside a rank's block
    loss_map: Optional[torch.Tensor] = None  # lazily built by sharded_bpr_loss

    @property
    def lo(self) -> int:
        return int(self.bounds[self.rank])

    @property
    def hi(self) -> int:
        return int(self.bounds[self.rank + 1])

    @property
    def P(self) -> int:
        return self.world * self.R

    def owned(self, rank: Optional[int] = None):
        """[(lo, hi, row offset in the block, padded rows)] per segment of a rank."""
        r = self.rank if rank is None else rank
        return [(int(b[r]), int(b[r + 1]), off, Rs) for b, off, Rs in zip(self.seg_bounds, self.seg_off, self.seg_R)]

    def owned_users(self, n_users: int, rank: Optional[int] = None):
        """(u0, u1): the rank's users (one contiguous range at the top of its block)."""
        rng = [(max(lo, 0), min(hi, n_users), off) for lo, hi, off, _ in self.owned(rank) if min(hi, n_users) > lo]
        if not rng:
            return 0, 0
        assert len(rng) == 1 and rng[0][2] == 0, "users must be one range at the top of the block"
        return rng[0][0], rng[0][1]


def _hip_csr(ei, P):
    from .hip_ops import csr_build
    return csr_build(ei, P)


def _hip_sched(ptr, E):
    from .hip_ops import schedule_build
    return schedule_build(ptr, E)


def build_dist_graph(edge_index: torch.Tensor, n_nodes: int, world: int, rank: int,
                     csr_builder: Callable = _hip_csr, sched_builder: Optional[Callable] = _hip_sched,
                     node_weight: float = 4.0, segments=None) -> DistGraph:
    """Every rank calls this with the same global edge_index (LongTensor [2, E], original
    node ids) and gets its own slices.  ``segments``: contiguous node-id ranges covering
    [0, N) in order, each split over the ranks (default one segment).  Deterministic: all
    ranks agree on every array."""
    dev = edge_index.device
    N = int(n_nodes)
    E = int(edge_index.size(1))
    segs = [(0, N)] if segments is None else [(int(a), int(b)) for a, b in segments]
    assert segs[0][0] == 0 and segs[-1][1] == N and all(segs[k][1] == segs[k + 1][0] for k in range(len(segs) - 1))
    deg = (torch.bincount(edge_index[1], minlength=N) + torch.bincount(edge_index[0], minlength=N)).cpu().numpy()
    seg_bounds, seg_R, seg_off = [], [], []
    off = 0
    for a, b in segs:
        bnd = a + partition_bounds(deg[a:b].astype(np.float64) + node_weight, world)
        seg_bounds.append(bnd)
        Rs = max(int(np.max(np.diff(bnd))), 1 if len(segs) == 1 else 0)
        seg_R.append(Rs)
        seg_off.append(off)
        off += Rs
    R = max(off, 1)
    row_map_np = np.empty(N, np.int64)
    for (a, b), bnd, o in zip(segs, seg_bounds, seg_off):
        owner = np.repeat(np.arange(world), np.diff(bnd))
        row_map_np[a:b] = owner * R + o + (np.arange(a, b) - bnd[owner])
    row_map = torch.from_numpy(row_map_np).to(dev)
    ei_p = row_map[edge_index]                       # [2, E] padded ids
    P = world * R
    G = csr_builder(ei_p, P)
    rowptr = G.rowptr.to(torch.int64)
    colptr = G.colptr.to(torch.int64)
    starts = rowptr[torch.arange(world, device=dev) * R].cpu().numpy()
    ends = rowptr[torch.arange(1, world + 1, device=dev) * R].cpu().numpy()
    e_max = max(int(np.max(ends - starts)), 1)
    r0, r1 = rank * R, (rank + 1) * R
    e0, e1 = int(starts[rank]), int(ends[rank])
    c0, c1 = int(colptr[r0].item()), int(colptr[r1].item())
    v_rowptr = (rowptr[r0:r1 + 1] - e0).to(torch.int32).contiguous()
    v_colptr = (colptr[r0:r1 + 1] - c0).to(torch.int32).contiguous()
    row = G.row[c0:c1].contiguous()
    glob_slot = G.csc2csr[c0:c1].to(torch.int64)
    dst_owner = row.to(torch.int64) // R
    starts_t = torch.from_numpy(starts).to(dev)
    dz_slot = (dst_owner * e_max + glob_slot - starts_t[dst_owner]).to(torch.int32).contiguous()
    view = LocalView(R, v_rowptr, G.col[e0:e1].contiguous(), G.csr_eid[e0:e1].contiguous(), e1 - e0,
                     v_colptr, row, G.csc_eid[c0:c1].contiguous(), dz_slot, c1 - c0)
    if sched_builder is not None:
        view.fwd_sched = sched_builder(v_rowptr, e1 - e0)
        view.bwd_sched = sched_builder(v_colptr, c1 - c0)
    return DistGraph(world, rank, N, E, seg_bounds[0], R, row_map.to(torch.int32), e_max, view,
                     seg_bounds, seg_R, seg_off)


# ---------------------------------------------------------------------------
# the sharded layer
# ---------------------------------------------------------------------------
class _ShardedGAT(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, att_src, att_dst, bias, dg: DistGraph, comm: Comm, stages, heads: int, C: int, mode: int,
                slope: float, p: float, seed: int):
        h = h.contiguous()
        a_s = att_src.detach().reshape(heads, C).contiguous()
        a_d = att_dst.detach().reshape(heads, C).contiguous()
        b = bias.detach().contiguous() if bias is not None else None
        s_src, s_dst = stages.scores(h, a_s, a_d, heads, C)
        h_full = comm.all_gather_rows(h)
        s_src_full = comm.all_gather_rows(s_src)
        need = any(ctx.needs_input_grad[:4])
        out, m, inv_l, agg = stages.fwd(dg.view, h_full, s_src_full, s_dst, b, heads, C, mode, slope, p, seed,
                                        need and heads > 1)
        if need:
            empty = torch.empty(0, device=h.device)
            ctx.save_for_backward(h, a_s, a_d, s_src, s_dst, out, m, inv_l, agg if agg is not None else empty,
                                  b if b is not None else empty)
        ctx.dg, ctx.comm, ctx.stages = dg, comm, stages
        ctx.meta = (heads, C, mode, slope, p, seed, bias is not None, agg is not None)
        ctx.att_shapes = (att_src.shape, att_dst.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        h, a_s, a_d, s_src, s_dst, out, m, inv_l, agg, b = ctx.saved_tensors
        heads, C, mode, slope, p, seed, has_bias, has_agg = ctx.meta
        dg, comm, st = ctx.dg, ctx.comm, ctx.stages
        g = g.contiguous()
        want_db = has_bias and ctx.needs_input_grad[3]
        nstate, dbias = st.bwd_prologue(g, out, agg if has_agg else None, b if has_bias else None, s_dst, m, inv_l,
                                        heads, C, mode, want_db)
        g_full = comm.all_gather_rows(g)
        nstate_full = comm.all_gather_rows(nstate)
        dz = torch.zeros(dg.world * dg.e_max * heads, dtype=h.dtype, device=h.device)
        grad_h, ds_src = st.bwd_edges(dg.view, h, s_src, nstate_full, g_full, dz, heads, C, mode, slope, p, seed)
        dz_local = comm.reduce_scatter_rows(dz.view(dg.world, dg.e_max * heads)).reshape(-1)
        datt_src, datt_dst = st.bwd_epilogue(dg.view, h, a_s, a_d, ds_src, dz_local, grad_h, heads, C)
        return (grad_h, datt_src.view(ctx.att_shapes[0]), datt_dst.view(ctx.att_shapes[1]), dbias,
                None, None, None, None, None, None, None, None, None)


def _dropout_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


class ShardedPyGGAT(torch.nn.Module):
    """PyGGAT (train_gat_pyg.py:68-88) with row-sharded nodes.  Built from a full model
    constructed identically on every rank (same seed), so the sharded and single-GPU runs
    start from the same parameters; ``full_state_dict`` reassembles the reference keys."""

    def __init__(self, full, dg: DistGraph, comm: Comm, stages=None):
        super().__init__()
        from .hip_ops import HipStages
        self.dg, self.comm = dg, comm
        self.stages = stages if stages is not None else HipStages()
        self.n_users, self.n_items = full.n_users, full.n_items
        nu = self.n_users
        self.u0, self.u1 = dg.owned_users(nu)
        self.user_emb_local = torch.nn.Parameter(full.user_emb.weight.detach()[self.u0:self.u1].clone())
        self.item_proj = full.item_proj
        self.convs = full.convs

    def dense_parameters(self):
        return [p for n, p in self.named_parameters() if n != "user_emb_local"]

    def node_features(self, item_feats):
        """The rank's block: per segment, its users (user_emb rows) then its items
        (item_proj of the feature rows), padded to the segment's row count."""
        nu = self.n_users
        parts = []
        for lo, hi, _, Rs in self.dg.owned():
            n = 0
            if min(hi, nu) > lo:
                parts.append(self.user_emb_local[max(lo, 0) - self.u0:min(hi, nu) - self.u0])
                n += min(hi, nu) - lo
            a, b = max(lo, nu), hi
            if b > a:
                parts.append(self.stages.linear(item_feats[a - nu:b - nu].contiguous(), self.item_proj.weight,
                                                self.item_proj.bias))
                n += b - a
            if Rs > n:
                parts.append(torch.zeros(Rs - n, self.user_emb_local.size(1), dtype=self.user_emb_local.dtype,
                                         device=self.user_emb_local.device))
        if self.u1 == self.u0:  # no users here: keep user_emb_local in the graph (a defined, empty grad)
            parts.insert(0, self.user_emb_local[:0])
        return torch.cat(parts, 0)

    def forward(self, item_feats):
        x = self.node_features(item_feats)
        for conv in self.convs:
            h = self.stages.linear(x, conv.lin.weight, None)
            p = float(conv.dropout) if self.training else 0.0
            seed = _dropout_seed() if p > 0 else 0
            x = _ShardedGAT.apply(h, conv.att_src, conv.att_dst, conv.bias, self.dg, self.comm, self.stages,
                                  conv.heads, conv.out_channels, _lib.MODE_PYG, float(conv.negative_slope), p, seed)
        return x  # own rows of Z, [R, C] (pad rows last)

    def allreduce_grads(self):
        """One flat all-reduce of every dense parameter gradient (replicated params)."""
        if not self.comm.active:
            return
        ps = self.dense_parameters()
        for p in ps:  # a rank whose block has no items never touched item_proj: its share is 0
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        self.comm.all_reduce_(flat)
        views, off = [], 0
        for p in ps:
            n = p.grad.numel()
            views.append(flat[off:off + n].view_as(p.grad))
            off += n
        torch._foreach_copy_([p.grad for p in ps], views)  # one multi-tensor launch, not one copy per tensor

    def full_state_dict(self):
        """Reference-keyed state_dict (user_emb gathered from the owners)."""
        dev = self.user_emb_local.device
        C = self.user_emb_local.size(1)
        blk = torch.zeros(self.dg.R, C, dtype=torch.float32, device=dev)
        blk[:self.u1 - self.u0] = self.user_emb_local.detach()
        allb = self.comm.all_gather_rows(blk)
        rows = []
        for r in range(self.dg.world):
            u0, u1 = self.dg.owned_users(self.n_users, r)
            rows.append(allb[r * self.dg.R: r * self.dg.R + (u1 - u0)])
        sd = {"user_emb.weight": torch.cat(rows, 0)}
        for k, v in self.state_dict().items():
            if k != "user_emb_local":
                sd[k] = v
        return sd


def _item_loss_map(dg: DistGraph, n_users: int) -> torch.Tensor:
    """Node id -> row of [own block's user rows ; all_gather of every rank's item slice]:
    own users -> their block row, other users -> -1 (triple skipped), items -> gathered row."""
    if dg.loss_map is None:
        (ub, ib), (RU, RI) = dg.seg_bounds, dg.seg_R
        N = dg.n_nodes
        m = np.full(N, -1, np.int64)
        u0, u1 = int(ub[dg.rank]), int(ub[dg.rank + 1])
        m[u0:u1] = np.arange(u1 - u0)
        owner = np.repeat(np.arange(dg.world), np.diff(ib))
        m[n_users:] = RU + owner * RI + (np.arange(n_users, N) - ib[owner])
        dg.loss_map = torch.from_numpy(m).to(torch.int32).to(dg.row_map.device)
    return dg.loss_map


def sharded_bpr_loss(Z_local, dg: DistGraph, comm: Comm, u, i, j, n_users: int, n_items: int, loss: str = "bpr",
                     stages=None):
    """The BPR/BCE loss of train_gat_pyg.py:313-322 over row-sharded Z; the ranks' returned
    values add up to the reference's mean loss.

    (users, items) segments: every rank evaluates the triples of its own users against
    the all-gathered item rows (n_items x C), item gradients return by reduce_scatter.
    Otherwise: all_gather of Z and a contiguous share of the triples."""
    if stages is None:
        from .hip_ops import HipStages
        stages = HipStages()
    S = int(u.numel())
    segs = dg.seg_bounds
    if len(segs) == 2 and int(segs[0][0]) == 0 and int(segs[0][-1]) == n_users:
        RU, RI = dg.seg_R
        I_full = all_gather_rows(Z_local[RU:RU + RI], comm)
        Zl = torch.cat([Z_local[:RU], I_full], 0)
        return stages.bpr(Zl, n_users, n_items, _item_loss_map(dg, n_users), u, i, j, loss)
    a, b = S * comm.rank // comm.world, S * (comm.rank + 1) // comm.world
    Z_full = all_gather_rows(Z_local, comm)
    part = stages.bpr(Z_full, n_users, n_items, dg.row_map, u[a:b], i[a:b], j[a:b], loss)
    return part * ((b - a) / max(S, 1))


def gather_rows_to_global(Z_local, dg: DistGraph, comm: Comm) -> torch.Tensor:
    """[R, C] own rows -> [N, C] in node-id order (every rank gets the full matrix)."""
    Z_full = comm.all_gather_rows(Z_local.contiguous())
    return Z_full.index_select(0, dg.row_map.to(torch.int64))


# ---------------------------------------------------------------------------
# replicated-item partition: users sharded, the (small) item segment on every rank
# ---------------------------------------------------------------------------
# The U-I graph is bipartite (train_gat_pyg.py:139-147: every column joins a user and an
# item).  Sharding only the users and keeping every item row on every rank gives each
# edge exactly one home -- the owner of its user endpoint -- with every row it touches
# local, so no node features are gathered at all:
#   forward : user destinations are complete locally; an item destination sees the in-edges
#             of the rank's users only, so its softmax is split over the ranks.  Each rank
#             runs the fused kernel on its local graph, then the item rows are merged
#             exactly: all_reduce(MAX) of the per-rank maxima, all_reduce(SUM) of
#             [c_r * agg_r | c_r] with c_r = l_r * exp(m_r - m) (the log-sum-exp merge of
#             the hub pieces in ppgat_fwd, across ranks).  The merged rows (and their m,
#             1/l) are bitwise identical on every rank.
#   backward: item-row gradients arrive as per-rank partial sums (each rank's loss covers
#             its own users' triples; each rank's edges feed its share of dx), so each
#             layer's backward starts with one all_reduce of the item rows of grad_out;
#             after that every quantity of the layer backward is a sum over the rank's own
#             edges (dh, ds_src, ds_dst of item rows, datt, dW) and is left partial for
#             the next all_reduce (item rows) or the dense-gradient all_reduce.
# Per layer and step: 2 all_reduces of n_items x (C+1) floats (32.5 MB at config 2)
# against 2 all_gathers of N x C (131 MB) for the row-sharded scheme above.  Item-item
# columns (config 3's kNN relation) have no user endpoint: they go to the rank owning the
# destination item's contiguous share.  User-user columns would need a user halo and are
# refused.
@dataclass
class RepGraph:
    world: int
    rank: int
    n_nodes: int
    n_edges: int
    n_users: int
    n_items: int
    user_bounds: np.ndarray     # [world + 1] user-id range bounds
    RU: int                     # this rank's user rows (the top of its local row space)
    RU_max: int                 # the largest RU over the ranks (block size of user-row gathers)
    view: LocalView             # local CSR/CSC over [RU user rows | n_items item rows]
    loss_map: torch.Tensor      # [N] int32: node id -> local row, -1 for other ranks' users
    item_live: torch.Tensor     # [n_items] bool: item rows with local in-edges
    bounds: np.ndarray = None   # = user_bounds (the DistGraph field the tests read)
    graph: object = None        # the local view as a hip_ops.CSRGraph (fused layer path)

    @property
    def R(self) -> int:
        return self.RU + self.n_items

    def owned_users(self, n_users: int, rank: Optional[int] = None):
        r = self.rank if rank is None else rank
        return int(self.user_bounds[r]), int(self.user_bounds[r + 1])


def build_replicated_graph(edge_index: torch.Tensor, n_nodes: int, n_users: int, world: int, rank: int,
                           csr_builder: Callable = _hip_csr, sched_builder: Optional[Callable] = _hip_sched,
                           node_weight: float = 4.0) -> RepGraph:
    """Every rank calls this with the same global edge_index (LongTensor [2, E], node ids
    users [0, n_users), items [n_users, N)); users are cut into `world` contiguous ranges
    balanced by degree + node_weight.  Deterministic: all ranks agree on every array."""
    dev = edge_index.device
    N, nu = int(n_nodes), int(n_users)
    ni = N - nu
    E = int(edge_index.size(1))
    src, dst = edge_index[0], edge_index[1]
    su, du = src < nu, dst < nu
    if bool((su & du).any()):
        raise NotImplementedError("replicated-item partition: user-user columns need a user halo")
    uend = torch.where(su, src, dst)
    deg = torch.bincount(uend[su | du], minlength=nu).cpu().numpy().astype(np.float64)
    ub = partition_bounds(deg + node_weight, world)
    RU_max = int(np.max(np.diff(ub))) if nu else 0
    RU = int(ub[rank + 1] - ub[rank])
    ub_t = torch.from_numpy(ub).to(dev)
    owner = torch.bucketize(uend, ub_t[1:-1], right=True)            # the user endpoint's rank
    ii_owner = torch.div((dst - nu).clamp_min(0) * world, max(ni, 1), rounding_mode="floor")
    owner = torch.where(su | du, owner, ii_owner)
    local = torch.nonzero(owner == rank).squeeze(1)
    u0, u1 = int(ub[rank]), int(ub[rank + 1])
    rm = np.full(N, -1, np.int64)
    rm[u0:u1] = np.arange(u1 - u0)
    rm[nu:] = RU + np.arange(ni)
    row_map = torch.from_numpy(rm).to(dev)
    R = RU + ni
    ei_l = row_map[edge_index[:, local]]
    El = int(local.numel())
    G = csr_builder(ei_l, R)
    lid = local.to(torch.int32)
    orig = (lambda t: lid[t.long()].contiguous()) if El else (lambda t: t[:0].contiguous())
    view = LocalView(R, G.rowptr.contiguous(), G.col[:El].contiguous(), orig(G.csr_eid[:El]), El,
                     G.colptr.contiguous(), G.row[:El].contiguous(), orig(G.csc_eid[:El]),
                     G.csc2csr[:El].contiguous(), El)
    graph = None
    if sched_builder is not None:
        view.fwd_sched = sched_builder(view.rowptr, El)
        view.bwd_sched = sched_builder(view.colptr, El)
        from .hip_ops import CSRGraph
        graph = CSRGraph(R, El, view.rowptr, view.col, view.csr_eid, view.colptr, view.row, view.csc_eid,
                         view.dz_slot, view.fwd_sched, view.bwd_sched)
    rp = G.rowptr.to(torch.int64)
    item_live = (rp[RU + 1:] - rp[RU:-1]) > 0
    return RepGraph(world, rank, N, E, nu, ni, ub, RU, RU_max, view, row_map.to(torch.int32), item_live, ub, graph)


class RepHooks:
    """The two exchange points of the fused layer (hip_ops.GATLayer ``rep``): the item-row
    merge after the forward kernel (ppgat_rep_merge + 2 all_reduces) and the item-row
    all_reduce of grad_out before the backward."""

    def __init__(self, rg: RepGraph, comm: Comm):
        self.rg, self.comm = rg, comm
        self.RU, self.rank = rg.RU, comm.rank

    def merge_fwd(self, out, m, inv_l, agg, bias, heads: int, C: int):
        if not self.comm.active:
            return
        lib = _lib.load()
        rg, RU = self.rg, self.RU
        n = rg.n_items
        dev = out.device
        mx = torch.empty(n, heads, dtype=torch.float32, device=dev)
        pack = torch.empty(n * heads * (C + 1), dtype=torch.float32, device=dev)
        rp = rg.view.rowptr[RU:]
        args = (rp.data_ptr(), n, heads, C, out.data_ptr() + 4 * RU * C,
                agg.data_ptr() + 4 * RU * heads * C if agg is not None else None, _lib.ptr(bias),
                m.data_ptr() + 4 * RU * heads, inv_l.data_ptr() + 4 * RU * heads, mx.data_ptr(), pack.data_ptr(),
                _lib.stream_handle(dev))
        _lib.check(lib.ppgat_rep_merge(0, *args), "rep_merge")
        self.comm.all_reduce_(mx, dist.ReduceOp.MAX)
        _lib.check(lib.ppgat_rep_merge(1, *args), "rep_merge")
        self.comm.all_reduce_(pack)
        _lib.check(lib.ppgat_rep_merge(2, *args), "rep_merge")

    def reduce_grad(self, g):
        if self.comm.active:
            self.comm.all_reduce_(g[self.RU:])


def _merge_item_rows(rg: RepGraph, comm: Comm, out, m, inv_l, agg, bias, heads: int, C: int):
    """Exact cross-rank softmax merge of the item destination rows (PyG mode, eps 1e-16),
    in place on out / m / inv_l / agg."""
    eps = 1e-16
    RU = rg.RU
    live = rg.item_live[:, None]
    mi = m[RU:]
    mx = torch.where(live, mi, torch.full_like(mi, -float("inf")))
    comm.all_reduce_(mx, dist.ReduceOp.MAX)
    c = torch.where(live, (1.0 / inv_l[RU:] - eps) * torch.exp(mi - torch.where(live, mx, mi)), torch.zeros_like(mi))
    if agg is not None:
        a = agg[RU:]
    else:
        a = (out[RU:] - bias if bias is not None else out[RU:]).view(-1, 1, C)
    pack = torch.cat([a * c[..., None], c[..., None]], -1).contiguous()   # [n_items, H, C + 1]
    comm.all_reduce_(pack)
    L = pack[..., C]
    ag = pack[..., :C] / (L + eps)[..., None]
    inv_l[RU:] = 1.0 / (L + eps)
    m[RU:] = torch.where(L > 0, mx, torch.zeros_like(mx))
    if agg is not None:
        agg[RU:] = ag
    o = ag.mean(1)
    out[RU:] = o + bias if bias is not None else o


class _ReplicatedGAT(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, att_src, att_dst, bias, rg: RepGraph, comm: Comm, stages, heads: int, C: int, mode: int,
                slope: float, p: float, seed: int):
        h = h.contiguous()
        a_s = att_src.detach().reshape(heads, C).contiguous()
        a_d = att_dst.detach().reshape(heads, C).contiguous()
        b = bias.detach().contiguous() if bias is not None else None
        s_src, s_dst = stages.scores(h, a_s, a_d, heads, C)
        out, m, inv_l, agg = stages.fwd(rg.view, h, s_src, s_dst, b, heads, C, mode, slope, p, seed, heads > 1)
        if comm.active:
            _merge_item_rows(rg, comm, out, m, inv_l, agg, b, heads, C)
        if any(ctx.needs_input_grad[:4]):
            empty = torch.empty(0, device=h.device)
            ctx.save_for_backward(h, a_s, a_d, s_src, s_dst, out, m, inv_l, agg if agg is not None else empty,
                                  b if b is not None else empty)
        ctx.rg, ctx.comm, ctx.stages = rg, comm, stages
        ctx.meta = (heads, C, mode, slope, p, seed, bias is not None, agg is not None)
        ctx.att_shapes = (att_src.shape, att_dst.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        h, a_s, a_d, s_src, s_dst, out, m, inv_l, agg, b = ctx.saved_tensors
        heads, C, mode, slope, p, seed, has_bias, has_agg = ctx.meta
        rg, comm, st = ctx.rg, ctx.comm, ctx.stages
        RU = rg.RU
        g = g.contiguous()
        if comm.active:  # item rows: per-rank partial sums -> the full gradient on every rank
            g = g.clone()
            gi = g[RU:].contiguous()
            comm.all_reduce_(gi)
            g[RU:] = gi
        nstate, _ = st.bwd_prologue(g, out, agg if has_agg else None, b if has_bias else None, s_dst, m, inv_l,
                                    heads, C, mode, False)
        dz = torch.zeros(max(rg.view.n_bwd_edges, 1) * heads, dtype=h.dtype, device=h.device)
        grad_h, ds_src = st.bwd_edges(rg.view, h, s_src, nstate, g, dz, heads, C, mode, slope, p, seed)
        datt_src, datt_dst = st.bwd_epilogue(rg.view, h, a_s, a_d, ds_src, dz, grad_h, heads, C)
        dbias = None
        if has_bias and ctx.needs_input_grad[3]:
            dbias = g[:RU].sum(0)  # own users; the replicated item rows are counted on rank 0 only
            if comm.rank == 0:
                dbias = dbias + g[RU:].sum(0)
        return (grad_h, datt_src.view(ctx.att_shapes[0]), datt_dst.view(ctx.att_shapes[1]), dbias,
                None, None, None, None, None, None, None, None, None)


class ReplicatedPyGGAT(ShardedPyGGAT):
    """PyGGAT with the users sharded and the item rows replicated (see above).  Local rows:
    [own users | every item]; ``forward`` returns them (Z's item rows are the same on every
    rank).  With the HIP stages (default) each layer is the fused hip_ops.GATLayer on the
    local graph with RepHooks at its two exchange points; other stages objects (the CPU
    restatement of the tests) run the staged _ReplicatedGAT."""

    def __init__(self, full, dg, comm: Comm, stages=None):
        super().__init__(full, dg, comm, stages)
        self.fused = stages is None
        self.hooks = RepHooks(dg, comm)

    def node_features(self, item_feats):
        x_items = self.stages.linear(item_feats.contiguous(), self.item_proj.weight, self.item_proj.bias)
        return torch.cat([self.user_emb_local, x_items], 0)

    def forward(self, item_feats):
        if self.fused:
            from .hip_ops import gat_layer
            x_items = self.stages.linear(item_feats.contiguous(), self.item_proj.weight, self.item_proj.bias)
            x = self.user_emb_local
            for li, conv in enumerate(self.convs):
                p = float(conv.dropout) if self.training else 0.0
                seed = _dropout_seed() if p > 0 else 0
                x = gat_layer(x, conv.lin.weight, conv.att_src, conv.att_dst, conv.bias, self.dg.graph, conv.heads,
                              conv.out_channels, _lib.MODE_PYG, float(conv.negative_slope), p, seed,
                              x_items=x_items if li == 0 else None, rep=self.hooks)
            return x
        x = self.node_features(item_feats)
        for conv in self.convs:
            h = self.stages.linear(x, conv.lin.weight, None)
            p = float(conv.dropout) if self.training else 0.0
            seed = _dropout_seed() if p > 0 else 0
            x = _ReplicatedGAT.apply(h, conv.att_src, conv.att_dst, conv.bias, self.dg, self.comm, self.stages,
                                     conv.heads, conv.out_channels, _lib.MODE_PYG, float(conv.negative_slope), p,
                                     seed)
        return x


def _replicated_full_state_dict(self):
    """Reference-keyed state_dict (user_emb gathered from the owners)."""
    rg = self.dg
    C = self.user_emb_local.size(1)
    blk = torch.zeros(rg.RU_max, C, dtype=torch.float32, device=self.user_emb_local.device)
    blk[:rg.RU] = self.user_emb_local.detach()
    allb = self.comm.all_gather_rows(blk)
    ub = rg.user_bounds
    sd = {"user_emb.weight": torch.cat([allb[r * rg.RU_max: r * rg.RU_max + int(ub[r + 1] - ub[r])]
                                        for r in range(rg.world)], 0)}
    for k, v in self.state_dict().items():
        if k != "user_emb_local":
            sd[k] = v
    return sd


ReplicatedPyGGAT.full_state_dict = _replicated_full_state_dict


def replicated_bpr_loss(Z_local, rg: RepGraph, comm: Comm, u, i, j, n_users: int, n_items: int,
                        loss: str = "bpr", stages=None):
    """The BPR/BCE loss of train_gat_pyg.py:313-322: each rank takes the triples of its own
    users against its (replicated) item rows -- no exchange; the ranks' values add up to
    the reference's mean loss and their item-row gradients are partial sums (merged by the
    next layer backward's all_reduce)."""
    if stages is None:
        from .hip_ops import HipStages
        stages = HipStages()
    return stages.bpr(Z_local, n_users, n_items, rg.loss_map, u, i, j, loss)


def replicated_rows_to_global(Z_local, rg: RepGraph, comm: Comm) -> torch.Tensor:
    """[RU + n_items, C] local rows -> [N, C] in node-id order (every rank gets it)."""
    blk = Z_local.new_zeros(rg.RU_max, Z_local.size(1))
    blk[:rg.RU] = Z_local[:rg.RU]
    users = comm.all_gather_rows(blk)
    ub = rg.user_bounds
    idx = np.concatenate([r * rg.RU_max + np.arange(ub[r + 1] - ub[r]) for r in range(rg.world)]).astype(np.int64)
    return torch.cat([users.index_select(0, torch.from_numpy(idx).to(users.device)), Z_local[rg.RU:]], 0)
