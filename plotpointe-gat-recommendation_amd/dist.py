"""Multi-GPU GAT: one process per GPU, RCCL (torch "nccl") over xGMI.

Two partitions of the node rows, both exact (every result equals the single-device layer):

Halo partition (``build_halo_graph`` / ``HaloPyGGAT``, any graph; configs 4 and 5).
  Users and items are two segments: users cut into `world` contiguous ranges balanced by
  degree, items dealt to the ranks by degree (``halo_owner``), so every rank owns a slice of
  both: its "own" rows, users first then items.
  Every edge_index column lives on the rank that owns its DESTINATION, so a rank holds the
  complete in-edge list (CSR) of each own row.  The sources those edges read that belong to
  other ranks are its halo rows; the local row space is [own rows | halo rows], the halo
  grouped by owner rank in the owner's row order.  The graph is static, so the exchange
  plan is built once (ExchangePlan: which own rows go to which peer, how many rows arrive
  from each):
    forward : per layer one RCCL all_to_all_single of the halo rows of the layer's
              exchanged operand -- the pre-projection x when H*C > C_in (config 5: 1 KB per
              row instead of 4 KB of h, the projection recomputed on the halo rows), else the
              projected h (config 4: 512 B, nothing recomputed) -- then the fused kernels on
              the local CSR (own destination rows, columns into [own | halo]).
    backward: the edge pass by source over the local CSC writes gradients for own AND halo
              source rows; one reverse all_to_all returns the halo rows' gradients to their
              owners, which add them in peer order (ppgat_rows_return_add: deterministic).
              Logit gradients of an edge stay on its destination's rank: no other exchange.
  Loss: a rank takes the triples of its own users; the item rows they read come by one
  all_to_all of exactly those rows (a plan per triple set), and go back the same way.
  Dense parameters are replicated and all-reduced once per step; user-embedding rows are
  owner-held.

Replicated-item partition (``build_replicated_graph`` / ``ReplicatedPyGGAT``; the U-I
graph of configs 2/3, default of ``bench.py --gpus N`` there): see its section below.

Dropout masks are keyed by the original edge_index column and a per-layer seed every rank
agrees on (``SharedSeeds``: a base drawn on rank 0 and broadcast once, then a counter), so
a source-side backward and a destination-side forward regenerate the same mask whatever
the ranks' own RNG states.
"""
from __future__ import annotations

import ctypes
import os
import weakref
from dataclasses import dataclass
from types import SimpleNamespace
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

    def all_to_all_rows(self, t: torch.Tensor, send_counts, recv_counts, out: Optional[torch.Tensor] = None):
        """all_to_all_single of row blocks: rows [sum(send_counts[:r]), +send_counts[r]) of t go
        to rank r; the result holds recv_counts[s] rows from each rank s, in rank order.
        ``out`` (optional): a contiguous [sum(recv_counts), ...] destination."""
        t = t.contiguous()
        n_out = int(sum(recv_counts))
        shape = (n_out,) + tuple(t.shape[1:])
        if out is None:
            out = torch.empty(shape, dtype=t.dtype, device=t.device)
        if not self.active:
            if n_out:
                out.copy_(t[:n_out])
            return out
        sc, rc = [int(c) for c in send_counts], [int(c) for c in recv_counts]
        if self.backend == "gloo" and t.is_cuda:  # several ranks sharing one GPU in a test: stage through host
            host = torch.empty(shape, dtype=t.dtype)
            dist.all_to_all_single(host, t.cpu(), rc, sc, group=self.group)
            out.copy_(host)
            return out
        dist.all_to_all_single(out, t, rc, sc, group=self.group)
        return out

    def p2p(self, sends, recvs):
        """One group of point-to-point transfers: ``sends`` / ``recvs`` are lists of (peer,
        contiguous tensor); between a pair of ranks the k-th send matches the k-th receive
        (RCCL: one ncclGroupStart/End through batch_isend_irecv; gloo: tag-ordered pairs).
        Device tensors under gloo (ranks sharing one GPU in a test) are staged through host."""
        if not sends and not recvs:
            return
        stage = self.backend == "gloo" and any(t.is_cuda for _, t in list(sends) + list(recvs))
        hs = [(p, t.cpu() if stage else t) for p, t in sends]
        hr = [(p, torch.empty(t.shape, dtype=t.dtype) if stage else t) for p, t in recvs]
        ops = [dist.P2POp(dist.isend, t, p, group=self.group) for p, t in hs]
        ops += [dist.P2POp(dist.irecv, t, p, group=self.group) for p, t in hr]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if stage:
            for (_, t), (_, h) in zip(recvs, hr):
                t.copy_(h)

    def exchange(self, plan: "ExchangePlan", src: torch.Tensor, out: torch.Tensor, part: Optional[int] = None
                 ) -> torch.Tensor:
        """A plan's forward exchange without packing: the own rows of ``src`` (own-local row
        order) in each peer's send runs leave straight from ``src``; ``out`` [n_recv, ...]
        receives each peer's rows in peer order, each peer's runs back to back (the halo rows'
        order, build_halo_graph) -- no gather into a send buffer, no copy out of a receive buffer."""
        sends, recvs, off = [], [], 0
        if part is not None:  # one of the two halves (run_plan): the other half's rows untouched
            sp, rp = plan.parts[part]
            for q, runs in enumerate(sp):
                sends += [(q, src[a:a + n]) for a, n in runs if n]
            for r, runs in enumerate(rp):
                recvs += [(r, out[o:o + n]) for o, n in runs if n]
            self.p2p(sends, recvs)
            return out
        for q, runs in enumerate(plan.send_runs):
            sends += [(q, src[a:a + n]) for a, n in runs]
        for r, lens in enumerate(plan.recv_runs):
            for n in lens:
                recvs.append((r, out[off:off + n]))
                off += n
        self.p2p(sends, recvs)
        return out

    def exchange_back(self, plan: "ExchangePlan", halo: torch.Tensor, out: Optional[torch.Tensor] = None):
        """The reverse of ``exchange``: the halo rows [n_recv, ...] go back to their owners in the
        same runs; ``out`` [n_send, ...] gets each peer's returned copies in send_idx order (peer
        order, each peer's runs back to back) -- the layout ret_ptr / ret_pos index."""
        if out is None:
            out = torch.empty((plan.n_send,) + tuple(halo.shape[1:]), dtype=halo.dtype, device=halo.device)
        sends, recvs, off = [], [], 0
        for r, lens in enumerate(plan.recv_runs):
            for n in lens:
                sends.append((r, halo[off:off + n]))
                off += n
        off = 0
        for q, runs in enumerate(plan.send_runs):
            for _, n in runs:
                recvs.append((q, out[off:off + n]))
                off += n
        self.p2p(sends, recvs)
        return out

    def broadcast_int(self, value: int, src: int = 0) -> int:
        if not self.active:
            return int(value)
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else "cpu"
        t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
        dist.broadcast(t, src, group=self.group)
        return int(t.item())

    def all_to_all_counts(self, counts) -> list:
        """Every rank sends counts[r] to rank r; returns what each rank sent here (host ints)."""
        if not self.active:
            return [int(c) for c in counts]
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else "cpu"
        src = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=dev)
        dst = torch.empty_like(src)
        dist.all_to_all_single(dst, src, group=self.group)
        return [int(v) for v in dst.cpu().tolist()]


# ---------------------------------------------------------------------------
# dropout seeds every rank agrees on
# ---------------------------------------------------------------------------
def _dropout_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


def derive_seed(base: int, k: int) -> int:
    """splitmix64(base + k * golden gamma): the k-th layer call's dropout seed."""
    x = (int(base) + (int(k) + 1) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return (x ^ (x >> 31)) & ((1 << 62) - 1)


class SharedSeeds:
    """Per-layer-call dropout seeds identical on every rank: the base is drawn from torch's
    CPU generator on rank 0 at the first draw and broadcast once (the only host sync), then
    call k uses derive_seed(base, k).  Ranks call the model the same number of times, so
    their counters agree; per-rank seeding of torch's RNG does not matter."""

    def __init__(self, comm: "Comm"):
        self.comm = comm
        self.base = None
        self.count = 0

    def next(self) -> int:
        if self.base is None:
            self.base = self.comm.broadcast_int(_dropout_seed() if self.comm.rank == 0 else 0)
        s = derive_seed(self.base, self.count)
        self.count += 1
        return s


# ---------------------------------------------------------------------------
# exchange plans: static all_to_all of rows (RCCL) and the ordered return of gradients
# ---------------------------------------------------------------------------
@dataclass
class ExchangePlan:
    """This rank sends its own rows ``send_idx`` (concatenated per peer, peers in rank
    order, send_counts[r] rows to rank r) and receives recv_counts[s] rows from each peer
    s, appended after its n_own own rows in peer order.  Backward: the peers return the
    gradients of the rows they received; own row o adds its copies ret_pos[ret_ptr[o] :
    ret_ptr[o+1]] (positions in the returned block) in that order -- peer order."""
    n_own: int
    send_idx: torch.Tensor      # int64 [n_send]
    send_counts: list
    recv_counts: list
    ret_ptr: torch.Tensor       # int32 [n_own + 1]
    ret_pos: torch.Tensor       # int32 [n_send]
    # the halo plans (build_halo_graph): per peer the runs [(own row, count), ...] send_idx is made
    # of, and per peer the lengths of the runs it sends here -- Comm.exchange moves rows straight
    # from / into the row tables; None for the loss plans (gather + all_to_all)
    send_runs: Optional[list] = None
    recv_runs: Optional[list] = None
    parts: Optional[list] = None    # [(send runs, recv (offset, count) runs) per peer] of the two halves

    @property
    def n_send(self) -> int:
        return int(sum(self.send_counts))

    @property
    def n_recv(self) -> int:
        return int(sum(self.recv_counts))


def make_plan(n_own: int, send_idx: np.ndarray, send_counts, recv_counts, device, send_runs=None,
              recv_runs=None) -> ExchangePlan:
    send_idx = np.asarray(send_idx, np.int64)
    order = np.argsort(send_idx, kind="stable")           # by own row, peer order kept
    ptr = np.zeros(n_own + 1, np.int64)
    np.cumsum(np.bincount(send_idx, minlength=n_own), out=ptr[1:])
    return ExchangePlan(int(n_own), torch.from_numpy(send_idx).to(device), [int(c) for c in send_counts],
                        [int(c) for c in recv_counts], torch.from_numpy(ptr.astype(np.int32)).to(device),
                        torch.from_numpy(order.astype(np.int32)).to(device), send_runs, recv_runs)


def _runs(b: np.ndarray):
    """(starts, lengths) of the runs of True in a boolean array."""
    d = np.diff(np.concatenate([[0], b.astype(np.int8), [0]]))
    st = np.flatnonzero(d == 1)
    return st, np.flatnonzero(d == -1) - st


def run_plan(n_own: int, masks_own: np.ndarray, base: int, world: int, recv: list, device) -> ExchangePlan:
    """The halo plan of one row class: own rows [base, base + len(masks_own)) in own-local order,
    masks_own their peer sets (bit q: rank q holds the row as a halo row); ``recv[r]`` = (starts,
    lengths, class rows): the runs rank r sends here, as positions in r's own rows of the class,
    and r's row count of the class.  send_idx = per peer (rank order) its runs expanded.
    The plan can also move in two parts split at half of each owner's class rows (exchange
    ``part``): a producer that finishes the first half of its rows sends them at once."""
    send_runs, idx, counts = [], [], []
    for q in range(world):
        st, ln = _runs(((masks_own >> np.uint32(q)) & np.uint32(1)).astype(bool))
        send_runs.append([(int(a) + base, int(n)) for a, n in zip(st, ln)])
        idx.append(np.concatenate([np.arange(a, a + n) for a, n in send_runs[-1]]) if len(st) else
                   np.zeros(0, np.int64))
        counts.append(int(ln.sum()))
    recv_runs = [[int(n) for n in ln] for _, ln, _ in recv]
    plan = make_plan(n_own, np.concatenate(idx) if idx else np.zeros(0, np.int64), counts,
                     [sum(l) for l in recv_runs], device, send_runs, recv_runs)
    # the two parts: sends clipped at base + len // 2; each owner's runs clipped at its class // 2,
    # landing at their places inside that owner's block of the halo slice
    cut = base + len(masks_own) // 2
    sp = [[], []]
    for runs in send_runs:
        lo, hi = [], []
        for a, n in runs:
            if a + n <= cut:
                lo.append((a, n))
            elif a >= cut:
                hi.append((a, n))
            else:
                lo.append((a, cut - a))
                hi.append((cut, a + n - cut))
        sp[0].append(lo)
        sp[1].append(hi)
    rp, off = [[], []], 0
    for st, ln, cnt in recv:
        ocut = int(cnt) // 2
        lo, hi = [], []
        for a, n in zip(st, ln):
            a, n = int(a), int(n)
            if a + n <= ocut:
                lo.append((off, n))
            elif a >= ocut:
                hi.append((off, n))
            else:
                lo.append((off, ocut - a))
                hi.append((off + ocut - a, a + n - ocut))
            off += n
        rp[0].append(lo)
        rp[1].append(hi)
    plan.parts = [(sp[0], rp[0]), (sp[1], rp[1])]
    return plan


def peer_masks(src: np.ndarray, od: np.ndarray, owner: np.ndarray, world: int) -> np.ndarray:
    """[N] uint32: bit q of node v set iff an edge v -> d has d owned by rank q != owner(v) --
    the ranks that hold v as a halo row (they home an edge that reads v)."""
    if world > 32:
        raise NotImplementedError("halo partition: at most 32 ranks (peer sets are 32-bit masks)")
    N = len(owner)
    mask = np.zeros(N, np.uint32)
    for q in range(world):
        mask[src[od == q]] |= np.uint32(1 << q)
    mask &= ~(np.uint32(1) << owner.astype(np.uint32))
    return mask


def send_order_key(mask: np.ndarray, owner: np.ndarray, world: int) -> np.ndarray:
    """Sort key of a node within its owner's rows: the position of its peer set (bits rotated
    so the owner's peers are bits 0..W-2) in the binary-reflected Gray sequence.  Rows sorted by
    it leave each peer's rows in few runs (about 2^(W-2) runs over all peers, one for the top
    bit), so Comm.exchange sends straight from the row table instead of packing."""
    rel = np.zeros(len(mask), np.uint32)
    o = owner.astype(np.int64)
    for q in range(world):
        bit = (mask >> np.uint32(q)) & np.uint32(1)
        rel |= bit << ((q - o - 1) % world).astype(np.uint32)
    key = rel.copy()
    sh = 1
    while sh < 32:  # inverse Gray code: prefix xor of the higher bits
        key ^= key >> np.uint32(sh)
        sh <<= 1
    return key


class _Exchange(torch.autograd.Function):
    """[n_own, ...] own rows -> [n_own + sum n_recv (+ n_tail), ...] = [own | rows received
    under each plan, in plan order | tail]: ``tail`` (nullable) are rows the rank computes
    itself (the first layer's halo items, from the replicated item features)."""

    @staticmethod
    def forward(ctx, t_own, tail, plans, comm: "Comm", stages, inplace_grad: bool = False,
                handoff: Optional[dict] = None):
        t_own = t_own.contiguous()
        n_tail = tail.size(0) if tail is not None else 0
        n_own = plans[0].n_own
        n_out = n_own + sum(p.n_recv for p in plans) + n_tail
        row = t_own[0].numel() if t_own.dim() > 1 else 1
        st_ = t_own.untyped_storage()
        if (inplace_grad and t_own.dim() == 2 and n_tail == 0 and t_own.size(0) == n_own and
                st_.nbytes() >= (t_own.storage_offset() + n_out * row) * t_own.element_size()):
            # the own rows lie at the top of a buffer with room for the received rows (the top
            # layer's output, HaloPyGGAT._top_out): receive behind them, no copy of the own rows
            out = t_own.new_empty(0).set_(st_, t_own.storage_offset(), (n_out, row), (row, 1))
        else:
            out = torch.empty((n_out,) + tuple(t_own.shape[1:]), dtype=t_own.dtype, device=t_own.device)
            out[:n_own].copy_(t_own)
        ctx.inplace_grad, ctx.handoff = inplace_grad, handoff
        off = n_own
        for plan in plans:
            if plan.send_runs is not None:  # the halo plans: straight from the own rows
                comm.exchange(plan, t_own, out[off:off + plan.n_recv])
            else:
                send = stages.gather_rows(t_own, plan.send_idx)
                comm.all_to_all_rows(send, plan.send_counts, plan.recv_counts, out=out[off:off + plan.n_recv])
            off += plan.n_recv
        if n_tail:
            out[off:].copy_(tail)
        ctx.plans, ctx.comm, ctx.stages, ctx.has_tail = plans, comm, stages, tail is not None
        return out

    @staticmethod
    def backward(ctx, g):
        plans, comm, st = ctx.plans, ctx.comm, ctx.stages
        g = g.contiguous()
        n_own = plans[0].n_own
        # the own rows' sums in place in the incoming gradient (a buffer of its own: the loss's or
        # the layer's fresh gradient) instead of a copy of them (1.9 GB at world 8 on config 5)
        g_own = g[:n_own] if (g._base is None or ctx.inplace_grad) else g[:n_own].clone()
        if ctx.handoff is not None:
            # the loss's dZ buffer: hand it to the top layer's backward by object identity (a later
            # tensor at the same address is never taken for it)
            ctx.handoff["g"] = weakref.ref(g_own)
        off = n_own
        for plan in plans:  # each plan touches its own rows (users / items): independent sums
            st.return_add(g_own, _return(comm, plan, g[off:off + plan.n_recv]), plan.ret_ptr, plan.ret_pos)
            off += plan.n_recv
        return g_own, (g[off:] if ctx.has_tail else None), None, None, None, None, None


def _return(comm: "Comm", plan: ExchangePlan, halo: torch.Tensor) -> torch.Tensor:
    """The halo rows' values back to their owners -> [n_send, ...] in send_idx order."""
    if plan.send_runs is not None:
        return comm.exchange_back(plan, halo)
    return comm.all_to_all_rows(halo, plan.recv_counts, plan.send_counts)


def exchange(t_own, plan: ExchangePlan, comm: "Comm", stages, inplace_grad: bool = False,
             handoff: Optional[dict] = None):
    """``inplace_grad``: the incoming gradient is a buffer of the caller's own (the loss's dZ):
    the own rows' sums are formed in place in it; ``handoff``: a dict that receives a weak
    reference to the own rows' gradient (key "g") for the layer below."""
    return _Exchange.apply(t_own, None, [plan], comm, stages, inplace_grad, handoff)


def halo_exchange(t_own, hg: "HaloGraph", comm: "Comm", stages, halo_items: Optional[torch.Tensor] = None):
    """[own | halo users | halo items] rows of one layer: the halo users by the user plan's
    all_to_all; the halo items by the item plan's, or -- first layer -- ``halo_items``
    computed locally from the replicated item features (no exchange, no return)."""
    if halo_items is not None:
        return _Exchange.apply(t_own, halo_items, [hg.plan_u], comm, stages)
    return _Exchange.apply(t_own, None, [hg.plan_u, hg.plan_i], comm, stages)


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
    """A rank's slice of a CSR (destination rows) / CSC (source rows) the stages run on."""
    n_rows: int                 # rows this view's stage iterates / writes
    rowptr: torch.Tensor        # CSR of destination rows (rebased)
    col: torch.Tensor           # [E_fwd] source row ids (local row space)
    csr_eid: torch.Tensor       # [E_fwd] original edge_index columns (dropout hash key)
    n_fwd_edges: int
    colptr: torch.Tensor        # CSC of source rows (rebased)
    row: torch.Tensor           # [E_bwd] destination row ids
    csc_eid: torch.Tensor       # [E_bwd]
    dz_slot: torch.Tensor       # [E_bwd] CSR slot of each CSC edge (the logit-gradient buffer)
    n_bwd_edges: int
    fwd_sched: object = None
    bwd_sched: object = None


def _hip_csr(ei, P):
    from .hip_ops import csr_build
    return csr_build(ei, P)


def _hip_sched(ptr, E):
    from .hip_ops import schedule_build
    return schedule_build(ptr, E)


@dataclass
class HaloGraph:
    world: int
    rank: int
    n_nodes: int
    n_edges: int
    n_users: int
    user_bounds: np.ndarray     # [world + 1]: rank r owns the users [b_r, b_{r+1}) (node ids)
    n_own: int                  # own rows: the users of [u0, u1), then the own items (halo_owner), each in
                                # send order (send_order_key)
    n_halo: int                 # halo rows: users (by owner) then items (by owner), in the owner's order
    plan_u: ExchangePlan        # the layer halo exchange of user rows
    plan_i: ExchangePlan        # ... of item rows
    fwd_view: LocalView         # CSR over the own destination rows (n_rows = n_own)
    bwd_view: LocalView         # CSC over [own | halo] source rows (n_rows = n_own + n_halo)
    local_of: np.ndarray        # [N] int64: node id -> own row, -1 elsewhere (host)
    owner: np.ndarray           # [N] int32 node owner (host)
    loss_plans: dict = None
    halo_items: torch.Tensor = None  # [n_halo_i] int64 item indices (node id - n_users) of the halo items
    bwd_sched_own: object = None   # backward schedule over the own source rows
    bwd_sched_halo: object = None  # ... over the halo source rows (row ids relative to n_own)
    n_own_u: int = 0               # own rows [0, n_own_u) are users, [n_own_u, n_own) items
    bipartite: bool = False        # every edge joins a user and an item (the U-I graph)
    fwd_sched_u: object = None     # forward schedule over the own user destinations
    fwd_sched_i: object = None     # ... over the own item destinations (rows relative to n_own_u)
    own_items: torch.Tensor = None # [n_own - n_own_u] int64 item indices (node id - n_users), own-local order
    own_pos: np.ndarray = None     # [N] int32: each node's row at its owner (host)
    own_users: np.ndarray = None   # [n_own_u] int64: the own users' node ids in own-local order (host)
    halo_ids: np.ndarray = None    # [n_halo] int64: the halo rows' node ids in table order (host)
    item_partition: str = "dealt"
    # symmetric edge list (every column j -> i has its i -> j, as build_edge_index's U-I graph):
    # the rows a rank needs as sources (forward) are exactly the rows it needs as destinations of
    # its own rows' out-edges, so the backward can run at the SOURCE's owner (_halo_xgat_backward)
    symmetric: bool = False
    src_views: object = None       # hip_ops.XViews of the edges whose source is own (CSC over own rows,
                                   # CSR over the [own | halo] destination table)
    src_sched_u: object = None     # their schedule over the own user sources
    src_sched_i: object = None     # ... over the own item sources (rows relative to n_own_u)

    @property
    def R(self) -> int:
        return self.n_own + self.n_halo

    @property
    def n_halo_u(self) -> int:
        return self.plan_u.n_recv

    @property
    def n_send(self) -> int:
        return self.plan_u.n_send + self.plan_i.n_send

    @property
    def bounds(self) -> np.ndarray:
        return self.user_bounds

    def owned_users(self, n_users: int = 0, rank: Optional[int] = None):
        """(u0, u1): the node-id range of a rank's users."""
        r = self.rank if rank is None else rank
        return int(self.user_bounds[r]), int(self.user_bounds[r + 1])

    def own_node_ids(self, rank: Optional[int] = None) -> np.ndarray:
        """A rank's own rows as global node ids, in its own-local row order (host)."""
        r = self.rank if rank is None else rank
        ids = np.flatnonzero(self.owner == r)   # users first (ids below n_users), then items
        nu = int(np.searchsorted(ids, self.n_users))
        u, it = ids[:nu], ids[nu:]
        return np.concatenate([u[np.argsort(self.own_pos[u], kind="stable")],
                               it[np.argsort(self.own_pos[it], kind="stable")]])

    def own_user_ids(self, rank: Optional[int] = None) -> np.ndarray:
        """A rank's own users' node ids in its own-local row order (host)."""
        if rank is None or rank == self.rank:
            return self.own_users
        return self.own_node_ids(rank)[:int(self.user_bounds[rank + 1] - self.user_bounds[rank])]

    def xviews(self):
        """The local edge lists as hip_ops.XViews (aggregate-then-transform layer): CSR over the
        own destination rows, CSC over [own | halo] sources."""
        from .hip_ops import XViews
        f, b = self.fwd_view, self.bwd_view
        return XViews(self.n_own, self.R, f.n_fwd_edges, f.col, f.csr_eid, f.fwd_sched, b.row, b.csc_eid, b.dz_slot,
                      b.bwd_sched, self.bwd_sched_own, self.bwd_sched_halo, rowptr=f.rowptr, colptr=b.colptr)


def halo_owner(deg: np.ndarray, n_users: int, world: int, item_partition: str = "dealt"):
    """Row ownership of the halo partition -> (owner [N] int32, user bounds [world + 1]).

    Users: contiguous id ranges with equal degree sums (users are uniform: each rank sends
    about the same number of user rows).  Items (``item_partition``):
      "dealt"      -- items sorted by degree (descending, ties by id) and dealt to the ranks in
                      snake order 0..W-1, W-1..0, ...: every rank gets the same mix of hub and
                      tail items, so the degree sums, the row counts AND the halo sends (a hub
                      goes to every peer, a tail item to few) are balanced together;
      "contiguous" -- contiguous id ranges with equal degree sums (with popularity-ordered
                      ids, e.g. config 5's Zipf items, one rank then owns all the hubs and
                      another the long tail: equal edges but 2x the sends of the mean).
    Deterministic: every rank computes the same owner array."""
    N, nu = len(deg), int(n_users)
    owner = np.empty(N, np.int32)
    ub = partition_bounds(deg[:nu], world)
    owner[:nu] = np.repeat(np.arange(world, dtype=np.int32), np.diff(ub))
    if item_partition == "dealt":
        order = np.argsort(-deg[nu:], kind="stable")
        pos = np.arange(N - nu)
        k, cyc = pos % world, pos // world
        owner[nu + order] = np.where(cyc % 2 == 0, k, world - 1 - k).astype(np.int32)
    elif item_partition == "contiguous":
        ib = partition_bounds(deg[nu:], world)
        owner[nu:] = np.repeat(np.arange(world, dtype=np.int32), np.diff(ib))
    else:
        raise ValueError(f"item_partition must be 'dealt' or 'contiguous', not {item_partition!r}")
    return owner, ub


def _mix64(k: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser over uint64 keys (wrapping arithmetic)."""
    k = k.astype(np.uint64)
    k = (k ^ (k >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    k = (k ^ (k >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return k ^ (k >> np.uint64(31))


def edges_symmetric(src: np.ndarray, dst: np.ndarray, n: int) -> bool:
    """Whether the multiset of columns (src, dst) equals that of (dst, src): equal in- and
    out-degrees and equal sums of a 64-bit hash of the ordered pair (a multiset hash; a false
    positive needs a 2^-64 collision).  build_edge_index's U-I graph (u -> i and i -> u per
    interaction) is symmetric."""
    with np.errstate(over="ignore"):
        if not np.array_equal(np.bincount(src, minlength=n), np.bincount(dst, minlength=n)):
            return False
        a = _mix64(src.astype(np.uint64) * np.uint64(n) + dst.astype(np.uint64)).sum(dtype=np.uint64)
        b = _mix64(dst.astype(np.uint64) * np.uint64(n) + src.astype(np.uint64)).sum(dtype=np.uint64)
    return bool(a == b)


def build_halo_graph(edge_index: torch.Tensor, n_nodes: int, n_users: int, world: int, rank: int,
                     csr_builder: Callable = _hip_csr, sched_builder: Optional[Callable] = _hip_sched,
                     node_weight: float = 4.0, item_partition: Optional[str] = None) -> HaloGraph:
    """Every rank calls this with the same global edge_index (LongTensor [2, E], users
    [0, n_users), items [n_users, N)) and gets its own slices; deterministic, so all ranks
    agree on the plan without exchanging it.  ``item_partition``: halo_owner's (default
    "dealt", or $PPGAT_ITEM_PARTITION)."""
    dev = edge_index.device
    N, nu = int(n_nodes), int(n_users)
    E = int(edge_index.size(1))
    ei = edge_index.cpu().numpy()
    src, dst = ei[0], ei[1]
    deg = (np.bincount(dst, minlength=N) + np.bincount(src, minlength=N)).astype(np.float64) + node_weight
    item_partition = item_partition or os.environ.get("PPGAT_ITEM_PARTITION", "dealt")
    owner, ub = halo_owner(deg, nu, world, item_partition)
    u0, u1 = int(ub[rank]), int(ub[rank + 1])
    od, osrc = owner[dst], owner[src]
    # every node's peer set and its row order at its owner: users then items, each sorted by the
    # Gray position of the peer set (then id), so that what a rank sends a peer is a few runs of
    # its row table (Comm.exchange, no packing); the halo rows of an owner arrive in that order
    mask = peer_masks(src, od, owner, world)
    ids = np.arange(N)
    cls = (ids >= nu).astype(np.int8)
    go = np.lexsort((ids, send_order_key(mask, owner, world), cls, owner))   # by owner, class, key, id
    bnd = np.searchsorted(owner[go] * 2 + cls[go], np.arange(2 * world + 1), side="left")
    own_pos = np.empty(N, np.int32)  # each node's row at its owner
    for r in range(world):
        a, b = bnd[2 * r], bnd[2 * r + 2]
        own_pos[go[a:b]] = np.arange(b - a, dtype=np.int32)
    own_u, own_it = go[bnd[2 * rank]:bnd[2 * rank + 1]], go[bnd[2 * rank + 1]:bnd[2 * rank + 2]]
    own_items = own_it                                     # node ids in own-local order
    n_own = len(own_u) + len(own_it)
    local_of = np.full(N, -1, np.int64)
    local_of[own_u] = np.arange(len(own_u))
    local_of[own_it] = len(own_u) + np.arange(len(own_it))
    loc = np.flatnonzero(od == rank)                       # edges homed here (destination owned)
    lsrc = src[loc]
    need = ((mask >> np.uint32(rank)) & np.uint32(1)).astype(bool)
    # the halo rows: every node whose peer set holds this rank, grouped by owner in the owner's order
    halo_u = np.concatenate([go[bnd[2 * r]:bnd[2 * r + 1]][need[go[bnd[2 * r]:bnd[2 * r + 1]]]]
                             for r in range(world)])
    halo_i = np.concatenate([go[bnd[2 * r + 1]:bnd[2 * r + 2]][need[go[bnd[2 * r + 1]:bnd[2 * r + 2]]]]
                             for r in range(world)])
    lidx = local_of.copy()
    lidx[halo_u] = n_own + np.arange(len(halo_u))
    lidx[halo_i] = n_own + len(halo_u) + np.arange(len(halo_i))
    # what each owner r sends here: the runs of its rows (in its order) whose peer set holds this rank
    recv_u = [_runs(need[go[bnd[2 * r]:bnd[2 * r + 1]]]) + (bnd[2 * r + 1] - bnd[2 * r],) for r in range(world)]
    recv_i = [_runs(need[go[bnd[2 * r + 1]:bnd[2 * r + 2]]]) + (bnd[2 * r + 2] - bnd[2 * r + 1],)
              for r in range(world)]
    plan_u = run_plan(n_own, mask[own_u], 0, world, recv_u, dev)
    plan_i = run_plan(n_own, mask[own_it], len(own_u), world, recv_i, dev)
    del go, mask, need
    halo = np.concatenate([halo_u, halo_i])
    R = n_own + len(halo)
    ei_l = torch.from_numpy(np.stack([lidx[lsrc], lidx[dst[loc]]])).to(dev)
    El = len(loc)
    G = csr_builder(ei_l, R)
    gid = torch.from_numpy(loc.astype(np.int32)).to(dev)
    orig = (lambda t: gid[t.long()].contiguous()) if El else (lambda t: t[:0].contiguous())
    rowptr_own = G.rowptr[:n_own + 1].contiguous()
    col, csr_eid = G.col[:El].contiguous(), orig(G.csr_eid[:El])
    row, csc_eid, slot = G.row[:El].contiguous(), orig(G.csc_eid[:El]), G.csc2csr[:El].contiguous()
    fwd_view = LocalView(n_own, rowptr_own, col, csr_eid, El, G.colptr.contiguous(), row, csc_eid, slot, El)
    bwd_view = LocalView(R, G.rowptr.contiguous(), col, csr_eid, El, G.colptr.contiguous(), row, csc_eid, slot, El)
    hg = HaloGraph(world, rank, N, E, nu, ub, n_own, len(halo), plan_u, plan_i, fwd_view, bwd_view, local_of,
                   owner, {}, torch.from_numpy(halo_i - nu).to(dev))
    hg.own_items = torch.from_numpy(own_items - nu).to(dev)
    hg.own_pos = own_pos
    hg.halo_ids = halo
    hg.own_users = own_u
    hg.item_partition = item_partition
    hg.n_own_u = u1 - u0
    hg.bipartite = bool(np.all((src < nu) != (dst < nu)))  # the same decision on every rank
    hg.symmetric = edges_symmetric(src, dst, N)
    if hg.symmetric:
        # the edges whose SOURCE this rank owns: source rows own-local, destinations in the
        # [own | halo] table (by symmetry every such destination is own or a halo row)
        sh = np.flatnonzero(osrc == rank)
        dl = lidx[dst[sh]]
        assert (dl >= 0).all(), "symmetric graph: every out-neighbour of an own row is own or halo"
        Gb = csr_builder(torch.from_numpy(np.stack([local_of[src[sh]], dl])).to(dev), R)
        Eb = len(sh)
        gidb = torch.from_numpy(sh.astype(np.int32)).to(dev)
        origb = (lambda t: gidb[t.long()].contiguous()) if Eb else (lambda t: t[:0].contiguous())
        hg.src_views = _src_views(n_own, R, Eb, Gb, origb)
    if dev.type == "cuda" and _lib.debug_build():  # debug build: plans and views within bounds
        for pname, plan in (("plan_u", plan_u), ("plan_i", plan_i)):
            _lib.check_index_range(plan.send_idx, 0, n_own, f"halo.{pname}.send_idx")
            _lib.check_index_range(plan.ret_pos, 0, max(plan.n_send, 1), f"halo.{pname}.ret_pos")
        _lib.check_index_range(col, 0, R, "halo.col")
        _lib.check_index_range(row, 0, n_own, "halo.row")
        _lib.check_index_range(slot, 0, max(El, 1), "halo.dz_slot")
        _lib.check_index_range(hg.halo_items, 0, N - nu, "halo.halo_items")
    if sched_builder is not None:
        fwd_view.fwd_sched = sched_builder(rowptr_own, El)
        bwd_view.bwd_sched = sched_builder(bwd_view.colptr, El)
        bwd_view.fwd_sched = fwd_view.fwd_sched
        # the backward edge pass split by source class: halo sources first (their input
        # gradients go back to their owners while the own sources are processed)
        hg.bwd_sched_own = sched_builder(bwd_view.colptr[:n_own + 1].contiguous(), El)
        hg.bwd_sched_halo = sched_builder(bwd_view.colptr[n_own:].contiguous(), El)
        # the forward split by destination class (bipartite graphs: a class's sources are the
        # other class, so a phase needs only that class's halo rows; _HaloLayerX)
        hg.fwd_sched_u = sched_builder(rowptr_own[:hg.n_own_u + 1].contiguous(), El)
        hg.fwd_sched_i = sched_builder(rowptr_own[hg.n_own_u:].contiguous(), El)
        if int(os.environ.get("PPGAT_HALO_PARTS", "2")) == 2:
            # each class's destinations in two halves (_halo_phases), split where the plans split
            nu_, n0_ = hg.n_own_u, n_own
            mu, mi = nu_ // 2, nu_ + (n0_ - nu_) // 2
            hg.fwd_sched_halves = {"u": (sched_builder(rowptr_own[:mu + 1].contiguous(), El),
                                         sched_builder(rowptr_own[mu:nu_ + 1].contiguous(), El)),
                                   "i": (sched_builder(rowptr_own[nu_:mi + 1].contiguous(), El),
                                         sched_builder(rowptr_own[mi:].contiguous(), El))}
        if hg.src_views is not None:
            sv = hg.src_views
            sv.fwd_sched = sched_builder(sv.rowptr, sv.n_edges)   # destination sums over the R table rows
            hg.src_sched_u = sched_builder(sv.colptr[:hg.n_own_u + 1].contiguous(), sv.n_edges)
            hg.src_sched_i = sched_builder(sv.colptr[hg.n_own_u:].contiguous(), sv.n_edges)
            sv.bwd_sched = sched_builder(sv.colptr, sv.n_edges)
    return hg


def _src_views(n_own: int, R: int, Eb: int, Gb, orig):
    """hip_ops.XViews of the edges whose source is own: CSC over the own source rows (row = the
    destination's row in the [own | halo] table, dz in CSC order), CSR over the table rows (the
    per-destination partial sums, read through csr2csc); edge ids mapped to edge_index columns."""
    from .hip_ops import XViews
    c2r = Gb.csc2csr[:Eb].long()
    csr2csc = torch.empty(Eb, dtype=torch.int32, device=c2r.device)  # CSR slot -> CSC position
    csr2csc[c2r] = torch.arange(Eb, dtype=torch.int32, device=c2r.device)
    return XViews(R, n_own, Eb, Gb.col[:Eb].contiguous(), orig(Gb.csr_eid[:Eb]), None, Gb.row[:Eb].contiguous(),
                  orig(Gb.csc_eid[:Eb]), None, None, csr2csc=csr2csc,
                  rowptr=Gb.rowptr.contiguous(), colptr=Gb.colptr[:n_own + 1].contiguous())


# ---------------------------------------------------------------------------
# the layer on a rank's local rows
# ---------------------------------------------------------------------------
class _LocalGAT(torch.autograd.Function):
    """h_loc [own + halo rows, H*C] -> out [own rows, C]: node scores, the fused forward over
    the own destination rows; backward over the local CSC (own and halo source rows)."""

    @staticmethod
    def forward(ctx, h, att_src, att_dst, bias, hg: HaloGraph, stages, heads: int, C: int, mode: int, slope: float,
                p: float, seed: int):
        h = h.contiguous()
        a_s = att_src.detach().reshape(heads, C).contiguous()
        a_d = att_dst.detach().reshape(heads, C).contiguous()
        b = bias.detach().contiguous() if bias is not None else None
        s_src, s_dst = stages.scores(h, a_s, a_d, heads, C)
        s_dst = s_dst[:hg.n_own].contiguous()
        need = any(ctx.needs_input_grad[:4])
        seed_buf = stages.seed_buffer(p, h.device) if need else None
        out, m, inv_l, agg = stages.fwd(hg.fwd_view, h, s_src, s_dst, b, heads, C, mode, slope, p, seed,
                                        need and heads > 1, seed_buf=seed_buf)
        if need:
            empty = torch.empty(0, device=h.device)
            ctx.save_for_backward(h, a_s, a_d, s_src, s_dst, out, m, inv_l, agg if agg is not None else empty,
                                  b if b is not None else empty)
        ctx.hg, ctx.stages, ctx.seed_buf = hg, stages, seed_buf
        ctx.meta = (heads, C, mode, slope, p, seed, bias is not None, agg is not None)
        ctx.att_shapes = (att_src.shape, att_dst.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        h, a_s, a_d, s_src, s_dst, out, m, inv_l, agg, b = ctx.saved_tensors
        heads, C, mode, slope, p, seed, has_bias, has_agg = ctx.meta
        hg, st = ctx.hg, ctx.stages
        g = g.contiguous()
        want_db = has_bias and ctx.needs_input_grad[3]
        nstate, dbias = st.bwd_prologue(g, out, agg if has_agg else None, b if has_bias else None, s_dst, m, inv_l,
                                        heads, C, mode, want_db)
        dz = torch.zeros(max(hg.bwd_view.n_bwd_edges, 1) * heads, dtype=h.dtype, device=h.device)
        grad_h, ds_src = st.bwd_edges(hg.bwd_view, h, s_src, nstate, g, dz, heads, C, mode, slope, p, seed,
                                      seed_buf=ctx.seed_buf)
        datt_src, datt_dst = st.bwd_epilogue(hg.bwd_view, h, a_s, a_d, ds_src, dz, grad_h, heads, C)
        return (grad_h, datt_src.view(ctx.att_shapes[0]), datt_dst.view(ctx.att_shapes[1]), dbias,
                None, None, None, None, None, None, None, None)


_COMM_STREAMS = {}


def _comm_stream(dev) -> torch.cuda.Stream:
    s = _COMM_STREAMS.get(dev.index)
    if s is None:
        s = torch.cuda.Stream(device=dev)
        _COMM_STREAMS[dev.index] = s
    return s


class HaloRows:
    """The input rows [own | halo users | halo items] of one multi-head halo layer and the state
    of its two halo classes ("u", "i").  A class's rows are either received -- ``start(cls,
    src)`` gathers the owner's rows of ``src`` each peer needs and runs the all_to_all, on the
    communication stream under RCCL, as soon as the owner has them (for layer l+1 right after
    the phase of layer l that produced them) -- or computed locally (``set_local``: the first
    layer's halo items).  ``wait(cls)`` orders the current stream after that class's rows."""

    def __init__(self, hg: "HaloGraph", comm: "Comm", stages, width: int, like: torch.Tensor,
                 x: Optional[torch.Tensor] = None):
        self.hg, self.comm, self.stages = hg, comm, stages
        # x: a caller's [R, width] table (the first layer's persistent one, HaloPyGGAT._first_table)
        self.x = x if x is not None else torch.empty((hg.R, width), dtype=like.dtype, device=like.device)
        self.events = {}
        self.local = set()
        self.started = []   # exchanged classes, in start order
        self.last = []      # exchanged classes, in the order of their latest start (complete last = last)
        self.keep = {}      # class -> the source tensors of its exchange in flight
        self.s = self.s_dst = self.A = None  # the consuming layer's node scores (enable_scores)

    def enable_scores(self, A: torch.Tensor):
        """The rows' node scores under the consuming multi-head layer's A [2, H, K] travel with
        them: the owner computes s_src / s_dst of its own rows (score_rows, as each producing
        phase finishes) and start() sends s_src beside the rows (H floats per row), so the
        consuming layer runs no score pass over its 11M table rows (hip_ops.xgat_forward
        ``scores``; the same kernel on the same rows: the same values)."""
        H = A.size(1)
        self.A = A
        self.s = torch.empty((self.hg.R, H), dtype=torch.float32, device=self.x.device)
        self.s_dst = torch.empty((max(self.hg.n_own, 1), H), dtype=torch.float32, device=self.x.device)

    def score_rows(self, out: torch.Tensor, d0: int, d1: int):
        """Scores of the own rows [d0, d1) of ``out`` (the producing layer's output)."""
        from .hip_ops import xgat_scores_rows
        xgat_scores_rows(out[d0:d1], self.A, self.s[d0:d1], self.s_dst[d0:d1])

    def span(self, cls):
        hg = self.hg
        return (hg.n_own, hg.n_own + hg.n_halo_u) if cls == "u" else (hg.n_own + hg.n_halo_u, hg.R)

    def plan(self, cls) -> ExchangePlan:
        return self.hg.plan_u if cls == "u" else self.hg.plan_i

    def set_local(self, cls, rows: torch.Tensor):
        a, b = self.span(cls)
        if b > a and rows.data_ptr() != self.x[a:b].data_ptr():  # (computed in place: nothing to copy)
            self.x[a:b].copy_(rows)
        self.local.add(cls)

    def start(self, cls, src: torch.Tensor, part: Optional[int] = None):
        """Send the own rows of ``src`` (own-local row order) of class ``cls`` to the peers;
        ``part`` (0 / 1): only that half of the class (run_plan), the other half sent by a later
        call -- wait(cls) then waits for both (one stream: the last event covers the first)."""
        plan, (a, b) = self.plan(cls), self.span(cls)
        if cls not in self.started:
            self.started.append(cls)
        if cls in self.last:
            self.last.remove(cls)
        self.last.append(cls)
        comm, st = self.comm, self.stages
        n0 = self.hg.n_own
        kw = {} if part is None else {"part": part}

        def send():  # straight from the own rows into the table's halo slice (no pack, no unpack)
            comm.exchange(plan, src, self.x[a:b], **kw)
            if self.s is not None:
                comm.exchange(plan, self.s[:n0], self.s[a:b], **kw)
        self._launch(cls, send, src)

    def start_touched(self, cls, src: torch.Tensor, tp: "TouchPlan"):
        """start() for a table whose halo rows are zero except the rows ``tp`` lists (the loss's
        gradient: nonzero only on the rows the triples touch, _touch_plans): only those rows
        travel -- gathered at the owner, one all_to_all, scattered into their places in the
        halo slice; every other halo row keeps the zero the table holds (the caller's part)."""
        a, b = self.span(cls)
        if cls not in self.started:
            self.started.append(cls)
        comm, st = self.comm, self.stages

        def send():
            buf = st.gather_rows(src, tp.send_idx) if tp.n_send else src.new_empty((0, src.size(1)))
            got = comm.all_to_all_rows(buf, tp.send_counts, tp.recv_counts)
            if tp.n_recv:
                self.x[a:b].index_copy_(0, tp.recv_pos, got)
        self._launch(cls, send, src)

    def _launch(self, cls, send, src):
        """Run ``send`` on the communication stream (RCCL) after the current stream's work so
        far, recording the class's event; inline under gloo or an inactive communicator."""
        comm = self.comm
        if comm.backend != "nccl" or not comm.active:
            send()
            return
        dev = self.x.device
        main, cs = torch.cuda.current_stream(dev), _comm_stream(dev)
        cs.wait_stream(main)
        # no record_stream: the tables are this object's and ``src`` is held here until the
        # current stream has waited for the exchange (wait / wait_all), so every block the comm
        # stream reads or writes is released in stream order after that wait.  (record_stream
        # defers each freed block to an event query; with 11-GB tables and steps enqueued ahead
        # the caching allocator then ran short and synchronised the host on the comm stream.)
        with torch.cuda.stream(cs):
            send()
            ev = torch.cuda.Event()
            ev.record(cs)
        self.events[cls] = ev
        self.keep.setdefault(cls, []).append(src)

    def wait(self, cls):
        ev = self.events.pop(cls, None)
        if ev is not None:
            torch.cuda.current_stream(self.x.device).wait_event(ev)
        self.keep.pop(cls, None)

    def wait_all(self):
        for cls in list(self.events):
            self.wait(cls)


class _CatInto(torch.autograd.Function):
    """torch.cat([a, b]) written into ``holder[0]`` (a preallocated [len(a) + len(b), C] buffer:
    the own rows of a halo layer's input table) and returned as that buffer, so the layer finds
    its own rows in place (one copy of them, not two).  The buffer travels in a list, not as a
    tensor argument: an in-place write to a tensor input (mark_dirty) would hang the whole 11-GB
    table on the autograd graph (CopySlices over its base; measured +7 ms per step at world 8)."""

    @staticmethod
    def forward(ctx, holder, a, b):
        dest = holder[0]
        na = a.size(0)
        for part, src in ((dest[:na], a), (dest[na:], b)):
            if src.numel() and part.data_ptr() != src.data_ptr():  # (a block already in place: no copy)
                part.copy_(src)
        ctx.na = na
        return dest

    @staticmethod
    def backward(ctx, g):
        return None, g[:ctx.na], g[ctx.na:]


def _halo_phases(hg: "HaloGraph", rows_in: HaloRows, rows_out: Optional[HaloRows]):
    """The phases of a halo layer's forward (hip_ops.XPhase).  On a bipartite graph the user
    destinations read item sources only and the item destinations user sources only, so each
    phase waits for one halo class: the phase whose class is local or arrives first runs first,
    and right after it the rows it produced start towards the next layer's peers (its output
    rows of that destination class).  Otherwise one phase after both classes."""
    from .hip_ops import XPhase

    def send(cls, d0=0, d1=0, part=None):
        if rows_out is None:
            return lambda out: None

        def go(out):
            if rows_out.s is not None:  # the next layer's scores of the rows this phase produced
                rows_out.score_rows(out, d0, d1)
            rows_out.start(cls, out, part)
        return go
    if not (hg.bipartite and hg.fwd_sched_u is not None and hg.fwd_sched_i is not None):
        def after_all(out):
            if rows_out is not None:
                if rows_out.s is not None:
                    rows_out.score_rows(out, 0, hg.n_own)
                rows_out.start("u", out)
                rows_out.start("i", out)
        return [XPhase(0, hg.n_own, hg.fwd_view.fwd_sched, (rows_in.span("u"), rows_in.span("i")), rows_in.wait_all,
                       after_all)]
    # destination class -> (rows, schedule, the source class it reads)
    ph = {"u": (0, hg.n_own_u, hg.fwd_sched_u, "i"), "i": (hg.n_own_u, hg.n_own, hg.fwd_sched_i, "u")}
    # the class whose rows complete first (its latest start earliest) first
    order = sorted(ph, key=lambda d: (ph[d][3] not in rows_in.local,
                                      rows_in.last.index(ph[d][3]) if ph[d][3] in rows_in.last else 0))
    halves = getattr(hg, "fwd_sched_halves", None) if rows_out is not None else None
    if not halves:
        return [XPhase(ph[d][0], ph[d][1], ph[d][2], (rows_in.span(ph[d][3]),),
                       (lambda c: (lambda: rows_in.wait(c)))(ph[d][3]), send(d, ph[d][0], ph[d][1])) for d in order]
    # each destination class in two halves (the plans' parts): the first half's output rows start
    # towards the peers while the second half is computed, so the next layer's rows arrive half a
    # phase earlier.  Per destination the same kernels and order as one phase: the same results.
    # Link order (PPGAT_HALO_DEFER=1, the default): the first class's second half leaves after the
    # second class's two halves, so the class the next layer's second phase needs is the one
    # still on the wire while its first phase runs -- with the exchange at 640 GB/s the forward
    # is link-bound and ends with the next layer's second phase.
    out = []
    defer = os.environ.get("PPGAT_HALO_DEFER", "1") == "1" and len(order) == 2
    held = []
    for k, d in enumerate(order):
        d0, d1, _, need = ph[d]
        dm = d0 + (d1 - d0) // 2
        (s0, s1) = halves[d]
        out.append(XPhase(d0, dm, s0, (rows_in.span(need),), (lambda c: (lambda: rows_in.wait(c)))(need),
                          send(d, d0, dm, 0)))
        if defer and k == 0:
            go = send(d, dm, d1, 1)
            held.append(go)
            out.append(XPhase(dm, d1, s1, (), None, (lambda o: None)))
        elif defer:
            last = send(d, dm, d1, 1)
            out.append(XPhase(dm, d1, s1, (), None, (lambda o, a=last, b=held: (a(o), [f(o) for f in b]))))
        else:
            out.append(XPhase(dm, d1, s1, (), None, send(d, dm, d1, 1)))
    return out


class _HaloLayerX(torch.autograd.Function):
    """One multi-head layer on the halo partition, aggregate-then-transform (hip_ops.xgat_*):
    forward = the layer over [own | halo] sources, its halo rows of x received by all_to_all
    (users, then items -- or, first layer, the halo items' rows computed locally:
    ``x_halo_items``), in phases by destination class that each wait only for the halo class
    they read (``HaloRows``, ``_halo_phases``); with ``rows_out`` the layer starts sending its
    own output rows to the next layer's peers as each phase finishes, so that exchange runs
    beside this layer's remaining work.  Backward = the halo sources' edge pass first, their
    input gradients sent back to the owners on a communication stream (RCCL all_to_all) while
    the own sources' edge pass and the weight-gradient GEMMs run, then the owners add the
    returned rows in peer order."""

    @staticmethod
    def forward(ctx, x_own, x_halo_items, weight, att_src, att_dst, bias, hg: "HaloGraph", comm: "Comm", stages,
                heads: int, C: int, slope: float, p: float, seed: int, rows_in: Optional[HaloRows] = None,
                rows_out: Optional[HaloRows] = None, link_in: Optional[dict] = None,
                link_out: Optional[dict] = None, out_buf: Optional[list] = None):
        from .hip_ops import xgat_forward
        x_own = x_own.contiguous()
        if rows_in is None:
            rows_in = HaloRows(hg, comm, stages, x_own.size(1), x_own)
            if x_halo_items is not None:
                rows_in.set_local("i", x_halo_items)
            for cls in ("u", "i"):
                if cls not in rows_in.local:
                    rows_in.start(cls, x_own)
        elif x_halo_items is not None:
            rows_in.set_local("i", x_halo_items)
        x_loc = rows_in.x
        if x_loc.data_ptr() != x_own.data_ptr():
            x_loc[:hg.n_own].copy_(x_own)
        if rows_in.s is not None and x_halo_items is not None:
            # the first layer: the own users' scores went out with their rows; the own items'
            # and the locally computed halo items' are computed here
            from .hip_ops import xgat_scores_rows
            nu, n0 = hg.n_own_u, hg.n_own
            xgat_scores_rows(x_loc[nu:n0], rows_in.A, rows_in.s[nu:n0], rows_in.s_dst[nu:n0])
            a, b = rows_in.span("i")
            xgat_scores_rows(x_halo_items, rows_in.A, rows_in.s[a:b])
        # the output rows go straight into the next layer's table (its own rows)
        dest = rows_out.x[:hg.n_own] if rows_out is not None and rows_out.x.size(1) == C else None
        if dest is None and out_buf is not None:  # the top layer: rows reserved after its own (the loss's)
            dest = out_buf[0][:hg.n_own]
        scores = (rows_in.s, rows_in.s_dst) if rows_in.s is not None else None
        out, ctx.saved = xgat_forward(x_loc, weight, att_src, att_dst, bias, hg.xviews(), heads, C, slope, p, seed,
                                      phases=_halo_phases(hg, rows_in, rows_out), out=dest, scores=scores,
                                      keep_agg=True)  # the halo backward's weight gradient reads agg
        rows_in.wait_all()
        if (source_homed_backward(hg) and os.environ.get("PPGAT_XGAT_GATHER") != "g"
                and any(ctx.needs_input_grad[:6])):
            _ntab_forward(ctx.saved, hg, comm, stages, x_own.device)
        # links between consecutive halo layers (_halo_xgat_backward_deferred_d): this layer's
        # state for the layer above, whose backward starts this layer's exchanges early
        if link_out is not None:
            link_out["saved"] = ctx.saved
        ctx.link_in, ctx.link_out = link_in, link_out
        ctx.hg, ctx.comm, ctx.stages = hg, comm, stages
        ctx.plans = [rows_in.plan(c) for c in ("u", "i") if c not in rows_in.local]
        ctx.att_shapes = (att_src.shape, att_dst.shape)
        ctx.local_items = "i" in rows_in.local
        return out

    @staticmethod
    def backward(ctx, g):
        from .hip_ops import xgat_backward
        hg, comm, st, plans = ctx.hg, ctx.comm, ctx.stages, ctx.plans
        dev = g.device
        if source_homed_backward(hg):
            pre = ctx.link_out.pop("pre", None) if ctx.link_out is not None else None
            dx, dW, datt_src, datt_dst, dbias = _halo_xgat_backward(ctx.saved, g, hg, comm, st,
                                                                    ctx.needs_input_grad[5], pre=pre,
                                                                    link_in=ctx.link_in)
            ctx.saved = None
            if ctx.link_out is not None:
                ctx.link_out.clear()
            # every input gradient of an own row is complete here (its out-edges live on this
            # rank); the halo rows' -- incl. the first layer's locally computed halo items -- are
            # their owners' business
            return (dx, None, dW, datt_src.view(ctx.att_shapes[0]), datt_dst.view(ctx.att_shapes[1]), dbias,
                    None, None, None, None, None, None, None, None, None, None, None, None, None)
        pending = {}

        def a2a_back(dx_halo):
            rets, off = [], 0
            for plan in plans:
                rets.append(_return(comm, plan, dx_halo[off:off + plan.n_recv]))
                off += plan.n_recv
            return rets

        def send_back(dx_halo):
            if comm.backend != "nccl" or not comm.active:
                pending["ret"] = a2a_back(dx_halo)
                return
            main, cs = torch.cuda.current_stream(dev), _comm_stream(dev)
            cs.wait_stream(main)
            dx_halo.record_stream(cs)
            with torch.cuda.stream(cs):
                pending["ret"] = a2a_back(dx_halo)
            pending["stream"] = cs

        dx, dW, datt_src, datt_dst, dbias = xgat_backward(ctx.saved, g, ctx.needs_input_grad[5], halo_hook=send_back)
        ctx.saved = None
        dx_own = dx[:hg.n_own]
        if "stream" in pending:
            main = torch.cuda.current_stream(dev)
            main.wait_stream(pending["stream"])
            for r in pending["ret"]:
                r.record_stream(main)
        for plan, ret in zip(plans, pending["ret"]):
            st.return_add(dx_own, ret, plan.ret_ptr, plan.ret_pos)
        d_items = dx[hg.n_own + hg.n_halo_u:] if ctx.local_items else None
        return (dx_own, d_items, dW, datt_src.view(ctx.att_shapes[0]), datt_dst.view(ctx.att_shapes[1]), dbias,
                None, None, None, None, None, None, None, None, None, None, None, None, None)


def source_homed_backward(hg: "HaloGraph") -> bool:
    """The multi-head halo layer's backward runs at the source rows' owners (_halo_xgat_backward)
    on a symmetric edge list unless PPGAT_HALO_BWD=dst (the round-3 backward: edges at their
    destination's owner, halo sources' input gradients returned)."""
    return hg.src_views is not None and os.environ.get("PPGAT_HALO_BWD", "src") != "dst"


def _halo_xgat_backward(saved: dict, g: torch.Tensor, hg: "HaloGraph", comm: "Comm", stages,
                        want_bias_grad: bool, pre=None, link_in: Optional[dict] = None):
    """Backward of the multi-head halo layer with every edge processed at its SOURCE's owner.

    The forward ran each edge at its destination's owner (the aggregation needs a destination's
    whole in-edge list).  The backward's edge pass is by source (pass B), and on the round-3 path
    it also ran at the destination's owner: every rank then computed hs = x W^T / H and
    dx = acc W / H for all of its local rows -- own AND halo, 11M rows against 1.9M own at 8 ranks
    on config 5 -- and returned the halo rows' dx.  On a symmetric edge list the destinations of
    an own row's out-edges are exactly the rows the rank already holds as [own | halo], so here:
      1. the own rows' destination state: gt = g W_g, nstate {s_dst, m, inv_l, D = gt . agg}
         (the g-gathering formulation; D needs agg, which only the destination's owner has);
      2. g and nstate of the halo rows arrive by the forward's plans (the same rows; g starts
         at once, beside the gt GEMM, the prologue and the hs GEMM; nstate after the prologue);
      3. hs = x W^T / H over the OWN rows only; the edge pass over the own sources' out-edges in
         two phases by source class (item sources read user rows and vice versa), each waiting
         only for its class of halo rows: dz per edge, ds_src and acc per own source;
      4. ds_dst: per destination row of the table, this rank's partial sum; the halo rows'
         partials go back to their owners (H floats per row), added after the own partial in
         peer order (ppgat_rows_return_add: deterministic);
      5. dx = acc W / H + ds_src A_src + ds_dst A_dst over the own rows (rank terms in the
         GEMM's epilogue) -- the complete input gradient, nothing returned;
      6. dW from G = g^T agg (own destinations) and GV = S^T x (own rows), datt, dbias.
    Exchanges per layer: g + nstate of the halo rows (the forward's x volume) and the partial
    ds_dst return, instead of the halo rows' dx; per-rank GEMMs over own rows only.
    This is the PPGAT_XGAT_GATHER=g variant; by default D is deferred instead
    (_halo_xgat_backward_deferred_d: no gt GEMM, D's partials go home and back out)."""
    from . import hip_ops as O
    lib = _lib.load()
    x, W, A = saved["x"], saved["W"], saved["A"]
    s_src, s_dst, agg, m, inv_l = saved["s_src"], saved["s_dst"], saved["agg"], saved["m"], saved["inv_l"]
    H, C, K, slope, p, seed, has_bias = saved["meta"]
    dev = x.device
    st = _lib.stream_handle(dev)
    n0, R, sv = hg.n_own, hg.R, hg.src_views
    E = sv.n_edges
    g = g.contiguous()
    if os.environ.get("PPGAT_XGAT_GATHER") != "g":
        return _halo_xgat_backward_deferred_d(saved, g, hg, comm, stages, want_bias_grad, pre, link_in)
    gtab = HaloRows(hg, comm, stages, C, g)
    gtab.x[:n0].copy_(g)
    for cls in ("u", "i"):
        gtab.start(cls, g)
    # 1. destination state of the own rows
    Wg = torch.empty(C, H * K, dtype=torch.float32, device=dev)
    _lib.check(lib.ppgat_xgat_weights(W.data_ptr(), None, None, H, C, K, None, None, Wg.data_ptr(), st),
               "xgat_weights")
    gt = O.gemm_nn(g, Wg, 0, H * K)
    nst = torch.empty(max(n0, 1), 4 * H, dtype=torch.float32, device=dev)
    _lib.check(lib.ppgat_xgat_bwd_prologue(gt.data_ptr(), agg.data_ptr(), s_dst.data_ptr(), m.data_ptr(),
                                           inv_l.data_ptr(), n0, K, H, nst.data_ptr(), st), "xgat_bwd_prologue")
    del gt, Wg
    nst = nst[:n0]
    ntab = HaloRows(hg, comm, stages, 4 * H, nst)
    ntab.x[:n0].copy_(nst)
    for cls in ("u", "i"):
        ntab.start(cls, nst)
    # 3. own sources
    hs = O.gemm_nn(x[:n0], W, 1, H * C, alpha=1.0 / H)
    acc = torch.empty(n0, H * C, dtype=torch.float32, device=dev)
    S = torch.zeros(max(n0, 1), 2 * H, dtype=torch.float32, device=dev)
    dz = torch.empty(max(E, 1) * H, dtype=torch.float32, device=dev)
    phases = ([("i", hg.src_sched_i, hg.n_own_u, "u"), ("u", hg.src_sched_u, 0, "i")] if hg.bipartite else
              [("all", sv.bwd_sched, 0, None)])
    for _, sched, base, need in phases:
        for tab in (gtab, ntab):
            tab.wait_all() if need is None else tab.wait(need)
        O._xgat_edges_bwd_g(lib, sched, sv, base, hs, s_src, ntab.x, gtab.x, acc, S, dz, H, C, slope, p, seed,
                            saved["seed_buf"], st)
    gtab.wait_all()
    ntab.wait_all()
    del hs
    # 4. ds_dst: partial sums over the table rows, the halo rows' back to their owners
    dsd = torch.zeros(max(R, 1), H, dtype=torch.float32, device=dev)
    O._xgat_dst_sum(lib, sv, dz, dsd, H, E, st, col0=0, ld=H)
    del dz
    S = S[:n0]
    S[:, H:].copy_(_partials_home(hg, comm, stages, dsd))
    # 5. the complete input gradient of the own rows
    dx = O.gemm_nn(acc, W, 0, K, alpha=1.0 / H, rank=(S, A.view(2 * H, K))) if n0 else \
        torch.zeros(0, K, dtype=torch.float32, device=dev)
    del acc
    # 6. weight gradients (the sums over ranks: the dense all-reduce)
    return O._xgat_weight_grads(lib, saved, g, S, dx, want_bias_grad, st, x_rows=x[:n0],
                                xbits=_source_colmax_bits(x[:n0], hg, comm, saved))


def _source_colmax_bits(x_own: torch.Tensor, hg: "HaloGraph", comm: "Comm", saved=None) -> torch.Tensor:
    """The column bound of the weight-gradient GEMM's aggregate operand (hip_ops._xgat_weight_grads):
    |agg_i[k]| <= max |x_j[k]| over i's sources j.  The exact set -- every table row with an edge
    into an own destination -- is 11M rows (11 GB) per rank at world 8 on config 5; instead each
    rank takes its OWN rows with an out-edge (src_views.colptr: on the symmetric edge list the
    table rows' out-edges are their owners' own out-edges) and the ranks' maxima are combined by
    an all_reduce(MAX) of K int32 (IEEE bits of non-negative floats order as the floats): the
    maximum over every row with an out-edge anywhere, a superset of the sources, never a
    row without one.  At world 1 it is the exact set.  With the forward's own maxima (``saved``
    xbits: gathered by its edge pass over this rank's destinations, halo sources included) the
    all_reduce(MAX) of those is exactly the maximum over every source, and x is not read again."""
    from . import hip_ops as O
    xb = saved.get("xbits") if saved is not None else None
    bits = xb.clone() if xb is not None else O.colmax_abs(x_own, hg.src_views.colptr)
    return comm.all_reduce_(bits, op=dist.ReduceOp.MAX)


def _small_class_first(hg: "HaloGraph") -> tuple:
    """The halo classes in exchange order: the one with fewer nodes in the whole graph first
    (every rank computes the same order -- the all_to_alls must match -- and on a bipartite
    graph a class's halo rows scale with its node count)."""
    n_items = hg.n_nodes - hg.n_users
    return ("i", "u") if n_items <= hg.n_users else ("u", "i")


def _partials_home(hg: "HaloGraph", comm: "Comm", stages, part: torch.Tensor) -> torch.Tensor:
    """part [R, w]: this rank's partial sums per table row -> the own rows' complete sums (the
    halo rows' partials returned to their owners by the reverse plans, each own row adding its
    copies after its own partial, in peer order: deterministic)."""
    own = part[:hg.n_own]
    off = hg.n_own
    for plan in (hg.plan_u, hg.plan_i):
        stages.return_add(own, _return(comm, plan, part[off:off + plan.n_recv]), plan.ret_ptr, plan.ret_pos)
        off += plan.n_recv
    return own


def _bwd_tables(saved: dict, hg: "HaloGraph", comm: "Comm", stages, g_width: int, dev,
                g_table: Optional[torch.Tensor] = None):
    """The backward's row tables of one multi-head halo layer: g [R, C] (own rows to be filled;
    ``g_table``: a caller's buffer) and the softmax state nstate {s_dst, m, inv_l, .} [R, 4H]
    (own rows filled here)."""
    n0 = hg.n_own
    ntab = saved.pop("ntab", None)  # started at the end of the forward (_ntab_forward)
    if ntab is None:
        ntab = _ntab_make(saved, hg, comm, stages, dev)
    nst = ntab.x[:n0]
    gtab = HaloRows(hg, comm, stages, g_width, nst, x=g_table)
    return gtab, ntab, nst


def _ntab_make(saved: dict, hg: "HaloGraph", comm: "Comm", stages, dev) -> "HaloRows":
    """The softmax-state table {s_dst, m, inv_l, .} [R, 4H] of a multi-head halo layer, the own
    rows filled (straight into the table, no copy)."""
    lib = _lib.load()
    s_dst, m, inv_l = saved["s_dst"], saved["m"], saved["inv_l"]
    H = saved["meta"][0]
    ntab = HaloRows(hg, comm, stages, 4 * H, s_dst)
    _lib.check(lib.ppgat_xgat_nstate(s_dst.data_ptr(), m.data_ptr(), inv_l.data_ptr(), None, hg.n_own, H,
                                     ntab.x.data_ptr(), _lib.stream_handle(dev)), "xgat_nstate")
    return ntab


def _ntab_forward(saved: dict, hg: "HaloGraph", comm: "Comm", stages, dev):
    """The backward's softmax state depends on the forward only: build the table and start its
    exchange as the forward ends (the communication stream is idle then, after the next layer's
    rows), so the backward waits only for g (saved["ntab"], taken by _bwd_tables)."""
    ntab = _ntab_make(saved, hg, comm, stages, dev)
    for cls in _small_class_first(hg):
        ntab.start(cls, ntab.x[:hg.n_own])
    saved["ntab"] = ntab


def _bwd_start(hg: "HaloGraph", gtab: "HaloRows", ntab: "HaloRows", nst, g):
    """Both tables of the smaller halo class first (the same order on every rank: it is decided
    from the global segment sizes), so the phase that reads it starts while the other class is
    still on the wire."""
    for cls in _small_class_first(hg):
        if cls not in ntab.started:  # (not already started by the forward)
            ntab.start(cls, nst)
        gtab.start(cls, g)


def _halo_xgat_backward_deferred_d(saved: dict, g, hg: "HaloGraph", comm: "Comm", stages, want_bias_grad: bool,
                                   pre=None, link_in: Optional[dict] = None):
    """_halo_xgat_backward with D deferred (the single-GPU default): no gt GEMM
    and no prologue.  nstate {s_dst, m, inv_l, .} of the own rows goes out with g at once; the
    edge pass writes dalpha and beta dalpha per edge; D_i = sum_j beta dalpha is summed per table
    row, the halo rows' partials go home and the completed D of the own rows back out (H floats
    per row each way); then the dz pass, ds_dst (partials home again) and the own rows' GEMMs.

    ``pre``: the tables with their exchanges already started by the layer above (its backward
    wrote this layer's g into the table and started it before its own weight-gradient GEMMs);
    ``link_in``: the link to the layer below -- when it is a halo layer too, this layer's input
    gradient is written straight into the layer below's g table and its exchanges start before
    this layer's weight gradients, so they run beside them."""
    from . import hip_ops as O
    lib = _lib.load()
    x, W, A, s_src = saved["x"], saved["W"], saved["A"], saved["s_src"]
    H, C, K, slope, p, seed, has_bias = saved["meta"]
    dev = x.device
    st = _lib.stream_handle(dev)
    n0, R, sv = hg.n_own, hg.R, hg.src_views
    E = sv.n_edges
    seed_buf = saved["seed_buf"]
    order = _small_class_first(hg)
    handed = getattr(hg, "grad_handoff", {}).pop("g", None)
    if pre is None and handed is not None and handed() is g and g.is_contiguous() and n0 and \
            g.data_ptr() == g.untyped_storage().data_ptr() and g.untyped_storage().nbytes() >= R * C * 4:
        # g is the top of an [R, C] buffer (the loss backward's dZ, halo_bpr_loss grad_rows): it is
        # the g table, its own rows already in place (its rows past n0 held the loss's received
        # rows' gradients, already returned to their owners in stream order before this point)
        gtab, ntab, nst = _bwd_tables(saved, hg, comm, stages, C, dev,
                                      g_table=g.new_empty(0).set_(g.untyped_storage(), 0, (R, C), (C, 1)))
        touch = getattr(hg, "top_touch", None)
        if touch is not None and touch["buf"] is not None and touch["buf"].data_ptr() == g.data_ptr():
            # the persistent table of halo_bpr_loss: only the touched rows travel; the rows the
            # loss's own exchange received (now returned to their owners) go back to zero first
            tail = int(getattr(hg, "loss_tail_rows", 0))
            if tail:
                gtab.x[n0:n0 + tail].zero_()
            for cls in order:
                if cls not in ntab.started:
                    ntab.start(cls, nst)
                gtab.start_touched(cls, g, touch[cls])
        else:
            _bwd_start(hg, gtab, ntab, nst, g)
    elif pre is not None:
        # started by the layer above from its dx, which is g when nothing sits between the two
        # layers (HaloPyGGAT links a layer only to the one consumer of its output).  If autograd
        # hands over another tensor (a hook, a residual, an activation in between), the halo rows
        # already sent carry the old values: wait for those exchanges and redo them from the real
        # g.  The branch is structural, so every rank takes it alike and the collectives match.
        gtab, ntab, nst = pre
        if gtab.x.data_ptr() != g.data_ptr():
            gtab.wait_all()
            gtab.x[:n0].copy_(g)
            for cls in order:
                gtab.start(cls, g)
    else:
        gtab, ntab, nst = _bwd_tables(saved, hg, comm, stages, C, dev)
        gtab.x[:n0].copy_(g)
        _bwd_start(hg, gtab, ntab, nst, g)
    hs = torch.empty(max(n0, 1), H * C, dtype=torch.float32, device=dev)
    acc = torch.empty(max(n0, 1), H * C, dtype=torch.float32, device=dev)
    dz = torch.empty(max(E, 1) * H, dtype=torch.float32, device=dev)
    pdal = torch.empty(max(E, 1) * H, dtype=torch.float32, device=dev)
    gbits = torch.zeros(C, dtype=torch.int32, device=dev)  # |g| over the gathered table rows (A bound of G)
    nu = hg.n_own_u
    by_need = {"i": (hg.src_sched_u, 0, "i"), "u": (hg.src_sched_i, nu, "u")}  # user sources read items
    phases = [by_need[c] for c in order] if hg.bipartite else [(sv.bwd_sched, 0, None)]
    for sched, base, need in phases:  # dalpha (into dz) and beta dalpha per edge, acc per own source
        # hs = x W^T / H of this phase's sources, while its class of halo rows is on the wire
        # (on the large-M fp16 kernel each row's result depends on that row alone)
        r0, r1 = ((0, nu) if base == 0 else (nu, n0)) if need is not None else (0, n0)
        if r1 > r0:
            O.gemm_nn(x[r0:r1], W, 1, H * C, alpha=1.0 / H, out=hs[r0:r1])
        for tab in (gtab, ntab):
            tab.wait_all() if need is None else tab.wait(need)
        nbytes = ctypes.c_size_t(0)
        _lib.check(lib.ppgat_xgat_bwd_g_workspace_bytes(sched.n_hub_items, C, H, ctypes.byref(nbytes)), "xgat_g_ws")
        ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=dev)
        cs = sched.cstruct()
        _lib.check(lib.ppgat_xgat_bwd_edges_gd_colmax(ctypes.byref(cs), _lib.ptr(sv.row) if E else None,
                                                      _lib.ptr(sv.csc_eid) if E else None, None, E, C, H,
                                                      hs.data_ptr() + 4 * base * H * C,
                                                      s_src.data_ptr() + 4 * base * H, ntab.x.data_ptr(),
                                                      gtab.x.data_ptr(), C, float(slope), float(p),
                                                      int(seed) & (2**64 - 1), _lib.ptr(seed_buf),
                                                      acc.data_ptr() + 4 * base * H * C, dz.data_ptr(),
                                                      pdal.data_ptr(), gbits.data_ptr(), ws.data_ptr(), nbytes.value,
                                                      st), "xgat_bwd_edges_gd_colmax")
    gtab.wait_all()
    ntab.wait_all()
    del hs
    # D: per table row partial sums of beta dalpha, completed at the owner, sent back out
    Dp = torch.zeros(max(R, 1), H, dtype=torch.float32, device=dev)
    O._xgat_dst_sum(lib, sv, pdal, Dp, H, E, st, col0=0, ld=H)
    del pdal
    Dtab = HaloRows(hg, comm, stages, H, Dp)
    Dtab.x[:n0].copy_(_partials_home(hg, comm, stages, Dp))
    del Dp
    for cls in ("u", "i"):
        Dtab.start(cls, Dtab.x[:n0])
    Dtab.wait_all()
    Dx = Dtab.x.contiguous()  # nstate {s_dst, m, inv_l, D} of every table row
    _lib.check(lib.ppgat_xgat_nstate_set_d(ntab.x.data_ptr(), Dx.data_ptr(), R, H, st), "xgat_nstate_set_d")
    del Dtab
    # dz in place over dalpha, ds_src per own source
    S = torch.zeros(max(n0, 1), 2 * H, dtype=torch.float32, device=dev)
    for sched, base, _ in phases:
        nbytes = ctypes.c_size_t(0)
        _lib.check(lib.ppgat_xgat_bwd_dz_workspace_bytes(sched.n_hub_items, H, ctypes.byref(nbytes)), "xgat_dz_ws")
        ws = torch.empty(max(int(nbytes.value), 4), dtype=torch.uint8, device=dev)
        cs = sched.cstruct()
        _lib.check(lib.ppgat_xgat_bwd_dz(ctypes.byref(cs), _lib.ptr(sv.row) if E else None,
                                         _lib.ptr(sv.csc_eid) if E else None, None, E, H,
                                         s_src.data_ptr() + 4 * base * H, ntab.x.data_ptr(), float(slope), float(p),
                                         int(seed) & (2**64 - 1), _lib.ptr(seed_buf), dz.data_ptr(),
                                         S.data_ptr() + 4 * base * 2 * H, 2 * H, ws.data_ptr(), nbytes.value, st),
                   "xgat_bwd_dz")
    # ds_dst: partials per table row, completed at the owner
    dsd = torch.zeros(max(R, 1), H, dtype=torch.float32, device=dev)
    O._xgat_dst_sum(lib, sv, dz, dsd, H, E, st, col0=0, ld=H)
    del dz
    S = S[:n0]
    S[:, H:].copy_(_partials_home(hg, comm, stages, dsd))
    del dsd
    # the weight-gradient bound's all_reduce now, before any exchange of the layer below is
    # started on the communication stream: no two collectives of one communicator in flight on
    # two streams (the comm stream's start waits for this stream's work so far)
    # (one all_reduce(MAX) for both bounds: the union over the ranks of the rows each edge pass
    # gathered is every source / every destination with an edge -- a rank's own g rows may have
    # their in-edges homed elsewhere, so its local g maxima alone would not cover them)
    xb = saved.get("xbits")
    if xb is not None:
        both = comm.all_reduce_(torch.cat([xb, gbits]), op=dist.ReduceOp.MAX)
        xbits, gbits = both[:K], both[K:]
    else:
        xbits = _source_colmax_bits(x[:n0], hg, comm, saved)
        gbits = comm.all_reduce_(gbits, op=dist.ReduceOp.MAX)
    below = link_in.get("saved") if link_in is not None else None
    if below is not None and n0:
        # the layer below's g = this dx: straight into its table, its exchanges started now
        gtab1, ntab1, nst1 = _bwd_tables(below, hg, comm, stages, K, dev)
        dx = gtab1.x[:n0]
        A2 = A.view(2 * H, K)
        if getattr(hg, "fwd_sched_halves", None) and hg.bipartite:
            # the GEMM by class in exchange order, the larger class in the plans' two halves, each
            # piece's rows sent as soon as they exist (per row the same kernel: the same bits)
            nu = hg.n_own_u
            span = {"u": (0, nu), "i": (nu, n0)}
            for k, cls in enumerate(_small_class_first(hg)):
                c0, c1 = span[cls]
                cuts = [(c0, c1, None)] if k == 0 else [(c0, c0 + (c1 - c0) // 2, 0), (c0 + (c1 - c0) // 2, c1, 1)]
                if cls not in ntab1.started:
                    ntab1.start(cls, nst1)
                for p0, p1, part in cuts:
                    if p1 > p0:
                        O.gemm_nn(acc[p0:p1], W, 0, K, alpha=1.0 / H, rank=(S[p0:p1], A2), out=dx[p0:p1])
                    gtab1.start(cls, dx, part)
        else:
            O.gemm_nn(acc[:n0], W, 0, K, alpha=1.0 / H, rank=(S, A2), out=dx)
            _bwd_start(hg, gtab1, ntab1, nst1, dx)
        link_in["pre"] = (gtab1, ntab1, nst1)
    else:
        dx = O.gemm_nn(acc[:n0], W, 0, K, alpha=1.0 / H, rank=(S, A.view(2 * H, K))) if n0 else \
            torch.zeros(0, K, dtype=torch.float32, device=dev)
    del acc
    return O._xgat_weight_grads(lib, saved, g, S, dx, want_bias_grad, st, x_rows=x[:n0], xbits=xbits, gbits=gbits)


class _ShardedBase(torch.nn.Module):
    """Shared parts of the sharded PyGGAT variants (train_gat_pyg.py:68-88): built from a
    full model constructed identically on every rank, so the sharded and single-GPU runs
    start from the same parameters; ``full_state_dict`` reassembles the reference keys."""

    def __init__(self, full, dg, comm: "Comm", stages=None):
        super().__init__()
        from .hip_ops import HipStages
        self.dg, self.comm = dg, comm
        self.stages = stages if stages is not None else HipStages()
        self.n_users, self.n_items = full.n_users, full.n_items
        self.u0, self.u1 = dg.owned_users(self.n_users)
        # the own users' rows in the graph's own-local order (the halo partition sorts them by
        # peer set; the replicated one keeps id order)
        ids = torch.from_numpy(np.asarray(dg.own_user_ids(), np.int64)).to(full.user_emb.weight.device)
        self.user_emb_local = torch.nn.Parameter(full.user_emb.weight.detach().index_select(0, ids).clone())
        self.item_proj = full.item_proj
        self.convs = full.convs
        self.seeds = SharedSeeds(comm)

    def layer_seed(self, conv) -> int:
        return self.seeds.next() if (self.training and float(conv.dropout) > 0) else 0

    def dense_parameters(self):
        return [p for n, p in self.named_parameters() if n != "user_emb_local"]

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

    def _user_rows_global(self, rows: torch.Tensor, pad: int) -> torch.Tensor:
        """Own user rows of a [*, C] tensor (own-local order) -> every rank's, in user-id order
        (all_gather)."""
        C = rows.size(1)
        blk = rows.new_zeros(pad, C)
        blk[:rows.size(0)] = rows
        allb = self.comm.all_gather_rows(blk)
        idx = np.empty(self.n_users, np.int64)
        for r in range(self.comm.world):
            ids = np.asarray(self.dg.own_user_ids(r), np.int64)
            idx[ids] = r * pad + np.arange(len(ids))
        return allb.index_select(0, torch.from_numpy(idx).to(allb.device))

    def full_state_dict(self):
        """Reference-keyed state_dict (user_emb gathered from the owners)."""
        pad = max(int(b - a) for a, b in (self.dg.owned_users(self.n_users, r) for r in range(self.comm.world)))
        sd = {"user_emb.weight": self._user_rows_global(self.user_emb_local.detach(), max(pad, 1))}
        for k, v in self.state_dict().items():
            if k != "user_emb_local":
                sd[k] = v
        return sd


def _unalias_local(module, state_dict, prefix, local_metadata):
    """state_dict hook: user_emb_local may share the first-layer table's storage
    (HaloPyGGAT._first_table); hand out its own copy (torch.save would write the whole table)."""
    k = prefix + "user_emb_local"
    v = state_dict.get(k)
    if v is not None and v.untyped_storage().nbytes() > v.numel() * v.element_size():
        state_dict[k] = v.clone()


class HaloPyGGAT(_ShardedBase):
    """PyGGAT with row-sharded users and items and halo all_to_all exchange (module doc).
    ``forward`` returns the own rows [n_own, C]: own users, then own items."""

    def __init__(self, full, dg, comm: "Comm", stages=None):
        super().__init__(full, dg, comm, stages)
        self._register_state_dict_hook(_unalias_local)

    def _item_feats(self, item_feats, which: str) -> torch.Tensor:
        """The item feature rows of the own ("own") or halo ("halo") items, gathered once per
        feature tensor: the features are a constant input and the partition is static, so the
        gathers (0.6 + 2.9 GB at world 8 on config 5) leave the step, and the item projection's
        weight-gradient operand is the same tensor every step (its column bound is cached,
        hip_ops._const_colmax)."""
        key = (item_feats.data_ptr(), item_feats._version, tuple(item_feats.shape), str(item_feats.device))
        cache = getattr(self, "_feat_cache", None)
        if cache is None or cache[0] != key:
            cache = (key, {})
            self._feat_cache = cache
        hit = cache[1].get(which)
        if hit is None:
            idx = self.dg.own_items if which == "own" else self.dg.halo_items
            hit = self.stages.gather_rows(item_feats, idx)
            cache[1][which] = hit
        return hit

    def _first_table(self, width: int, like: torch.Tensor) -> torch.Tensor:
        """The first layer's input table [R, width], kept across steps, whose first rows ARE the
        user embedding's storage (re-pointed once, as model.node_table): the own users' rows need
        no copy into it, the item projections write their rows in place."""
        hg = self.dg
        t = getattr(self, "_tab0", None)
        if t is None or tuple(t.shape) != (hg.R, width) or t.device != like.device or t.dtype != like.dtype:
            t = torch.empty((hg.R, width), dtype=like.dtype, device=like.device)
            self._tab0 = t
        w = self.user_emb_local
        if w.size(0) and w.data_ptr() != t.data_ptr():
            t[:w.size(0)].copy_(w.detach())
            w.data = t[:w.size(0)]
        return t

    def _top_out(self, C: int, like: torch.Tensor):
        """The top layer's output rows, with room after them for the rows the loss receives
        (halo_bpr_loss sets hg.loss_tail_rows once its plan exists): the loss's exchange then
        receives straight behind the own rows instead of copying them (_Exchange)."""
        tail = int(getattr(self.dg, "loss_tail_rows", 0))
        if not tail:
            return None
        return [torch.empty((self.dg.n_own + tail, C), dtype=like.dtype, device=like.device)]

    def node_features(self, item_feats, into: Optional[torch.Tensor] = None):
        """[own users | own items] input rows; ``into``: write them there (the first halo layer's
        table) instead of a new tensor."""
        f = self._item_feats(item_feats, "own")
        if into is not None:
            nu = self.user_emb_local.size(0)
            x_items = self.stages.linear(f, self.item_proj.weight, self.item_proj.bias, out=into[nu:])
            return _CatInto.apply([into], self.user_emb_local, x_items)
        x_items = self.stages.linear(f, self.item_proj.weight, self.item_proj.bias)
        return torch.cat([self.user_emb_local, x_items], 0)

    @staticmethod
    def exchanges_input(conv) -> bool:
        """Exchange the pre-projection rows when they are narrower than h (H*C > C_in)."""
        return conv.heads * conv.out_channels > conv.in_channels

    def halo_item_input(self, item_feats, out: Optional[torch.Tensor] = None):
        """The first layer's input rows of the halo items, item_proj(features) computed on this
        rank (the item features are on every rank): they are neither received nor returned;
        their gradient reaches item_proj here and is summed by the dense all-reduce.  ``out``:
        write them there (the first halo layer's table) instead of a new tensor."""
        f = self._item_feats(item_feats, "halo")
        if out is not None:
            return self.stages.linear(f, self.item_proj.weight, self.item_proj.bias, out=out)
        return self.stages.linear(f, self.item_proj.weight, self.item_proj.bias)

    def _x_path(self, li: int) -> bool:
        conv = self.convs[li]
        return self.exchanges_input(conv) and getattr(self.stages, "supports_x", lambda c: False)(conv)

    def forward(self, item_feats):
        from .hip_ops import xgat_att_proj
        hg = self.dg
        rows = link_in = None
        if self._x_path(0):
            # the first layer's halo user rows are parameters: their exchange starts before
            # the item projections (the own and the halo items' rows) are computed
            rows = HaloRows(hg, self.comm, self.stages, self.user_emb_local.size(1), self.user_emb_local,
                            x=self._first_table(self.user_emb_local.size(1), self.user_emb_local))
            c0 = self.convs[0]
            rows.enable_scores(xgat_att_proj(c0.lin.weight, c0.att_src, c0.att_dst, c0.heads, c0.out_channels))
            rows.score_rows(self.user_emb_local.detach(), 0, hg.n_own_u)  # sent beside the user rows
            rows.start("u", self.user_emb_local.detach())
        # the own rows go straight into the first layer's table when it has one
        x = self.node_features(item_feats, into=rows.x[:hg.n_own] if rows is not None else None)
        for li, conv in enumerate(self.convs):
            p = float(conv.dropout) if self.training else 0.0
            seed = self.layer_seed(conv)
            xh = None
            if li == 0 and hg.plan_i.n_recv:
                # on the x path straight into the first layer's table (HaloRows.set_local: no copy)
                xh = self.halo_item_input(item_feats, out=rows.x[slice(*rows.span("i"))]
                                          if rows is not None and self._x_path(0) else None)
            if li == 0 and xh is None:
                xh = x.new_zeros(0, x.size(1))
            if self.exchanges_input(conv):
                if self._x_path(li):
                    # aggregate-then-transform on the local rows: no halo projection; the next
                    # layer's halo rows start moving as this layer's phases finish, and the
                    # return of the halo gradients overlaps the own rows' backward
                    nxt = link_out = out_buf = None
                    if li + 1 == len(self.convs):
                        out_buf = self._top_out(conv.out_channels, x)
                        # the loss's dZ in an [R, C] buffer: this layer's backward takes it as its g table
                        hg.loss_grad_rows = hg.R if source_homed_backward(hg) else 0
                    if li + 1 < len(self.convs) and self._x_path(li + 1):
                        nxt = HaloRows(hg, self.comm, self.stages, conv.out_channels, x)
                        cn = self.convs[li + 1]
                        nxt.enable_scores(xgat_att_proj(cn.lin.weight, cn.att_src, cn.att_dst, cn.heads,
                                                        cn.out_channels))
                        link_out = {}
                    x = _HaloLayerX.apply(x, xh, conv.lin.weight, conv.att_src, conv.att_dst, conv.bias, hg,
                                          self.comm, self.stages, conv.heads, conv.out_channels,
                                          float(conv.negative_slope), p, seed, rows, nxt, link_in, link_out,
                                          out_buf)
                    rows, link_in = nxt, link_out
                    continue
                h = self.stages.linear(halo_exchange(x, hg, self.comm, self.stages, xh), conv.lin.weight, None)
            else:
                hh = self.stages.linear(xh, conv.lin.weight, None) if xh is not None and xh.size(0) else xh
                h = halo_exchange(self.stages.linear(x, conv.lin.weight, None), hg, self.comm, self.stages, hh)
            x = _LocalGAT.apply(h, conv.att_src, conv.att_dst, conv.bias, hg, self.stages, conv.heads,
                                conv.out_channels, _lib.MODE_PYG, float(conv.negative_slope), p, seed)
        return x


@dataclass
class TouchPlan:
    """One halo class of the top layer's g exchange restricted to the rows the loss touches
    (_touch_plans): this rank's own rows ``send_idx`` (per peer in rank order, ``send_counts``),
    and the positions ``recv_pos`` in the class's halo slice of the rows each owner sends here
    (owners in rank order, ``recv_counts``)."""
    send_idx: torch.Tensor      # int64 [n_send] own-local rows
    send_counts: list
    recv_pos: torch.Tensor      # int64 [n_recv] rows of the class's halo slice
    recv_counts: list

    @property
    def n_send(self) -> int:
        return int(sum(self.send_counts))

    @property
    def n_recv(self) -> int:
        return int(sum(self.recv_counts))


def _touch_plans(hg: HaloGraph, comm: "Comm", un: np.ndarray, inn: np.ndarray, jn: np.ndarray, dev):
    """The loss reads the rows of the triples only (users u, items i and j,
    train_gat_pyg.py:313-322), so the top layer's incoming gradient is exactly zero on every
    other row (the loss backward writes those zeros).  The top layer's source-homed backward
    needs g of its halo rows: only the touched ones carry anything, a few percent of the 9M
    halo rows at config 5 -- so they alone travel (HaloRows.start_touched) and the rest of the
    table stays zero, the same table the dense exchange would deliver, bit for bit.

    Every rank derives the touched set from the full triple arrays it was given (each rank
    passes the same draw and keeps its own users' triples, _loss_plan), so the plans need no
    exchange; one all_reduce of a hash of the arrays confirms the ranks agree, else (or with
    PPGAT_SPARSE_TOP_G=0, or the destination-homed backward) the dense exchange stays: None.
    -> {"u": TouchPlan, "i": TouchPlan, "buf": None (the persistent zeroed g table, made by
    halo_bpr_loss)}."""
    if hg.src_views is None or hg.halo_ids is None or os.environ.get("PPGAT_SPARSE_TOP_G", "1") == "0":
        return None
    nu, N, n0 = hg.n_users, hg.n_nodes, hg.n_own
    rows = np.concatenate([un, inn + nu, jn + nu]).astype(np.int64)
    with np.errstate(over="ignore"):
        h = int(_mix64(rows.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) +
                       np.arange(len(rows), dtype=np.uint64)).sum(dtype=np.uint64) >> np.uint64(2))
    chk = torch.tensor([h, -h], dtype=torch.int64, device=dev if comm.backend == "nccl" else "cpu")
    chk = comm.all_reduce_(chk, op=dist.ReduceOp.MAX).cpu()
    if int(chk[0]) != -int(chk[1]):
        return None  # different triple sets on different ranks: keep the dense exchange
    T = np.zeros(N, bool)
    T[rows[(rows >= 0) & (rows < N)]] = True
    own = np.flatnonzero(hg.local_of >= 0)
    own_ids = np.empty(n0, np.int64)
    own_ids[hg.local_of[own]] = own
    t_own = T[own_ids]
    out = {"buf": None}
    halo_t = T[hg.halo_ids]
    for cls, plan, h0 in (("u", hg.plan_u, 0), ("i", hg.plan_i, hg.n_halo_u)):
        sidx, scnt = [], []
        for runs in plan.send_runs:
            idx = (np.concatenate([np.arange(a, a + n, dtype=np.int64) for a, n in runs]) if runs
                   else np.zeros(0, np.int64))
            idx = idx[t_own[idx]]
            sidx.append(idx)
            scnt.append(len(idx))
        tm = halo_t[h0:h0 + plan.n_recv]
        rpos, rcnt, off = [], [], 0
        for c in plan.recv_counts:
            p_ = np.flatnonzero(tm[off:off + c]) + off
            rpos.append(p_)
            rcnt.append(len(p_))
            off += c
        out[cls] = TouchPlan(torch.from_numpy(np.concatenate(sidx)).to(dev), scnt,
                             torch.from_numpy(np.concatenate(rpos).astype(np.int64)).to(dev), rcnt)
    return out


def _loss_plan(hg: HaloGraph, comm: "Comm", u, i, j, plan_key=None):
    """Exchange plan + row map for the triples of this rank's own users: the item rows they
    read that other ranks own come by one all_to_all.

    Reuse across calls is keyed ONLY on the caller's ``plan_key`` (e.g. the epoch of the
    triple draw, or a constant for a fixed triple set), which the caller passes identically on
    every rank -- the cache decision then agrees across ranks by construction, so no rank can
    skip the request exchange while another enters it.  Tensor identity (data_ptr/_version)
    is not a key: a new draw written in place (the device sampler) or placed at a freed
    address would hit a stale plan.  ``plan_key=None`` rebuilds the plan on every call."""
    if plan_key is not None:
        hit = hg.loss_plans.get(plan_key)
        if hit is not None:
            return hit
    nu, N = hg.n_users, hg.n_nodes
    u0, u1 = hg.owned_users()
    un, inn, jn = (t.detach().cpu().numpy().astype(np.int64) for t in (u, i, j))
    mine = (un >= u0) & (un < u1)
    items = np.unique(np.concatenate([inn[mine], jn[mine]])) + nu if mine.any() else np.zeros(0, np.int64)
    items = items[(items >= nu) & (items < N)]
    req = items[hg.owner[items] != hg.rank]                    # ascending ids, grouped by owner below
    req = req[np.argsort(hg.owner[req], kind="stable")]
    recv_counts = np.bincount(hg.owner[req], minlength=hg.world)
    send_counts = comm.all_to_all_counts(recv_counts)          # what each peer asks of this rank
    dev = u.device
    ids_in = comm.all_to_all_rows(torch.from_numpy(req).to(dev if comm.backend == "nccl" else "cpu"),
                                  recv_counts, send_counts).cpu().numpy()
    plan = make_plan(hg.n_own, hg.local_of[ids_in], send_counts, recv_counts, dev)
    rmap = np.full(N, -1, np.int64)
    rmap[u0:u1] = hg.local_of[u0:u1]
    own_items = items[hg.owner[items] == hg.rank]
    rmap[own_items] = hg.local_of[own_items]
    rmap[req] = hg.n_own + np.arange(len(req))
    res = (plan, torch.from_numpy(rmap.astype(np.int32)).to(dev), _touch_plans(hg, comm, un, inn, jn, dev))
    hg.loss_plans.clear()  # one live triple set at a time (an epoch's draw)
    if plan_key is not None:
        hg.loss_plans[plan_key] = res
    return res


def halo_bpr_loss(Z_own, hg: HaloGraph, comm: "Comm", u, i, j, n_users: int, n_items: int, loss: str = "bpr",
                  stages=None, plan_key=None):
    """The BPR/BCE loss of train_gat_pyg.py:313-322 over row-sharded Z: each rank takes the
    triples of its own users; the ranks' returned values add up to the reference's mean.
    ``plan_key``: identifies the triple set, the same value on every rank (see _loss_plan)."""
    if stages is None:
        from .hip_ops import HipStages
        stages = HipStages()
    plan, rmap, touch = _loss_plan(hg, comm, u, i, j, plan_key)
    hg.loss_tail_rows = plan.n_recv  # the next forward's top layer leaves room for these rows
    grad_rows = int(getattr(hg, "loss_grad_rows", 0))
    hg.grad_handoff = {}
    hg.top_touch = None
    Zl = exchange(Z_own, plan, comm, stages, inplace_grad=True, handoff=hg.grad_handoff if grad_rows else None)
    if grad_rows and getattr(stages, "bpr_grad_rows", False):
        # dZ inside an [R, C] buffer: the top layer's backward uses it as its g table (no copy)
        if touch is not None and grad_rows == hg.R:
            # ... a persistent one, zeroed once per triple set: the touched rows' exchange
            # (_touch_plans) leaves every other halo row of it at that zero
            C = Z_own.size(1)
            buf = touch["buf"]
            if buf is None or buf.shape != (hg.R, C) or buf.dtype != Z_own.dtype or buf.device != Z_own.device:
                buf = touch["buf"] = torch.zeros(hg.R, C, dtype=Z_own.dtype, device=Z_own.device)
            hg.top_touch = touch
            return stages.bpr(Zl, n_users, n_items, rmap, u, i, j, loss, grad_rows=grad_rows, grad_buf=buf)
        return stages.bpr(Zl, n_users, n_items, rmap, u, i, j, loss, grad_rows=grad_rows)
    return stages.bpr(Zl, n_users, n_items, rmap, u, i, j, loss)


def halo_rows_to_global(Z_own, hg: HaloGraph, comm: "Comm") -> torch.Tensor:
    """[n_own, C] own rows -> [N, C] in node-id order on every rank (all_gather; export and
    test helper, not on the training path)."""
    ids = [hg.own_node_ids(r) for r in range(hg.world)]
    pad = max(len(a) for a in ids)
    blk = Z_own.new_zeros(max(pad, 1), Z_own.size(1))
    blk[:hg.n_own] = Z_own
    allb = comm.all_gather_rows(blk)
    idx = np.empty(hg.n_nodes, np.int64)
    for r in range(hg.world):
        idx[ids[r]] = r * max(pad, 1) + np.arange(len(ids[r]))
    return allb.index_select(0, torch.from_numpy(idx).to(allb.device))


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

    def own_user_ids(self, rank: Optional[int] = None) -> np.ndarray:
        """A rank's users in its local row order: the id range itself."""
        a, b = self.owned_users(self.n_users, rank)
        return np.arange(a, b)


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
        # opt-in (PPGAT_FWD_SPLIT=1): measured 0.06-0.08 ms/step of fork/join and split-launch
        # cost per rank, more than the user rows hide from the merge at N >= 4
        if os.environ.get("PPGAT_FWD_SPLIT", "0") == "1":
            graph.fwd_split = (RU, sched_builder(view.rowptr[:RU + 1].contiguous(), El),
                               sched_builder(view.rowptr[RU:].contiguous(), El))
        if not bool((~su & ~du).any()):  # bipartite (no I-I columns): item sources reach users only
            graph.bwd_split = (RU, sched_builder(view.colptr[:RU + 1].contiguous(), El),
                               sched_builder(view.colptr[RU:].contiguous(), El))
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

    def merge_fwd_async(self, out, m, inv_l, agg, bias, heads: int, C: int):
        """merge_fwd on the communication stream, after the main stream's work so far (the
        item destinations' forward); ``wait`` joins it back.  It touches the item rows only."""
        dev = out.device
        main, cs = torch.cuda.current_stream(dev), _comm_stream(dev)
        cs.wait_stream(main)
        for t in (out, m, inv_l, agg, bias):
            if t is not None:
                t.record_stream(cs)
        with torch.cuda.stream(cs):
            self.merge_fwd(out, m, inv_l, agg, bias, heads, C)
        return (main, cs)

    def reduce_grad(self, g):
        if self.comm.active:
            self.comm.all_reduce_(g[self.RU:])

    def async_capable(self) -> bool:
        """RCCL on device tensors: the item-row all_reduce can run on the communication stream."""
        return self.comm.active and self.comm.backend == "nccl"

    def reduce_grad_async(self, g):
        """all_reduce of the item rows of g on the communication stream, after the main
        stream's work so far; ``wait`` joins it back."""
        dev = g.device
        main, cs = torch.cuda.current_stream(dev), _comm_stream(dev)
        cs.wait_stream(main)
        g.record_stream(cs)
        with torch.cuda.stream(cs):
            self.comm.all_reduce_(g[self.RU:])
        return (main, cs)

    def wait(self, pending):
        main, cs = pending
        main.wait_stream(cs)


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
        seed_buf = stages.seed_buffer(p, h.device)
        out, m, inv_l, agg = stages.fwd(rg.view, h, s_src, s_dst, b, heads, C, mode, slope, p, seed, heads > 1,
                                        seed_buf=seed_buf)
        if comm.active:
            _merge_item_rows(rg, comm, out, m, inv_l, agg, b, heads, C)
        if any(ctx.needs_input_grad[:4]):
            empty = torch.empty(0, device=h.device)
            ctx.save_for_backward(h, a_s, a_d, s_src, s_dst, out, m, inv_l, agg if agg is not None else empty,
                                  b if b is not None else empty)
        ctx.rg, ctx.comm, ctx.stages, ctx.seed_buf = rg, comm, stages, seed_buf
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
        grad_h, ds_src = st.bwd_edges(rg.view, h, s_src, nstate, g, dz, heads, C, mode, slope, p, seed,
                                      seed_buf=ctx.seed_buf)
        datt_src, datt_dst = st.bwd_epilogue(rg.view, h, a_s, a_d, ds_src, dz, grad_h, heads, C)
        dbias = None
        if has_bias and ctx.needs_input_grad[3]:
            dbias = g[:RU].sum(0)  # own users; the replicated item rows are counted on rank 0 only
            if comm.rank == 0:
                dbias = dbias + g[RU:].sum(0)
        return (grad_h, datt_src.view(ctx.att_shapes[0]), datt_dst.view(ctx.att_shapes[1]), dbias,
                None, None, None, None, None, None, None, None, None)


class ReplicatedPyGGAT(_ShardedBase):
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
                seed = self.layer_seed(conv)
                x = gat_layer(x, conv.lin.weight, conv.att_src, conv.att_dst, conv.bias, self.dg.graph, conv.heads,
                              conv.out_channels, _lib.MODE_PYG, float(conv.negative_slope), p, seed,
                              x_items=x_items if li == 0 else None, rep=self.hooks)
            return x
        x = self.node_features(item_feats)
        for conv in self.convs:
            h = self.stages.linear(x, conv.lin.weight, None)
            p = float(conv.dropout) if self.training else 0.0
            seed = self.layer_seed(conv)
            x = _ReplicatedGAT.apply(h, conv.att_src, conv.att_dst, conv.bias, self.dg, self.comm, self.stages,
                                     conv.heads, conv.out_channels, _lib.MODE_PYG, float(conv.negative_slope), p,
                                     seed)
        return x


def replicated_bpr_loss(Z_local, rg: RepGraph, comm: Comm, u, i, j, n_users: int, n_items: int,
                        loss: str = "bpr", stages=None, plan_key=None):
    """The BPR/BCE loss of train_gat_pyg.py:313-322: each rank takes the triples of its own
    users against its (replicated) item rows -- no exchange (so no plan: ``plan_key`` is
    accepted for the halo loss's signature and unused); the ranks' values add up to
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
