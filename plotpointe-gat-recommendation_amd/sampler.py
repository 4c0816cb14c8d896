"""BPR triple sampler on the GPU -- scripts/train_gat_pyg.py:179-190 (sample_bpr_epoch).

``BPRSampler(user_ptr, user_items, n_items, device)`` sorts each user's train items once
(``ppgat_bpr_sampler_prepare``); ``sample(S, seed, offset=0)`` returns device int64 tensors
(u, i, j) drawn by ``ppgat_bpr_sample`` with the reference's rule -- u uniform over users
with train items, i uniform over u's train list, j uniform over the items u has not
interacted with (rejection, as :185-188) -- from a counter-based stream: triple t depends
only on (seed, offset + t), so an epoch can be drawn in pieces.  The stream is not Python's
``random``; parity runs that need the reference's exact triples keep
``data.sample_bpr_epoch``.  No CPU path: the library must be loaded and tensors live on
a ROCm device.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


class BPRSampler:
    def __init__(self, user_ptr, user_items, n_items: int, device=None):
        lib = _lib.load()
        dev = torch.device(device) if device is not None else (
            user_ptr.device if isinstance(user_ptr, torch.Tensor) else torch.device("cuda"))
        if dev.type != "cuda":
            raise RuntimeError("BPRSampler: needs a ROCm device (there is no CPU path)")
        ptr = torch.as_tensor(np.asarray(user_ptr) if not isinstance(user_ptr, torch.Tensor) else user_ptr)
        items = torch.as_tensor(np.asarray(user_items) if not isinstance(user_items, torch.Tensor) else user_items)
        self.ptr = ptr.to(dev, torch.int64).contiguous()
        items = items.to(dev, torch.int32).contiguous()
        self.n_users = self.ptr.numel() - 1
        self.nnz = items.numel()
        self.n_items = int(n_items)
        self.device = dev
        if self.n_users < 0:
            raise ValueError("BPRSampler: user_ptr must have n_users + 1 entries")
        self.items = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=dev)
        self.eligible = torch.empty(max(self.n_users, 1), dtype=torch.int32, device=dev)
        self.n_eligible = torch.zeros(1, dtype=torch.int64, device=dev)
        nb = ctypes.c_size_t(0)
        _lib.check(lib.ppgat_bpr_sampler_workspace_bytes(self.n_users, self.nnz, ctypes.byref(nb)),
                   "bpr_sampler_workspace_bytes")
        ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
        _lib.check(lib.ppgat_bpr_sampler_prepare(self.ptr.data_ptr(), items.data_ptr() if self.nnz else None,
                                                 self.n_users, self.nnz, self.items.data_ptr(),
                                                 self.eligible.data_ptr(), self.n_eligible.data_ptr(),
                                                 ws.data_ptr(), nb.value, _lib.stream_handle(dev)),
                   "bpr_sampler_prepare")
        self._bad = torch.zeros(1, dtype=torch.int32, device=dev)

    def sample(self, samples: int, seed: int = 42, offset: int = 0, check: bool = True):
        """-> (u, i, j) int64 [samples] on the sampler's device.  ``check`` syncs once to
        raise if no user has items or a negative could not be drawn (user holds ~all items)."""
        lib = _lib.load()
        out = torch.empty(3, samples, dtype=torch.int64, device=self.device)
        _lib.check(lib.ppgat_bpr_sample(self.ptr.data_ptr(), self.items.data_ptr(), self.eligible.data_ptr(),
                                        self.n_eligible.data_ptr(), self.n_items, samples,
                                        int(seed) & 0xFFFFFFFFFFFFFFFF, int(offset), out[0].data_ptr(),
                                        out[1].data_ptr(), out[2].data_ptr(), self._bad.data_ptr(),
                                        _lib.stream_handle(self.device)), "bpr_sample")
        if check and samples > 0:
            bad = int(self._bad.item())
            if bad & 1:
                raise ValueError("BPRSampler: no user has train items")
            if bad & 2:
                raise ValueError("BPRSampler: a user holds (almost) every item; no negative found")
        return out[0], out[1], out[2]

    def eval_candidates(self, users, pos, n_neg: int, seed: int = 0, check: bool = True) -> torch.Tensor:
        """eval_sampled's candidates (train_gat_pyg.py:157-167) on the device: [B, n_neg + 1]
        int64, column 0 the held-out positive, then n_neg negatives drawn uniformly from the
        items outside the user's train list and != the positive (ppgat_eval_sample)."""
        lib = _lib.load()
        u = torch.as_tensor(users).to(self.device, torch.int64).contiguous()
        p = torch.as_tensor(pos).to(self.device, torch.int64).contiguous()
        if u.numel() != p.numel():
            raise ValueError("eval_candidates: users and pos must have the same length")
        cands = torch.empty(u.numel(), int(n_neg) + 1, dtype=torch.int64, device=self.device)
        _lib.check(lib.ppgat_eval_sample(self.ptr.data_ptr(), self.items.data_ptr(), u.data_ptr(), p.data_ptr(),
                                         u.numel(), int(n_neg), self.n_items, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                         cands.data_ptr(), self._bad.data_ptr(), _lib.stream_handle(self.device)),
                   "eval_sample")
        if check and u.numel() > 0 and int(self._bad.item()) & 2:
            raise ValueError("eval_candidates: a user holds (almost) every item; no negative found")
        return cands
