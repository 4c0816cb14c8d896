"""Adam on the device in one launch per 16 tensors (include/ppgat.h ppgat_adam_step).

Drop-in for ``torch.optim.Adam(model.parameters(), lr=cfg.lr, weight_decay=cfg.l2)``
(scripts/train_gat_pyg.py:299, train_gat_custom.py's equivalent) with the same
hyper-parameters, the same per-parameter state keys (``step``, ``exp_avg``,
``exp_avg_sq``) and the same update rule (L2 weight decay added to the gradient, bias
corrections, eps after the square root), so optimizer state_dicts move between the two.
Supported: fp32 dense tensors on one ROCm device, amsgrad=False, maximize=False.

``capturable=True`` (torch.optim.Adam's flag of the same name): every parameter's step
count ``state["step"]`` is a device float (as in torch's capturable Adam), incremented with
one multi-tensor launch and turned into the bias corrections on the stream
(``ppgat_adam_step_device``), so ``step()`` can be captured in a hipGraph and replayed; a
parameter without a gradient keeps its count, and saved state has one count per parameter.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False, maximize: bool = False, capturable: bool = False):
        if amsgrad or maximize:
            raise NotImplementedError("ppgat Adam: amsgrad / maximize not implemented")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError("invalid Adam hyper-parameter")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, capturable=bool(capturable)))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        cap = int(lib.ppgat_adam_max_tensors())
        for group in self.param_groups:
            b1, b2 = group["betas"]
            batch = []
            if group.get("capturable", False):
                self._step_device(lib, cap, group)
                continue
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("ppgat Adam: sparse gradients are not supported")
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and g.is_contiguous()
                        and g.dtype == torch.float32):
                    raise RuntimeError("ppgat Adam: fp32 contiguous ROCm parameters and gradients only")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] += 1
                t = float(st["step"].item())
                batch.append((p, g, st["exp_avg"], st["exp_avg_sq"], group["lr"] / (1.0 - b1 ** t),
                              math.sqrt(1.0 - b2 ** t)))
                if len(batch) == cap:
                    self._launch(lib, batch, group, b1, b2)
                    batch = []
            if batch:
                self._launch(lib, batch, group, b1, b2)
        return loss

    def _step_device(self, lib, cap, group):
        b1, b2 = group["betas"]
        ps = [p for p in group["params"] if p.grad is not None]
        if not ps:
            return
        for p in ps:
            g = p.grad
            if g.is_sparse or not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and g.is_contiguous()
                                   and g.dtype == torch.float32):
                raise RuntimeError("ppgat Adam: fp32 contiguous dense ROCm parameters and gradients only")
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            elif not (st["step"].is_cuda and st["step"].device == p.device and st["step"].dtype == torch.float32):
                # a state_dict loaded from a host-step run: the count moves to the device once
                st["step"] = st["step"].to(device=p.device, dtype=torch.float32).reshape(())
        steps = [self.state[p]["step"] for p in ps]
        torch._foreach_add_(steps, 1.0)  # one launch, on the stream: graph replays advance every count
        for k in range(0, len(ps), cap):
            chunk = ps[k:k + cap]
            n = len(chunk)
            dev = chunk[0].device
            P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in chunk])
            G = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p in chunk])
            M = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg"].data_ptr() for p in chunk])
            V = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg_sq"].data_ptr() for p in chunk])
            NE = (ctypes.c_int64 * n)(*[p.numel() for p in chunk])
            T = (ctypes.c_void_p * n)(*[self.state[p]["step"].data_ptr() for p in chunk])
            _lib.check(lib.ppgat_adam_step_device(n, P, G, M, V, NE, T, float(group["lr"]), float(b1), float(b2),
                                                  float(group["eps"]), float(group["weight_decay"]),
                                                  _lib.stream_handle(dev)), "adam_step_device")

    @staticmethod
    def _launch(lib, batch, group, b1, b2):
        n = len(batch)
        dev = batch[0][0].device
        for p, *_ in batch:
            if p.device != dev:
                raise RuntimeError("ppgat Adam: all parameters of a group must be on one device")
        P = (ctypes.c_void_p * n)(*[b[0].data_ptr() for b in batch])
        G = (ctypes.c_void_p * n)(*[b[1].data_ptr() for b in batch])
        M = (ctypes.c_void_p * n)(*[b[2].data_ptr() for b in batch])
        V = (ctypes.c_void_p * n)(*[b[3].data_ptr() for b in batch])
        NE = (ctypes.c_int64 * n)(*[b[0].numel() for b in batch])
        SS = (ctypes.c_float * n)(*[b[4] for b in batch])
        BC = (ctypes.c_float * n)(*[b[5] for b in batch])
        _lib.check(lib.ppgat_adam_step(n, P, G, M, V, NE, SS, BC, float(b1), float(b2), float(group["eps"]),
                                       float(group["weight_decay"]), _lib.stream_handle(dev)), "adam_step")
