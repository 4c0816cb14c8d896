"""Multimodal fusion (the north star's MFMA target):
embeddings/fuse_modal.py.

``FusionMLP``             -- :18-36, same modules/keys (mlp.0, mlp.3, txt_proj, img_proj) and
                             construction order (seeded construction = reference weights).
                             Eval-mode forward runs the fused matrix-core kernel
                             (``ppgat_fusion_fwd``); train-mode forward is autograd over the
                             ppgat GEMMs (hip_ops.linear) with torch's Dropout (its RNG stream).
``contrastive_fusion_loss`` -- :39-72 (InfoNCE, tau = 0.07, both modalities), autograd; the
                             similarity products on the ppgat GEMM.
``fusion_train_step``      -- the same forward + loss + backward on the device kernels: the four
                             Linear layers on the fp32 matrix-core GEMMs (ppgat_gemm_nn, weight
                             grads ppgat_gemm_tn_big + ppgat_colsum), ReLU/Dropout and its
                             backward (ppgat_relu_dropout, counter-hash mask), InfoNCE loss and
                             gradient (ppgat_infonce).  Writes .grad; the loss stays on the device.
``infer_fused_embeddings``  -- :220-244: all items, mean-image fallback for items without an
                             image, L2-normalised; the per-row host->device image copy loop
                             becomes an index gather inside the kernel.
``train_fusion``            -- :167-214 training loop (Adam, contiguous batches); native step
                             by default, ``native=False`` keeps the torch-autograd step.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from . import hip_ops


def fusion_forward(txt: torch.Tensor, img: Optional[torch.Tensor], W1, b1, W2, b2, normalize: bool,
                   img_index: Optional[torch.Tensor] = None, img_fallback: Optional[torch.Tensor] = None,
                   want_z1: bool = False):
    lib = _lib.load()
    if not txt.is_cuda or txt.dtype != torch.float32:
        raise RuntimeError("fusion_forward: fp32 ROCm tensors required (no CPU path)")
    dev = txt.device
    txt = txt.contiguous()
    n, Dt = txt.shape
    Di = W1.size(1) - Dt
    H1, Do = W1.size(0), W2.size(0)
    out = torch.empty(n, Do, dtype=torch.float32, device=dev)
    z1 = torch.empty(n, H1, dtype=torch.float32, device=dev) if want_z1 else None
    ptr = _lib.ptr
    # keep every converted tensor alive until the launch is enqueued
    imgc = img.contiguous() if img is not None else None
    idx32 = img_index.to(torch.int32).contiguous() if img_index is not None else None
    fb = img_fallback.contiguous() if img_fallback is not None else None
    W1c, b1c, W2c, b2c = (t.detach().contiguous() for t in (W1, b1, W2, b2))
    nbytes = ctypes.c_size_t(0)
    _lib.check(lib.ppgat_fusion_fwd_workspace_bytes(Dt, Di, H1, Do, ctypes.byref(nbytes)), "fusion_fwd_workspace")
    ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=dev)  # the pre-split W1 / W2 images
    _lib.check(lib.ppgat_fusion_fwd_ws(ptr(txt), ptr(imgc), ptr(idx32), ptr(fb), n, Dt, Di, W1c.data_ptr(),
                                       b1c.data_ptr(), H1, W2c.data_ptr(), b2c.data_ptr(), Do, 1 if normalize else 0,
                                       out.data_ptr(), ptr(z1), ws.data_ptr(), nbytes.value, _lib.stream_handle(dev)),
               "fusion_fwd")
    return (out, z1) if want_z1 else out


class FusionMLP(nn.Module):
    """embeddings/fuse_modal.py:18-36."""

    def __init__(self, text_dim, img_dim, output_dim=128, hidden_dim=256):
        super().__init__()
        input_dim = text_dim + img_dim
        self.mlp = nn.Sequential(
            nn.Linear(input_dim, hidden_dim),
            nn.ReLU(),
            nn.Dropout(0.1),
            nn.Linear(hidden_dim, output_dim),
        )
        self.txt_proj = nn.Linear(text_dim, output_dim)
        self.img_proj = nn.Linear(img_dim, output_dim)
        self.text_dim, self.img_dim = text_dim, img_dim

    def project_txt(self, t):
        """txt_proj (fuse_modal.py:31) on the ppgat GEMM."""
        return hip_ops.linear(t.contiguous(), self.txt_proj.weight, self.txt_proj.bias)

    def project_img(self, t):
        """img_proj (fuse_modal.py:32) on the ppgat GEMM."""
        return hip_ops.linear(t.contiguous(), self.img_proj.weight, self.img_proj.bias)

    def forward(self, text_emb, img_emb):
        if not text_emb.is_cuda:
            raise RuntimeError("FusionMLP runs on ROCm devices only; there is no CPU path")
        if self.training:  # autograd through the ppgat GEMMs; Dropout keeps torch's RNG draw (:29)
            l1, l2 = self.mlp[0], self.mlp[3]
            h = torch.relu(hip_ops.linear(torch.cat([text_emb, img_emb], dim=-1), l1.weight, l1.bias))
            return hip_ops.linear(self.mlp[2](h), l2.weight, l2.bias)
        return fusion_forward(text_emb, img_emb, self.mlp[0].weight, self.mlp[0].bias, self.mlp[3].weight,
                              self.mlp[3].bias, normalize=False)


def contrastive_fusion_loss(fused, txt_emb, img_emb, temperature=0.07):
    """embeddings/fuse_modal.py:39-72 -> (loss, loss_txt, loss_img)."""
    import torch.nn.functional as F
    batch_size = fused.size(0)
    fused_norm = F.normalize(fused, dim=-1)
    txt_norm = F.normalize(txt_emb, dim=-1)
    img_norm = F.normalize(img_emb, dim=-1)
    # fused_norm @ txt_norm.T as x W^T on ppgat_gemm_nn, differentiable in both operands
    sim_fused_txt = hip_ops.linear(fused_norm.contiguous(), txt_norm.contiguous()) / temperature
    sim_fused_img = hip_ops.linear(fused_norm.contiguous(), img_norm.contiguous()) / temperature
    labels = torch.arange(batch_size, device=fused.device)
    loss_txt = F.cross_entropy(sim_fused_txt, labels)
    loss_img = F.cross_entropy(sim_fused_img, labels)
    loss = (loss_txt + loss_img) / 2
    return loss, loss_txt.item(), loss_img.item()


def infonce(fused: torch.Tensor, txt_p: torch.Tensor, img_p: torch.Tensor, temperature: float = 0.07):
    """contrastive_fusion_loss forward and gradient on the device (ppgat_infonce) ->
    (loss [3] = {loss, loss_txt, loss_img}, d_fused, d_txt_p, d_img_p)."""
    lib = _lib.load()
    for name, t in (("fused", fused), ("txt_p", txt_p), ("img_p", img_p)):
        if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.is_contiguous()):
            raise RuntimeError(f"infonce: {name} must be a contiguous fp32 ROCm [B, D] tensor (no CPU path)")
    B, D = fused.shape
    if txt_p.shape != (B, D) or img_p.shape != (B, D):
        raise ValueError("infonce: fused, txt_p, img_p must share [B, D]")
    nbytes = ctypes.c_size_t(0)
    _lib.check(lib.ppgat_infonce_workspace_bytes(B, D, ctypes.byref(nbytes)), "infonce_workspace_bytes")
    dev = fused.device
    ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=dev)
    loss = torch.empty(3, dtype=torch.float32, device=dev)
    dF, dT, dI = (torch.empty(B, D, dtype=torch.float32, device=dev) for _ in range(3))
    _lib.check(lib.ppgat_infonce(fused.data_ptr(), txt_p.data_ptr(), img_p.data_ptr(), B, D, float(temperature),
                                 loss.data_ptr(), dF.data_ptr(), dT.data_ptr(), dI.data_ptr(), ws.data_ptr(),
                                 nbytes.value, _lib.stream_handle(dev)), "infonce")
    return loss, dF, dT, dI


def relu_dropout(z: torch.Tensor, p: float, seed: int, grad: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Forward (grad None): relu(z) * mask.  Backward: grad * mask * [z > 0], in place on grad.
    The mask is a counter hash of (seed, element) (ppgat_relu_dropout), identical both ways."""
    lib = _lib.load()
    if not (z.is_cuda and z.dtype == torch.float32 and z.is_contiguous()):
        raise RuntimeError("relu_dropout: contiguous fp32 ROCm tensor required (no CPU path)")
    out = torch.empty_like(z) if grad is None else grad
    if grad is not None and (grad.shape != z.shape or not grad.is_contiguous()):
        raise ValueError("relu_dropout: grad must be contiguous and shaped like z")
    _lib.check(lib.ppgat_relu_dropout(z.data_ptr(), z.numel(), float(p), int(seed) & (2**64 - 1),
                                      0 if grad is None else 1, out.data_ptr(), _lib.stream_handle(z.device)),
               "relu_dropout")
    return out


def _accumulate(p: torch.Tensor, g: torch.Tensor):
    if p.grad is None:
        p.grad = g
    else:
        p.grad.add_(g)


def fusion_train_step(model: FusionMLP, txt: torch.Tensor, img: torch.Tensor, seed: int = 0,
                      temperature: float = 0.07) -> torch.Tensor:
    """One forward + contrastive loss + backward of FusionMLP on the device kernels (the
    reference's opt.zero_grad/forward/loss/backward, fuse_modal.py:185-193, minus the step).
    Dropout p is model.mlp[2].p (0 in eval-equivalent checks), drawn from ``seed``.
    Accumulates into each parameter's .grad and returns the device loss [3] =
    {loss, loss_txt, loss_img}."""
    if not txt.is_cuda:
        raise RuntimeError("fusion_train_step runs on ROCm devices only; there is no CPU path")
    txt, img = txt.contiguous(), img.contiguous()
    l1, l2 = model.mlp[0], model.mlp[3]
    p = float(model.mlp[2].p) if model.training else 0.0
    W1, b1, W2, b2 = (t.detach() for t in (l1.weight, l1.bias, l2.weight, l2.bias))
    Wt, bt, Wi, bi = (t.detach() for t in (model.txt_proj.weight, model.txt_proj.bias, model.img_proj.weight,
                                             model.img_proj.bias))
    x = torch.cat([txt, img], 1)
    z1 = hip_ops.gemm_nn(x, W1, 1, W1.size(0), bias=b1)                 # [B, hidden]
    a = relu_dropout(z1, p, seed)
    fused = hip_ops.gemm_nn(a, W2, 1, W2.size(0), bias=b2)              # [B, out]
    tp = hip_ops.gemm_nn(txt, Wt, 1, Wt.size(0), bias=bt)
    ip = hip_ops.gemm_nn(img, Wi, 1, Wi.size(0), bias=bi)
    loss, dF, dT, dI = infonce(fused, tp, ip, temperature)
    dW2, db2, _ = hip_ops.gemm_tn(dF, a, want_colsum=True)
    da = hip_ops.gemm_nn(dF, W2, 0, W2.size(1))                         # dF W2 [B, hidden]
    dz = relu_dropout(z1, p, seed, grad=da)
    dW1, db1, _ = hip_ops.gemm_tn(dz, x, want_colsum=True)
    dWt, dbt, _ = hip_ops.gemm_tn(dT, txt, want_colsum=True)
    dWi, dbi, _ = hip_ops.gemm_tn(dI, img, want_colsum=True)
    for prm, g in ((l1.weight, dW1), (l1.bias, db1), (l2.weight, dW2), (l2.bias, db2), (model.txt_proj.weight, dWt),
                   (model.txt_proj.bias, dbt), (model.img_proj.weight, dWi), (model.img_proj.bias, dbi)):
        _accumulate(prm, g)
    return loss


def train_fusion(model: FusionMLP, txt_aligned: torch.Tensor, img_aligned: torch.Tensor, epochs: int = 5,
                 batch_size: int = 512, lr: float = 1e-3, native: bool = True, seed: int = 0):
    """fuse_modal.py:167-214 (tensors already on the device).  The native path keeps the
    per-batch losses on the device and reads them once per epoch (the reference's
    loss.item() per batch is a host sync per step)."""
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    model.train()
    history = []
    step = 0
    for _ in range(epochs):
        if native:
            acc = torch.zeros(3, dtype=torch.float32, device=txt_aligned.device)
            nb = 0
            for i in range(0, len(txt_aligned), batch_size):
                bt, bi = txt_aligned[i:i + batch_size], img_aligned[i:i + batch_size]
                opt.zero_grad(set_to_none=True)
                acc += fusion_train_step(model, bt, bi, seed=(seed * 1_000_003 + step) & (2**64 - 1))
                opt.step()
                nb += 1
                step += 1
            tot, tt, ti = (acc / nb).tolist()
            history.append((tot, tt, ti))
            continue
        tot = tt = ti = 0.0
        nb = 0
        for i in range(0, len(txt_aligned), batch_size):
            bt, bi = txt_aligned[i:i + batch_size], img_aligned[i:i + batch_size]
            opt.zero_grad()
            fused = model(bt, bi)
            loss, lt, li = contrastive_fusion_loss(fused, model.project_txt(bt), model.project_img(bi))
            loss.backward()
            opt.step()
            tot += loss.item(); tt += lt; ti += li
            nb += 1
        history.append((tot / nb, tt / nb, ti / nb))
    return history


def infer_fused_embeddings(model: FusionMLP, txt_emb: torch.Tensor, img_aligned: torch.Tensor,
                           img_index: torch.Tensor, chunk: int = 1 << 17) -> torch.Tensor:
    """fuse_modal.py:220-244: fused, L2-normalised embeddings for ALL items.

    img_index[g] = row of img_aligned holding item g's image, or -1 (use the mean image
    embedding, :211-213,231).  One fused MFMA launch per ``chunk`` items."""
    model.eval()
    mean_img = img_aligned.mean(dim=0)
    out = torch.empty(txt_emb.size(0), model.mlp[3].out_features, dtype=torch.float32, device=txt_emb.device)
    with torch.no_grad():
        for s in range(0, txt_emb.size(0), chunk):
            e = min(s + chunk, txt_emb.size(0))
            out[s:e] = fusion_forward(txt_emb[s:e], img_aligned, model.mlp[0].weight, model.mlp[0].bias,
                                      model.mlp[3].weight, model.mlp[3].bias, normalize=True,
                                      img_index=img_index[s:e], img_fallback=mean_img)
    return out


def image_index_for_items(n_items: int, img_indices: np.ndarray) -> np.ndarray:
    """fuse_modal.py:147-151: item g -> local image row (img_idx_map), -1 if none."""
    idx = np.full(n_items, -1, np.int32)
    idx[np.asarray(img_indices, np.int64)] = np.arange(len(img_indices), dtype=np.int32)
    return idx
