"""I-I kNN graph on the GPU -- graphs/build_ii_knn.py (the second relation of config 3).

``build_ii_knn(embeddings, k=20, min_similarity=0.3)`` returns the reference's COO triplet
(rows = item, cols = neighbour, sims = cosine) in the reference's order (items ascending,
neighbours by similarity descending), for ``scipy.sparse.coo_matrix((sims, (rows, cols)))``
and ``save_npz`` exactly as build_ii_knn.py:104-116 writes it.

Steps (build_ii_knn.py line refs): rows normalised as e / (||e|| + 1e-8) (:57-59) and again
by sklearn's cosine_similarity (:76); per block of query rows the similarity block
E_q E^T is one ``ppgat_gemm_nn`` launch on the matrix cores through an operand split -- the
bf16 three-term split (<= 2^-24 relative per product) or, for blocks of >= 1,024 rows, the
fp16 two-term split with per-row / per-column power-of-two scales (<= 2^-21 per product;
DESIGN.md §4.3) -- NOT bitwise sklearn's fp32 dot products: where two candidates'
similarities, or a similarity and ``min_similarity``, are within ~1e-6 the order or the
membership can differ from the reference's (tests/test_knn.py pins the lists against the
reference script's own output with a 1e-5 near-tie / threshold rule).  The rows are copied
once into a zero-padded [n_p, d_p] buffer (exact zeros; the kernel's widths), so the
embeddings are held twice during the build; the selection -- self excluded, top-k, sorted,
thresholded (:79-95) -- is libppgat's ``ppgat_knn_topk`` kernel.  The full n x n matrix is
never materialised (block_rows x n at a time).
"""
from __future__ import annotations

import torch

from . import _lib
from . import hip_ops


def build_ii_knn(embeddings: torch.Tensor, k: int = 20, min_similarity: float = 0.3, block_rows: int = 8192):
    lib = _lib.load()
    if not (isinstance(embeddings, torch.Tensor) and embeddings.is_cuda and embeddings.dim() == 2):
        raise RuntimeError("build_ii_knn: embeddings must be a 2-D ROCm tensor (there is no CPU path)")
    if k < 1 or k > int(lib.ppgat_knn_max_k()):
        raise NotImplementedError(f"build_ii_knn: k={k} outside [1, {int(lib.ppgat_knn_max_k())}]")
    e = embeddings.to(torch.float32).contiguous()
    n = e.size(0)
    dev = e.device
    d = e.size(1)
    n_p, d_p = -(-n // 128) * 128, -(-max(d, 1) // 32) * 32
    exp = torch.zeros(n_p, d_p, dtype=torch.float32, device=dev)  # padded rows/columns are exact zeros
    en = e / (torch.linalg.vector_norm(e, dim=1, keepdim=True) + 1e-8)
    n2 = torch.linalg.vector_norm(en, dim=1, keepdim=True)
    # sklearn.preprocessing.normalize, written straight into the padded operand (no third copy)
    torch.div(en, torch.where(n2 == 0, torch.ones_like(n2), n2), out=exp[:n, :d])
    del en, n2
    idx = torch.empty(n, k, dtype=torch.int32, device=dev)
    sim = torch.empty(n, k, dtype=torch.float32, device=dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev)
    st = _lib.stream_handle(dev)
    for q0 in range(0, n, block_rows):
        q1 = min(q0 + block_rows, n)
        S = hip_ops.gemm_nn(exp[q0:q1], exp, 1, n_p)  # [q, n_p]: the similarity block, columns >= n unused
        _lib.check(lib.ppgat_knn_topk(S.data_ptr(), n_p, q1 - q0, n, q0, k, float(min_similarity),
                                      idx[q0:].data_ptr(), sim[q0:].data_ptr(), cnt[q0:].data_ptr(), st),
                   "knn_topk")
    keep = torch.arange(k, device=dev)[None, :] < cnt[:, None].to(torch.int64)
    rows = torch.arange(n, device=dev, dtype=torch.int32)[:, None].expand(n, k)[keep]
    return rows, idx[keep], sim[keep]
