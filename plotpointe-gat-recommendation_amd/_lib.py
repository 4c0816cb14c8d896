"""ctypes binding of libppgat.so (include/ppgat.h).

The product path has no CPU fallback: if the shared library is missing or fails to
load, every op raises ``RuntimeError`` (build it with ``python -c "import
__graft_entry__ as g; g.build()"`` or ``make -C plotpointe-gat-recommendation_amd/csrc``).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("PPGAT_LIB", _HERE / "libppgat.so"))

c_int, c_i64, c_u64, c_f, c_vp, c_sz = (ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float,
                                         ctypes.c_void_p, ctypes.c_size_t)



class Schedule(ctypes.Structure):
    """include/ppgat.h ppgat_schedule"""
    _fields_ = [("item_row", c_vp), ("item_beg", c_vp), ("item_end", c_vp), ("n_items", c_i64),
                ("n_hub_items", c_i64), ("hub_row", c_vp), ("hub_ptr", c_vp), ("n_hubs", c_i64),
                ("n_long_items", c_i64)]


SP = ctypes.POINTER(Schedule)

# name -> (restype, argtypes); mirrors include/ppgat.h
SIGNATURES = {
    "ppgat_version": (c_int, []),
    "ppgat_last_error": (ctypes.c_char_p, []),
    "ppgat_supported_channels": (c_int, [c_int]),
    "ppgat_csr_workspace_bytes": (c_int, [c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "ppgat_csr_build": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz,
                                c_vp]),
    "ppgat_schedule_capacity": (c_i64, [c_i64, c_i64, ctypes.c_int32]),
    "ppgat_schedule_workspace_bytes": (c_int, [c_i64, ctypes.POINTER(c_sz)]),
    "ppgat_schedule_build": (c_int, [c_vp, c_i64, c_i64, ctypes.c_int32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_sz, c_vp]),
    "ppgat_node_scores": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp]),
    "ppgat_fwd_workspace_bytes": (c_int, [c_i64, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_fwd": (c_int, [SP, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_f, c_f,
                          c_u64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_bwd_workspace_bytes": (c_int, [c_i64, c_i64, c_i64, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_bwd": (c_int, [SP, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                          c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_f, c_f, c_u64, c_vp, c_vp, c_vp, c_vp, c_vp,
                          c_vp, c_sz, c_vp]),
    "ppgat_bwd_partial_rows": (c_i64, [c_i64]),
    "ppgat_bwd_prologue": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_vp,
                                   c_vp, c_vp]),
    "ppgat_bwd_edges": (c_int, [SP, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_f, c_f,
                                c_u64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_bwd_dst_sum": (c_int, [c_vp, c_i64, c_int, c_vp, c_vp, c_i64, c_vp, c_sz, c_vp]),
    "ppgat_bwd_dst_sum_csc": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_vp, c_sz, c_vp]),
    "ppgat_invert_index": (c_int, [c_vp, c_i64, c_vp, c_vp]),
    "ppgat_bwd_epilogue": (c_int, [c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   c_vp]),
    "ppgat_bpr_workspace_bytes": (c_int, [c_i64, c_i64, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_bpr_fwd": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp,
                              c_vp, c_vp, c_sz, c_vp]),
    "ppgat_bpr_bwd": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                              c_vp, c_sz, c_vp]),
    "ppgat_bpr_bwd_prepare": (c_int, [c_i64, c_i64, c_i64, c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_vp, c_sz, c_vp]),
    "ppgat_bpr_bwd_prepared": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                       c_vp, c_vp, c_sz, c_vp]),
    "ppgat_bpr_bwd_producer": (c_int, [c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                       c_vp, c_vp, c_vp, c_vp, c_f, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_gemm_tn_workspace_bytes": (c_int, [c_i64, c_int, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_gemm_tn": (c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp,
                              c_vp, c_sz, c_vp]),
    "ppgat_gemm_tn_seg": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_int, c_int, c_vp, c_vp,
                                  c_vp, c_i64, c_int, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_project_supported": (c_int, [c_int, c_int]),
    "ppgat_project": (c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_i64, c_int, c_vp, c_vp, c_vp,
                              c_vp, c_i64, c_vp, c_vp, c_vp]),
    "ppgat_project_bwd_input": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_vp,
                                        c_i64, c_vp]),
    "ppgat_project_bwd_fused_supported": (c_int, [c_int]),
    "ppgat_project_bwd_fused_workspace_bytes": (c_int, [c_i64, ctypes.POINTER(c_sz)]),
    "ppgat_project_bwd_fused": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_int, c_vp,
                                        c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_project_bwd_fused_producer": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64,
                                                 c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                                 c_vp, c_vp, c_f, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_weight_grads": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "ppgat_adam_max_tensors": (c_int, []),
    "ppgat_adam_step": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_double, ctypes.c_double,
                                c_f, c_f, c_vp]),
    "ppgat_adam_step_device": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, c_f, c_f, c_vp]),
    "ppgat_dropout_advance": (c_int, [c_vp]),
    "ppgat_rep_merge": (c_int, [c_int, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ppgat_dropout_set_epoch": (c_int, [ctypes.c_uint64, c_vp]),
    "ppgat_rows_gather": (c_int, [c_vp, c_i64, c_vp, c_i64, c_int, c_vp, c_i64, c_vp]),
    "ppgat_rows_return_add": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_int, c_vp]),
    "ppgat_knn_max_k": (c_int, []),
    "ppgat_knn_topk": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_int, c_f, c_vp, c_vp, c_vp, c_vp]),
    "ppgat_bpr_sampler_workspace_bytes": (c_int, [c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "ppgat_bpr_sampler_prepare": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_bpr_sample": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_u64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ppgat_eval_sample": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_u64, c_vp, c_vp, c_vp]),
    "ppgat_sampled_rank": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "ppgat_serve_topk_workspace_bytes": (c_int, [c_i64, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_serve_topk": (c_int, [c_vp, c_i64, c_int, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_fusion_fwd": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_int,
                                 c_int, c_vp, c_vp, c_vp]),
    "ppgat_fusion_fwd_workspace_bytes": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_fusion_fwd_ws": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_int,
                                    c_int, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_infonce_workspace_bytes": (c_int, [c_i64, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_infonce": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_f, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_relu_dropout": (c_int, [c_vp, c_i64, c_f, c_u64, c_int, c_vp, c_vp]),
    "ppgat_gemm_nn_supported": (c_int, [c_i64, c_int, c_int, c_int]),
    "ppgat_gemm_nn": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_i64, c_int, c_int, c_f, c_vp, c_vp, c_i64, c_vp]),
    "ppgat_gemm_nn_workspace_bytes": (c_int, [c_i64, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_gemm_nn_ws": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_i64, c_int, c_int, c_f, c_vp, c_vp, c_i64, c_vp, c_sz,
                                 c_vp]),
    "ppgat_gemm_nn_rank": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_i64, c_int, c_int, c_f, c_vp, c_vp, c_i64, c_int,
                                   c_vp, c_i64, c_vp, c_i64, c_vp, c_sz, c_vp]),
    "ppgat_gemm_tn_big_workspace_bytes": (c_int, [c_i64, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_gemm_tn_big": (c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_gemm_tn_big_bounded": (c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_int, c_f, c_vp, c_vp,
                                          c_sz, c_vp]),
    "ppgat_gemm_tn_big_bounds": (c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_vp, c_int, c_f, c_vp,
                                         c_vp, c_sz, c_vp]),
    "ppgat_gemm_tn_big_colsum": (c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_vp, c_int, c_f, c_vp,
                                         c_vp, c_vp, c_sz, c_vp]),
    "ppgat_colmax_abs": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp]),
    "ppgat_colmax_abs_sources": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp]),
    "ppgat_colsum_workspace_bytes": (c_int, [c_i64, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_colsum": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_xgat_supported": (c_int, [c_int, c_int, c_int]),
    "ppgat_xgat_weights": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "ppgat_xgat_scores": (c_int, [c_vp, c_i64, c_i64, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "ppgat_xgat_fwd_workspace_bytes": (c_int, [c_i64, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_xgat_fwd": (c_int, [SP, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_i64, c_vp, c_vp, c_f, c_f, c_u64,
                               c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_xgat_fwd_colmax": (c_int, [SP, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_i64, c_vp, c_vp, c_f, c_f,
                                      c_u64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_xgat_bwd_prologue": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp]),
    "ppgat_xgat_bwd_workspace_bytes": (c_int, [c_i64, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_xgat_bwd_edges": (c_int, [SP, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                     c_f, c_f, c_u64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_xgat_bwd_g_workspace_bytes": (c_int, [c_i64, c_int, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_xgat_bwd_edges_g": (c_int, [SP, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64,
                                       c_f, c_f, c_u64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_xgat_bwd_edges_gd": (c_int, [SP, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64,
                                        c_f, c_f, c_u64, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_xgat_bwd_edges_gd_colmax": (c_int, [SP, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp,
                                               c_i64, c_f, c_f, c_u64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ppgat_xgat_nstate": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp]),
    "ppgat_xgat_nstate_set_d": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp]),
    "ppgat_xgat_bwd_dz_workspace_bytes": (c_int, [c_i64, c_int, ctypes.POINTER(c_sz)]),
    "ppgat_xgat_bwd_dz": (c_int, [SP, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_f, c_f, c_u64, c_vp, c_vp, c_vp,
                                  c_i64, c_vp, c_sz, c_vp]),
    "ppgat_xgat_bwd_epilogue": (c_int, [c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_vp, c_i64, c_vp]),
    "ppgat_att_proj": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp]),
    "ppgat_rows_rank_update": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_i64, c_int, c_vp, c_i64, c_vp]),
    "ppgat_xgat_weight_grads": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "ppgat_stream_copy": (c_int, [c_vp, c_vp, c_i64, c_vp]),
    "ppgat_debug_build": (c_int, []),
    "ppgat_check_index_range": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, ctypes.POINTER(c_i64), c_vp]),
    "ppgat_profile_enable": (c_int, [c_int]),
    "ppgat_profile_reset": (c_int, []),
    "ppgat_profile_read": (c_int, [c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_i64)]),
}

KERNELS = {"csr": 0, "scores": 1, "fwd": 2, "bwd_pro": 3, "bwd_src": 4, "bwd_epi": 5, "bwd_red": 6, "sched": 7,
           "gemm_tn": 8, "fusion": 9, "proj": 10, "adam": 11,
           "sample": 12, "infonce": 13, "proj_bwd": 14}
MODE_PYG, MODE_CUSTOM = 0, 1

_lib = None
_load_error = None


def load(path: Path = None):
    """Load (once) and return the ctypes library; raise RuntimeError if unavailable.

    torch must be imported first so the already-loaded HIP runtime
    (soname libamdhip64.so.7) is shared with torch's streams and allocator.
    """
    global _lib, _load_error
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (HIP runtime first)
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        _load_error = f"libppgat.so not found at {p}; build it first (make -C {_HERE / 'csrc'})"
        raise RuntimeError(_load_error)
    try:
        lib = ctypes.CDLL(str(p))
    except OSError as e:  # pragma: no cover
        _load_error = f"failed to load {p}: {e}"
        raise RuntimeError(_load_error) from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.ppgat_last_error().decode() if _lib is not None else "library not loaded"
        if rc == 2:
            raise NotImplementedError(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_handle(device) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def debug_build() -> bool:
    """True when the loaded library is libppgat_debug.so (PPGAT_LIB=.../libppgat_debug.so)."""
    return bool(load().ppgat_debug_build())


def check_index_range(t, lo: int, hi: int, what: str):
    """Raise if any entry of the int32/int64 device tensor t is outside [lo, hi)
    (ppgat_check_index_range; synchronises).  The debug build's graph/plan validation."""
    import torch
    lib = load()
    if t is None or t.numel() == 0:
        return
    if t.dtype not in (torch.int32, torch.int64) or not t.is_cuda or not t.is_contiguous():
        raise RuntimeError(f"check_index_range({what}): contiguous int32/int64 device tensor required")
    n_bad = ctypes.c_int64(0)
    check(lib.ppgat_check_index_range(t.data_ptr(), t.element_size(), t.numel(), int(lo), int(hi), ctypes.byref(n_bad),
                                      stream_handle(t.device)), "check_index_range")
    if n_bad.value:
        raise RuntimeError(f"{what}: {n_bad.value} of {t.numel()} indices outside [{lo}, {hi})")


def profile_enable(on: bool = True):
    lib = load()
    check(lib.ppgat_profile_enable(1 if on else 0), "profile_enable")


def profile_reset():
    lib = load()
    check(lib.ppgat_profile_reset(), "profile_reset")


def profile_read(kernel: str):
    lib = load()
    ms = ctypes.c_double(0.0)
    n = ctypes.c_int64(0)
    check(lib.ppgat_profile_read(KERNELS[kernel], ctypes.byref(ms), ctypes.byref(n)), "profile_read")
    return ms.value, n.value


def dropout_advance(device=None):
    """Enqueue the dropout-epoch increment (include/ppgat.h ppgat_dropout_advance) on the
    current stream: call once at the top of a training step that is captured in a graph."""
    import torch
    lib = load()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    check(lib.ppgat_dropout_advance(stream_handle(dev)), "dropout_advance")


def dropout_set_epoch(epoch: int, device=None):
    import torch
    lib = load()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    check(lib.ppgat_dropout_set_epoch(int(epoch) & (2**64 - 1), stream_handle(dev)), "dropout_set_epoch")
