"""ctypes binding of the C ABI in include/pcfm.h (libpcfm_hip.so, gfx950).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
point-cloud-flow-matching_amd/csrc``).  Nothing here falls back: if the
library is missing, every op on a HIP tensor raises.  (CPU tensors never reach
this module -- pcfm.ops sends them to the pure-PyTorch pcfm.cpu_ops.)
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "csrc", "libpcfm_hip.so")
# PCFM_LIB: load a measurement variant built by `make variant` (dev knob)
LIB_PATH = os.environ.get("PCFM_LIB", LIB_PATH)

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_Z = ctypes.c_size_t
_L = ctypes.c_longlong
_D = ctypes.c_double
_DP = ctypes.POINTER(ctypes.c_double)  # host array

# name -> (restype, argtypes); must list every symbol of include/pcfm.h.
SIGNATURES = {
    "pcfm_abi_version": (_I, []),
    "pcfm_last_error": (ctypes.c_char_p, []),
    "pcfm_avg_voxelize_fwd_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_avg_voxelize_fwd": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _Z, _P]),
    "pcfm_avg_voxelize_bwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "pcfm_trilinear_devoxelize_fwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "pcfm_trilinear_devoxelize_bwd_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_trilinear_devoxelize_bwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_ball_query": (_I, [_P, _P, _I, _I, _I, _F, _I, _P, _P]),
    "pcfm_grouping_fwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "pcfm_grouping_bwd_workspace_bytes": (_Z, [_I, _I, _I, _I, _I]),
    "pcfm_grouping_bwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_chamfer_workspace_bytes": (_Z, [_I, _I, _I]),
    "pcfm_chamfer_fwd": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _Z, _P]),
    "pcfm_chamfer_bwd": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "pcfm_emd_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_emd_approxmatch_f32": (_I, [_P, _P, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_emd_approxmatch_f64": (_I, [_P, _P, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_emd_approxmatch_cost_f32": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _Z, _P]),
    "pcfm_emd_approxmatch_cost_f64": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _Z, _P]),
    "pcfm_emd_matchcost_f32": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_emd_matchcost_f64": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_emd_matchcost_bwd_f32": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _Z, _P]),
    "pcfm_emd_matchcost_bwd_f64": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _Z, _P]),
    "pcfm_conv3d_weight_bytes": (_Z, [_I, _I]),
    "pcfm_conv3d_prep_weight": (_I, [_P, _I, _I, _I, _P, _P]),
    "pcfm_conv3d_supported": (_I, [_I, _I, _I, _I]),
    "pcfm_conv3d_igemm": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_conv3d_igemm_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_conv3d_split_bytes": (_Z, [_I, _I, _I]),
    "pcfm_conv3d_split": (_I, [_P, _I, _I, _I, _P, _P]),
    "pcfm_conv3d_igemm_cl_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_conv3d_igemm_cl": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_conv3d_wgrad_cl": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_conv3d_occupancy_bytes": (_Z, [_I, _I]),
    "pcfm_conv3d_occupancy": (_I, [_P, _I, _I, _P, _P]),
    "pcfm_conv3d_igemm_cl_occ": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P, _Z, _P]),
    "pcfm_conv3d_vlist_bytes": (_Z, [_I, _I]),
    "pcfm_conv3d_vlist": (_I, [_P, _I, _I, _P, _P]),
    "pcfm_conv3d_igemm_cl_list": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _I, _P, _P, _Z, _P]),
    "pcfm_conv3d_wgrad_occ_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_conv3d_wgrad_cl_occ": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _Z, _P]),
    "pcfm_conv3d_wgrad_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_conv3d_wgrad": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_pointwise_weight_bytes": (_Z, [_I, _I]),
    "pcfm_pointwise_prep_weight": (_I, [_P, _I, _I, _I, _P, _P]),
    "pcfm_pointwise_gemm": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "pcfm_pointwise_wgrad_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_pointwise_wgrad": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_trilinear_devoxelize_scale_add_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P,
                                                     _P, _P]),
    "pcfm_debug_devox_verify": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "pcfm_se_mlp_fwd": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "pcfm_se_mlp_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P, _P, _P, _P]),
    "pcfm_trilinear_devoxelize_bn_scale_add_fwd": (_I, [_P, _P, _P, _P, _P, _P, _F, _P, _P, _P,
                                                       _P, _P, _P, _F, _I, _I, _I, _I, _I, _P,
                                                       _P, _P, _P]),
    "pcfm_bn_fwd_stats": (_I, [_P, _P, _I, _I, _I, _I, _F, _F, _P, _P, _P, _P, _P, _P, _Z, _P]),
    "pcfm_bn_act_fwd_rowmean_workspace_bytes": (_Z, [_I, _I, _I]),
    "pcfm_bn_act_fwd_rowmean": (_I, [_P, _P, _P, _I, _I, _I, _F, _F, _F, _P, _P, _P, _P, _P, _P,
                                     _P, _Z, _P]),
    "pcfm_bn_se_bwd_workspace_bytes": (_Z, [_I, _I, _I]),
    "pcfm_bn_se_bwd_stats": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P, _P, _Z, _P]),
    "pcfm_bn_se_bwd_apply_split": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P,
                                        _P, _P, _P, _P, _Z, _P]),
    "pcfm_rows_dot": (_I, [_P, _P, _L, _I, _F, _P, _P]),
    "pcfm_rows_affine": (_I, [_P, _P, _P, _L, _I, _P]),
    "pcfm_rows_colsum_workspace_bytes": (_Z, [_I, _L, _I]),
    "pcfm_rows_colsum": (_I, [_P, _I, _I, _L, _I, _P, _P, _Z, _P]),
    "pcfm_avg_voxelize_bwd_add": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "pcfm_gn_silu_fwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _F, _P, _P, _P, _P, _Z, _P]),
    "pcfm_gn_silu_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _Z, _P]),
    "pcfm_tgate_fwd": (_I, [_P, _P, _P, _I, _I, _I, _P, _P]),
    "pcfm_tgate_bwd": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "pcfm_pointwise_gemm_parts": (_I, [_I, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "pcfm_pointwise_wgrad_parts": (_I, [_I, _P, _P, _P, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_rows_wgrad_workspace_bytes": (_Z, [_L, _I, _I]),
    "pcfm_rows_wgrad_bf16": (_I, [_P, _I, _P, _I, _L, _I, _I, _P, _P, _Z, _P]),
    "pcfm_rows_max_workspace_bytes": (_Z, [_I, _I, _I]),
    "pcfm_rows_max_bf16": (_I, [_P, _I, _I, _I, _P, _P, _P, _Z, _P]),
    "pcfm_head_film_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P, _P, _P,
                                   _P, _P]),
    "pcfm_head_silu_fwd": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "pcfm_head_bwd_workspace_bytes": (_Z, [_I, _I, _I]),
    "pcfm_head_film_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I,
                                   _P, _P, _P, _P, _P, _P, _P, _P, _P, _Z, _P]),
    "pcfm_head_silu_bwd": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _Z, _P]),
    "pcfm_bn_workspace_bytes": (_Z, [_I, _I, _I]),
    "pcfm_bn_act_fwd": (_I, [_P, _P, _P, _I, _I, _I, _F, _F, _F, _P, _P, _P, _P, _P, _P, _P,
                             _Z, _P]),
    "pcfm_pointwise_bnstats_groups": (_I, [_I, _I, _I, _I]),
    "pcfm_pointwise_gemm_bnstats": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "pcfm_bn_act_fwd_parts": (_I, [_P, _P, _I, _P, _P, _I, _I, _I, _F, _F, _F, _P, _P, _P, _P,
                                   _P, _P, _P]),
    "pcfm_bn_act_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P, _P, _P, _P, _P, _Z,
                             _P]),
    "pcfm_bn_act_fwd_split": (_I, [_P, _P, _P, _I, _I, _I, _F, _F, _F, _P, _P, _P, _P, _P, _P,
                                   _P, _Z, _P]),
    "pcfm_bn_act_bwd_split_workspace_bytes": (_Z, [_I, _I, _I]),
    "pcfm_bn_act_bwd_split": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P, _P, _P, _P, _P,
                                   _Z, _P]),
    "pcfm_gn_film_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_gn_film_res_fwd": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _P, _P, _P, _P, _Z,
                                  _P]),
    "pcfm_gn_film_res_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P,
                                  _P, _P, _Z, _P]),
    "pcfm_debug_devox_verify_bn": (_I, [_P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P, _P, _F,
                                        _P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "pcfm_gn_film_res_fwd_bnin": (_I, [_P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _I, _I, _I, _I,
                                       _F, _P, _P, _P, _P, _Z, _P]),
    "pcfm_gn_bnin_parts": (_I, [_I, _I]),
    "pcfm_gn_film_res_bwd_bnin": (_I, [_P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P, _I, _I,
                                       _I, _I, _P, _P, _P, _P, _P, _P, _P, _Z, _P]),
    "pcfm_bn_act_bwd_apply_parts": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _P, _P,
                                         _P, _P, _P, _Z, _P]),
    "pcfm_seg_plan_bytes": (_Z, [_I, _I, _I, _I]),
    "pcfm_seg_apply_workspace_bytes": (_Z, [_I, _I, _I, _I, _I]),
    "pcfm_avg_voxelize_plan": (_I, [_P, _I, _I, _I, _P, _P, _P, _Z, _P]),
    "pcfm_avg_voxelize_fwd_planned": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_trilinear_devoxelize_bwd_plan": (_I, [_P, _P, _I, _I, _I, _P, _Z, _P]),
    "pcfm_trilinear_devoxelize_bwd_planned": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _Z, _P]),
    "pcfm_adamw_chunk_elems": (_I, []),
    "pcfm_adamw_workspace_bytes": (_Z, [_I]),
    "pcfm_adamw_grad_norm": (_I, [_P, _I, _P, _I, _P, _F, _P, _P, _P, _Z, _P]),
    "pcfm_adamw_ema_step": (_I, [_P, _P, _I, _P, _P, _I, _DP, _DP, _D, _D, _D, _D, _P]),
}

ABI_VERSION = 20

_lock = threading.Lock()
_lib = None


class PcfmError(RuntimeError):
    """A pcfm_* entry point returned a non-zero status."""


def load() -> ctypes.CDLL:
    """Load libpcfm_hip.so once and declare every signature.  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"pcfm: HIP library {LIB_PATH} is not built; run "
                    "`python -c 'import __graft_entry__ as g; g.build()'` "
                    "(HIP tensors have no fallback)")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            v = lib.pcfm_abi_version()
            if v != ABI_VERSION:
                raise RuntimeError(f"pcfm: ABI version {v} != expected {ABI_VERSION}; rebuild")
            _lib = lib
    return _lib


def call(name: str, *args) -> None:
    """Call pcfm_<name>; raise PcfmError with the library's message on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.pcfm_last_error().decode(errors="replace")
        raise PcfmError(f"{name} failed (status {rc}): {msg}")


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))
