"""ctypes binding of ``libwats_hip.so`` (C ABI: ``include/wats_hip.h``).

The library is built in-tree by ``make -C efficient-gnn_amd/csrc`` (or
``__graft_entry__.build()``).  There is no fallback: if the library is missing
or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# WATS_HIP_LIB selects an experimental build (csrc/Makefile VARIANT=...) for A/B timing.
LIB_PATH = os.environ.get("WATS_HIP_LIB") or os.path.join(_HERE, "libwats_hip.so")

WG_FLAG_NONE = 0
WG_FLAG_NO_REORDER = 1
WG_FLAG_TRANSPOSE = 2
WG_FLAG_KEEP_COLUMN_ORDER = 4

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_u32 = ctypes.c_uint32
c_f64 = ctypes.c_double
c_vp = ctypes.c_void_p


class LaplacianInfo(ctypes.Structure):
    _fields_ = [
        ("n_rows", c_i64),
        ("n_cols", c_i64),
        ("nnz_input", c_i64),
        ("nnz", c_i64),
        ("n_isolated", c_i64),
        ("max_row_nnz", c_i64),
        ("n_segments", c_i32),
        ("reordered", c_i32),
        ("n_closed_form", c_i64),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


# name -> (restype, argtypes); every symbol declared in include/wats_hip.h
SIGNATURES = {
    "wg_last_error": (ctypes.c_char_p, []),
    "wg_abi_version": (ctypes.c_int, []),
    "wg_dense_to_csr_count": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, ctypes.POINTER(c_i64), c_vp]),
    "wg_dense_to_csr_fill": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "wg_column_degree": (ctypes.c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wg_laplacian_create": (ctypes.c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_u32, c_vp,
                                           ctypes.POINTER(c_vp)]),
    "wg_operator_create": (ctypes.c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_u32, c_vp, ctypes.POINTER(c_vp)]),
    "wg_laplacian_destroy": (ctypes.c_int, [c_vp]),
    "wg_laplacian_get_info": (ctypes.c_int, [c_vp, ctypes.POINTER(LaplacianInfo)]),
    "wg_laplacian_export": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wg_log1p_degree": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "wg_cheb_step": (ctypes.c_int, [c_vp, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_f64, c_f64, c_vp]),
    "wg_permute_rows": (ctypes.c_int, [c_vp, c_i32, c_i64, c_vp, c_vp, c_vp]),
    "wg_wavelet_features": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_f64, c_vp, c_vp, c_vp]),
    "wg_laplacian_tune": (ctypes.c_int, [c_vp, ctypes.c_char_p, c_i64]),
    "wg_laplacian_describe": (ctypes.c_char_p, [c_vp, c_i64]),
    "wg_laplacian_set_halo_groups": (ctypes.c_int, [c_vp, c_i32, c_vp]),
    "wg_profile_enable": (ctypes.c_int, [c_vp, c_i32]),
    "wg_profile_durations": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double), c_i64, ctypes.POINTER(c_i64)]),
    "wg_profile_collect": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_i64),
                                          ctypes.POINTER(ctypes.c_double)]),
    "wg_row_l1_normalize": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_vp]),
    "wg_laplacian_map_rows": (ctypes.c_int, [c_vp, c_i32, c_vp, c_i64, c_vp, c_vp]),
    "wg_gather_rows": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "wg_cheb_u_len": (ctypes.c_int, [c_vp, ctypes.POINTER(c_i64)]),
    "wg_scale_dinv": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    "wg_lds_plan_info": (ctypes.c_int, [c_vp, c_i32, ctypes.POINTER(c_i64)]),
    "wg_cheb_step_u": (ctypes.c_int, [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f64, c_f64, c_vp]),
    "wg_clenshaw_step": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f64, c_f64, c_i32, c_vp]),
    "wg_rownorm_create": (ctypes.c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_u32, c_vp, ctypes.POINTER(c_vp)]),
    "wg_spmm": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    "wg_wats_head_forward": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i32] + [c_vp] * 8 + [c_vp]),
    "wg_wats_head_workspace": (ctypes.c_int, [c_i64, c_i64, c_i32, ctypes.POINTER(c_i64)]),
    "wg_wats_head_backward": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i32] + [c_vp] * 15 + [c_vp]),
    "wg_dist_unique_id": (ctypes.c_int, [c_vp]),
    "wg_dist_create": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, ctypes.POINTER(c_vp)]),
    "wg_dist_destroy": (ctypes.c_int, [c_vp]),
    "wg_dist_set_graph": (ctypes.c_int, [c_vp, c_i32]),
    "wg_dist_wavelet_features": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_f64, c_vp, c_vp, c_vp]),
    "wg_dist_info": (ctypes.c_int, [c_vp, ctypes.POINTER(c_i64)]),
    "wg_dist_profile_collect": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_i64)]),
    "wg_dist_ipc_local": (ctypes.c_int, [c_vp, c_i64, c_vp]),
    "wg_dist_ipc_connect": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "wg_dist_ipc_sdma": (ctypes.c_int, [c_vp, c_vp]),
    "wg_dist_status": (ctypes.c_int, [c_vp, ctypes.POINTER(c_i32)]),
    "wg_chain_status": (ctypes.c_int, [c_vp, ctypes.POINTER(c_i32)]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and type the HIP library; raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"wats_hip: HIP library not found at {LIB_PATH}; build it with "
            "`make -C efficient-gnn_amd/csrc` (there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class WaveletError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().wg_last_error()
        raise WaveletError(f"wats_hip{(' ' + what) if what else ''}: status {rc}: "
                           f"{msg.decode() if msg else '?'}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()
