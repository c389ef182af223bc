"""ctypes binding of libniidmix.so (the C-ABI in include/niidmix.h).

This is the same stub a maintainer would add to the reference.  There is NO CPU
fallback: if the HIP library is missing the import fails loudly.

torch is imported first on purpose: torch ships its own libamdhip64.so (SONAME libamdhip64.so.7);
once it is loaded, the dynamic loader binds libniidmix.so to that same HIP runtime, so device
pointers and hipStream_t handles coming from torch are valid in our calls.
"""
import ctypes
import os

import torch  # noqa: F401  (must be loaded before libniidmix.so, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NIIDMIX_LIB") or os.path.join(_HERE, "libniidmix.so")

OK, EINVAL, EALIAS, EHIP, EUNSUPPORTED = 0, 1, 2, 3, 4
MODE_EXACT, MODE_FAST = 0, 1
ABI_VERSION = 5

_i64, _i32, _vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p


class CliquePlanC(ctypes.Structure):
    """Mirror of struct niidmix_clique_plan (include/niidmix.h)."""
    _fields_ = [("n_cliques", _i32), ("n_members", _i32), ("n_groups", _i32), ("max_clique", _i32),
                ("max_clique_res", _i32), ("clique_ptr", _vp), ("member_row", _vp), ("member_group", _vp), ("coef", _vp),
                ("res_ptr", _vp), ("res_col", _vp), ("res_val", _vp), ("res_member", _vp),
                ("csr_ptr", _vp), ("csr_col", _vp), ("csr_val", _vp)]


class TilePlanC(ctypes.Structure):
    """Mirror of struct niidmix_tile_plan (include/niidmix.h)."""
    _fields_ = [("n_sub", _i64), ("rt", _i32), ("reserved", _i32), ("sub_ptr", _vp), ("sub_rows", _vp),
                ("sub_wself", _vp), ("pos_src", _vp), ("pos_mask", _vp), ("pos_w", _vp)]


class TileLdsPlanC(ctypes.Structure):
    """Mirror of struct niidmix_tile_lds_plan (include/niidmix.h)."""
    _fields_ = [("n_sub", _i64), ("rt", _i32), ("n_grp", _i32), ("max_src", _i32), ("max_tiles", _i32),
                ("sub_ptr", _vp), ("sub_rows", _vp), ("sub_slot", _vp), ("sub_wself", _vp),
                ("pos_slot", _vp), ("pos_mask", _vp), ("pos_w", _vp), ("grp_tile_ptr", _vp),
                ("grp_src_ptr", _vp), ("grp_src_rows", _vp), ("seg_ptr", _vp), ("seg", _vp),
                ("seg_w", _vp), ("mf_ptr", _vp), ("mf", _vp), ("rem_rows", _vp),
                ("rem_regs", ctypes.c_int32)]


class ShardC(ctypes.Structure):
    """Mirror of struct niidmix_shard (include/niidmix.h)."""
    _fields_ = [("device", _i32), ("n_peers", _i32), ("n_local", _i64), ("rows_in", _i64),
                ("x", _vp), ("y", _vp), ("row_ptr", _vp), ("col", _vp), ("val", _vp),
                ("peer", _vp), ("send_ptr", _vp), ("send_rows", _vp), ("send_buf", _vp),
                ("recv_row", _vp), ("recv_count", _vp), ("stream", _vp)]


# every symbol include/niidmix.h declares, with its ctypes signature
SIGNATURES = {
    "niidmix_abi_version": (ctypes.c_int, []),
    "niidmix_last_error": (ctypes.c_char_p, []),
    "niidmix_mix_csr_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp,
                                           ctypes.c_int, _vp]),
    "niidmix_mix_ell_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, ctypes.c_int, _vp, _vp,
                                           _vp, ctypes.c_int, _vp]),
    "niidmix_mix_band_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, ctypes.c_int,
                                            ctypes.c_int, _vp, _vp, _vp, ctypes.c_int, _vp]),
    "niidmix_mix_strip_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, ctypes.c_int, _vp,
                                             _vp, _vp, ctypes.c_int, _vp]),
    "niidmix_mix_clique_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64,
                                              ctypes.POINTER(CliquePlanC), _vp]),
    "niidmix_mix_clique_blocked_f32": (ctypes.c_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64,
                                                      ctypes.POINTER(CliquePlanC), _vp]),
    "niidmix_mix_tile_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64,
                                            ctypes.POINTER(TilePlanC), ctypes.c_int, _vp]),
    "niidmix_mix_tile_lds_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64,
                                                ctypes.POINTER(TileLdsPlanC), ctypes.c_int, _vp]),
    "niidmix_mix_dense_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp,
                                             _vp, _vp]),
    "niidmix_dense_split_elems": (_i64, [_i64]),
    "niidmix_dense_split_w": (ctypes.c_int, [_vp, _i64, _vp, _vp]),
    "niidmix_mix_dense_bf16x6_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp,
                                                    _vp, _vp]),
    "niidmix_mean_rows_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, ctypes.c_int, _vp]),
    "niidmix_grad_segment_mean_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp,
                                                     _vp, _vp]),
    "niidmix_grad_segment_mean_blocked_f32": (ctypes.c_int, [_vp, _vp, _i64, _i64, _i64, _i64,
                                                             _i64, _i64, _i64, _vp, _vp, _vp]),
    "niidmix_update_rows_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp]),
    "niidmix_sgd_step_rows_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _vp, _i64,
                                                 ctypes.c_float, _vp]),
    "niidmix_sharded_create": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.POINTER(_vp)]),
    "niidmix_sharded_destroy": (ctypes.c_int, [_vp]),
    "niidmix_sharded_is_loopback": (ctypes.c_int, [_vp]),
    "niidmix_mix_sharded_f32": (ctypes.c_int, [_vp, ctypes.POINTER(ShardC), _i64, ctypes.c_int]),
    "niidmix_hbm_alloc": (ctypes.c_void_p, [ctypes.c_ssize_t, ctypes.c_int, _vp]),
    "niidmix_hbm_free": (None, [_vp, ctypes.c_ssize_t, ctypes.c_int, _vp]),
    "niidmix_copy2d_async": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, ctypes.c_int, _vp]),
    "niidmix_stream_copy_f32": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
}


def lib_sha16(path=None):
    """First 16 hex digits of the SHA-256 of the loaded library: identifies the kernels a
    measurement (e.g. a PMC traffic entry in profiles/traffic.json) was taken with."""
    import hashlib
    with open(path or LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


class NiidmixError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libniidmix.so not found at {LIB_PATH}: build it with `python -m niidmix.build` "
            "(or __graft_entry__.build()); there is no CPU fallback for the mixing kernels")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.niidmix_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"libniidmix.so ABI {v} != expected {ABI_VERSION}; rebuild it")
    return lib


lib = _load()


def check(rc, what=""):
    if rc != OK:
        msg = lib.niidmix_last_error().decode(errors="replace")
        raise NiidmixError(f"{what}: niidmix error {rc}: {msg}")
