"""ctypes binding of libcnnitmo.so (include/cnn_itmo.h).

The product path has exactly one implementation: the HIP kernels in this
library.  If the library is missing or a call fails, we raise -- there is no
CPU or PyTorch fallback.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CNNITMO_LIB") or os.path.join(HERE, "lib", "libcnnitmo.so")  # override: experiments

F32 = 0
BF16 = 1
RELU = 1
STATS = 2
AFFINE = 4
DROPOUT = 1
NO_BN = 2
PARITY = 4
BIAS_PER_COL = 8
CONSUMER_ROWS = 64

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_long
f32 = C.c_float
f64 = C.c_double
u64 = C.c_uint64
sz = C.c_size_t

# name -> (restype, argtypes).  Mirrors include/cnn_itmo.h exactly.
SIGNATURES = {
    "cnnitmo_version": (i32, []),
    "cnnitmo_consumer_rows": (i32, []),
    "cnnitmo_last_error": (C.c_char_p, []),
    "cnnitmo_augment_affine": (i32, [i32, vp, i32, i32, i32, i32, vp, vp, f32, vp, vp]),
    "cnnitmo_tonemap_workspace_bytes": (sz, [i32]),
    "cnnitmo_tonemap_stats": (i32, [i32, vp, i32, i32, i32, vp, vp, vp, sz, vp]),
    "cnnitmo_tonemap_apply": (i32, [i32, vp, i32, i32, i32, vp, vp, vp, i32, vp, vp]),
    "cnnitmo_inverse_reinhard_apply": (i32, [i32, vp, i32, i32, i32, vp, vp, f64, f64, vp, vp]),
    "cnnitmo_conv3x3_fwd": (i32, [i32, vp, i32, i32, i32, i32, i32, i32, vp, vp, i32, vp, i32, i32, i32, vp, vp, vp, vp, vp]),
    "cnnitmo_conv3x3_fwd_cat": (i32, [i32, vp, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, vp, vp, i32, vp, i32,
                                      i32, i32, vp, vp, vp, vp, vp]),
    "cnnitmo_conv3x3_fwd_cat_supported": (i32, [i32] * 7),
    "cnnitmo_conv3x3_fwd_pool": (i32, [i32, vp, i32, i32, i32, i32, i32, i32, vp, vp, i32, vp, i32, i32, i32, vp, vp, vp,
                                       vp, vp, i32, vp, vp, vp]),
    "cnnitmo_conv3x3_pool_supported": (i32, [i32] * 6),
    "cnnitmo_conv3x3_fwd_head": (i32, [i32, vp, i32, i32, i32, i32, i32, i32, vp, vp, i32, i32, vp, vp, i32, vp, vp,
                                       vp, vp]),
    "cnnitmo_conv3x3_head_supported": (i32, [i32] * 6),
    "cnnitmo_pool_bnsums_pooled": (i32, [i32, vp, vp, i32, i32, i32, i32, vp, vp, vp, vp]),
    "cnnitmo_wgrad_cat_workspace_bytes": (sz, [i32, i32, i32, i32, i32, i32]),
    "cnnitmo_wgrad_cat_kernel_name": (C.c_char_p, [i32, i32, i32, i32, i32, i32]),
    "cnnitmo_conv_wgrad_cat": (i32, [i32, vp, i32, i32, i32, vp, i32, i32, vp, i32, i32, i32, i32, i32, vp, vp, vp,
                                     vp, vp, vp, vp, sz, vp]),
    "cnnitmo_fwd_stat_rows": (i32, [i32, i64, i32]),
    "cnnitmo_tconv2x2_dgrad_bn_rows": (i64, [i32, i32, i32, i32, i32, i32]),
    "cnnitmo_tconv2x2_dgrad_bn": (i32, [i32, vp, i32, i32, i32, i32, vp, i32, vp, vp, i32, i32, vp, vp, vp]),
    "cnnitmo_conv3x3_dgrad_bn_rows": (i64, [i32, i32, i32, i32, i32, i32, i32, i32]),
    "cnnitmo_conv3x3_dgrad_bn": (i32, [i32, vp, i32, i32, i32, i32, vp, i32, vp, i32, i32, i32, i32, vp, vp, i32,
                                       i32, vp, vp, i32, vp]),
    "cnnitmo_conv3x3_dgrad_bn_pooled_rows": (i64, [i32] * 6),
    "cnnitmo_conv3x3_dgrad_bn_pooled": (i32, [i32, vp, i32, i32, i32, i32, vp, i32, vp, vp, i32, i32, vp, vp, vp,
                                              vp, vp]),
    "cnnitmo_conv3x3_dgrad_bn_pooled_kernel_name": (C.c_char_p, [i32] * 6),
    "cnnitmo_conv3x3_dgrad": (i32, [i32, vp, i32, i32, i32, i32, vp, i32, vp, i32, i32, vp]),
    "cnnitmo_wgrad_workspace_bytes": (sz, [i32, i32, i32, i32, i32, i32, i32]),
    "cnnitmo_conv_wgrad": (i32, [i32, i32, vp, i32, i32, vp, i32, i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, vp, sz, vp]),
    "cnnitmo_im2col_c3": (i32, [i32, vp, i32, i32, i32, i32, vp, vp]),
    "cnnitmo_conv_c3_stat_rows": (i64, [i32, i32, i32]),
    "cnnitmo_bn_bwd_apply_g3": (i32, [i32, vp, vp, vp, i32, i32, i64, i32, vp, vp, vp, vp]),
    "cnnitmo_head_fwd_bwd_g3": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, f64, vp]),
    "cnnitmo_conv_c3_fwd": (i32, [i32, vp, i32, i32, i32, i32, vp, vp, vp, i32, i32, i32, vp, vp, vp, vp]),
    "cnnitmo_conv_c3_wgrad_workspace_bytes": (sz, [i32, i32, i32]),
    "cnnitmo_conv_c3_wgrad": (i32, [i32, vp, i32, i32, i32, i32, vp, vp, vp, sz, vp]),
    "cnnitmo_conv1tap_fwd": (i32, [i32, vp, i32, i64, vp, vp, i32, vp, i32, i32, i32, vp, vp, vp, vp]),
    "cnnitmo_tconv2x2_fwd": (i32, [i32, vp, i32, i32, i32, i32, vp, vp, i32, vp, i32, i32, i32, vp, vp, vp, vp]),
    "cnnitmo_tconv2x2_dgrad": (i32, [i32, vp, i32, i32, i32, i32, vp, i32, vp, vp]),
    "cnnitmo_tconv2x2_wgrad": (i32, [i32, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, sz, vp]),
    "cnnitmo_tconv2x2_wgrad_workspace_bytes": (sz, [i32, i32, i32, i32, i32, i32]),
    "cnnitmo_prep_conv3x3_weights": (i32, [i32, vp, i32, i32, vp, vp, vp]),
    "cnnitmo_prep_tconv2x2_weights": (i32, [i32, vp, i32, i32, vp, vp, vp]),
    "cnnitmo_prep_c3_weights": (i32, [i32, vp, i32, vp, vp]),
    "cnnitmo_maxpool2x2_fwd": (i32, [i32, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp]),
    "cnnitmo_maxpool2x2_bwd": (i32, [i32, vp, vp, i32, i32, i32, i32, vp, i32, i32, vp]),
    "cnnitmo_reduce_workspace_bytes": (sz, [i64, i32]),
    "cnnitmo_bn_fwd_finalize": (i32, [vp, i64, i32, i32, f64, vp, vp, vp, vp, f32, f32, vp, vp, vp, vp, vp, vp]),
    "cnnitmo_bn_infer_coeffs": (i32, [i32, vp, vp, vp, vp, f32, vp, vp, vp]),
    "cnnitmo_bn_apply": (i32, [i32, vp, i64, i32, vp, vp, vp, i32, i32, i32, u64, i32, vp]),
    "cnnitmo_bn_bwd_rows": (i32, [i64, i32]),
    "cnnitmo_bn_bwd_reduce": (i32, [i32, vp, i32, i32, vp, i32, i32, i64, i32, vp, vp, i32, u64, i32, vp, vp]),
    "cnnitmo_bn_bwd_finalize": (i32, [vp, i64, i32, f64, vp, vp, vp, vp, vp, vp, vp, vp]),
    "cnnitmo_bn_bwd_apply": (i32, [i32, vp, i32, i32, vp, i32, i32, i64, i32, vp, i32, u64, i32, i32, i32, vp, vp, vp]),
    "cnnitmo_colsum": (i32, [vp, i64, i32, i32, vp, vp, vp]),
    "cnnitmo_head_fwd": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp]),
    "cnnitmo_head_rows": (i32, [i64]),
    "cnnitmo_head_fwd_bwd": (i32, [i32, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, f64, vp]),
    "cnnitmo_head_finalize": (i32, [vp, i64, i32, f64, vp, vp, vp, vp, vp, vp, vp, vp]),
    "cnnitmo_bn_consumer_sums": (i32, [i32, vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp]),
    "cnnitmo_pool_bnsums": (i32, [i32, vp, vp, i32, i32, i32, i32, vp, i32, i32, vp, vp, vp, vp]),
    "cnnitmo_bn_bwd_apply_pooled": (i32, [i32, vp, i32, i32, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp,
                                          vp, vp]),
    "cnnitmo_fold_conv3x3": (i32, [i32, vp, vp, vp, vp, i32, i32, vp, vp, vp, vp]),
    "cnnitmo_fold_tconv2x2": (i32, [i32, vp, vp, vp, vp, i32, i32, vp, vp, vp]),
    "cnnitmo_border_rows": (i32, [i32]),
    "cnnitmo_conv3x3_stat_rows": (i64, [i32, i32, i32, i32, i32, i32]),
    "cnnitmo_tconv2x2_stat_rows": (i64, [i32, i32, i32, i32, i32, i32]),
    "cnnitmo_conv3x3_kernel_name": (C.c_char_p, [i32, i32, i32, i32, i32, i32, i32]),
    "cnnitmo_wgrad_kernel_name": (C.c_char_p, [i32, i32, i32, i32, i32, i32, i32]),
    "cnnitmo_tconv2x2_kernel_name": (C.c_char_p, [i32, i32, i32, i32, i32, i32, i32]),
    "cnnitmo_conv3x3_dgrad_bn_kernel_name": (C.c_char_p, [i32] * 8),
    "cnnitmo_tconv2x2_dgrad_bn_kernel_name": (C.c_char_p, [i32] * 6),
    "cnnitmo_border_sums": (i32, [i32, vp, i32, i32, i32, i32, vp, vp]),
    "cnnitmo_rmsprop": (i32, [vp, vp, vp, i64, f32, f32, f32, f32, vp]),
}


class CnnItmoError(RuntimeError):
    pass


_lib = None


def load(path: str | None = None):
    """Load libcnnitmo.so and bind every symbol; raises if anything is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise CnnItmoError(
            f"libcnnitmo.so not found at {p}: build it with `python -m cnn_itmo_amd.build` "
            "(there is no CPU fallback)")
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the export is missing
        fn.restype = res
        fn.argtypes = args
    if lib.cnnitmo_consumer_rows() != CONSUMER_ROWS:  # a compile-time sizing constant of the ABI
        raise CnnItmoError(f"{p}: built with {lib.cnnitmo_consumer_rows()} consumer-sum rows, "
                           f"the binding sizes {CONSUMER_ROWS} (cnnitmo_version {lib.cnnitmo_version()})")
    if path is None:
        _lib = lib
    return lib


def call(name: str, *args):
    """Invoke a status-returning entry point; raise CnnItmoError on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.cnnitmo_last_error().decode(errors="replace")
        raise CnnItmoError(f"{name} failed ({rc}): {msg}")
    return rc


def query(name: str, *args):
    return getattr(load(), name)(*args)
