"""ctypes binding of libdauc.so — the C ABI declared in include/dauc.h.

The product path has exactly one implementation: the gfx950 HIP kernels in
this library. If the library is missing or cannot be loaded this module raises
immediately; there is no CPU fallback anywhere in ``distributedauc_amd``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import re
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("DAUC_LIB", PKG_DIR / "libdauc.so"))
HEADER = PKG_DIR.parent / "include" / "dauc.h"

DAUC_OK = 0
DAUC_EINVAL = -100000
LABEL_I8, LABEL_I32, LABEL_I64 = 1, 2, 3
DTYPE_F32, DTYPE_BF16 = 1, 2
MODE_REFERENCE, MODE_PAPER = 0, 1


class DaucError(RuntimeError):
    """A libdauc.so call returned a non-zero status."""


class GradSeg(ctypes.Structure):
    """dauc_grad_seg: one parameter's gradient and its offset in the flat buffer."""

    _fields_ = [("grad", ctypes.c_void_p), ("offset", ctypes.c_int64), ("numel", ctypes.c_int64)]


_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_f32 = ctypes.c_float
_sz = ctypes.c_size_t

# name -> (restype, argtypes); must list every function include/dauc.h declares
SIGNATURES = {
    "dauc_version": (_int, []),
    "dauc_strerror": (ctypes.c_char_p, [_int]),
    "dauc_label_map_phat": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp]),
    "dauc_surrogate_workspace_size": (_sz, [_i64]),
    "dauc_surrogate_fwdbwd": (_int, [_vp, _i64, _vp, _int, _i64, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                     _vp, _sz, _vp]),
    "dauc_class_sums": (_int, [_vp, _i64, _vp, _int, _i64, _vp, _int, _vp, _sz, _vp]),
    "dauc_surrogate_status": (_int, [_vp, _sz, _vp, _int, _vp]),
    "dauc_alpha_from_sums": (_int, [_vp, _vp, _vp]),
    "dauc_surrogate_logits_fwdbwd": (_int, [_vp, _int, _i64, _vp, _int, _i64, _vp, _vp, _vp, _i64, _vp, _vp,
                                            _vp, _vp, _vp, _sz, _vp]),
    "dauc_class_sums_logits": (_int, [_vp, _int, _i64, _vp, _int, _i64, _vp, _vp, _int, _vp, _sz, _vp]),
    "dauc_pd_update": (_int, [_vp, _vp, _vp, ctypes.POINTER(GradSeg), _int, _vp, _vp, _vp, _f32, _f32,
                              _int, _vp]),
    "dauc_pd_update_dense": (_int, [_vp, _vp, _vp, _vp, _i64, _f32, _f32, _vp]),
    "dauc_coda_finalize": (_int, [_vp, _i64, _int, _vp, _vp, _vp]),
    "dauc_scale_div": (_int, [_vp, _i64, _f32, _vp]),
    "dauc_split_workspace_size": (_sz, [_i64]),
    "dauc_split_scores": (_int, [_vp, _vp, _int, _i64, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dauc_pair_count": (_int, [_vp, _i64, _vp, _i64, _vp, _vp]),
    "dauc_sort_workspace_size": (_sz, [_i64]),
    "dauc_auc_counts_sorted": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _sz, _vp]),
    "dauc_auc_counts_sorted_labeled": (_int, [_vp, _i64, _vp, _vp, _int, _i64, _i64, _vp, _vp, _vp, _sz, _vp]),
    "dauc_compact_workspace_size": (_sz, [_i64]),
    "dauc_auc_eval_workspace_size": (_sz, [_i64]),
    "dauc_auc_eval_enqueue": (_int, [_vp, _vp, _int, _i64, _int, _int, _vp, _vp, _sz, _vp]),
    "dauc_auc_eval_counts": (_int, [_vp, _vp, _int, _i64, _vp, _vp, _vp, _sz, _vp]),
    "dauc_auc_eval_counts_part": (_int, [_vp, _vp, _int, _i64, _int, _int, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dauc_auc_slot_bytes": (_sz, [_i64, _int]),
    "dauc_auc_eval_compact_part": (_int, [_vp, _vp, _int, _i64, _int, _int, _vp, _vp, _sz, _vp]),
    "dauc_auc_eval_query_part": (_int, [_vp, _vp, _int, _i64, _int, _int, _vp, _vp, _vp, _sz, _vp]),
    "dauc_auc_eval_query_part_sorted": (_int, [_vp, _vp, _int, _i64, _int, _int, _vp, _i64, _vp, _vp, _sz, _vp]),
    "dauc_compact_positives": (_int, [_vp, _vp, _int, _i64, _vp, _vp, _vp, _sz, _vp]),
    "dauc_sort_keys": (_int, [_vp, _i64, _vp, _vp, _sz, _vp]),
    "dauc_bn_workspace_size": (_sz, [_i64, _int]),
    "dauc_bn_act_forward": (_int, [_vp, _int, _i64, _int, _vp, _int, _vp, _vp, _vp, _vp, _f32, _f32, _vp, _vp, _vp,
                                   _vp, _vp, _sz, _vp]),
    "dauc_bn_act_backward": (_int, [_vp, _vp, _vp, _vp, _int, _i64, _int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _vp, _sz, _vp]),
    "dauc_maxpool2d_forward": (_int, [_vp, _int, _i64, _int, _int, _int, _int, _int, _int, _vp, _vp, _int, _int,
                                      _vp]),
    "dauc_slab_sum": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "dauc_conv3x3_wgrad_workspace_size": (_sz, [_i64, _int, _int, _int, _int]),
    "dauc_conv3x3_wgrad": (_int, [_vp, _vp, _int, _i64, _int, _int, _int, _int, _int, _int, _int, _vp, _vp, _sz,
                                  _vp]),
    "dauc_maxpool2d_backward": (_int, [_vp, _vp, _int, _i64, _int, _int, _int, _int, _int, _int, _int, _int, _vp,
                                       _vp]),
    "dauc_conv7x7s2_stem_forward": (_int, [_vp, _vp, _int, _i64, _int, _int, _int, _int, _vp, _vp]),
    "dauc_conv7x7s2_stem_wgrad_workspace_size": (_sz, [_i64, _int, _int]),
    "dauc_conv7x7s2_stem_wgrad": (_int, [_vp, _vp, _int, _i64, _int, _int, _int, _int, _vp, _vp, _sz, _vp]),
    "dauc_strided_pick": (_int, [_vp, _int, _i64, _int, _int, _int, _int, _vp, _vp]),
    "dauc_strided_add": (_int, [_vp, _int, _i64, _int, _int, _int, _int, _vp, _vp]),
    "dauc_broadcast_hw": (_int, [_vp, _int, _i64, _i64, _int, _vp, _vp]),
}

# tuning builds only (tuning/libdauc_tuning.so, -DDAUC_TUNING; include/dauc_tuning.h): measured
# alternatives of the product kernels, selectable by number
TUNING_SIGNATURES = {
    "dauc_surrogate_fwdbwd_variant": (_int, [_vp, _i64, _vp, _int, _i64, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                             _vp, _sz, _int, _vp]),
    "dauc_pd_update_dense_variant": (_int, [_vp, _vp, _vp, _vp, _i64, _f32, _f32, _int, _vp]),
    "dauc_pair_count_variant": (_int, [_vp, _i64, _vp, _i64, _vp, _int, _vp]),
    "dauc_set_search_mode": (_int, [_int]),
    "dauc_set_direct_fault": (_int, [_int]),
    "dauc_set_index_form": (_int, [_int]),
    "dauc_probe_tr16": (_int, [_vp, _vp]),
    "dauc_set_wgrad_form": (_int, [_int]),
}
TUNING_LIB_PATH = Path(os.environ.get("DAUC_TUNING_LIB", PKG_DIR.parent / "tuning" / "libdauc_tuning.so"))

_lib = None
_tuning = None


@contextlib.contextmanager
def using(lib: ctypes.CDLL):
    """Run the ops against another loaded build of the library (tests: the tuning build)."""
    global _lib
    prev = load()
    _lib = lib
    try:
        yield lib
    finally:
        _lib = prev


def header_functions(header: Path = HEADER) -> list[str]:
    """Names of every function the C header declares (used by the ABI tests)."""
    text = re.sub(r"/\*.*?\*/", "", header.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(dauc_[a-z0-9_]+)\s*\(", text)) - {"dauc_grad_seg"})


def load() -> ctypes.CDLL:
    """Load libdauc.so and attach the prototypes. Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} not found: the HIP library must be built first "
            "(python -c 'import __graft_entry__ as g; g.build()' or python distributedauc_amd/build.py). "
            "distributedauc_amd has no CPU fallback."
        )
    _lib = _attach(ctypes.CDLL(str(LIB_PATH)))
    return _lib


def _attach(lib: ctypes.CDLL) -> ctypes.CDLL:
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in TUNING_SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    return lib


def tuning() -> ctypes.CDLL:
    """The library that exports the tuning entry points: the loaded one if it is a tuning build
    (DAUC_LIB), else tuning/libdauc_tuning.so (built by build.py next to the product library).
    Tests and micro-benchmarks only; the product path never calls it."""
    global _tuning
    lib = load()
    if all(hasattr(lib, n) for n in TUNING_SIGNATURES):
        return lib
    if _tuning is None:
        if not TUNING_LIB_PATH.exists():
            raise ImportError(f"{TUNING_LIB_PATH} not found: build it with python distributedauc_amd/build.py")
        _tuning = _attach(ctypes.CDLL(str(TUNING_LIB_PATH)))
    return _tuning


def strerror(rc: int) -> str:
    return load().dauc_strerror(rc).decode()


def check(rc: int, what: str) -> None:
    if rc != DAUC_OK:
        raise DaucError(f"{what} failed: {strerror(rc)} (status {rc})")
