"""The C-ABI boundary: libdauc.so loads, exports exactly what include/dauc.h declares,
and validates arguments on the host (these calls return before touching a GPU)."""
from __future__ import annotations

import ctypes
import subprocess

import pytest
import torch

from distributedauc_amd import _lib


def test_library_loads_and_exports_header():
    lib = _lib.load()
    declared = _lib.header_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib.SIGNATURES), "Python prototypes out of sync with include/dauc.h"


def _exports(path):
    """Every defined dynamic symbol of the library (not only dauc_*: internals must not leak)."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_exported_symbols_are_c_linkage():
    """libdauc.so exports exactly the product header's entry points (no tuning variants)."""
    syms = _exports(_lib.LIB_PATH)
    assert syms == set(_lib.header_functions()), syms ^ set(_lib.header_functions())
    assert not (syms & set(_lib.TUNING_SIGNATURES))


def test_tuning_library_exports_tuning_header():
    """tuning/libdauc_tuning.so (-DDAUC_TUNING) = the product entry points + include/dauc_tuning.h's."""
    tuning_header = _lib.HEADER.parent / "dauc_tuning.h"
    declared = set(_lib.header_functions(tuning_header))
    assert declared == set(_lib.TUNING_SIGNATURES)
    syms = _exports(_lib.TUNING_LIB_PATH)
    assert syms == set(_lib.header_functions()) | declared
    lib = _lib.tuning()
    null = ctypes.c_void_p(0)
    assert lib.dauc_pair_count_variant(null, 0, null, 0, ctypes.c_void_p(8), 7, null) == _lib.DAUC_OK  # empty: no-op
    assert lib.dauc_pair_count_variant(null, 5, null, 5, ctypes.c_void_p(8), 12, null) == _lib.DAUC_EINVAL
    assert lib.dauc_set_search_mode(3) == _lib.DAUC_EINVAL


def test_library_is_gfx950_code_object():
    """The embedded device code object targets gfx950 (hipcc --offload-arch=gfx950)."""
    data = _lib.LIB_PATH.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_version_and_strerror():
    assert _lib.load().dauc_version() == 100
    assert _lib.strerror(0) == "success"
    assert _lib.strerror(_lib.DAUC_EINVAL) == "invalid argument"


def test_workspace_sizes():
    L = _lib.load()
    assert L.dauc_surrogate_workspace_size(1) >= 256
    assert L.dauc_surrogate_workspace_size(1 << 26) > L.dauc_surrogate_workspace_size(4096)
    assert L.dauc_split_workspace_size(1 << 24) >= (1 << 24) // 8192 * 20  # 8192-score tiles


def test_invalid_arguments_return_einval():
    L = _lib.load()
    null = ctypes.c_void_p(0)
    assert L.dauc_pair_count(null, -1, null, 5, null, null) == _lib.DAUC_EINVAL
    assert L.dauc_pair_count(null, 5, null, 5, ctypes.c_void_p(8), null) == _lib.DAUC_EINVAL
    assert L.dauc_pair_count(null, 0, null, 0, ctypes.c_void_p(8), null) == _lib.DAUC_OK  # empty: no-op
    assert L.dauc_surrogate_fwdbwd(null, 1, null, 1, 0, null, null, null, 1, null, null, null, null, 0,
                                   null) == _lib.DAUC_EINVAL
    assert L.dauc_pd_update(null, null, null, None, 0, null, null, null, 0.1, 0.1, 0, null) == _lib.DAUC_EINVAL
    assert L.dauc_pd_update(ctypes.c_void_p(16), ctypes.c_void_p(16), null, None, 0, null, null, null, 0.1, 0.1,
                            9, null) == _lib.DAUC_EINVAL
    assert L.dauc_coda_finalize(null, 10, 2, null, null, null) == _lib.DAUC_EINVAL
    assert L.dauc_split_scores(null, null, 1, 10, null, null, null, null, 0, null) == _lib.DAUC_EINVAL
    assert L.dauc_label_map_phat(null, 0, 4, null, null, null, null, null) == _lib.DAUC_EINVAL
    a = ctypes.c_void_p(256)
    # max-pool: Ho/Wo must be the floor-mode sizes, C a whole bf16 vector, pad <= kernel / 2
    assert L.dauc_maxpool2d_forward(a, 2, 2, 112, 112, 64, 3, 2, 1, a, a, 55, 56, null) == _lib.DAUC_EINVAL
    assert L.dauc_maxpool2d_forward(a, 2, 2, 112, 112, 60, 3, 2, 1, a, a, 56, 56, null) == _lib.DAUC_EINVAL
    assert L.dauc_maxpool2d_forward(a, 2, 2, 112, 112, 64, 3, 2, 2, a, a, 57, 57, null) == _lib.DAUC_EINVAL
    assert L.dauc_maxpool2d_backward(a, null, 2, 2, 112, 112, 64, 3, 2, 1, 56, 56, a, null) == _lib.DAUC_EINVAL
    assert L.dauc_maxpool2d_backward(a, a, 3, 2, 112, 112, 64, 3, 2, 1, 56, 56, a, null) == _lib.DAUC_EINVAL
    with pytest.raises(_lib.DaucError, match="invalid argument"):
        _lib.check(_lib.DAUC_EINVAL, "x")


def test_cpu_tensors_are_refused():
    """No CPU fallback: every product op refuses host tensors loudly."""
    from distributedauc_amd import ops

    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.scale_div(torch.zeros(4), 2.0)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.pair_count(torch.zeros(4), torch.zeros(4), torch.zeros(2, dtype=torch.int64))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.surrogate_fwdbwd(torch.zeros(4), torch.zeros(4, dtype=torch.int8), torch.zeros(3), torch.zeros(1))


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", tmp_path / "libdauc.so")
    with pytest.raises(ImportError, match="no CPU fallback"):
        _lib.load()


def test_ctypes_signatures_match_header_arity():
    """Every ctypes prototype has as many parameters as the C declaration in include/dauc.h."""
    import re

    text = re.sub(r"/\*.*?\*/", "", _lib.HEADER.read_text(), flags=re.S)
    decls = dict(re.findall(r"\b(dauc_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text))
    text = re.sub(r"/\*.*?\*/", "", (_lib.HEADER.parent / "dauc_tuning.h").read_text(), flags=re.S)
    decls.update(re.findall(r"\b(dauc_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text))
    for name, (_, args) in list(_lib.SIGNATURES.items()) + list(_lib.TUNING_SIGNATURES.items()):
        params = decls[name].strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert n == len(args), (name, n, len(args))
