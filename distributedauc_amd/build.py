"""Build libdauc.so (the gfx950 HIP kernels + C ABI) in-tree with hipcc.

The shared library is written next to this file so that it travels with the
repository snapshot to the GPU box. No JIT cache, no torch extension: the
product boundary is the plain C ABI declared in ``include/dauc.h``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
OBJ_DIR = PKG_DIR / "build"
LIB_PATH = PKG_DIR / "libdauc.so"
# linker version script: only the dauc_* C entry points are exported (no C++ internals)
EXPORTS = CSRC / "exports.map"
# the tuning build: the same sources with -DDAUC_TUNING, which adds the measured alternatives'
# entry points (include/dauc_tuning.h); tests and micro-benchmarks load it, the product never does
TUNING_LIB_PATH = REPO / "tuning" / "libdauc_tuning.so"
ARCH = os.environ.get("DAUC_OFFLOAD_ARCH", "gfx950")

HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

# -ffp-contract=off: the update kernel must reproduce the reference's separately
# rounded fp32 ops bit for bit (it also uses __f*_rn intrinsics explicitly).
# Denormals are kept (default): exact pair counting compares subnormal scores.
CFLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-ffp-contract=off",
    "-Wall",
    "-Wno-unused-function",
    f"-I{REPO / 'include'}",
]


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _needs_build(target: Path = LIB_PATH) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    deps = sources() + sorted(CSRC.glob("*.h")) + sorted((REPO / "include").glob("*.h")) + [Path(__file__), EXPORTS]
    return any(p.stat().st_mtime > t for p in deps)


def _compile(src: Path, obj_dir: Path = OBJ_DIR, defines: tuple = ()) -> Path:
    obj = obj_dir / (src.stem + ".o")
    cmd = [HIPCC, *CFLAGS, *[f"-D{d}" for d in defines], "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build_library(force: bool = False, verbose: bool = False, out: Path | None = None,
                  defines: tuple = ()) -> Path:
    """Compile every csrc/*.hip for gfx950 and link libdauc.so (incremental).

    ``out``/``defines`` build a tuning variant of the library side by side
    (e.g. ``defines=("DAUC_SURROGATE_SLOTS=2",)``); the product loads LIB_PATH.
    """
    target = Path(out) if out is not None else LIB_PATH
    if out is None and not defines and not force and not _needs_build():
        return LIB_PATH
    if target == TUNING_LIB_PATH and tuple(defines) == ("DAUC_TUNING",) and not force and not _needs_build(target):
        return target
    obj_dir = OBJ_DIR if out is None else OBJ_DIR / target.stem
    obj_dir.mkdir(parents=True, exist_ok=True)
    target.parent.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, obj_dir, tuple(defines)), srcs))
    tmp = target.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", f"-Wl,--version-script={EXPORTS}", *map(str, objs),
           "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, target)
    if verbose:
        print(f"built {target}", file=sys.stderr)
    return target


def build_tuning(force: bool = False, verbose: bool = False) -> Path:
    """tuning/libdauc_tuning.so: the product sources with -DDAUC_TUNING."""
    return build_library(force=force, verbose=verbose, out=TUNING_LIB_PATH, defines=("DAUC_TUNING",))


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--out", default=None, help="write a tuning variant here instead of libdauc.so")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--tuning", action="store_true", help="also build tuning/libdauc_tuning.so")
    a = ap.parse_args()
    build_library(force=a.force, verbose=True, out=a.out, defines=tuple(a.defines))
    if a.tuning:
        build_tuning(force=a.force, verbose=True)
