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


def _needs_build() -> bool:
    if not LIB_PATH.exists():
        return True
    t = LIB_PATH.stat().st_mtime
    deps = sources() + sorted(CSRC.glob("*.h")) + [REPO / "include" / "dauc.h", Path(__file__)]
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
    obj_dir = OBJ_DIR if out is None else OBJ_DIR / target.stem
    obj_dir.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, obj_dir, tuple(defines)), srcs))
    tmp = target.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, target)
    if verbose:
        print(f"built {target}", file=sys.stderr)
    return target


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--out", default=None, help="write a tuning variant here instead of libdauc.so")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    build_library(force=a.force, verbose=True, out=a.out, defines=tuple(a.defines))
