"""Builds ``librescore.so`` in-tree with hipcc for gfx950 (no JIT cache, no pip install).

Each ``csrc/*.hip`` (hipcc) and host-only ``csrc/*.cpp`` (g++) is compiled to an object in
``csrc/build/`` (in parallel), then linked into ``asr-rescoring_amd/librescore.so``.  Rebuilds
only what changed, judged by CONTENT: every object and the library carry a ``.stamp`` with the
sha256 of their inputs (source, headers, command line), so a copied-in or stale artefact whose
stamp does not match its sources is rebuilt (mtimes are not trusted).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(CSRC, "build")
LIB = os.path.join(PKG, "librescore.so")
REPO = os.path.dirname(PKG)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
ARCH = os.environ.get("RS_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-I", os.path.join(REPO, "include")]


def _digest(deps, cmd) -> str:
    h = hashlib.sha256(" ".join(cmd).encode())
    for d in sorted(deps):
        h.update(d.encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _needs(target: str, deps, cmd) -> bool:
    """True unless ``target`` exists with a stamp equal to the digest of deps + cmd."""
    stamp = target + ".stamp"
    if not (os.path.exists(target) and os.path.exists(stamp)):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest(deps, cmd)


def _stamp(target: str, deps, cmd) -> None:
    with open(target + ".stamp", "w") as f:
        f.write(_digest(deps, cmd))


def _compile(src: str, csrc: str = CSRC, objdir: str = OBJ, include: str = os.path.join(REPO, "include"),
             defines=()) -> str:
    host = src.endswith(".cpp")                     # host-only C++ (tokenizer / JSON front end)
    obj = os.path.join(objdir, os.path.basename(src).rsplit(".", 1)[0] + ".o")
    deps = [src] + glob.glob(os.path.join(csrc, "*.h")) + glob.glob(os.path.join(csrc, "*.inc")) \
        + glob.glob(os.path.join(include, "*.h"))
    flags = [f if f != os.path.join(REPO, "include") else include for f in FLAGS]
    cmd = ([CXX, "-O2", "-std=c++17", "-fPIC", "-Wall", "-I", include] if host
           else [HIPCC] + flags + [f"-D{d}" for d in defines]) + ["-c", src, "-o", obj]
    if _needs(obj, deps, cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
        _stamp(obj, deps, cmd)
    return obj


def build_library(verbose: bool = False, diag: bool = False, csrc: str = CSRC, out: str = None,
                  include: str = None) -> str:
    """The shipped library (default), or with ``diag`` the timing-diagnostic build
    ``librescore_diag.so`` (-DRS_DIAG=1: the wrong-results GEMM variants and the stamp build the
    probe tools under tools/ use; never loaded by the scoring path, tests or bench).  ``csrc`` /
    ``out`` / ``include``: build another source tree (an A/B of two revisions, tools/build_rev.py)."""
    include = include or os.path.join(REPO, "include")
    lib = out or (os.path.join(PKG, "librescore_diag.so") if diag else LIB)
    objdir = os.path.join(os.path.dirname(lib), "build_" + os.path.basename(lib).split(".")[0]) \
        if (out or diag) else OBJ
    os.makedirs(objdir, exist_ok=True)
    defines = ("RS_DIAG=1",) if diag else ()
    srcs = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda f: _compile(f, csrc, objdir, include, defines), srcs))
    # rocBLAS: the trainer's RS_TRAIN_ROCBLAS=1 baseline GEMMs (its soname matches the copy torch loads first)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs + \
        ["-L/opt/rocm/lib", "-lrocblas", "-lpthread"]
    if _needs(lib, objs, cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        _stamp(lib, objs, cmd)
    if verbose:
        print("built", lib, file=sys.stderr)
    return lib


if __name__ == "__main__":
    build_library(verbose=True, diag="--diag" in sys.argv)
