"""Builds ``librescore.so`` in-tree with hipcc for gfx950 (no JIT cache, no pip install).

Each ``csrc/*.hip`` (hipcc) and host-only ``csrc/*.cpp`` (g++) is compiled to an object in
``csrc/build/`` (in parallel), then linked into ``asr-rescoring_amd/librescore.so``.  Rebuilds only what changed.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
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


def _needs(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str) -> str:
    host = src.endswith(".cpp")                     # host-only C++ (tokenizer / JSON front end)
    obj = os.path.join(OBJ, os.path.basename(src).rsplit(".", 1)[0] + ".o")
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc")) \
        + glob.glob(os.path.join(REPO, "include", "*.h"))
    if _needs(obj, deps):
        cmd = ([CXX, "-O2", "-std=c++17", "-fPIC", "-Wall", "-I", os.path.join(REPO, "include")] if host
               else [HIPCC] + FLAGS) + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj


def build_library(verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if _needs(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        # rocBLAS: fp32 GEMMs of the trainer (its soname matches the copy torch loads first)
        r = subprocess.run(cmd + ["-L/opt/rocm/lib", "-lrocblas", "-lpthread"], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    if verbose:
        print("built", LIB, file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build_library(verbose=True)
