"""Build ``magic_amd/libmvae.so`` (HIP for gfx950) in-tree with hipcc.

``python -m magic_amd.build`` or ``magic_amd.build.build()``. Sources are compiled to
objects under ``magic_amd/_build/`` in parallel and relinked only when a source changed.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libmvae.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MVAE_ARCH", "gfx950")
SOURCES = ["mvae_api.cpp", "gemm_f32.hip", "gemm_bf16.hip", "gemm_valu.hip", "mvae_kernels.hip",
           "conv_tower.hip", "conv_mfma.hip"]
HEADERS = ["mvae_internal.h", "gemm_common.h", os.path.join("..", "..", "include", "mvae.h")]
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result",
          "-Wno-unused-value", "-I", os.path.join(ROOT, "include")]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _compile(src: str, force: bool) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src + ".o")
    deps = [s] + [os.path.join(CSRC, h) for h in HEADERS]
    if force or _mtime(o) < max(_mtime(d) for d in deps):
        cmd = [HIPCC, *CFLAGS, "-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return o


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
