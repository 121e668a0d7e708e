"""Build ``magic_amd/libmvae.so`` (HIP for gfx950) in-tree with hipcc.

``python -m magic_amd.build`` or ``magic_amd.build.build()``. Sources are compiled to
objects under ``magic_amd/_build/`` in parallel and relinked only when a source changed.
The library carries ``source_hash()`` of the sources it was built from (``mvae_build_id``);
``magic_amd._lib.load`` compares it with the sources on disk.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
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
SOURCES = ["mvae_api.cpp", "gemm_f32.hip", "gemm_bf16.hip", "gemm_bf16e.hip", "gemm_valu.hip", "mvae_kernels.hip",
           "conv_tower.hip", "conv_mfma.hip", "enc_chain.hip"]
HEADERS = ["mvae_internal.h", "gemm_common.h", "deint_bits.h", os.path.join("..", "..", "include", "mvae.h")]
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result",
          "-Wno-unused-value", "-I", os.path.join(ROOT, "include")]


def source_files() -> list[str]:
    """The files the library is compiled from: SOURCES and HEADERS (include/mvae.h among them).
    Nothing else under csrc/ (editor files, -save-temps output) enters the build id."""
    return sorted(os.path.normpath(os.path.join(CSRC, f)) for f in SOURCES + HEADERS)


def source_hash() -> str:
    """First 16 hex digits of SHA-256 over (relative path, NUL, contents) of source_files().
    Raises FileNotFoundError naming the missing file when a source is absent."""
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.relpath(p, ROOT).replace(os.sep, "/").encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _compile(src: str, force: bool, bid: str) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src + ".o")
    deps = [s] + [os.path.join(CSRC, h) for h in HEADERS]
    extra = []
    if src == "mvae_api.cpp":  # the build id: recompiled whenever any source changed
        extra = [f'-DMVAE_BUILD_ID="{bid}"']
        stamp = os.path.join(OBJ, "build_id.txt")
        old = open(stamp).read().strip() if os.path.exists(stamp) else ""
        if old != bid:
            force = True
    if force or _mtime(o) < max(_mtime(d) for d in deps):
        cmd = [HIPCC, *CFLAGS, *extra, "-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return o


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    bid = source_hash()
    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, bid), SOURCES))
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    with open(os.path.join(OBJ, "build_id.txt"), "w") as f:
        f.write(bid + "\n")
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
