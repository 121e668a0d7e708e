"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every
symbol ``include/mvae.h`` declares (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

from magic_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mvae.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mvae_[a-z_0-9]+)\s*\(", src)))


def test_library_loads_and_exports_header():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.EXPORTED), set(syms) ^ set(_lib.EXPORTED)
    assert lib.mvae_abi_version() == _lib.ABI_VERSION


def test_struct_layout_matches_header(tmp_path):
    """ctypes mirrors of mvae_cfg / mvae_tensor agree with the C compiler's layout."""
    import shutil
    import subprocess
    got = (ctypes.sizeof(_lib.mvae_cfg), _lib.mvae_cfg.seed.offset, ctypes.sizeof(_lib.mvae_tensor))
    if shutil.which("gcc") is None:
        assert got == (112, 104, 72)
        return
    src = tmp_path / "s.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\n'
                   'int main(){printf("%%zu %%zu %%zu", sizeof(mvae_cfg), offsetof(mvae_cfg, seed),'
                   ' sizeof(mvae_tensor));}\n' % os.path.join(ROOT, "include", "mvae.h"))
    exe = tmp_path / "s"
    subprocess.check_call(["gcc", str(src), "-o", str(exe)])
    want = tuple(int(v) for v in subprocess.check_output([str(exe)]).split())
    assert got == want


def test_create_rejects_bad_config_without_gpu_work():
    lib = _lib.load()
    c = _lib.mvae_cfg()
    c.image_size = 0
    h = ctypes.c_void_p()
    rc = lib.mvae_create(ctypes.byref(c), 0, ctypes.byref(h))
    assert rc < 0 and h.value is None
    assert b"positive" in lib.mvae_last_error(None)
    assert lib.mvae_create(None, 0, ctypes.byref(h)) < 0


def test_engine_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from magic_amd.engine import Engine
    from magic_amd.config import preset
    with pytest.raises(_lib.MVAELibraryError):
        Engine(preset("8c", image_size=10, batch=4))


def test_missing_library_is_an_error(tmp_path):
    with pytest.raises(_lib.MVAELibraryError):
        _lib.load(str(tmp_path / "nope.so"))


def test_build_id_ties_library_to_sources():
    """libmvae.so carries the hash of the sources it was built from; the loader refuses a
    library whose id differs from the sources on disk (a stale or foreign build)."""
    from magic_amd.build import source_files, source_hash
    lib = _lib.load()
    assert lib.mvae_build_id().decode() == source_hash()
    assert any(p.endswith("mvae_api.cpp") for p in source_files())
    assert any(p.endswith(os.path.join("include", "mvae.h")) for p in source_files())
    with pytest.raises(_lib.MVAELibraryError, match="stale"):
        _lib.verify_build(lib, expected="0" * 16)


def test_build_id_ignores_stray_files_and_names_missing_sources(tmp_path, monkeypatch):
    """Only the compiled sources enter the build id (a stray file under csrc/ does not make the
    library "stale"); a missing source raises MVAELibraryError naming it, not a bare OSError."""
    from magic_amd import build
    lib = _lib.load()
    stray = os.path.join(build.CSRC, "zz_stray_editor_file.orig")
    with open(stray, "w") as f:
        f.write("not a source\n")
    try:
        assert _lib.verify_build(lib) == build.source_hash()
    finally:
        os.remove(stray)
    monkeypatch.setattr(build, "SOURCES", build.SOURCES + ["does_not_exist.hip"])
    with pytest.raises(_lib.MVAELibraryError, match="does_not_exist.hip"):
        _lib.verify_build(lib)
