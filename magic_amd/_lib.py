"""ctypes binding of ``libmvae.so`` (the C ABI declared in ``include/mvae.h``).

The library is the product path: nothing here falls back to a CPU or PyTorch
implementation. If the shared object is missing or cannot be loaded, importing the
engine raises ``MVAELibraryError`` with the reason.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MVAE_LIB", os.path.join(HERE, "libmvae.so"))

MVAE_MAX_ENC = 8
MARKER_GRID = 4096   # mvae_region_marker workgroups = MARKER_GRID + region (mvae_internal.h)
ABI_VERSION = 4

ACT = {"tanh": 0, "elu": 1}
METRIC = {"cosine": 0, "sqdiff": 1}
PREC = {"f32": 0, "bf16": 1, "f32x": 2}

KIND_PARAM, KIND_GRAD1, KIND_GRAD2, KIND_M1, KIND_V1, KIND_M2, KIND_V2 = range(7)
(BUF_PARAMS, BUF_GRADS, BUF_ADAM, BUF_LOSSES, BUF_COLSQ, BUF_COLDOT, BUF_DIST, BUF_GRADS_DEC,
 BUF_DEAD, BUF_EPS, BUF_DYN) = range(11)


class MVAELibraryError(RuntimeError):
    pass


class MVAEError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libmvae error {code}: {msg}")
        self.code = code


class mvae_cfg(C.Structure):
    _fields_ = [
        ("image_size", C.c_int), ("batch", C.c_int), ("global_batch", C.c_int),
        ("n_enc", C.c_int), ("enc", C.c_int * MVAE_MAX_ENC), ("dec", C.c_int * 2),
        ("latent", C.c_int), ("act", C.c_int), ("metric", C.c_int), ("reciprocal", C.c_int),
        ("deform_weight", C.c_float), ("lr", C.c_float * 2),
        ("beta1", C.c_float), ("beta2", C.c_float), ("epsilon", C.c_float),
        ("precision", C.c_int), ("seed", C.c_uint64), ("conv", C.c_int),
    ]


class mvae_tensor(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("data", C.c_void_p), ("rows", C.c_int),
                ("cols", C.c_int), ("ld", C.c_int), ("trained_by", C.c_int)]


_SIGS = {
    "mvae_abi_version": ([], C.c_int),
    "mvae_build_id": ([], C.c_char_p),
    "mvae_create": ([C.POINTER(mvae_cfg), C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "mvae_create_ex": ([C.POINTER(mvae_cfg), C.c_int, C.c_char_p, C.POINTER(C.c_void_p)], C.c_int),
    "mvae_destroy": ([C.c_void_p], C.c_int),
    "mvae_last_error": ([C.c_void_p], C.c_char_p),
    "mvae_param_count": ([C.c_void_p], C.c_int),
    "mvae_param_info": ([C.c_void_p, C.c_int, C.c_int, C.POINTER(mvae_tensor)], C.c_int),
    "mvae_buffer": ([C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)], C.c_int),
    "mvae_get_step": ([C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)], C.c_int),
    "mvae_set_step": ([C.c_void_p, C.c_int64, C.c_int64], C.c_int),
    "mvae_set_shard": ([C.c_void_p, C.c_int64], C.c_int),
    "mvae_get_rng": ([C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)], C.c_int),
    "mvae_set_rng": ([C.c_void_p, C.c_uint64, C.c_uint64], C.c_int),
    "mvae_sync_params": ([C.c_void_p, C.c_void_p], C.c_int),
    "mvae_forward": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_metric": ([C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_backward": ([C.c_void_p, C.c_void_p], C.c_int),
    "mvae_backward_part": ([C.c_void_p, C.c_int, C.c_void_p], C.c_int),
    "mvae_backward_nparts": ([C.c_void_p], C.c_int),
    "mvae_grad_range": ([C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)], C.c_int),
    "mvae_set_option": ([C.c_void_p, C.c_char_p, C.c_int], C.c_int),
    "mvae_adam": ([C.c_void_p, C.c_void_p], C.c_int),
    "mvae_train_step": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                         C.c_void_p], C.c_int),
    "mvae_predict": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_predict_encode": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_predict_finish": ([C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_transform": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_reconstruct": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_generate": ([C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_make_batch": ([C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                         C.c_float, C.c_void_p, C.c_void_p], C.c_int),
    "mvae_timing_enable": ([C.c_void_p, C.c_int], C.c_int),
    "mvae_timing_select": ([C.c_void_p, C.c_int], C.c_int),
    "mvae_timing_marker": ([C.c_void_p, C.c_int, C.c_int], C.c_int),
    "mvae_timing_regions": ([C.c_void_p], C.c_int),
    "mvae_timing_name": ([C.c_void_p, C.c_int], C.c_char_p),
    "mvae_timing_read": ([C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int64)], C.c_int),
    "mvae_timing_reset": ([C.c_void_p], C.c_int),
    "mvae_bench_gemm": ([C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                         C.c_void_p, C.POINTER(C.c_float)], C.c_int),
    "mvae_bench_deint": ([C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_float)], C.c_int),
    "mvae_debug_conv2": ([C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                          C.c_void_p], C.c_int),
    "mvae_debug_gemm": ([C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                         C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                         C.c_int, C.c_void_p], C.c_int),
}

EXPORTED = tuple(_SIGS)

_lib = None


def load(path: str | None = None):
    """Load and type the library once. Raises MVAELibraryError if it is unavailable."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise MVAELibraryError(
            f"{p} not found: build it with `python -m magic_amd.build` (hipcc, gfx950). "
            "There is no CPU fallback for the product path.")
    # torch first: it carries the process's HIP runtime (same soname as ours), so the
    # library binds to the runtime that owns torch's device pointers and streams.
    import torch  # noqa: F401
    try:
        lib = C.CDLL(p)
    except OSError as e:
        raise MVAELibraryError(f"cannot load {p}: {e}") from e
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    v = lib.mvae_abi_version()
    if v != ABI_VERSION:
        raise MVAELibraryError(f"ABI version mismatch: library {v}, binding {ABI_VERSION}")
    verify_build(lib)
    if path is None:
        _lib = lib
    return lib


def verify_build(lib, expected: str | None = None) -> str:
    """The library's build id must equal the hash of the sources on disk (magic_amd/build.py
    source_hash): a libmvae.so built from other sources (stale, or shipped from another tree)
    is refused. Returns the id."""
    from .build import source_hash
    got = lib.mvae_build_id().decode()
    try:
        want = expected if expected is not None else source_hash()
    except FileNotFoundError as e:
        raise MVAELibraryError(
            f"cannot verify libmvae.so (build id {got}): source file missing ({e.filename}); the "
            "library is only loaded from a tree holding the sources it was built from") from e
    if got != want:
        raise MVAELibraryError(
            f"libmvae.so build id {got} does not match the sources on disk ({want}): the library "
            "is stale; rebuild it with `python -m magic_amd.build`")
    return got


def check(lib, ctx, rc):
    if rc != 0:
        msg = lib.mvae_last_error(ctx)
        raise MVAEError(rc, msg.decode() if msg else "")
    return rc


# ------------------------------------------------------------------------- DLPack
# Zero-copy torch views of context-owned device memory (params, grads, Adam slots):
# a DLManagedTensor (device kDLROCM) wrapped in a "dltensor" PyCapsule.
class _DLDevice(C.Structure):
    _fields_ = [("device_type", C.c_int32), ("device_id", C.c_int32)]


class _DLDataType(C.Structure):
    _fields_ = [("code", C.c_uint8), ("bits", C.c_uint8), ("lanes", C.c_uint16)]


class _DLTensor(C.Structure):
    _fields_ = [("data", C.c_void_p), ("device", _DLDevice), ("ndim", C.c_int32),
                ("dtype", _DLDataType), ("shape", C.POINTER(C.c_int64)),
                ("strides", C.POINTER(C.c_int64)), ("byte_offset", C.c_uint64)]


class _DLManagedTensor(C.Structure):
    pass


_DELETER = C.CFUNCTYPE(None, C.POINTER(_DLManagedTensor))
_DLManagedTensor._fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", C.c_void_p),
                             ("deleter", _DELETER)]

_KDLROCM = 10
_KDLFLOAT = 2
_PyCapsule_New = C.pythonapi.PyCapsule_New
_PyCapsule_New.restype = C.py_object
_PyCapsule_New.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p]


def device_view(ptr: int, shape, strides, device: int, keepalive: list):
    """torch.float32 tensor aliasing device memory at ``ptr`` (owned by a libmvae context).

    ``keepalive`` must outlive the tensor (the engine keeps it); the view must not be used
    after the context is destroyed."""
    import torch
    nd = len(shape)
    shp = (C.c_int64 * nd)(*shape)
    std = (C.c_int64 * nd)(*strides)
    mt = _DLManagedTensor()
    mt.dl_tensor.data = ptr
    mt.dl_tensor.device = _DLDevice(_KDLROCM, device)
    mt.dl_tensor.ndim = nd
    mt.dl_tensor.dtype = _DLDataType(_KDLFLOAT, 32, 1)
    mt.dl_tensor.shape = shp
    mt.dl_tensor.strides = std
    mt.dl_tensor.byte_offset = 0
    mt.manager_ctx = None
    mt.deleter = _DELETER()  # NULL: memory belongs to the context
    keepalive.extend([shp, std, mt])
    cap = _PyCapsule_New(C.addressof(mt), b"dltensor", None)
    return torch.utils.dlpack.from_dlpack(cap)
