"""shorthair_amd -- MI355X-native Cauchy Reed-Solomon codec (drop-in for catid/shorthair cauchy_256).

The product is the C-ABI shared library ``libcauchy256.so`` (HIP kernels for gfx950 + host code);
this module is a thin ctypes binding used by the tests and the benchmark. It mirrors the
reference interface (cauchy_256.h: ``cauchy_256_init`` / ``cauchy_256_encode`` /
``cauchy_256_decode`` with the same argument meaning and return codes) and exposes the batched
device-resident API (``include/cauchy_256_batch.h``) on torch tensors.

There is no CPU fallback: if the library is missing this import fails, and without a GPU every
codec call returns -2 (see the library's stderr message).
"""
import ctypes
import os

__all__ = ["lib", "Block", "CAUCHY_256_VERSION", "cauchy_256_init", "cauchy_256_encode",
           "cauchy_256_decode", "encode_batch", "decode_batch", "decode_batch_out",
           "fill_synthetic", "erasure_pattern", "batch_reserve", "batch_errors", "has_fixed", "path", "default_stream", "sync", "LIB_PATH",
           "EXPORTED_SYMBOLS"]

CAUCHY_256_VERSION = 2
LIB_PATH = os.environ.get("SH_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                         "libcauchy256.so")

# Every function declared in include/*.h (cauchy_256.h, cauchy_256_batch.h, gf256.h).
EXPORTED_SYMBOLS = [
    "_cauchy_256_init", "cauchy_256_encode", "cauchy_256_decode",
    "cauchy_256_batch_init", "cauchy_256_encode_batch", "cauchy_256_decode_batch",
    "cauchy_256_decode_batch_out", "cauchy_256_batch_reserve", "cauchy_256_batch_reserve_stream",
    "cauchy_256_batch_errors", "cauchy_256_batch_path", "cauchy_256_fill_synthetic",
    "cauchy_256_erasure_pattern",
    "cauchy_256_default_stream", "cauchy_256_sync", "cauchy_256_profile", "cauchy_256_profile_read",
    "gf256_init_", "gf256_add_mem", "gf256_add2_mem", "gf256_addset_mem", "gf256_mul_mem",
    "gf256_muladd_mem", "gf256_memswap",
    "shorthair_recovery_packet_bytes", "shorthair_encode_groups", "shorthair_recover_groups",
]

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} not built: run `python shorthair_amd/build.py` "
                      "(the codec has no CPU fallback)")

# One HIP runtime per process. PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 with
# the same SONAMEs as /opt/rocm's: loaded after torch, the library binds to torch's copies; loaded
# before, the process gets two HSA runtimes and whichever initialises second sees no GPU
# (measured on the box: "No HIP GPUs are available" / our -2). So torch, when present, loads
# first. Callers without torch are unaffected.
try:
    import torch  # noqa: F401
except ImportError:
    pass
lib = ctypes.CDLL(LIB_PATH)


class Block(ctypes.Structure):
    """Reference Block descriptor (cauchy_256.h:52-55)."""
    _fields_ = [("data", ctypes.c_void_p), ("row", ctypes.c_ubyte)]


_c = ctypes
lib._cauchy_256_init.argtypes = [_c.c_int]
lib._cauchy_256_init.restype = _c.c_int
lib.cauchy_256_encode.argtypes = [_c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_int]
lib.cauchy_256_encode.restype = _c.c_int
lib.cauchy_256_decode.argtypes = [_c.c_int, _c.c_int, _c.c_void_p, _c.c_int]
lib.cauchy_256_decode.restype = _c.c_int
lib.cauchy_256_batch_init.argtypes = [_c.c_int]
lib.cauchy_256_batch_init.restype = _c.c_int
lib.cauchy_256_encode_batch.argtypes = [_c.c_int] * 4 + [_c.c_void_p] * 3
lib.cauchy_256_encode_batch.restype = _c.c_int
lib.cauchy_256_decode_batch.argtypes = [_c.c_int] * 4 + [_c.c_void_p] * 3
lib.cauchy_256_decode_batch.restype = _c.c_int
lib.cauchy_256_decode_batch_out.argtypes = [_c.c_int] * 4 + [_c.c_void_p] * 6
lib.cauchy_256_decode_batch_out.restype = _c.c_int
lib.cauchy_256_batch_reserve.argtypes = [_c.c_int] * 4
lib.cauchy_256_batch_reserve.restype = _c.c_int
lib.cauchy_256_batch_reserve_stream.argtypes = [_c.c_int] * 4 + [_c.c_void_p]
lib.cauchy_256_batch_reserve_stream.restype = _c.c_int
lib.cauchy_256_batch_errors.argtypes = [_c.c_void_p]
lib.cauchy_256_batch_errors.restype = _c.c_int
lib.cauchy_256_batch_path.argtypes = [_c.c_int] * 3
lib.cauchy_256_batch_path.restype = _c.c_int
lib.cauchy_256_fill_synthetic.argtypes = [_c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                          _c.c_ulonglong, _c.c_ulonglong, _c.c_void_p]
lib.cauchy_256_fill_synthetic.restype = _c.c_int
lib.cauchy_256_erasure_pattern.argtypes = [_c.c_ulonglong, _c.c_int, _c.c_int, _c.c_ulonglong, _c.c_int,
                                           _c.c_void_p]
lib.cauchy_256_erasure_pattern.restype = _c.c_int
lib.cauchy_256_default_stream.argtypes = []
lib.cauchy_256_default_stream.restype = _c.c_void_p
lib.cauchy_256_sync.argtypes = [_c.c_void_p]
lib.cauchy_256_sync.restype = _c.c_int
lib.cauchy_256_profile.argtypes = [_c.c_int]
lib.cauchy_256_profile.restype = _c.c_int
lib.cauchy_256_profile_read.argtypes = [_c.c_void_p]
lib.cauchy_256_profile_read.restype = _c.c_int


class CodecError(RuntimeError):
    pass


def _check(rc, what):
    if rc == -2:
        raise CodecError(f"{what}: GPU/runtime failure (see stderr)")
    return rc


# ---- reference-shaped single-group API (host buffers; numpy arrays or anything with .ctypes) ----

def cauchy_256_init(version=CAUCHY_256_VERSION):
    """_cauchy_256_init: 0 ok, -1 version mismatch (reference cauchy_256.cpp:390-399)."""
    return _check(lib._cauchy_256_init(version), "cauchy_256_init")


def cauchy_256_encode(k, m, data_ptrs, recovery_ptr, block_bytes):
    """data_ptrs: sequence of k integer addresses; recovery_ptr: address of m*block_bytes."""
    arr = (ctypes.c_void_p * max(k, 1))(*[int(p) for p in data_ptrs])
    return _check(lib.cauchy_256_encode(k, m, arr, int(recovery_ptr), block_bytes), "encode")


def cauchy_256_decode(k, m, blocks, block_bytes):
    """blocks: ctypes array of Block (modified in place, like the reference)."""
    return _check(lib.cauchy_256_decode(k, m, blocks, block_bytes), "decode")


# ---- batched device-resident API on torch tensors ----

def _ptr(t):
    return None if t is None else int(t.data_ptr())


def _stream(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return stream


def encode_batch(k, m, block_bytes, groups, data, recovery, stream=None):
    """data: uint8 cuda tensor [groups][k][B]; recovery: [groups][m][B]."""
    return _check(lib.cauchy_256_encode_batch(k, m, block_bytes, groups, _ptr(data), _ptr(recovery),
                                              _stream(stream)), "encode_batch")


def decode_batch(k, m, block_bytes, groups, blocks, rows, stream=None):
    """In place on blocks [groups][k][B] and rows [groups][k] (uint8 cuda tensors)."""
    return _check(lib.cauchy_256_decode_batch(k, m, block_bytes, groups, _ptr(blocks), _ptr(rows),
                                              _stream(stream)), "decode_batch")


def decode_batch_out(k, m, block_bytes, groups, blocks, rows, out, out_rows, out_count, stream=None):
    """Read-only blocks/rows; out [groups][min(k,m)][B], out_rows [groups][min(k,m)], out_count int32 [groups]."""
    return _check(lib.cauchy_256_decode_batch_out(k, m, block_bytes, groups, _ptr(blocks), _ptr(rows),
                                                  _ptr(out), _ptr(out_rows), _ptr(out_count),
                                                  _stream(stream)), "decode_batch_out")


def fill_synthetic(out, n, block_bytes, groups, g0, cfg, stream=None):
    return _check(lib.cauchy_256_fill_synthetic(_ptr(out), n, block_bytes, groups, g0, cfg,
                                                _stream(stream)), "fill_synthetic")


def erasure_pattern(g, k, m, cfg, e_fixed=0):
    """Synthetic decoder input rows of group g (host, no GPU): returns (e, rows uint8[k])."""
    import numpy as np
    rows = np.zeros(k, np.uint8)
    e = lib.cauchy_256_erasure_pattern(g, k, m, cfg, e_fixed, rows.ctypes.data)
    if e < 0:
        raise ValueError("erasure_pattern: bad arguments")
    return e, rows


def batch_reserve(k, m, block_bytes, groups):
    return _check(lib.cauchy_256_batch_reserve(k, m, block_bytes, groups), "batch_reserve")


def batch_errors(stream=None):
    """Malformed decode groups since the last call (waits for the stream)."""
    return _check(lib.cauchy_256_batch_errors(_stream(stream)), "batch_errors")


def has_fixed(k, m, block_bytes):
    """True when (k, m, block_bytes) runs on compile-time-scheduled kernels."""
    return lib.cauchy_256_batch_path(k, m, block_bytes) == 1


def path(k, m, block_bytes):
    """Kernel family that codes (k, m, block_bytes): "fixed" (compile-time schedules), "tile"
    (runtime-coefficient snippet tiles), "generic" (per-column kernels, B/8 < 16) or "invalid".
    Host-only: never initialises the GPU."""
    rc = lib.cauchy_256_batch_path(k, m, block_bytes)
    return {1: "fixed", 2: "tile", 0: "generic"}.get(rc, "invalid")


def default_stream():
    return lib.cauchy_256_default_stream()


def sync(stream=None):
    return _check(lib.cauchy_256_sync(stream), "sync")


def profile(capacity=64):
    """Record HIP events around the stages of the next `capacity` batched decodes (0: off;
    negative: only the two events around stage A of the next -capacity decodes)."""
    return _check(lib.cauchy_256_profile(int(capacity)), "profile")


def profile_read():
    """Mean (setup_ms, stageA_ms, stageB_ms) over the recorded decodes, or None."""
    ms = (ctypes.c_float * 3)()
    return tuple(ms) if lib.cauchy_256_profile_read(ms) > 0 else None
