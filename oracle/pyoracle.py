"""ctypes access to the CPU checkers -- TEST INFRASTRUCTURE ONLY.

Loads oracle/_ref/liboracle.so (our C restatement, cauchy_oracle.c) and, when present,
oracle/_ref/libref_cauchy.so (the reference codec compiled from /root/reference by
oracle/Makefile). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (shorthair_amd) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")


class Block(ctypes.Structure):
    """Reference Block descriptor (cauchy_256.h:52-55)."""
    _fields_ = [("data", ctypes.c_void_p), ("row", ctypes.c_ubyte)]


def build():
    """Compile the oracle (always) and the reference (when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load(name):
    path = os.path.join(REF_DIR, name)
    if not os.path.exists(path):
        return None
    return ctypes.CDLL(path)


class Codec:
    """Common numpy-level API over either C library (same C signatures)."""

    def __init__(self, lib, enc, dec):
        self.lib = lib
        self._enc = enc
        self._dec = dec
        self._enc.restype = ctypes.c_int
        self._enc.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        self._dec.restype = ctypes.c_int
        self._dec.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]

    def encode(self, k, m, blocks, block_bytes, out=None):
        """blocks: (k, B) uint8 array or list of 1-D arrays. Returns (rc, (m, B) recovery)."""
        ptrs = (ctypes.c_void_p * max(k, 1))()
        for i in range(k):
            ptrs[i] = blocks[i].ctypes.data
        if out is None:
            out = np.zeros((m, block_bytes), np.uint8)
        rc = self._enc(k, m, ptrs, out.ctypes.data, block_bytes)
        return rc, out

    def decode(self, k, m, datas, rows, block_bytes):
        """datas: list of k writable 1-D uint8 arrays (modified in place); rows: list of k ints.
        Returns (rc, new_rows)."""
        arr = (Block * k)()
        for i in range(k):
            arr[i].data = datas[i].ctypes.data
            arr[i].row = int(rows[i])
        rc = self._dec(k, m, arr, block_bytes)
        return rc, [arr[i].row for i in range(k)]


def oracle():
    lib = _load("liboracle.so")
    if lib is None:
        raise RuntimeError("oracle/_ref/liboracle.so missing: run `make -C oracle`")
    lib.ora_init()
    c = Codec(lib, lib.ora_encode, lib.ora_decode)
    lib.ora_cauchy_matrix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.ora_fill_block.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    lib.ora_erasure_pattern.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                        ctypes.c_int, ctypes.c_void_p]
    lib.ora_erasure_pattern.restype = ctypes.c_int
    lib.ora_gf_mul.restype = ctypes.c_ubyte
    lib.ora_gf_mul.argtypes = [ctypes.c_ubyte, ctypes.c_ubyte]
    lib.ora_gf_div.restype = ctypes.c_ubyte
    lib.ora_gf_div.argtypes = [ctypes.c_ubyte, ctypes.c_ubyte]
    lib.ora_gf_inv.restype = ctypes.c_ubyte
    lib.ora_gf_inv.argtypes = [ctypes.c_ubyte]
    return c


def reference():
    """The real reference codec, or None if it was not built (e.g. no /root/reference)."""
    lib = _load("libref_cauchy.so")
    if lib is None:
        return None
    lib._cauchy_256_init.restype = ctypes.c_int
    lib._cauchy_256_init.argtypes = [ctypes.c_int]
    if lib._cauchy_256_init(2) != 0:
        raise RuntimeError("reference _cauchy_256_init(2) failed")
    return Codec(lib, lib.cauchy_256_encode, lib.cauchy_256_decode)


def cauchy_matrix(k, m):
    """(m-1, k) uint8 generator rows 1..m-1 from the oracle."""
    c = oracle()
    out = np.zeros((m - 1, k), np.uint8)
    c.lib.ora_cauchy_matrix(k, m, out.ctypes.data)
    return out


def fill_group(g, k, block_bytes, cfg):
    """Synthetic input of group g: (k, B) uint8 (see ora_fill_block)."""
    c = oracle()
    out = np.empty((k, block_bytes), np.uint8)
    for x in range(k):
        c.lib.ora_fill_block(g, x, cfg, out[x].ctypes.data, block_bytes)
    return out


def erasure_pattern(g, k, m, cfg, e_fixed=0):
    """Decoder input rows for group g (survivors ascending, then recovery rows); returns (e, rows)."""
    c = oracle()
    rows = np.zeros(k, np.uint8)
    e = c.lib.ora_erasure_pattern(g, k, m, cfg, e_fixed, rows.ctypes.data)
    return e, rows
