"""ctypes wrapper of the CPU oracle (oracle/_build/liboracle_nw.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / baseline, never as the
product path.  Parity vs EMBOSS needle itself is unpinned (see nw_oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_int64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(BUILD, "liboracle_nw.so")
CLI = os.path.join(BUILD, "needle_oracle")


class OracleParams(ctypes.Structure):
    _fields_ = [("scale", c_int32), ("gap_open", c_int32), ("gap_extend", c_int32),
                ("gap_open_f", c_float), ("gap_extend_f", c_float), ("end_weight", c_int32),
                ("end_open", c_int32), ("end_extend", c_int32)]


class OracleResult(ctypes.Structure):
    _fields_ = [("aln_len", c_int32), ("n_ident", c_int32), ("n_sim", c_int32), ("n_gaps", c_int32),
                ("score", c_int32), ("end_i", c_int32), ("end_j", c_int32), ("read_end", c_int32),
                ("ref_end", c_int32)]


RESULT_DTYPE = np.dtype([(f, "<i4") for f, _ in OracleResult._fields_])

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    lib.oracle_params_init.argtypes = [POINTER(OracleParams), c_float, c_float]
    lib.oracle_params_init.restype = c_int
    lib.oracle_params_init_end.argtypes = [POINTER(OracleParams), c_float, c_float, c_int, c_float, c_float]
    lib.oracle_params_init_end.restype = c_int
    lib.oracle_align.argtypes = [c_char_p, c_int32, c_char_p, c_int32, POINTER(OracleParams),
                                 POINTER(OracleResult), c_void_p, c_void_p, c_void_p]
    lib.oracle_align.restype = c_int
    lib.oracle_score.argtypes = [c_char_p, c_int32, c_char_p, c_int32, POINTER(OracleParams)]
    lib.oracle_score.restype = c_int32
    lib.oracle_align_batch.argtypes = [c_char_p, c_int32, c_void_p, c_void_p, c_int32, POINTER(OracleParams),
                                       c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64]
    lib.oracle_align_batch.restype = c_int
    lib.oracle_format_srspair.argtypes = [c_void_p, c_int64, c_char_p, c_char_p, POINTER(OracleParams),
                                          POINTER(OracleResult), c_char_p, c_char_p, c_char_p]
    lib.oracle_format_srspair.restype = c_int64
    lib.oracle_code.argtypes = [ctypes.c_ubyte]
    lib.oracle_code.restype = c_int
    lib.oracle_sub.argtypes = [c_int, c_int]
    lib.oracle_sub.restype = c_int
    _lib = lib
    return lib


def params(gap_open: float = 10.0, gap_extend: float = 0.5, end_weight: bool = False, end_open: float = 10.0,
           end_extend: float = 0.5) -> OracleParams:
    p = OracleParams()
    if load().oracle_params_init_end(ctypes.byref(p), gap_open, gap_extend, int(bool(end_weight)), end_open,
                                     end_extend) != 0:
        raise ValueError("penalties not representable")
    return p


def align(amplicon: str, read: str, p: OracleParams | None = None):
    """-> (result dict, ref_aln, markup, read_aln)."""
    p = p or params()
    lib = load()
    a, b = amplicon.encode(), read.encode()
    cap = len(a) + len(b) + 1
    ra, mk, rb = (ctypes.create_string_buffer(cap) for _ in range(3))
    r = OracleResult()
    if lib.oracle_align(a, len(a), b, len(b), ctypes.byref(p), ctypes.byref(r), ra, mk, rb) != 0:
        raise ValueError("oracle_align failed")
    res = {f: getattr(r, f) for f, _ in OracleResult._fields_}
    return res, ra.value.decode(), mk.value.decode(), rb.value.decode()


def score(amplicon: str, read: str, p: OracleParams | None = None) -> int:
    p = p or params()
    a, b = amplicon.encode(), read.encode()
    return int(load().oracle_score(a, len(a), b, len(b), ctypes.byref(p)))


def align_batch(amplicon: str, buf: np.ndarray, offsets: np.ndarray, p: OracleParams | None = None,
                nthreads: int = 1):
    """-> (results structured array, aln uint8 [n, 3, stride])."""
    p = p or params()
    lib = load()
    n = len(offsets) - 1
    lens = np.diff(offsets)
    stride = len(amplicon) + (int(lens.max()) if n else 0) + 1
    res = np.zeros(n, dtype=RESULT_DTYPE)
    aln = np.zeros((n, 3, stride), dtype=np.uint8)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    a = amplicon.encode()
    base = aln.ctypes.data
    rc = lib.oracle_align_batch(a, len(a), buf.ctypes.data, offsets.ctypes.data, n, ctypes.byref(p), nthreads,
                                res.ctypes.data, base, base + stride, base + 2 * stride, 3 * stride)
    if rc != 0:
        raise ValueError("oracle_align_batch failed")
    return res, aln


def srspair(amplicon_name: str, read_name: str, result: dict, ref_aln: str, markup: str, read_aln: str,
            p: OracleParams | None = None) -> str:
    p = p or params()
    lib = load()
    r = OracleResult(*[result[f] for f, _ in OracleResult._fields_])
    args = (amplicon_name.encode(), read_name.encode(), ctypes.byref(p), ctypes.byref(r), ref_aln.encode(),
            markup.encode(), read_aln.encode())
    need = lib.oracle_format_srspair(None, 0, *args)
    buf = ctypes.create_string_buffer(int(need) + 1)
    lib.oracle_format_srspair(buf, int(need) + 1, *args)
    return buf.raw[:need].decode()
