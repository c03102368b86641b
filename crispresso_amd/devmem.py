"""Device buffers in the HIP runtime libcrispr_nw.so links (``/opt/rocm``'s
libamdhip64), for handing device-resident arrays between the C ABIs (e.g. the
aligner's output into nwq_run_device) without a host round trip.

torch is not used for this: it bundles a second HIP runtime, and whichever of
the two initialises second sees no GPU (probe: scripts/diag/torch_hip_order.py).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

_H2D, _D2H = 1, 2
_hip = None


def hip() -> ctypes.CDLL:
    global _hip
    if _hip is None:
        _lib.load()                                   # same runtime instance as the library's
        h = ctypes.CDLL("libamdhip64.so.7")
        h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        h.hipFree.argtypes = [ctypes.c_void_p]
        h.hipSetDevice.argtypes = [ctypes.c_int]
        _hip = h
    return _hip


class DeviceBuffer:
    """nbytes of device memory on `device`; .ptr is the device address (int)."""

    def __init__(self, nbytes: int, device: int = 0):
        h = hip()
        if h.hipSetDevice(int(device)) != 0:
            raise _lib.NativeLibraryError(f"hipSetDevice({device}) failed")
        p = ctypes.c_void_p()
        if h.hipMalloc(ctypes.byref(p), max(int(nbytes), 1)) != 0:
            raise _lib.NativeLibraryError(f"hipMalloc({nbytes}) failed")
        self.ptr, self.nbytes, self.device = int(p.value), int(nbytes), device

    @classmethod
    def from_array(cls, a: np.ndarray, device: int = 0) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes, device)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        if a.nbytes and hip().hipMemcpy(self.ptr, a.ctypes.data, a.nbytes, _H2D) != 0:
            raise _lib.NativeLibraryError("hipMemcpy H2D failed")

    def download(self, a: np.ndarray) -> np.ndarray:
        assert a.flags.c_contiguous and a.nbytes <= self.nbytes
        if a.nbytes and hip().hipMemcpy(a.ctypes.data, self.ptr, a.nbytes, _D2H) != 0:
            raise _lib.NativeLibraryError("hipMemcpy D2H failed")
        return a

    def free(self) -> None:
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()

    def __del__(self):  # pragma: no cover
        try:
            self.free()
        except Exception:
            pass
