"""ctypes binding of ``libcrispr_nw.so`` (C ABI declared in ``include/crispr_nw.h``).

This is the in-process replacement of the ``needle`` subprocess boundary of
CRISPResso (``CRISPResso/CRISPRessoCORE.py:1788-1806``).  The library is built
in-tree by ``__graft_entry__.build()`` (``crispresso_amd/csrc/Makefile``).  There
is deliberately no CPU fallback: if the library or a GPU is missing every entry
point raises :class:`NativeLibraryError`.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_int64, c_void_p

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                        os.environ.get("CRISPR_NW_LIB", "libcrispr_nw.so"))   # variant builds (experiments)

NW_OK = 0
NW_E_INVALID = -1
NW_E_INEXACT = -2
NW_E_UNSUPPORTED = -3
NW_E_HIP = -4
NW_E_NOMEM = -5
NW_E_STATE = -6
NW_E_CAPACITY = -7
NW_TIE_EMBOSS = 0
NW_FLAG_EMPTY = 1
NW_OUT_ROWS, NW_OUT_OPS = 0, 1
NW_RUN_M, NW_RUN_X, NW_RUN_Y = 0, 1, 2
TB_MODES = {0: "full-lds", 1: "full-global", 5: "diag-int16"}

# Field order of nw_stat (include/crispr_nw.h).
STAT_FIELDS = ("aln_len", "n_ident", "n_sim", "n_gaps", "score", "end_i", "end_j", "flags")
STAT_DTYPE = np.dtype([(f, "<i4") for f in STAT_FIELDS])

# Every symbol include/crispr_nw.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "nw_create", "nw_destroy", "nw_last_error", "nw_set_params", "nw_score_scale",
    "nw_set_reference", "nw_required_stride", "nw_align_batch", "nw_batch_upload", "nw_batch_upload_packed",
    "nw_batch_run_async", "nw_batch_sync", "nw_batch_download", "nw_batch_algo_bytes",
    "nw_batch_cells", "nw_batch_geometry", "nw_batch_fallbacks", "nw_batch_kernel_times",
    "nw_align_multi", "nw_required_stride_multi", "nw_format_srspair", "nw_batch_device_output",
    "nw_batch_set_output", "nw_batch_download_ops", "nw_align_ops", "nw_ops_times", "nw_host_alloc", "nw_host_free",
    "nw_host_register", "nw_host_unregister", "nw_host_threads", "nw_batch_set_lane_walk", "nw_batch_set_phase_events", "nw_set_known", "nw_expand_ops", "nw_batch_phase_times", "nw_batch_path_counts", "nw_batch_exact_reads",
    "nw_align_ops_packed_lens", "nw_align_multi_ops_packed_lens", "nw_align_dual_ops_packed_lens", "nw_read_lengths16", "nw_fastq_lens",
    "nw_align_ops_resident", "nw_align_multi_ops", "nw_align_multi_ops_packed", "nw_align_ops_packed", "nw_pack_reads",
    "nw_fastq_read", "nw_fastq_read_filtered", "nw_fastq_dropped", "nw_fastq_pass", "nw_fastq_count", "nw_fastq_seqs", "nw_fastq_offsets", "nw_fastq_names", "nw_fastq_free",
    "nw_expand_ops_subset", "nw_reads_equal_ref", "nw_reads_first_copy", "nw_names_to_ids", "nw_gunzip_parallel", "nw_ops_rows_concat", "nw_fastq_pack", "nw_batch_device_ops",
)

# Every symbol include/crispr_quant.h declares.
QUANT_EXPORTS = (
    "nwq_create", "nwq_destroy", "nwq_last_error", "nwq_set_params", "nwq_totals_words", "nwq_run",
    "nwq_run_device", "nwq_run_device_ops", "nwq_lane_fallbacks",
)


# Every symbol include/crispr_flash.h declares.
FLASH_EXPORTS = ("nwf_merge_batch", "nwf_last_error")

# Every symbol include/crispr_synth.h declares (bench / test input generator).
SYNTH_EXPORTS = ("nw_synth_offsets", "nw_synth_reads")
NWF_COMBINED, NWF_OUTIE = 1, 2


class NwfParams(ctypes.Structure):
    """nwf_params (include/crispr_flash.h)."""
    _fields_ = [("min_overlap", c_int32), ("max_overlap", c_int32), ("max_mismatch_density", c_float),
                ("allow_outies", c_int32), ("phred_offset", c_int32), ("cap_mismatch_quals", c_int32)]


class NwqParams(ctypes.Structure):
    """nwq_params (include/crispr_quant.h)."""
    _fields_ = [("len_amplicon", c_int32), ("include_mask", c_void_p), ("exon_mask", c_void_p),
                ("splicing_mask", c_void_p), ("ignore_substitutions", c_int32), ("ignore_insertions", c_int32),
                ("ignore_deletions", c_int32), ("window_around_sgrna", c_int32),
                ("hide_mutations_outside_window_nhej", c_int32), ("amplicon_has_n", c_int32)]


NWQ_PRE_UNMODIFIED, NWQ_PRE_HDR, NWQ_PRE_MIXED = 1, 2, 4
NWQ_NVEC, NWQ_NCOUNTERS = 15, 4
NWQ_READ_DTYPE = np.dtype([(f, "<i4") for f in ("cls", "n_mutated", "n_inserted", "n_deleted")])


class NativeLibraryError(RuntimeError):
    """The HIP library is missing, failed to load, or a call failed."""


_lib = None


def load() -> ctypes.CDLL:
    """Load and type the shared library once; raise loudly when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as exc:  # pragma: no cover - depends on the ROCm install
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {exc}") from exc
    ctx_p = c_void_p
    sig = {
        "nw_create": (c_int, [c_int, POINTER(c_void_p)]),
        "nw_destroy": (None, [ctx_p]),
        "nw_last_error": (c_char_p, [ctx_p]),
        "nw_set_params": (c_int, [ctx_p, c_float, c_float, c_int, c_float, c_float, c_char_p, c_int]),
        "nw_score_scale": (c_int, [ctx_p]),
        "nw_set_reference": (c_int, [ctx_p, c_char_p, c_int32]),
        "nw_required_stride": (c_int64, [ctx_p, c_int32]),
        "nw_align_batch": (c_int, [ctx_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p]),
        "nw_batch_upload": (c_int, [ctx_p, c_void_p, c_void_p, c_int64]),
        "nw_batch_upload_packed": (c_int, [ctx_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64]),
        "nw_batch_run_async": (c_int, [ctx_p]),
        "nw_batch_sync": (c_int, [ctx_p, POINTER(c_float)]),
        "nw_batch_download": (c_int, [ctx_p, c_void_p, c_int64, c_void_p]),
        "nw_batch_algo_bytes": (c_int64, [ctx_p]),
        "nw_batch_cells": (c_int64, [ctx_p]),
        "nw_batch_geometry": (c_int, [ctx_p] + [POINTER(c_int32)] * 5),
        "nw_batch_fallbacks": (c_int64, [ctx_p]),
        "nw_batch_kernel_times": (c_int, [ctx_p] + [POINTER(c_float)] * 3),
        "nw_align_multi": (c_int, [ctx_p, c_char_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int64,
                                   c_void_p, c_int64, c_void_p]),
        "nw_required_stride_multi": (c_int64, [c_void_p, c_int32, c_int32]),
        "nw_batch_device_output": (c_int, [ctx_p, POINTER(c_void_p), POINTER(c_int64), POINTER(c_void_p)]),
        "nw_batch_set_output": (c_int, [ctx_p, c_int]),
        "nw_batch_device_ops": (c_int, [ctx_p] + [POINTER(c_void_p)] * 5 + [POINTER(c_int64)] * 2),
        "nw_batch_phase_times": (c_int, [ctx_p, c_void_p]),
        "nw_batch_path_counts": (c_int, [ctx_p, c_void_p]),
        "nw_batch_exact_reads": (c_int64, [ctx_p]),
        "nw_batch_download_ops": (c_int, [ctx_p, c_void_p, c_int64, c_void_p, c_void_p]),
        "nw_align_ops": (c_int, [ctx_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
        "nw_align_ops_resident": (c_int, [ctx_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
        "nw_fastq_read": (c_int, [c_char_p, POINTER(c_void_p)]),
        "nw_fastq_read_filtered": (c_int, [c_char_p, c_int32, c_int32, POINTER(c_void_p)]),
        "nw_fastq_dropped": (c_int64, [c_void_p]),
        "nw_fastq_pass": (c_void_p, [c_void_p, POINTER(c_int64)]),
        "nw_expand_ops_subset": (c_int, [c_char_p, c_int32, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                         c_void_p, c_int64, c_int32]),
        "nw_ops_rows_concat": (c_int, [c_char_p, c_int32, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32]),
        "nw_reads_equal_ref": (c_int64, [c_char_p, c_int32, c_void_p, c_void_p, c_int64, c_void_p, c_int32]),
        "nw_reads_first_copy": (c_int64, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int32]),
        "nw_names_to_ids": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
        "nw_gunzip_parallel": (c_int, [c_void_p, c_int64, c_int32, c_void_p, c_int64, c_void_p]),
        "nw_fastq_count": (c_int64, [c_void_p]),
        "nw_fastq_seqs": (c_void_p, [c_void_p]),
        "nw_fastq_offsets": (c_void_p, [c_void_p]),
        "nw_fastq_names": (c_void_p, [c_void_p, POINTER(c_int64)]),
        "nw_fastq_free": (None, [c_void_p]),
        "nw_fastq_pack": (c_int, [c_void_p, c_int32] + [POINTER(c_void_p)] * 4 + [POINTER(c_int64)]),
        "nw_align_ops_packed": (c_int, [ctx_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p,
                                        c_int64, c_void_p, c_void_p]),
        "nw_pack_reads": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                                  c_int32]),
        "nw_align_multi_ops": (c_int, [ctx_p, c_char_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int64,
                                       c_void_p, c_int64, c_void_p, c_void_p]),
        "nw_align_multi_ops_packed": (c_int, [ctx_p, c_char_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                              c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                              c_void_p]),
        "nw_align_ops_packed_lens": (c_int, [ctx_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                                             c_void_p, c_int64, c_void_p, c_void_p]),
        "nw_align_multi_ops_packed_lens": (c_int, [ctx_p, c_char_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                                   c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_int64,
                                                   c_void_p, c_void_p]),
        "nw_align_dual_ops_packed_lens": (c_int, [ctx_p, c_char_p, c_int32, c_void_p, c_void_p, c_void_p, c_int64,
                                                  c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                                  c_void_p, c_int64, c_void_p, c_void_p]),
        "nw_read_lengths16": (c_int, [c_void_p, c_int64, c_void_p, c_int32]),
        "nw_fastq_lens": (c_int, [c_void_p, POINTER(c_void_p)]),
        "nw_ops_times": (c_int, [ctx_p, POINTER(c_float), POINTER(c_float), POINTER(c_int64), POINTER(c_int64)]),
        "nw_host_alloc": (c_int, [c_int64, POINTER(c_void_p)]),
        "nw_host_free": (None, [c_void_p]),
        "nw_host_threads": (c_int, []),
        "nw_batch_set_lane_walk": (c_int, [ctx_p, c_int]),
        "nw_batch_set_phase_events": (c_int, [ctx_p, c_int]),
        "nw_set_known": (c_int, [ctx_p, c_char_p, c_int32]),
        "nw_host_register": (c_int, [c_void_p, c_int64]),
        "nw_host_unregister": (c_int, [c_void_p]),
        "nw_expand_ops": (c_int, [c_char_p, c_int32, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                                  c_int32]),
        "nwf_merge_batch": (c_int, [c_int, POINTER(NwfParams)] + [c_void_p] * 6 + [c_int64] + [c_void_p] * 4
                            + [POINTER(c_float)]),
        "nwf_last_error": (c_char_p, []),
        "nwq_create": (c_int, [c_int, POINTER(c_void_p)]),
        "nwq_destroy": (None, [ctx_p]),
        "nwq_last_error": (c_char_p, [ctx_p]),
        "nwq_set_params": (c_int, [ctx_p, POINTER(NwqParams)]),
        "nwq_totals_words": (c_int64, [ctx_p, c_int64]),
        "nwq_run": (c_int, [ctx_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                            POINTER(c_float)]),
        "nwq_run_device": (c_int, [ctx_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                   c_void_p, POINTER(c_float)]),
        "nwq_lane_fallbacks": (c_int64, [ctx_p]),
        "nwq_run_device_ops": (c_int, [ctx_p, c_char_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p, POINTER(c_float)]),
        "nw_synth_offsets": (c_int64, [c_char_p, c_int32, c_int64, c_int64, ctypes.c_uint64, c_void_p, c_void_p,
                                        c_int32]),
        "nw_synth_reads": (c_int, [c_char_p, c_int32, c_int64, c_int64, ctypes.c_uint64, c_void_p, c_void_p,
                                   c_void_p, c_int32]),
        "nw_format_srspair": (
            c_int64,
            [c_void_p, c_int64, c_char_p, c_char_p, c_float, c_float, c_int32, c_int32, c_void_p, c_int64,
             c_void_p, c_int64],
        ),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None:   # a stale build: a use of the entry point says so (build() checks every symbol)
            _MISSING.add(name)
            setattr(lib, name, _stale(name))
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


_MISSING: set = set()


def _stale(name: str):
    def call(*_a, **_k):
        raise RuntimeError(f"libcrispr_nw.so is out of date: it does not export {name} "
                           "(rebuild it: make -C crispresso_amd/csrc)")
    return call


def has_symbol(name: str) -> bool:
    """Whether the loaded library exports ``name`` (False for an out-of-date build)."""
    lib = load()
    return name not in _MISSING and getattr(lib, name, None) is not None


def exported_symbols() -> dict:
    """Map of each declared symbol to whether the loaded library exports it."""
    lib = load()
    out = {}
    for name in EXPORTS + QUANT_EXPORTS + FLASH_EXPORTS + SYNTH_EXPORTS:
        try:
            getattr(lib, name)
            out[name] = name not in _MISSING
        except AttributeError:
            out[name] = False
    return out


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None else 0


class _PinnedOwner:
    """Owns one page-locked block (nw_host_alloc); numpy arrays made from it
    (``np.asarray``) keep it alive through their ``base``, and the block is freed when
    the last of them and its :class:`PinnedBuffer` are gone (or at an explicit close)."""

    def __init__(self, lib, p: int, nbytes: int):
        self._lib, self._p = lib, p
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "version": 3, "data": (p, False)}

    def free(self):
        if getattr(self, "_p", None):
            self._lib.nw_host_free(self._p)
            self._p = None

    def __del__(self):  # pragma: no cover - runs at garbage collection
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host memory (nw_host_alloc) viewed as a numpy array.  Batches in
    pinned memory let nw_align_ops copy at PCIe rate.  The memory lives while this
    object or any array viewing it does (``PinnedBuffer(n, dt).array`` alone is safe);
    ``close()`` frees it at once (the caller's promise that no view is used after)."""

    def __init__(self, shape, dtype):
        self.lib = load()
        dtype = np.dtype(dtype)
        count = int(np.prod(shape)) if np.ndim(shape) else int(shape)
        nbytes = max(count * dtype.itemsize, 1)
        p = ctypes.c_void_p()
        if self.lib.nw_host_alloc(nbytes, ctypes.byref(p)) != NW_OK:
            raise NativeLibraryError(f"nw_host_alloc({nbytes}) failed")
        self._p = p.value
        self._owner = _PinnedOwner(self.lib, self._p, nbytes)
        self.array = np.asarray(self._owner)[: count * dtype.itemsize].view(dtype).reshape(shape)

    def close(self):
        if getattr(self, "_p", None):
            self.array = None
            self._owner.free()
            self._p = None


def pinned_copy(a: np.ndarray) -> PinnedBuffer:
    """A pinned copy of `a` (same shape and dtype)."""
    pb = PinnedBuffer(a.shape, a.dtype)
    pb.array[...] = a
    return pb


class _Lease:
    """One view of pinned memory handed out by :class:`PinnedPool`: numpy arrays made
    from it (``np.asarray``) keep it alive through their ``base``; when the last one
    goes the block returns to the pool (it is never freed while a view exists)."""

    def __init__(self, pool: "PinnedPool", block: "PinnedBuffer", nbytes: int):
        self._pool, self._block = pool, block
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "version": 3,
                                    "data": (block._p, False)}

    def __del__(self):  # pragma: no cover - runs at garbage collection
        pool, block = getattr(self, "_pool", None), getattr(self, "_block", None)
        if pool is not None and block is not None:
            pool._release(block)


class PinnedPool:
    """Reusable page-locked blocks for the aligner's outputs (records, run offsets, runs).

    A call's results must land in pinned memory for the copies to run at PCIe rate, but
    page-locking a fresh buffer per call costs more than the call (hipHostMalloc of tens
    of MB).  ``array(shape, dtype)`` leases a block at least that large (reusing a free
    one); the block goes back to the pool when every array viewing it is gone, so results
    a caller keeps are never overwritten.  Blocks are kept (not freed) for the process's
    lifetime, up to ``keep_bytes`` of free blocks."""

    def __init__(self, keep_bytes: int = 2 << 30):
        import collections
        import threading

        self._free: list = []
        self._keep = keep_bytes
        self._mu = threading.Lock()
        # blocks handed back by _Lease.__del__: a lock-free hand-off, since a lease can be
        # finalised by the cyclic GC inside array() while this thread holds _mu
        self._returned = collections.deque()

    def array(self, shape, dtype) -> np.ndarray:
        dtype = np.dtype(dtype)
        count = int(np.prod(shape)) if np.ndim(shape) else int(shape)
        nbytes = max(count * dtype.itemsize, 1)
        with self._mu:
            self._drain()
            fits = [b for b in self._free if b.nbytes >= nbytes]
            block = min(fits, key=lambda b: b.nbytes) if fits else None
            if block is not None:
                self._free.remove(block)
        if block is None:
            # rounded up (steps of 1/16 of the size) so a slightly bigger batch reuses the block
            step = max(4096, 1 << max(0, nbytes.bit_length() - 4))
            cap = (nbytes + step - 1) // step * step
            block = PinnedBuffer(cap, np.uint8)
            block.nbytes = cap
        raw = np.asarray(_Lease(self, block, nbytes))
        return raw[: count * dtype.itemsize].view(dtype).reshape(shape)

    def _release(self, block: "PinnedBuffer") -> None:
        self._returned.append(block)   # no lock (deque.append is atomic); taken in by _drain
        # trim now when nobody holds the lock (a lease finalised by the cyclic GC inside array()
        # finds it held and leaves the trimming to the next array() / free_bytes())
        if self._mu.acquire(blocking=False):
            try:
                self._drain()
            finally:
                self._mu.release()

    def _drain(self) -> None:
        """Move returned blocks to the free list, trimmed to keep_bytes (caller holds _mu)."""
        while self._returned:
            self._free.append(self._returned.popleft())
        total = sum(b.nbytes for b in self._free)
        while total > self._keep and self._free:
            big = max(self._free, key=lambda b: b.nbytes)
            self._free.remove(big)
            total -= big.nbytes
            big.close()

    def free_bytes(self) -> int:
        with self._mu:
            self._drain()
            return sum(b.nbytes for b in self._free)


_pool = None


def pinned_pool() -> PinnedPool:
    """The process-wide pool of pinned output blocks."""
    global _pool
    if _pool is None:
        _pool = PinnedPool()
    return _pool
