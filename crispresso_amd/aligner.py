"""GPU aligner: the object that stands where one ``needle`` process stood.

Each ``needle`` invocation in the reference (``CRISPRessoCORE.py:1797-1801``
forward, ``1818-1822`` HDR, ``1913-1917`` RC, ``1926-1930`` RC-HDR) aligns a stream
of reads against ONE amplicon with the options of ``--needle_options_string``.
:class:`GpuAligner` is that, in-process: set the amplicon once, align batches.
Results come back as an :class:`AlignmentBatch` whose fields are exactly what
``parse_needle_output`` (``CRISPRessoCORE.py:1707-1786``) extracts from the
srspair text, plus the text itself when a file is wanted.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .needle_options import NeedleOptions


class NeedleError(RuntimeError):
    """Raised where the reference raises NeedleException (CRISPRessoCORE.py:381)."""


def pack_reads(reads: Sequence) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate reads (str or bytes) into one uint8 buffer + int64 offsets."""
    enc = [r.encode("ascii") if isinstance(r, str) else bytes(r) for r in reads]
    lens = np.fromiter((len(r) for r in enc), dtype=np.int64, count=len(enc))
    offsets = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    buf = np.frombuffer(b"".join(enc), dtype=np.uint8) if enc else np.zeros(0, np.uint8)
    return np.ascontiguousarray(buf), offsets


_ident_cache: dict = {}


def printed_percent(num: int, den: int) -> float:
    """Value parse_needle_output reads back: eval of the "%4.1f" identity token."""
    key = (int(num), int(den))
    v = _ident_cache.get(key)
    if v is None:
        v = float("%.1f" % (100.0 * num / den)) if den else 0.0
        _ident_cache[key] = v
    return v


@dataclass
class AlignmentBatch:
    """Alignments of one batch against one amplicon (host copies)."""

    stats: np.ndarray        # structured, _lib.STAT_DTYPE
    aln: np.ndarray          # uint8 [n, 3, stride]: aligned amplicon, markup, aligned read
    read_lens: np.ndarray    # int64 [n]
    scale: int
    awidth: int = 5000

    def __len__(self) -> int:
        return len(self.stats)

    def _cols(self, i: int) -> int:
        return int(min(self.stats["aln_len"][i], self.awidth))

    def ref_seq(self, i: int) -> str:
        return self.aln[i, 0, : self._cols(i)].tobytes().decode("ascii")

    def align_str(self, i: int) -> str:
        return self.aln[i, 1, : self._cols(i)].tobytes().decode("ascii")

    def align_seq(self, i: int) -> str:
        return self.aln[i, 2, : self._cols(i)].tobytes().decode("ascii")

    def identity(self, i: int) -> float:
        s = self.stats[i]
        return printed_percent(s["n_ident"], s["aln_len"])

    def score(self, i: int) -> float:
        return float(self.stats["score"][i]) / self.scale

    def read_end(self, i: int) -> str:
        """``split()[3]`` of the read line: last read coordinate on the first line."""
        seg = self.aln[i, 2, : self._cols(i)]
        return str(int(np.count_nonzero(seg != ord("-"))))

    def empty(self, i: int) -> bool:
        return bool(self.stats["flags"][i] & _lib.NW_FLAG_EMPTY)


class OpsBatch:
    """Alignments of one batch as traceback runs (nw_align_ops): what crosses PCIe.

    Read r's runs are ``ops[ops_off[r]:ops_off[r + 1]]`` (``type << 28 | length``,
    start -> end; ``_lib.NW_RUN_M / X / Y``).  :meth:`expand` rebuilds the three
    alignment rows on the host (``nw_expand_ops``).  ``read_lens`` may be given as the
    batch's offsets (``offsets=``) and is then computed on first use (not inside the
    aligner call)."""

    def __init__(self, stats: np.ndarray, ops: np.ndarray, ops_off: np.ndarray, read_lens: Optional[np.ndarray],
                 scale: int, awidth: int = 5000, offsets: Optional[np.ndarray] = None, has_runs: bool = True):
        self.stats = stats             # structured, _lib.STAT_DTYPE
        self.ops = ops                 # uint32 runs
        self.ops_off = ops_off         # int64 [n + 1] (a records-only batch: the runs' offsets, no runs)
        self.has_runs = has_runs
        self._read_lens = read_lens    # int64 [n]
        self._offsets = offsets
        self.scale = scale
        self.awidth = awidth

    @property
    def read_lens(self) -> np.ndarray:
        if self._read_lens is None:
            self._read_lens = np.diff(self._offsets)
        return self._read_lens

    def __len__(self) -> int:
        return len(self.stats)

    def runs(self, i: int) -> List[Tuple[int, int]]:
        seg = self.ops[self.ops_off[i]:self.ops_off[i + 1]]
        return [(int(v) >> 28, int(v) & 0x0FFFFFFF) for v in seg]

    def expand(self, reference: str, buf: np.ndarray, offsets: np.ndarray, nthreads: int = 0,
               rows: Optional[np.ndarray] = None) -> "AlignmentBatch":
        """The three rows per read (host C++, ``nthreads`` threads; 0 = all cores)."""
        lib = _lib.load()
        n = len(self)
        ref = reference.encode("ascii")
        max_len = int(self.read_lens.max()) if n else 1
        stride = (len(ref) + max(max_len, 1) + 15) & ~15
        if rows is None:
            rows = np.zeros((n, 3, stride), dtype=np.uint8)
        buf = np.ascontiguousarray(buf)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        ops = np.ascontiguousarray(self.ops, dtype=np.uint32)
        rc = lib.nw_expand_ops(ref, len(ref), _lib.ptr(buf), _lib.ptr(offsets), n, _lib.ptr(ops) if len(ops) else None,
                               _lib.ptr(self.ops_off), _lib.ptr(rows), rows.shape[2], int(nthreads))
        if rc != _lib.NW_OK:
            raise NeedleError(f"nw_expand_ops: runs do not match the reads (code {rc})")
        return AlignmentBatch(self.stats, rows, self.read_lens, self.scale, self.awidth)


@dataclass
class PackedReads:
    """A batch as 2 bits per base + exceptions (nw_pack_reads): what nw_align_ops_packed
    sends over PCIe.  ``packed`` is indexed by batch position (byte i // 4)."""

    packed: np.ndarray       # uint8
    offsets: np.ndarray      # int64 [n + 1], the text's offsets
    exc_pos: np.ndarray      # int64, ascending
    exc_byte: np.ndarray     # uint8
    lens: Optional[np.ndarray] = None   # uint16 [n] read lengths: they cross PCIe instead of the offsets


def read_lengths16(offsets: np.ndarray, out: Optional[np.ndarray] = None) -> Optional[np.ndarray]:
    """uint16 read lengths for nw_align_ops_packed_lens (nw_read_lengths16), or None when a
    read is longer than 65535.  ``out``: a preallocated (e.g. pinned) uint16 array of n."""
    lib = _lib.load()
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    n = len(offsets) - 1
    lens = out if out is not None else np.empty(max(n, 1), np.uint16)
    rc = lib.nw_read_lengths16(_lib.ptr(offsets), n, _lib.ptr(lens), 0)
    if rc == _lib.NW_E_UNSUPPORTED:
        return None
    if rc != _lib.NW_OK:
        raise NeedleError(f"nw_read_lengths16 failed (code {rc})")
    return lens[:n]


def pack_2bit(buf: np.ndarray, offsets: np.ndarray, nthreads: int = 0, packed: Optional[np.ndarray] = None,
              exc_cap: int = 0, lens: Optional[np.ndarray] = None) -> PackedReads:
    """2-bit pack a text batch (host C++, ``nthreads`` threads; 0 = all cores).  ``packed``
    may be a preallocated (e.g. pinned) uint8 array of (offsets[-1] + 3) // 4 bytes; the
    read lengths go into ``lens`` (uint16 [n], e.g. pinned) or a new array."""
    lib = _lib.load()
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    n = len(offsets) - 1
    nbytes = (int(offsets[-1]) + 3) // 4 if n else 0
    if packed is None:
        packed = np.zeros(max(nbytes, 1), np.uint8)
    cap = exc_cap or max(1024, (int(offsets[-1]) - int(offsets[0])) // 64 if n else 1024)
    for _ in range(2):
        pos = np.empty(cap, np.int64)
        byt = np.empty(cap, np.uint8)
        cnt = ctypes.c_int64()
        rc = lib.nw_pack_reads(_lib.ptr(buf), _lib.ptr(offsets), n, _lib.ptr(packed), _lib.ptr(pos), _lib.ptr(byt),
                               cap, ctypes.byref(cnt), int(nthreads))
        if rc == _lib.NW_E_CAPACITY:
            cap = int(cnt.value)
            continue
        if rc != _lib.NW_OK:
            raise NeedleError(f"nw_pack_reads failed (code {rc})")
        return PackedReads(packed, offsets, pos[: cnt.value], byt[: cnt.value], read_lengths16(offsets, lens))
    raise NeedleError("nw_pack_reads: exception list kept growing")


def _outputs(n: int, runs: bool = True):
    """(stats, ops, ops_off) for an n-read call, leased from the pinned pool."""
    pool = _lib.pinned_pool()
    return (pool.array(n, _lib.STAT_DTYPE), pool.array(2 * n + 4096 if runs else 0, np.uint32),
            pool.array(n + 1, np.int64))


def default_output_mode() -> str:
    """``CRISPR_NW_OUTPUT``: "ops" (default: runs over PCIe, rows built on the host)
    or "rows" (the kernels write the rows, which cross PCIe)."""
    mode = os.environ.get("CRISPR_NW_OUTPUT", "ops")
    if mode not in ("ops", "rows"):
        raise ValueError(f"CRISPR_NW_OUTPUT={mode!r}: expected 'ops' or 'rows'")
    return mode


class GpuAligner:
    """One GPU context aligning reads to one amplicon at a time."""

    ops_native = True   # align_ops runs on the device (host code may take the ops path)

    def __init__(self, device: int = 0, options: Optional[NeedleOptions] = None):
        self.lib = _lib.load()
        self.options = options or NeedleOptions()
        h = ctypes.c_void_p()
        rc = self.lib.nw_create(int(device), ctypes.byref(h))
        if rc != _lib.NW_OK:
            raise _lib.NativeLibraryError(f"nw_create(device={device}) failed with code {rc} (no usable GPU?)")
        self._h = h
        self.device = device
        o = self.options
        self._check(
            self.lib.nw_set_params(
                self._h, o.gap_open, o.gap_extend, int(o.end_weight), o.end_open, o.end_extend,
                o.matrix.encode(), _lib.NW_TIE_EMBOSS,
            ),
            "nw_set_params",
        )
        self.scale = int(self.lib.nw_score_scale(self._h))
        self.reference: Optional[str] = None

    def _check(self, rc: int, what: str) -> None:
        if rc != _lib.NW_OK:
            msg = self.lib.nw_last_error(self._h).decode(errors="replace")
            raise NeedleError(f"{what}: {msg} (code {rc})")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.nw_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_reference(self, seq: str) -> None:
        b = seq.encode("ascii")
        self._check(self.lib.nw_set_reference(self._h, b, len(b)), "nw_set_reference")
        self.reference = seq

    # -- device-resident path (bench) ------------------------------------
    def upload(self, buf: np.ndarray, offsets: np.ndarray) -> None:
        self._buf, self._off = buf, offsets
        self._check(self.lib.nw_batch_upload(self._h, _lib.ptr(buf), _lib.ptr(offsets), len(offsets) - 1),
                    "nw_batch_upload")

    def upload_packed(self, pr: "PackedReads") -> None:
        """Resident batch in the packed call's layout (nw_batch_upload_packed, ops output):
        run_async then times the kernels nw_align_ops_packed_lens runs (in one launch each over
        the whole batch; set_lane_walk(True) swaps the first level's walk for the lane walk)."""
        if pr.lens is None:
            raise NeedleError("upload_packed needs the reads' lengths (PackedReads.lens)")
        self.set_output("ops")
        n = len(pr.offsets) - 1
        self._buf, self._off = None, pr.offsets
        self._check(self.lib.nw_batch_upload_packed(
            self._h, _lib.ptr(pr.packed), _lib.ptr(pr.offsets), _lib.ptr(pr.lens), n,
            _lib.ptr(pr.exc_pos) if len(pr.exc_pos) else None, _lib.ptr(pr.exc_byte) if len(pr.exc_byte) else None,
            len(pr.exc_pos)), "nw_batch_upload_packed")

    def set_known(self, seq: Optional[str]) -> None:
        """nw_set_known: reads equal to `seq` take one alignment of it (the HDR amplicon during the
        amplicon pass of the dual alignment); None clears it."""
        b = (seq or "").encode("ascii")
        self._check(self.lib.nw_set_known(self._h, b, len(b)), "nw_set_known")

    def set_lane_walk(self, on: bool) -> None:
        """Resident passes: the first band level's lane walk + stop summary (nw_batch_set_lane_walk;
        what a pipelined call runs on its chunks of >= 65536 reads of one amplicon)."""
        self._check(self.lib.nw_batch_set_lane_walk(self._h, 1 if on else 0), "nw_batch_set_lane_walk")

    def set_phase_events(self, on: bool) -> None:
        """Resident passes: record the per-phase events phase_times() reads (default on; a timed
        pass turns them off: each writes back the L2 between two kernels)."""
        self._check(self.lib.nw_batch_set_phase_events(self._h, 1 if on else 0), "nw_batch_set_phase_events")

    def run_async(self) -> None:
        self._check(self.lib.nw_batch_run_async(self._h), "nw_batch_run_async")

    def sync(self) -> float:
        ms = ctypes.c_float(0.0)
        self._check(self.lib.nw_batch_sync(self._h, ctypes.byref(ms)), "nw_batch_sync")
        return float(ms.value)

    def algo_bytes(self) -> int:
        return int(self.lib.nw_batch_algo_bytes(self._h))

    def cells(self) -> int:
        return int(self.lib.nw_batch_cells(self._h))

    def geometry(self) -> dict:
        vals = [ctypes.c_int32() for _ in range(5)]
        self._check(self.lib.nw_batch_geometry(self._h, *[ctypes.byref(v) for v in vals]), "nw_batch_geometry")
        g = dict(zip(("rows_per_lane", "waves_per_block", "grid", "lds_bytes", "tb_mode"), (v.value for v in vals)))
        g["tb_mode"] = _lib.TB_MODES.get(g["tb_mode"], g["tb_mode"])
        return g

    def fallbacks(self) -> int:
        """Reads of the last run the 16- and 32-diagonal band levels did not certify (the
        128-diagonal wide level's input; nw_batch_fallbacks)."""
        return int(self.lib.nw_batch_fallbacks(self._h))

    def exact_reads(self) -> int:
        """Reads of the last run aligned by the exact int32 kernel (nw_batch_exact_reads)."""
        return int(self.lib.nw_batch_exact_reads(self._h))

    def kernel_times(self) -> dict:
        """Device ms of the last run: DP fill, traceback/emit kernel, the rest."""
        vals = [ctypes.c_float() for _ in range(3)]
        self._check(self.lib.nw_batch_kernel_times(self._h, *[ctypes.byref(v) for v in vals]),
                    "nw_batch_kernel_times")
        return dict(zip(("fill_ms", "walk_ms", "rest_ms"), (float(v.value) for v in vals)))

    def phase_times(self) -> dict:
        """Device ms of the last run by band-path phase (nw_batch_phase_times)."""
        v = np.zeros(5, np.float32)
        self._check(self.lib.nw_batch_phase_times(self._h, _lib.ptr(v)), "nw_batch_phase_times")
        return dict(zip(("sort_ms", "fill16_ms", "walk16_ms", "level32_ms", "rest_ms"), map(float, v)))

    def path_counts(self) -> dict:
        """Reads of the last run by path (nw_batch_path_counts)."""
        v = np.zeros(4, np.int64)
        self._check(self.lib.nw_batch_path_counts(self._h, _lib.ptr(v)), "nw_batch_path_counts")
        d = dict(zip(("exact_copies", "band16", "band32", "band_fallback"), map(int, v)))
        ex = self.exact_reads()   # of the 16 / 32 levels' give-ups: the wide level certified the rest
        d["wide128"] = d["band_fallback"] - ex
        d["exact_kernel"] = ex
        return d

    def device_output(self):
        """(d_aln, stride, d_stats) device pointers of the last run's resident output
        (nw_batch_device_output); valid until the next upload / align."""
        d_aln, d_stats, stride = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        self._check(self.lib.nw_batch_device_output(self._h, ctypes.byref(d_aln), ctypes.byref(stride),
                                                    ctypes.byref(d_stats)), "nw_batch_device_output")
        return int(d_aln.value), int(stride.value), int(d_stats.value)

    def device_ops(self) -> dict:
        """Device pointers of the last ops-mode run's resident output (nw_batch_device_ops):
        runs, run offsets, records, reads (+ their offsets and bias) and max_cols."""
        p = [ctypes.c_void_p() for _ in range(5)]
        bias, cols = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.nw_batch_device_ops(self._h, *[ctypes.byref(x) for x in p], ctypes.byref(bias),
                                                 ctypes.byref(cols)), "nw_batch_device_ops")
        d = dict(zip(("ops", "ops_off", "stats", "reads", "offsets"), (int(x.value or 0) for x in p)))
        d["reads_bias"], d["max_cols"] = int(bias.value), int(cols.value)
        return d

    def download(self, n: int, max_len: int) -> AlignmentBatch:
        stride = int(self.lib.nw_required_stride(self._h, max(int(max_len), 1)))
        stats = np.zeros(n, dtype=_lib.STAT_DTYPE)
        aln = np.zeros((n, 3, stride), dtype=np.uint8)
        self._check(self.lib.nw_batch_download(self._h, _lib.ptr(aln), stride, _lib.ptr(stats)),
                    "nw_batch_download")
        lens = np.diff(self._off)
        return AlignmentBatch(stats, aln, lens, self.scale, self.options.awidth)

    def set_output(self, mode: str) -> None:
        """Output mode of the upload/run path: "rows" (default) or "ops"; from the next upload."""
        self._check(self.lib.nw_batch_set_output(self._h, _lib.NW_OUT_OPS if mode == "ops" else _lib.NW_OUT_ROWS),
                    "nw_batch_set_output")

    def download_ops(self, n: int) -> OpsBatch:
        stats = np.zeros(n, dtype=_lib.STAT_DTYPE)
        ops_off = np.zeros(n + 1, dtype=np.int64)
        cap = 2 * n + 4096
        ops = np.empty(cap, dtype=np.uint32)
        rc = self.lib.nw_batch_download_ops(self._h, _lib.ptr(ops), cap, _lib.ptr(ops_off), _lib.ptr(stats))
        if rc == _lib.NW_E_CAPACITY:
            ops = np.empty(int(ops_off[n]), dtype=np.uint32)
            rc = self.lib.nw_batch_download_ops(self._h, _lib.ptr(ops), len(ops), _lib.ptr(ops_off), _lib.ptr(stats))
        self._check(rc, "nw_batch_download_ops")
        return OpsBatch(stats, ops[: int(ops_off[n])], ops_off, np.diff(self._off), self.scale, self.options.awidth)

    # -- synchronous path ----------------------------------------------------
    def align_ops(self, buf: Optional[np.ndarray], offsets: np.ndarray, out: Optional[tuple] = None,
                  resident: bool = False, records_only: bool = False) -> OpsBatch:
        """The call-level path (nw_align_ops): host reads in, records + runs out.

        ``out`` = (stats, ops, ops_off) preallocated (e.g. pinned) arrays; by default
        they are leased from the process's pinned pool (:func:`_lib.pinned_pool`: the
        copies back run at PCIe rate, and a block is reused once the returned arrays are
        gone).  An ops array too small for the batch is replaced.
        ``resident``: align the batch this aligner's last call uploaded (still in HBM;
        ``buf`` unused) against the current amplicon (nw_align_ops_resident) -- the HDR
        pass over the same reads.  ``records_only``: no runs are copied back (a
        scores-only pass); the returned batch has no runs."""
        if self.reference is None:
            raise NeedleError("no amplicon set")
        n = len(offsets) - 1
        if out is None:
            stats, ops, ops_off = _outputs(n, runs=not records_only)
        else:
            stats, ops, ops_off = out

        def call(ops_arr):
            o = None if records_only else _lib.ptr(ops_arr)
            cap = 0 if records_only else len(ops_arr)
            if resident:
                return self.lib.nw_align_ops_resident(self._h, _lib.ptr(offsets), n, o, cap, _lib.ptr(ops_off),
                                                      _lib.ptr(stats))
            return self.lib.nw_align_ops(self._h, _lib.ptr(buf), _lib.ptr(offsets), n, o, cap, _lib.ptr(ops_off),
                                         _lib.ptr(stats))

        rc = call(ops)
        if rc == _lib.NW_E_CAPACITY:   # rare: more runs than the buffer holds; run again with the size it said
            ops = _lib.pinned_pool().array(int(ops_off[n]), np.uint32)
            rc = call(ops)
        self._check(rc, "nw_align_ops")
        if records_only:
            return OpsBatch(stats, np.zeros(0, np.uint32), ops_off, None, self.scale, self.options.awidth,
                            offsets=offsets, has_runs=False)
        return OpsBatch(stats, ops[: int(ops_off[n])], ops_off, None, self.scale, self.options.awidth, offsets=offsets)

    def align_ops_packed(self, pr: "PackedReads", out: Optional[tuple] = None) -> OpsBatch:
        """nw_align_ops_packed: the batch crosses PCIe as 2 bits per base (+ exceptions)."""
        if self.reference is None:
            raise NeedleError("no amplicon set")
        offsets = pr.offsets
        n = len(offsets) - 1
        if out is None:
            stats, ops, ops_off = _outputs(n)
        else:
            stats, ops, ops_off = out

        exc = (_lib.ptr(pr.exc_pos) if len(pr.exc_pos) else None, _lib.ptr(pr.exc_byte) if len(pr.exc_byte) else None,
               len(pr.exc_pos))

        def call(o):
            if pr.lens is not None:   # the lengths cross PCIe instead of the offsets
                return self.lib.nw_align_ops_packed_lens(self._h, _lib.ptr(pr.packed), _lib.ptr(offsets),
                                                         _lib.ptr(pr.lens), n, *exc, _lib.ptr(o), len(o),
                                                         _lib.ptr(ops_off), _lib.ptr(stats))
            return self.lib.nw_align_ops_packed(self._h, _lib.ptr(pr.packed), _lib.ptr(offsets), n, *exc,
                                                _lib.ptr(o), len(o), _lib.ptr(ops_off), _lib.ptr(stats))

        rc = call(ops)
        if rc == _lib.NW_E_CAPACITY:
            ops = _lib.pinned_pool().array(int(ops_off[n]), np.uint32)
            rc = call(ops)
        self._check(rc, "nw_align_ops_packed")
        return OpsBatch(stats, ops[: int(ops_off[n])], ops_off, None, self.scale, self.options.awidth, offsets=offsets)

    def align_dual_packed(self, pr: "PackedReads", ref2: str, out: Optional[tuple] = None,
                          out2: Optional[tuple] = None, records_only2: bool = False) -> tuple:
        """nw_align_dual_ops_packed_lens: every read of the packed batch (with lengths) against
        the current amplicon and against ``ref2`` (the expected HDR amplicon, CORE:1808-1828) in
        one call -- one upload, the second pass interleaved with the first.  ``out`` / ``out2``:
        (stats, ops, ops_off) per pass (``out2``'s ops may be None with ``records_only2``: the
        second pass's runs stay on the device).  Returns the two OpsBatch (the second without runs
        when records_only2)."""
        if self.reference is None:
            raise NeedleError("no amplicon set")
        if pr.lens is None:
            raise NeedleError("the dual call takes a packed batch with its lengths")
        offsets = pr.offsets
        n = len(offsets) - 1
        stats, ops, ops_off = out if out is not None else _outputs(n)
        if out2 is not None:
            stats2, ops2, ops_off2 = out2
        else:
            stats2, ops2, ops_off2 = _outputs(n)
        if records_only2:
            ops2 = None
        exc = (_lib.ptr(pr.exc_pos) if len(pr.exc_pos) else None, _lib.ptr(pr.exc_byte) if len(pr.exc_byte) else None,
               len(pr.exc_pos))
        r2 = ref2.encode()

        def call(o, o2):
            return self.lib.nw_align_dual_ops_packed_lens(
                self._h, r2, len(r2), _lib.ptr(pr.packed), _lib.ptr(offsets), _lib.ptr(pr.lens), n, *exc,
                _lib.ptr(o), len(o), _lib.ptr(ops_off), _lib.ptr(stats),
                _lib.ptr(o2) if o2 is not None else None, len(o2) if o2 is not None else 0, _lib.ptr(ops_off2),
                _lib.ptr(stats2))

        rc = call(ops, ops2)
        if rc == _lib.NW_E_CAPACITY:
            if int(ops_off[n]) > len(ops):
                ops = _lib.pinned_pool().array(int(ops_off[n]), np.uint32)
            if ops2 is not None and int(ops_off2[n]) > len(ops2):
                ops2 = _lib.pinned_pool().array(int(ops_off2[n]), np.uint32)
            rc = call(ops, ops2)
        self._check(rc, "nw_align_dual_ops_packed_lens")
        ob = OpsBatch(stats, ops[: int(ops_off[n])], ops_off, None, self.scale, self.options.awidth, offsets=offsets)
        ob2 = OpsBatch(stats2, ops2[: int(ops_off2[n])] if ops2 is not None else np.empty(0, np.uint32), ops_off2,
                       None, self.scale, self.options.awidth, offsets=offsets, has_runs=ops2 is not None)
        return ob, ob2

    def ops_times(self) -> dict:
        """Last align_ops: upload span (ms); ``compute_ms`` = the device span from the first upload to
        the last chunk's end (uploads included; with CRISPR_NW_HOST_TIMING=1 the chunks' kernel spans
        summed); bytes each way (nw_ops_times)."""
        h2d, comp = ctypes.c_float(), ctypes.c_float()
        hb, db = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.nw_ops_times(self._h, ctypes.byref(h2d), ctypes.byref(comp), ctypes.byref(hb),
                                          ctypes.byref(db)), "nw_ops_times")
        return {"h2d_ms": float(h2d.value), "compute_ms": float(comp.value), "h2d_bytes": int(hb.value),
                "d2h_bytes": int(db.value)}

    def align_packed(self, buf: np.ndarray, offsets: np.ndarray, strings: bool = True,
                     mode: Optional[str] = None) -> AlignmentBatch:
        """Align a packed batch.  ``strings=False`` copies back only the per-read
        records (identity, score, ...): what a ``just_score`` pass (CORE:1740-1741) reads.
        ``mode`` "ops" (default, :func:`default_output_mode`): runs cross PCIe and the
        rows are built on the host; "rows": the kernels write the rows."""
        if self.reference is None:
            raise NeedleError("no amplicon set")
        if (mode or default_output_mode()) == "ops":
            ob = self.align_ops(buf, offsets)
            if not strings:
                return AlignmentBatch(ob.stats, np.empty((len(ob), 3, 0), np.uint8), ob.read_lens, self.scale,
                                      self.options.awidth)
            return ob.expand(self.reference, buf, offsets)
        n = len(offsets) - 1
        lens = np.diff(offsets)
        max_len = int(lens.max()) if n else 1
        stride = int(self.lib.nw_required_stride(self._h, max(max_len, 1)))
        stats = np.zeros(n, dtype=_lib.STAT_DTYPE)
        aln = np.empty((n, 3, stride if strings else 0), dtype=np.uint8)
        self._check(
            self.lib.nw_align_batch(self._h, _lib.ptr(buf), _lib.ptr(offsets), n,
                                    _lib.ptr(aln) if strings else None, stride, _lib.ptr(stats)),
            "nw_align_batch",
        )
        return AlignmentBatch(stats, aln, lens, self.scale, self.options.awidth)

    def align(self, reads: Sequence) -> AlignmentBatch:
        buf, offsets = pack_reads(reads)
        return self.align_packed(buf, offsets)

    def align_multi_ops(self, amplicons: Sequence[str], buf, offsets: np.ndarray,
                        amplicon_of_read: np.ndarray, out: Optional[tuple] = None) -> OpsBatch:
        """Pooled batch, ops output (nw_align_multi_ops): read r against
        amplicons[amplicon_of_read[r]]; records and runs in read order.  Reads grouped
        by amplicon are aligned in place.  Leaves no amplicon set on this aligner.
        ``buf`` a :class:`PackedReads` (offsets its own): nw_align_multi_ops_packed,
        reads grouped by amplicon."""
        packed = isinstance(buf, PackedReads)
        if packed:
            offsets = buf.offsets
        amps = [a.strip().upper() for a in amplicons]
        refs = "".join(amps).encode()
        roff = np.zeros(len(amps) + 1, dtype=np.int64)
        roff[1:] = np.cumsum([len(a) for a in amps])
        idx = np.ascontiguousarray(amplicon_of_read, dtype=np.int32)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        n = len(offsets) - 1
        if len(idx) != n:
            raise NeedleError(f"{len(idx)} amplicon indices for {n} reads")
        if out is None:
            stats = np.zeros(n, dtype=_lib.STAT_DTYPE)
            ops_off = np.zeros(n + 1, dtype=np.int64)
            ops = np.empty(2 * n + 4096, dtype=np.uint32)
        else:
            stats, ops, ops_off = out

        def call(o):
            if packed and buf.lens is not None:
                return self.lib.nw_align_multi_ops_packed_lens(
                    self._h, refs, _lib.ptr(roff), len(amps), _lib.ptr(buf.packed), _lib.ptr(offsets),
                    _lib.ptr(buf.lens), _lib.ptr(idx), n, _lib.ptr(buf.exc_pos) if len(buf.exc_pos) else None,
                    _lib.ptr(buf.exc_byte) if len(buf.exc_byte) else None, len(buf.exc_pos), _lib.ptr(o), len(o),
                    _lib.ptr(ops_off), _lib.ptr(stats))
            if packed:
                return self.lib.nw_align_multi_ops_packed(
                    self._h, refs, _lib.ptr(roff), len(amps), _lib.ptr(buf.packed), _lib.ptr(offsets),
                    _lib.ptr(idx), n, _lib.ptr(buf.exc_pos) if len(buf.exc_pos) else None,
                    _lib.ptr(buf.exc_byte) if len(buf.exc_byte) else None, len(buf.exc_pos), _lib.ptr(o), len(o),
                    _lib.ptr(ops_off), _lib.ptr(stats))
            return self.lib.nw_align_multi_ops(self._h, refs, _lib.ptr(roff), len(amps), _lib.ptr(buf),
                                               _lib.ptr(offsets), _lib.ptr(idx), n, _lib.ptr(o), len(o),
                                               _lib.ptr(ops_off), _lib.ptr(stats))

        rc = call(ops)
        if rc == _lib.NW_E_CAPACITY:
            ops = np.empty(int(ops_off[n]), dtype=np.uint32)
            rc = call(ops)
        self.reference = None
        self._check(rc, "nw_align_multi_ops_packed" if packed else "nw_align_multi_ops")
        return OpsBatch(stats, ops[: int(ops_off[n])], ops_off, None, self.scale, self.options.awidth, offsets=offsets)

    def align_multi(self, amplicons: Sequence[str], buf: np.ndarray, offsets: np.ndarray,
                    amplicon_of_read: np.ndarray) -> AlignmentBatch:
        """Pooled batch: read r against amplicons[amplicon_of_read[r]] (nw_align_multi).

        Results in read order; rows are as wide as the longest amplicon needs.
        Leaves no amplicon set on this aligner (call set_reference before
        align_packed again).
        """
        amps = [a.strip().upper() for a in amplicons]
        refs = "".join(amps).encode()
        roff = np.zeros(len(amps) + 1, dtype=np.int64)
        roff[1:] = np.cumsum([len(a) for a in amps])
        idx = np.ascontiguousarray(amplicon_of_read, dtype=np.int32)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        n = len(offsets) - 1
        if len(idx) != n:
            raise NeedleError(f"{len(idx)} amplicon indices for {n} reads")
        lens = np.diff(offsets)
        max_len = int(lens.max()) if n else 1
        stride = int(self.lib.nw_required_stride_multi(_lib.ptr(roff), len(amps), max(max_len, 1)))
        stats = np.zeros(n, dtype=_lib.STAT_DTYPE)
        aln = np.zeros((n, 3, stride), dtype=np.uint8)
        self._check(
            self.lib.nw_align_multi(self._h, refs, _lib.ptr(roff), len(amps), _lib.ptr(buf), _lib.ptr(offsets),
                                    _lib.ptr(idx), n, _lib.ptr(aln), stride, _lib.ptr(stats)),
            "nw_align_multi",
        )
        self.reference = None
        return AlignmentBatch(stats, aln, lens, self.scale, self.options.awidth)


def format_srspair(batch: AlignmentBatch, aname: str, bnames: Sequence[str], options: NeedleOptions) -> str:
    """srspair blocks of a batch (needle's default -aformat), via the C++ writer."""
    lib = _lib.load()
    names = b"".join(n.encode() + b"\0" for n in bnames)
    stride = batch.aln.shape[2]
    args = (aname.encode(), names, options.gap_open, options.gap_extend, batch.scale, options.awidth,
            _lib.ptr(batch.aln), stride, _lib.ptr(batch.stats), len(batch))
    need = lib.nw_format_srspair(None, 0, *args)
    buf = ctypes.create_string_buffer(int(need) + 1)
    got = lib.nw_format_srspair(buf, int(need) + 1, *args)
    assert got == need
    return buf.raw[:need].decode("ascii")
