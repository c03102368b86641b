"""Test doubles: an aligner with GpuAligner's interface backed by the CPU oracle.

Used only in CPU tests (no GPU in the build container) to exercise the host
logic around the aligner; the GPU path itself is covered by the -m gpu tests.
"""
import numpy as np

from crispresso_amd import _lib
from crispresso_amd.aligner import AlignmentBatch, OpsBatch, pack_reads
from crispresso_amd.needle_options import NeedleOptions
from oracle import oracle_py


def oracle_batch(amplicon, buf, offsets, awidth=5000, gap_open=10.0, gap_extend=0.5):
    p = oracle_py.params(gap_open, gap_extend)
    res, aln = oracle_py.align_batch(amplicon, buf, offsets, p, nthreads=4)
    n = len(offsets) - 1
    stats = np.zeros(n, dtype=_lib.STAT_DTYPE)
    for f in ("aln_len", "n_ident", "n_sim", "n_gaps", "score", "end_i", "end_j"):
        stats[f] = res[f]
    lens = np.diff(offsets)
    stats["flags"] = np.where(lens == 0, _lib.NW_FLAG_EMPTY, 0)
    stride = ((aln.shape[2] + 15) // 16) * 16
    out = np.zeros((n, 3, stride), dtype=np.uint8)
    out[:, :, : aln.shape[2]] = aln
    return AlignmentBatch(stats, out, lens, p.scale, awidth)


def runs_from_rows(ref_row: bytes, read_row: bytes):
    """Runs of an alignment whose inputs hold no '-' (then '-' marks a gap)."""
    out = []
    for a, b in zip(ref_row, read_row):
        t = _lib.NW_RUN_X if a == ord("-") else (_lib.NW_RUN_Y if b == ord("-") else _lib.NW_RUN_M)
        if out and out[-1][0] == t:
            out[-1][1] += 1
        else:
            out.append([t, 1])
    return [(t << 28) | n for t, n in out]


def ops_from_batch(batch: AlignmentBatch) -> OpsBatch:
    """The ops form of a rows batch (inputs without '-')."""
    ops, off = [], [0]
    for i in range(len(batch)):
        L = int(batch.stats["aln_len"][i])
        if not batch.empty(i):
            ops += runs_from_rows(batch.aln[i, 0, :L].tobytes(), batch.aln[i, 2, :L].tobytes())
        off.append(len(ops))
    return OpsBatch(batch.stats, np.array(ops, np.uint32), np.array(off, np.int64), batch.read_lens, batch.scale,
                    batch.awidth)


class OracleAligner:
    """Stand-in for GpuAligner (same methods the host code calls)."""

    def __init__(self, device=0, options=None):
        self.options = options or NeedleOptions()
        self.scale = oracle_py.params(self.options.gap_open, self.options.gap_extend).scale
        self.reference = None

    def set_reference(self, seq):
        self.reference = seq

    def align_packed(self, buf, offsets, strings=True):
        return oracle_batch(self.reference, buf, offsets, self.options.awidth, self.options.gap_open,
                            self.options.gap_extend)

    def align(self, reads):
        return self.align_packed(*pack_reads(reads))

    def align_ops(self, buf, offsets, out=None, resident=False, records_only=False):
        if resident:
            buf, offsets = self._resident
        ob = ops_from_batch(self.align_packed(buf, offsets))
        self._resident = (buf, offsets)
        return ob

    def align_multi_ops(self, amplicons, buf, offsets, amplicon_of_read):
        return ops_from_batch(self.align_multi(amplicons, buf, offsets, amplicon_of_read))

    def align_multi(self, amplicons, buf, offsets, amplicon_of_read):
        """Per-amplicon oracle runs, reassembled in read order (reference for nw_align_multi)."""
        offsets = np.asarray(offsets, dtype=np.int64)
        n = len(offsets) - 1
        lens = np.diff(offsets)
        stride = max(((len(a) + int(lens.max() if n else 1) + 15) // 16) * 16 for a in amplicons)
        stats = np.zeros(n, dtype=_lib.STAT_DTYPE)
        aln = np.zeros((n, 3, stride), dtype=np.uint8)
        for g, amp in enumerate(amplicons):
            sel = np.flatnonzero(np.asarray(amplicon_of_read) == g)
            if not len(sel):
                continue
            sub = [bytes(buf[offsets[r]:offsets[r + 1]]) for r in sel]
            part = self.__class__(options=self.options)
            part.set_reference(amp)
            b = part.align_packed(*pack_reads([x.decode() for x in sub]))
            stats[sel] = b.stats
            aln[sel, :, : b.aln.shape[2]] = b.aln
        return AlignmentBatch(stats, aln, lens, self.scale, self.options.awidth)

    def close(self):
        pass
