"""Paired-end read merge on the GPU with FLASH 1.2.11 semantics.

CRISPResso runs the external FLASH program on paired-end input before the
alignment (``CRISPResso/CRISPRessoCORE.py:1655-1677``)::

    flash R1 R2 --allow-outies --max-overlap M --min-overlap m -f LEN -r AVG -s STD -z -d OUT

and then reads ``out.extendedFrags.fastq.gz`` (``CORE:1679-1686``).  This module
is that step in-process: :func:`merge_pairs` merges packed read pairs through the
C ABI ``nwf_merge_batch`` (``include/crispr_flash.h``, kernel
``crispresso_amd/csrc/flash_merge.hip``); :func:`run_flash` reads the two FASTQ
files and writes FLASH's output files (merged reads, the not-combined pairs, the
length histogram).  There is no CPU fallback: without the library or a GPU every
call raises :class:`crispresso_amd._lib.NativeLibraryError`.
"""
from __future__ import annotations

import ctypes
import gzip
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _lib


class FlashError(RuntimeError):
    """A failed merge (the message is the library's)."""


@dataclass
class FlashOptions:
    """FLASH's options, defaulting to what CRISPResso passes (CORE:1655-1670 with the
    argparse defaults CORE:4119-4138: ``--allow-outies --max-overlap 100 --min-overlap 4``;
    FLASH's -x stays 0.25).  FLASH's own defaults (-m 10, -M 65, no outies) are
    ``FlashOptions.flash_defaults()``."""
    min_overlap: int = 4
    max_overlap: int = 100
    max_mismatch_density: float = 0.25
    allow_outies: bool = True
    phred_offset: int = 33
    cap_mismatch_quals: bool = False

    @staticmethod
    def flash_defaults() -> "FlashOptions":
        """FLASH 1.2.11 run without options: -m 10 -M 65 -x 0.25, innies only."""
        return FlashOptions(min_overlap=10, max_overlap=65, allow_outies=False)

    @staticmethod
    def max_overlap_for(read_len: float, fragment_len: float, fragment_len_stddev: float) -> int:
        """FLASH's -M default when it is not given: 2r - f + 2.5 s (truncated)."""
        return int(2 * read_len - fragment_len + 2.5 * fragment_len_stddev)


@dataclass
class MergeResult:
    seq: np.ndarray      # uint8, pair i's merged read at [off1[i] + off2[i], + length[i])
    qual: np.ndarray     # uint8 ASCII qualities, same layout
    length: np.ndarray   # int32 [n], 0 = not combined
    flags: np.ndarray    # int32 [n], NWF_COMBINED | NWF_OUTIE
    base: np.ndarray     # int64 [n], off1[i] + off2[i]
    kernel_ms: float

    def merged(self, i: int) -> Optional[Tuple[bytes, bytes, bool]]:
        n = int(self.length[i])
        if n == 0:
            return None
        b = int(self.base[i])
        return (self.seq[b:b + n].tobytes(), self.qual[b:b + n].tobytes(),
                bool(self.flags[i] & _lib.NWF_OUTIE))


def _pack(items: List[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    off = np.zeros(len(items) + 1, dtype=np.int64)
    np.cumsum([len(x) for x in items], out=off[1:])
    buf = np.frombuffer(b"".join(items), dtype=np.uint8) if items else np.zeros(0, np.uint8)
    return np.ascontiguousarray(buf), off


def merge_pairs(seq1: List[bytes], qual1: List[bytes], seq2: List[bytes], qual2: List[bytes],
                options: Optional[FlashOptions] = None, device: int = 0) -> MergeResult:
    """Merge read pairs (FASTQ sequence and quality lines, as bytes) on the GPU."""
    if not (len(seq1) == len(qual1) == len(seq2) == len(qual2)):
        raise FlashError("merge_pairs: the four lists must have the same length")
    for s, q in zip(seq1 + seq2, qual1 + qual2):
        if len(s) != len(q):
            raise FlashError("merge_pairs: a sequence and its quality line differ in length")
    s1, off1 = _pack(seq1)
    q1, _ = _pack(qual1)
    s2, off2 = _pack(seq2)
    q2, _ = _pack(qual2)
    return merge_packed(s1, q1, off1, s2, q2, off2, options, device)


def merge_packed(s1: np.ndarray, q1: np.ndarray, off1: np.ndarray, s2: np.ndarray, q2: np.ndarray,
                 off2: np.ndarray, options: Optional[FlashOptions] = None, device: int = 0) -> MergeResult:
    """merge_pairs on packed inputs: uint8 sequence / quality buffers and int64
    offsets (n + 1, from 0) per mate."""
    o = options or FlashOptions()
    s1, q1, s2, q2 = (np.ascontiguousarray(x, dtype=np.uint8) for x in (s1, q1, s2, q2))
    off1 = np.ascontiguousarray(off1, dtype=np.int64)
    off2 = np.ascontiguousarray(off2, dtype=np.int64)
    if len(off1) != len(off2) or len(off1) < 1 or off1[-1] > len(s1) or off2[-1] > len(s2) or \
            len(q1) < off1[-1] or len(q2) < off2[-1]:
        raise FlashError("merge_packed: offsets do not match the buffers")
    n = len(off1) - 1
    total = int(off1[-1] + off2[-1])
    out_seq = np.zeros(max(total, 1), dtype=np.uint8)
    out_qual = np.zeros(max(total, 1), dtype=np.uint8)
    length = np.zeros(n, dtype=np.int32)
    flags = np.zeros(n, dtype=np.int32)
    params = _lib.NwfParams(o.min_overlap, o.max_overlap, o.max_mismatch_density, int(o.allow_outies),
                            o.phred_offset, int(o.cap_mismatch_quals))
    ms = ctypes.c_float(0.0)
    lib = _lib.load()
    rc = lib.nwf_merge_batch(device, ctypes.byref(params), _lib.ptr(s1), _lib.ptr(q1), _lib.ptr(off1),
                             _lib.ptr(s2), _lib.ptr(q2), _lib.ptr(off2), n, _lib.ptr(out_seq), _lib.ptr(out_qual),
                             _lib.ptr(length), _lib.ptr(flags), ctypes.byref(ms))
    if rc != 0:
        raise FlashError(lib.nwf_last_error().decode())
    return MergeResult(out_seq, out_qual, length, flags, off1[:-1] + off2[:-1], float(ms.value))


def read_fastq(path: str) -> Tuple[List[bytes], List[bytes], List[bytes]]:
    """-> (header lines without '@', sequences, qualities) of a FASTQ(.gz) file."""
    with open(path, "rb") as f:
        gz = f.read(2) == b"\x1f\x8b"
    with (gzip.open(path, "rb") if gz else open(path, "rb")) as f:
        lines = f.read().split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    names = [h.rstrip(b"\r")[1:] for h in lines[0::4]]
    seqs = [s.rstrip(b"\r") for s in lines[1::4]]
    quals = [q.rstrip(b"\r") for q in lines[3::4]]
    n = min(len(names), len(seqs), len(quals))
    return names[:n], seqs[:n], quals[:n]


def run_flash(r1: str, r2: str, out_dir: str, prefix: str = "out", gz: bool = True,
              options: Optional[FlashOptions] = None, device: int = 0) -> Dict[str, int]:
    """FLASH's outputs for two FASTQ files: ``<prefix>.extendedFrags.fastq(.gz)``,
    ``<prefix>.notCombined_1/2.fastq(.gz)``, ``<prefix>.hist``, ``<prefix>.histogram``."""
    n1, s1, q1 = read_fastq(r1)
    n2, s2, q2 = read_fastq(r2)
    n = min(len(s1), len(s2))
    res = merge_pairs(s1[:n], q1[:n], s2[:n], q2[:n], options, device)
    os.makedirs(out_dir, exist_ok=True)
    op = (lambda p: gzip.open(p + ".gz", "wb", compresslevel=1)) if gz else (lambda p: open(p, "wb"))
    ext = op(os.path.join(out_dir, f"{prefix}.extendedFrags.fastq"))
    nc1 = op(os.path.join(out_dir, f"{prefix}.notCombined_1.fastq"))
    nc2 = op(os.path.join(out_dir, f"{prefix}.notCombined_2.fastq"))
    hist: Dict[int, int] = {}
    stats = {"pairs": n, "combined": 0, "innies": 0, "outies": 0}
    for i in range(n):
        m = res.merged(i)
        if m is None:
            nc1.write(b"@%s\n%s\n+\n%s\n" % (n1[i], s1[i], q1[i]))
            nc2.write(b"@%s\n%s\n+\n%s\n" % (n2[i], s2[i], q2[i]))
            continue
        s, q, outie = m
        name = n1[i][:-2] if n1[i].endswith(b"/1") else n1[i]
        ext.write(b"@%s\n%s\n+\n%s\n" % (name, s, q))
        stats["combined"] += 1
        stats["outies" if outie else "innies"] += 1
        hist[len(s)] = hist.get(len(s), 0) + 1
    for f in (ext, nc1, nc2):
        f.close()
    with open(os.path.join(out_dir, f"{prefix}.hist"), "w") as f:
        for k in sorted(hist):
            f.write(f"{k}\t{hist[k]}\n")
    with open(os.path.join(out_dir, f"{prefix}.histogram"), "w") as f:
        for k in sorted(hist):
            f.write(f"{k}\t{'*' * max(1, hist[k] * 80 // max(hist.values()))}\n")
    return stats
