"""FASTQ(.gz) -> the FASTA stream ``needle`` would have read.

Restates the shell stage of the reference pipeline
(``CRISPRessoCORE.py:1791-1797``, HDR re-stream ``1812-1818``)::

    cat F | gunzip | awk 'NR % 4 == 1 {print ">" $0} NR % 4 == 2 {print $0}' | sed 's/:/_/g'

and what EMBOSS's FASTA reader then keeps: the sequence name is the first
whitespace-delimited word of the header (here ``@`` + read id with every ``:``
turned into ``_``), and the sequence keeps letters and the characters
``*.~?#+-``.  Reads come back packed (one uint8 buffer + int64 offsets) so they
can go to the GPU without a per-read Python object on the hot path.
"""
from __future__ import annotations

import gzip
import io
import os
import re
from collections.abc import Sequence
from typing import List, Optional, Tuple

import numpy as np

_KEEP = np.zeros(256, dtype=bool)
for _c in range(256):
    ch = chr(_c)
    _KEEP[_c] = ch.isascii() and (ch.isalpha() or ch in "*.~?#+-")


def _open(path: str):
    with open(path, "rb") as f:
        magic = f.read(2)
    if magic == b"\x1f\x8b":
        return gzip.open(path, "rb")
    return open(path, "rb")


def fasta_name(header_line: bytes) -> str:
    """Name EMBOSS gives the record awk/sed made of a FASTQ header line."""
    h = header_line.rstrip(b"\r\n").replace(b":", b"_")
    tok = h.split()
    return tok[0].decode("ascii", "replace") if tok else ""


class NameList(Sequence):
    """The record names (a sequence of str) plus ``raw``: the same names as one uint8
    block, each followed by '\\n' -- what the native reader produced, kept so the
    DataFrame's ID column is built from it in bulk (needle._ids_of).  The str objects are
    made on first use (a 1M-read ingest does not pay for 1M of them when only the IDs are
    read); ``raw`` is empty when a name holds a byte outside ASCII."""

    def __init__(self, names: Optional[List[str]], raw: np.ndarray, n: Optional[int] = None,
                 text: Optional[np.ndarray] = None):
        self._list = names
        self._n = len(names) if names is not None else int(n)
        self._text = text
        self.raw = raw

    def _names(self) -> List[str]:
        if self._list is None:
            t = self._text if self._text is not None else self.raw
            self._list = t.tobytes().decode("ascii", "replace").split("\n")[:-1] if self._n else []
            self._text = None
        return self._list

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        return self._names()[i]

    def __iter__(self):
        return iter(self._names())

    def __eq__(self, other):
        if isinstance(other, (list, tuple, NameList)):
            return self._names() == list(other)
        return NotImplemented

    def __repr__(self):
        return f"NameList({self._names()!r})"


def read_fastq_as_fasta(path: str, min_bp_quality: int = 0,
                        min_single_bp_quality: int = 0) -> Tuple[List[str], np.ndarray, np.ndarray]:
    """-> (fasta names, packed sequences, offsets) in file order.

    Native ingest (``nw_fastq_read``, zlib + one C++ pass); the semantics are those
    of :func:`fastq_bytes_as_fasta` below (the Python restatement the tests hold the
    native reader to).  With a quality threshold only the records
    filter_se_fastq_by_qual (``CORE:270-308``) keeps are returned
    (``nw_fastq_read_filtered``; restated by :func:`quality_pass`)."""
    import ctypes

    from . import _lib

    lib = _lib.load()
    h = ctypes.c_void_p()
    if lib.nw_fastq_read_filtered(os.fsencode(path), int(min_bp_quality), int(min_single_bp_quality),
                                  ctypes.byref(h)) != _lib.NW_OK:
        raise OSError(f"cannot read FASTQ {path}")
    try:
        n = int(lib.nw_fastq_count(h))
        off = np.ctypeslib.as_array((ctypes.c_int64 * (n + 1)).from_address(lib.nw_fastq_offsets(h))).copy()
        nb = int(off[-1])
        seqs = (np.ctypeslib.as_array((ctypes.c_uint8 * nb).from_address(lib.nw_fastq_seqs(h))).copy()
                if nb else np.zeros(0, np.uint8))
        nm = ctypes.c_int64()
        p = lib.nw_fastq_names(h, ctypes.byref(nm))
        raw = (np.ctypeslib.as_array((ctypes.c_uint8 * nm.value).from_address(p)).copy() if nm.value
               else np.zeros(0, np.uint8))
    finally:
        lib.nw_fastq_free(h)
    ascii_ok = len(raw) and int(raw.max()) < 128
    return NameList(None, raw if ascii_ok else np.zeros(0, np.uint8), n, raw), seqs, off


class _Owner:
    """Frees a native ingest handle when the last array viewing its memory is gone."""

    def __init__(self, lib, h):
        self.lib, self.h = lib, h

    def __del__(self):  # pragma: no cover - runs at garbage collection
        if self.h:
            self.lib.nw_fastq_free(self.h)
            self.h = None


class _View:
    """``np.asarray(_View(...))``: an array over native memory that keeps its owner alive."""

    def __init__(self, owner, addr: int, nbytes: int):
        self._owner = owner
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "version": 3, "data": (addr or 0, False)}


def _native_array(owner, addr, count: int, dtype) -> np.ndarray:
    dtype = np.dtype(dtype)
    if count <= 0 or not addr:
        return np.zeros(0, dtype)
    return np.asarray(_View(owner, addr, count * dtype.itemsize)).view(dtype)


def read_fastq_packed(path: str, pinned: bool = True):
    """-> (names, text, offsets, packed): the FASTQ's reads as the aligner takes them.

    The native ingest (:func:`read_fastq_as_fasta` semantics, no quality filter: the
    reference filters the raw reads upstream, ``CORE:1547-1583``) plus ``nw_fastq_pack``:
    ``packed`` is an :class:`~crispresso_amd.aligner.PackedReads` whose 2-bit bases,
    exceptions and offsets sit in page-locked memory (``pinned``) ready for
    ``nw_align_ops_packed``; ``text`` (the bytes, for the alignment rows) and ``offsets``
    are views of the same native buffers -- nothing is copied into Python-owned memory.
    The buffers live as long as any of the returned arrays."""
    import ctypes

    from . import _lib
    from .aligner import PackedReads

    lib = _lib.load()
    h = ctypes.c_void_p()
    if lib.nw_fastq_read(os.fsencode(path), ctypes.byref(h)) != _lib.NW_OK:
        raise OSError(f"cannot read FASTQ {path}")
    owner = _Owner(lib, h)
    n = int(lib.nw_fastq_count(h))
    pk, po, ep, eb = (ctypes.c_void_p() for _ in range(4))
    ne = ctypes.c_int64()
    rc = lib.nw_fastq_pack(h, int(bool(pinned)), ctypes.byref(pk), ctypes.byref(po), ctypes.byref(ep),
                           ctypes.byref(eb), ctypes.byref(ne))
    if rc != _lib.NW_OK:
        raise _lib.NativeLibraryError(f"nw_fastq_pack failed (code {rc})")
    offsets = _native_array(owner, po.value, n + 1, np.int64)
    if n == 0:
        offsets = np.zeros(1, np.int64)
    nb = int(offsets[-1])
    text = _native_array(owner, lib.nw_fastq_seqs(h), nb, np.uint8)
    pl = ctypes.c_void_p()   # the read lengths (they cross PCIe instead of the offsets); None past 65535 bases
    lens = (_native_array(owner, pl.value, n, np.uint16)
            if n and lib.nw_fastq_lens(h, ctypes.byref(pl)) == _lib.NW_OK else None)
    packed = PackedReads(_native_array(owner, pk.value, (nb + 3) // 4 + 16, np.uint8), offsets,
                         _native_array(owner, ep.value, ne.value, np.int64),
                         _native_array(owner, eb.value, ne.value, np.uint8), lens)
    nm = ctypes.c_int64()
    p = lib.nw_fastq_names(h, ctypes.byref(nm))
    raw = _native_array(owner, p, nm.value, np.uint8).copy()
    ascii_ok = len(raw) and int(raw.max()) < 128
    return NameList(None, raw if ascii_ok else np.zeros(0, np.uint8), n, raw), text, offsets, packed


def read_fastq_as_fasta_py(path: str, min_bp_quality: int = 0,
                           min_single_bp_quality: int = 0) -> Tuple[List[str], np.ndarray, np.ndarray]:
    """The Python restatement (gzip + :func:`fastq_bytes_as_fasta`)."""
    with _open(path) as f:
        data = f.read()
    return fastq_bytes_as_fasta(data, min_bp_quality, min_single_bp_quality)


def quality_pass(qual_lines: List[bytes], min_bp_quality: int, min_single_bp_quality: int) -> List[bool]:
    """filter_se_fastq_by_qual's test per record (``CORE:296-305``): keep when
    ``mean(phred) >= min_bp_quality and min(phred) >= min_single_bp_quality``, Phred+33
    as Biopython's "fastq" parser reads it.  An empty quality line has a NaN mean: the
    record is not kept (the test short-circuits before ``min()``)."""
    out = []
    for q in qual_lines:
        ph = np.frombuffer(q.rstrip(b"\r"), dtype=np.uint8).astype(np.int64) - 33
        out.append(bool(len(ph)) and ph.mean() >= min_bp_quality and ph.min() >= min_single_bp_quality)
    return out


def fastq_bytes_as_fasta(data: bytes, min_bp_quality: int = 0,
                         min_single_bp_quality: int = 0) -> Tuple[List[str], np.ndarray, np.ndarray]:
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    headers = lines[0::4]
    seqs = lines[1::4][: len(headers)]
    if len(seqs) < len(headers):  # awk prints a header even without a sequence line
        seqs += [b""] * (len(headers) - len(seqs))
    if min_bp_quality > 0 or min_single_bp_quality > 0:
        quals = lines[3::4]
        quals += [b""] * (len(headers) - len(quals))
        keep = quality_pass(quals, min_bp_quality, min_single_bp_quality)
        headers = [h for h, k in zip(headers, keep) if k]
        seqs = [s for s, k in zip(seqs, keep) if k]
    names = [fasta_name(h) for h in headers]
    return (names,) + pack_filtered(seqs)


def _records(path: str) -> List[Tuple[bytes, bytes, bytes]]:
    """(header, sequence, quality) lines of every 4-line record."""
    with _open(path) as f:
        lines = f.read().split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    lines += [b""] * ((-len(lines)) % 4)
    return list(zip(lines[0::4], lines[1::4], lines[3::4]))


def _record_id(header: bytes) -> str:
    """Biopython's record.id: the title after '@' up to the first whitespace."""
    tok = header[1:].rstrip(b"\r").split()
    return tok[0].decode("ascii", "replace") if tok else ""


def get_ids_reads_to_remove(fastq_filename: str, min_bp_quality: int = 20, min_single_bp_quality: int = 0) -> set:
    """get_ids_reads_to_remove (``CORE:162-193``): ids of the records whose mean
    Phred quality is < min_bp_quality or whose lowest is < min_single_bp_quality."""
    out = set()
    for h, _, q in _records(fastq_filename):
        ph = np.frombuffer(q.rstrip(b"\r"), dtype=np.uint8).astype(np.int64) - 33
        if len(ph) == 0:
            raise ValueError(f"record {_record_id(h)} has no qualities")   # numpy: min() of an empty array
        if ph.mean() < min_bp_quality or ph.min() < min_single_bp_quality:
            out.add(_record_id(h))
    return out


def _write_records(path: str, recs) -> None:
    """Records as Biopython's FASTQ writer prints them: '@title', sequence, '+', qualities."""
    import gzip as _gz

    with _gz.open(path, "wb") as f:
        f.write(b"".join(h.rstrip(b"\r") + b"\n" + s.rstrip(b"\r") + b"\n+\n" + q.rstrip(b"\r") + b"\n"
                         for h, s, q in recs))


def _filtered_name(fastq_filename: str) -> str:
    return fastq_filename.replace(".fastq", "").replace(".gz", "") + "_filtered.fastq.gz"


def filter_se_fastq_by_qual(fastq_filename: str, output_filename: str = None, min_bp_quality: int = 20,
                            min_single_bp_quality: int = 0) -> str:
    """filter_se_fastq_by_qual (``CORE:270-308``): writes the records with mean
    quality >= min_bp_quality and none < min_single_bp_quality; returns the file name.
    (:func:`read_fastq_as_fasta` with the thresholds gives the same reads in memory.)"""
    output_filename = output_filename or _filtered_name(fastq_filename)
    recs = _records(fastq_filename)
    keep = quality_pass([q for _, _, q in recs], min_bp_quality, min_single_bp_quality)
    _write_records(output_filename, [r for r, k in zip(recs, keep) if k])
    return output_filename


def filter_pe_fastq_by_qual(fastq_r1: str, fastq_r2: str, output_filename_r1: str = None,
                            output_filename_r2: str = None, min_bp_quality: int = 20,
                            min_single_bp_quality: int = 0) -> Tuple[str, str]:
    """filter_pe_fastq_by_qual (``CORE:196-267``): a pair goes when either mate's id is
    in either file's get_ids_reads_to_remove set; returns the two file names."""
    drop = get_ids_reads_to_remove(fastq_r1, min_bp_quality, min_single_bp_quality) | \
        get_ids_reads_to_remove(fastq_r2, min_bp_quality, min_single_bp_quality)
    outs = []
    for src, dst in ((fastq_r1, output_filename_r1), (fastq_r2, output_filename_r2)):
        dst = dst or _filtered_name(src)
        _write_records(dst, [r for r in _records(src) if _record_id(r[0]) not in drop])
        outs.append(dst)
    return outs[0], outs[1]


def pack_filtered(seqs: List[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate, dropping bytes EMBOSS's reader would drop (sed ':' -> '_' first)."""
    joined = b"".join(s.replace(b":", b"_") for s in seqs)
    raw = np.frombuffer(joined, dtype=np.uint8)
    lens = np.fromiter((len(s) for s in seqs), dtype=np.int64, count=len(seqs))
    keep = _KEEP[raw]
    if keep.all():
        buf = raw.copy()
        kept_lens = lens
    else:
        seg = np.repeat(np.arange(len(seqs)), lens)
        kept_lens = np.bincount(seg[keep], minlength=len(seqs)).astype(np.int64)
        buf = raw[keep].copy()
    offsets = np.zeros(len(seqs) + 1, dtype=np.int64)
    np.cumsum(kept_lens, out=offsets[1:])
    return buf, offsets


def parse_fasta_text(text: str) -> Tuple[List[str], np.ndarray, np.ndarray]:
    """FASTA text (e.g. not_aligned_amplicon_forward.fa) after ``sed 's/:/_/g'``."""
    names: List[str] = []
    seqs: List[bytes] = []
    cur: List[bytes] = []
    for line in io.BytesIO(text.encode()):
        line = line.rstrip(b"\r\n")
        if line.startswith(b">"):
            if names:
                seqs.append(b"".join(cur))
            names.append(fasta_name(line[1:]))
            cur = []
        elif names:
            cur.append(line)
    if names:
        seqs.append(b"".join(cur))
    return (names,) + pack_filtered(seqs)


_ws = re.compile(r"\s+")


def count_reads(path: str) -> int:
    """``zcat | wc -l`` / 4, as get_n_reads_fastq (CRISPRessoCORE.py:331-346)."""
    with _open(path) as f:
        n = sum(1 for _ in f)
    return n // 4
