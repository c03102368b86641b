"""The alignment step of ``run_crispresso``, with the GPU aligner in place of ``needle``.

Mirrors, name for name, what ``CRISPResso/CRISPRessoCORE.py`` does around its
``needle`` calls so that code written against the reference reads the same:

* :func:`reverse_complement`, :func:`find_wrong_nt` -- ``CORE:129-159``
* :class:`NeedleException` -- ``CORE:381``; raised with the reference's messages
* :func:`parse_needle_output` -- restatement of the closure at ``CORE:1707-1786``
  (reads srspair text back into the DataFrame the quantification consumes)
* :func:`needle_pass` -- one ``needle`` invocation (``CORE:1791-1806``): FASTQ or
  FASTA in, DataFrame out, optional ``needle_output_*.txt.gz`` file
* :func:`align_reads` -- the whole block ``CORE:1788-2000``: forward pass, HDR
  pass, join, ``min_identity_score`` filter, reverse-complement retry, RC
  transform and ``_RC`` suffix, concatenation.

Reference quirks reproduced on purpose:
  1. retry inputs are ``align_seq.replace("_", "")``, so ``-`` gaps stay in them
     (``CORE:1846``, ``1867``);
  2. with an HDR amplicon the retry set tests ``score_ref`` twice (``CORE:1844-1845``);
  3. identities exactly equal to ``min_identity_score`` are neither kept nor
     retried (strict ``<`` / ``>``, ``CORE:1844-1851``, ``1866-1871``);
  4. the RC-HDR pass passes the literal text ``args.needle_options_string`` to
     needle (``CORE:1928``), so that needle run produces no alignments; the
     failure goes unnoticed because ``sb.call`` sees the exit status of the
     pipeline's last command, ``gzip`` (``CORE:1932-1934``).  The reference
     therefore joins an EMPTY repair table: RC rows get ``score_repaired`` and
     ``score_diff`` = NaN.  ``rc_hdr_quirk="reference"`` (default) reproduces
     that (pinned by tests/golden/syn_hdr_rcfail); ``"align"`` runs the pass the
     author evidently meant.  (The same exit-status rule means a failing needle
     never raises NeedleException in the reference; ours raises on real errors.)
  5. read ids lose real underscores (``sed 's/:/_/g'`` then ``_`` -> ``:``,
     ``CORE:1797``, ``1725``).
"""
from __future__ import annotations

import gzip
import os
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

from . import _lib, fastq
from .aligner import (AlignmentBatch, GpuAligner, NeedleError, OpsBatch, default_output_mode, format_srspair,
                      printed_percent)
from .needle_options import DEFAULT_NEEDLE_OPTIONS, NeedleOptions, UnsupportedNeedleOption


class NeedleException(Exception):
    """CRISPRessoCORE.py:381 -- mapped to exit code 6 by the reference CLI."""


_NT_COMPLEMENT = {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N", "_": "_", "-": "-"}


def reverse_complement(sequence: str) -> str:
    """CRISPRessoCORE.py:129-144 (KeyError on characters outside ACGTN_-, as there)."""
    return "".join([_NT_COMPLEMENT[c] for c in sequence.upper()[-1::-1]])


def find_wrong_nt(sequence: str) -> List[str]:
    """CRISPRessoCORE.py:147-159."""
    return list(set(sequence.upper()).difference(set(["A", "T", "C", "G", "N"])))


# ----------------------------------------------------------------- parsing

def parse_needle_output(needle_filename: str, name: str = "seq", just_score: bool = False) -> pd.DataFrame:
    """Restatement of the reference parser (CRISPRessoCORE.py:1707-1786).

    Reads srspair text (gzip or plain) line by line exactly as the reference
    does: find ``# Aligned_sequences``, skip 1, id = last token of the next line
    with ``_`` -> ``:``, skip 5, identity = last token of the next line stripped
    of ``%()``, then (unless ``just_score``) skip 7 and take ``split()[2]`` of
    the first alignment line, ``[21:]`` of the markup line, ``split()[2]`` and
    ``split()[3]`` of the read line.
    """
    needle_data = []
    try:
        opener = gzip.open if _is_gzip(needle_filename) else open
        with opener(needle_filename, mode="rb") as fh:
            rd = lambda: fh.readline().decode("UTF-8")  # noqa: E731
            line = rd()
            while line:
                while line and ("# Aligned_sequences" not in line):
                    line = rd()
                if line:
                    rd()
                    line = rd()
                    id_seq = line.split()[-1].replace("_", ":")
                    for _ in range(5):
                        rd()
                    line = rd()
                    identity_seq = float(line.strip().split(" ")[-1].replace("%", "").replace(")", "").replace("(", ""))
                    if just_score:
                        needle_data.append([id_seq, identity_seq])
                    else:
                        for _ in range(7):
                            rd()
                        line = rd()
                        aln_ref_seq = line.split()[2]
                        aln_str = rd()[21:].rstrip("\n")
                        line = rd()
                        aln_query_seq = line.split()[2]
                        aln_query_len = line.split()[3]
                        needle_data.append([id_seq, identity_seq, aln_query_len, aln_ref_seq, aln_str, aln_query_seq])
                    line = rd()
    except Exception as exc:
        raise NeedleException("Failed to parse the output of needle!") from exc
    if just_score:
        return pd.DataFrame(needle_data, columns=["ID", "score_" + name]).set_index("ID")
    return pd.DataFrame(
        needle_data, columns=["ID", "score_" + name, "length", "ref_seq", "align_str", "align_seq"]
    ).set_index("ID")


def _is_gzip(path: str) -> bool:
    with open(path, "rb") as f:
        return f.read(2) == b"\x1f\x8b"


def _ids_of(names: Sequence[str], keep: np.ndarray) -> np.ndarray:
    """``line.split()[-1].replace("_", ":")`` of each kept name (CORE:1725), in bulk,
    as an object array.  Names read natively (:class:`fastq.NameList`) are converted
    from their byte block without a per-name Python step."""
    raw = getattr(names, "raw", None)
    if raw is not None and len(raw):
        lib = _lib.load()
        raw = np.ascontiguousarray(raw, dtype=np.uint8)
        ids = np.empty(len(raw), np.uint8)
        off = np.empty(len(names) + 1, np.int64)
        if lib.nw_names_to_ids(_lib.ptr(raw), len(raw), len(names), _lib.ptr(ids), _lib.ptr(off)) == _lib.NW_OK:
            allids = _strings(ids, off, ascii_checked=True)
            return allids if len(keep) == len(names) else allids[keep]
    sel = [names[i] for i in keep] if len(keep) != len(names) else list(names)
    joined = "\n".join(sel)
    if joined.count("\n") == max(len(sel) - 1, 0) and not _WS.search(joined):
        out = joined.replace("_", ":").split("\n") if sel else []
    else:
        out = [nm.split()[-1].replace("_", ":") if nm.split() else "" for nm in sel]
    arr = np.empty(len(out), dtype=object)
    arr[:] = out
    return arr


_WS = __import__("re").compile(r"[ \t\r\f\v\x0b\x1c-\x1f\x85\xa0]")


def _strings(data: np.ndarray, off: np.ndarray, take: Optional[np.ndarray] = None,
             ascii_checked: bool = False) -> np.ndarray:
    """Object array of the ASCII strings data[off[i]:off[i + 1]] (only those i in
    ``take`` when given): built by pyarrow in one native pass when it is importable,
    else one decode + a slice per string."""
    n = len(off) - 1
    if n <= 0 or (take is not None and len(take) == 0):
        return np.empty(0, dtype=object)
    if not ascii_checked and len(data) and int(data.max()) >= 128:
        raise NeedleException("alignment row is not ASCII")
    try:
        import pyarrow as pa
    except ImportError:   # pragma: no cover - pyarrow is in the image
        pa = None
    if pa is not None:
        d = np.ascontiguousarray(data, dtype=np.uint8)
        o = np.ascontiguousarray(off - off[0], dtype=np.int64)
        arr = pa.LargeStringArray.from_buffers(n, pa.py_buffer(o), pa.py_buffer(d[int(off[0]):int(off[-1])]))
        if take is not None:
            arr = arr.take(pa.array(np.asarray(take, dtype=np.int64)))
        return arr.to_numpy(zero_copy_only=False)
    big = np.ascontiguousarray(data).tobytes().decode("ascii")
    idx = range(n) if take is None else np.asarray(take).tolist()
    offl = off.tolist()
    out = np.empty(len(idx), dtype=object)
    out[:] = [big[offl[i]:offl[i + 1]] for i in idx]
    return out


def _rows_to_str(mat: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """Row i's first lens[i] bytes as str, for every row (object array): the rows'
    bytes gathered contiguous by one mask, then :func:`_strings`."""
    n = mat.shape[0]
    if n == 0:
        return np.empty(0, dtype=object)
    w = max(int(lens.max()), 1)
    data = mat[:, :w][np.arange(w)[None, :] < lens[:, None]]
    off = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    return _strings(data, off)


def _printed_percents(num: np.ndarray, den: np.ndarray) -> np.ndarray:
    """printed_percent over arrays: formatted once per distinct (num, den) -- found through a
    dense (den, num) table when the values are small (alignment lengths), else by sorting."""
    if len(num) == 0:
        return np.zeros(0, dtype=np.float64)
    num = num.astype(np.int64)
    den = den.astype(np.int64)
    hi_n, hi_d = int(num.max()) + 1, int(den.max()) + 1
    if int(num.min()) >= 0 and int(den.min()) >= 0 and hi_n * hi_d <= (1 << 24):
        key = den * hi_n + num
        seen = np.zeros(hi_n * hi_d, dtype=bool)
        seen[key] = True
        uniq = np.flatnonzero(seen)
        lut = np.zeros(hi_n * hi_d, dtype=np.float64)
        lut[uniq] = [printed_percent(int(k % hi_n), int(k // hi_n)) for k in uniq.tolist()]
        return lut[key]
    key = (den << 32) | (num & 0xFFFFFFFF)
    uniq, inv = np.unique(key, return_inverse=True)
    vals = np.array([printed_percent(int(k & 0xFFFFFFFF), int(k >> 32)) for k in uniq.tolist()], dtype=np.float64)
    return vals[inv.reshape(-1)]


_INT_STR: List[str] = [str(i) for i in range(4096)]


def batch_to_dataframe(batch: AlignmentBatch, names: Sequence[str], name: str = "seq",
                       just_score: bool = False) -> pd.DataFrame:
    """The DataFrame parse_needle_output would build from this batch's srspair text.

    Fast path (no text, no gzip): identical columns, dtypes and values.  Reads
    needle skips (empty sequences) are absent, as they are from needle's output.
    Columns are built in bulk (one decode + split per string column) rather than
    row by row: 1M rows in about a second instead of eight.
    """
    st = batch.stats
    keep = np.flatnonzero((st["flags"] & _lib.NW_FLAG_EMPTY) == 0)
    ids = _ids_of(names, keep)
    ident = _printed_percents(st["n_ident"][keep], st["aln_len"][keep]).tolist()
    if just_score:
        return pd.DataFrame({"ID": ids, "score_" + name: ident}).set_index("ID")
    cols = np.minimum(st["aln_len"][keep], batch.awidth).astype(np.int64)
    aln = batch.aln if len(keep) == len(st) else batch.aln[keep]
    # "length" = split()[3] of the first read line: the non-'-' characters of the
    # aligned read within the first awidth columns (reads of the RC retry keep '-')
    ends = np.empty(len(keep), dtype=np.int64)
    w = max(int(cols.max()), 1) if len(keep) else 1
    pos = np.arange(w)[None, :]
    for lo in range(0, len(keep), 65536):
        blk = aln[lo:lo + 65536, 2, :w]
        ends[lo:lo + 65536] = np.count_nonzero((blk != ord("-")) & (pos < cols[lo:lo + 65536, None]), axis=1)
    length = [_INT_STR[e] if e < len(_INT_STR) else str(e) for e in ends.tolist()]
    data = {
        "ID": ids,
        "score_" + name: ident,
        "length": length,
        "ref_seq": _rows_to_str(aln[:, 0, :], cols),
        "align_str": _rows_to_str(aln[:, 1, :], cols),
        "align_seq": _rows_to_str(aln[:, 2, :], cols),
    }
    return pd.DataFrame(data, columns=["ID", "score_" + name, "length", "ref_seq", "align_str", "align_seq"]
                        ).set_index("ID")


def ops_to_dataframe(ob: OpsBatch, amplicon: str, buf: np.ndarray, offsets: np.ndarray, names: Sequence[str],
                     name: str = "seq", just_score: bool = False, nthreads: int = 0,
                     index: Optional[pd.Index] = None) -> pd.DataFrame:
    """batch_to_dataframe from the ops output: the same DataFrame, built without the
    rows of reads that are byte-for-byte the amplicon (CRISPResso's unmodified reads,
    most of a typical run): they share one ``ref_seq`` / ``align_str`` / ``align_seq``
    string, as do the ``ref_seq`` of every read whose amplicon row has no gap.  The other
    rows come from nw_ops_rows_concat (runs -> rows cut to ``awidth``, one C++ pass) and
    become strings in bulk (:func:`_strings`)."""
    st = ob.stats
    keep = np.flatnonzero((st["flags"] & _lib.NW_FLAG_EMPTY) == 0)
    ident = _printed_percents(st["n_ident"][keep], st["aln_len"][keep])
    if index is None or len(index) != len(keep) or len(keep) != len(st):
        index = pd.Index(_ids_of(names, keep), dtype=object, name="ID")
    if just_score:
        return pd.DataFrame({"score_" + name: ident}, index=index)
    lib = _lib.load()
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    ref = amplicon.encode("ascii")
    La = len(ref)
    # reads identical to the amplicon (unmodified, same case): one shared string per column
    eq = np.zeros(len(offsets) - 1, np.uint8)
    if La <= ob.awidth:
        lib.nw_reads_equal_ref(ref, La, _lib.ptr(buf), _lib.ptr(offsets), len(eq), _lib.ptr(eq), nthreads)
    other = np.flatnonzero(eq[keep] == 0)
    # row q's strings are entry which[q] of each column's table: 0 = the amplicon's rows,
    # 1 + p = distinct read p's (identical reads have identical rows: built once)
    which = np.zeros(len(keep), np.int64)
    ref_t, str_t, seq_t = [np.array([s], dtype=object) for s in (amplicon, "|" * La, amplicon)]
    end_t = np.array([La], np.int64)
    if len(other):
        rk = np.ascontiguousarray(keep[other], dtype=np.int64)
        rep = np.empty(len(rk), np.int64)
        lib.nw_reads_first_copy(_lib.ptr(buf), _lib.ptr(offsets), _lib.ptr(rk), len(rk), _lib.ptr(rep), nthreads)
        first = np.flatnonzero(rep == np.arange(len(rk)))
        rd = rk[first]
        slot = np.empty(len(rk), np.int64)
        slot[first] = np.arange(1, len(first) + 1)
        which[other] = slot[rep]
        cols = np.minimum(st["aln_len"][rd], ob.awidth).astype(np.int64)
        row_off = np.zeros(len(rd) + 1, np.int64)
        np.cumsum(cols, out=row_off[1:])
        tot = int(row_off[-1])
        r0, r1, r2 = (np.empty(max(tot, 1), np.uint8) for _ in range(3))
        nchar = np.empty(len(rd), np.int32)
        is_amp = np.empty(len(rd), np.uint8)
        ops = np.ascontiguousarray(ob.ops, dtype=np.uint32)
        rc = lib.nw_ops_rows_concat(ref, La, _lib.ptr(buf), _lib.ptr(offsets), _lib.ptr(rd), len(rd),
                                    _lib.ptr(ops) if len(ops) else None, _lib.ptr(ob.ops_off), _lib.ptr(row_off),
                                    _lib.ptr(r0), _lib.ptr(r1), _lib.ptr(r2), _lib.ptr(nchar), _lib.ptr(is_amp),
                                    nthreads)
        if rc != _lib.NW_OK:
            raise NeedleException("Failed to build the alignment rows (runs inconsistent with the reads, "
                                  "or a byte outside ASCII in a read)")
        refs = np.empty(len(rd) + 1, dtype=object)
        refs[0] = amplicon
        amp_row = np.flatnonzero(is_amp)
        refs[1 + amp_row] = amplicon
        if len(amp_row) < len(rd):   # the gapped amplicon rows (a few hundred distinct ones)
            sub = np.flatnonzero(is_amp == 0)
            refs[1 + sub] = _distinct_strings(lib, r0, row_off, sub, nthreads)
        ref_t = refs
        # markup rows repeat across reads (the same substitution positions): one str per distinct row
        str_t = np.concatenate([str_t, _distinct_strings(lib, r1, row_off, None, nthreads)])
        seq_t = np.concatenate([seq_t, _strings(r2, row_off, ascii_checked=True)])
        end_t = np.concatenate([end_t, nchar.astype(np.int64)])
    # the four str columns as one object block (pandas keeps a 2-D array as its block)
    block = np.empty((4, len(keep)), dtype=object)
    block[0] = _int_strings(end_t[which])
    for k, t in enumerate((ref_t, str_t, seq_t)):
        np.take(t, which, out=block[k + 1])
    df = pd.DataFrame(block.T, index=index, columns=["length", "ref_seq", "align_str", "align_seq"], copy=False)
    df.insert(0, "score_" + name, ident)
    return df


def _distinct_strings(lib, data: np.ndarray, off: np.ndarray, take: Optional[np.ndarray], nthreads: int) -> np.ndarray:
    """_strings(data, off, take) with one str object per distinct byte string (equal rows
    share it; nw_reads_first_copy finds the first of each)."""
    idx = np.arange(len(off) - 1, dtype=np.int64) if take is None else np.ascontiguousarray(take, dtype=np.int64)
    if len(idx) == 0:
        return np.empty(0, dtype=object)
    rep = np.empty(len(idx), np.int64)
    lib.nw_reads_first_copy(_lib.ptr(data), _lib.ptr(off), _lib.ptr(idx), len(idx), _lib.ptr(rep), nthreads)
    first = np.flatnonzero(rep == np.arange(len(idx)))
    uniq = _strings(data, off, take=idx[first], ascii_checked=True)
    if len(first) == len(idx):
        return uniq
    slot = np.empty(len(idx), np.int64)
    slot[first] = np.arange(len(first))
    return uniq[slot[rep]]


_INT_OBJ = np.array(_INT_STR, dtype=object)


def _int_strings(v: np.ndarray) -> np.ndarray:
    """str(v[i]) for every i as an object array (one shared string per value < 4096)."""
    if len(v) and int(v.max()) < len(_INT_OBJ) and int(v.min()) >= 0:
        return _INT_OBJ[v]
    out = np.empty(len(v), dtype=object)
    out[:] = [str(e) for e in v.tolist()]
    return out


# ----------------------------------------------------------------- passes

SRSPAIR_HEADER = (
    "########################################\n# Program: needle\n# Rundate: (crispresso_amd)\n"
    "# Commandline: needle\n#    -asequence {a}\n#    -bsequence /dev/stdin\n#    -outfile /dev/stdout\n"
    "# Align_format: srspair\n# Report_file: /dev/stdout\n########################################\n\n"
)
SRSPAIR_TRAILER = "#---------------------------------------\n#---------------------------------------\n"


@dataclass
class PassResult:
    names: Sequence[str]
    batch: Optional[AlignmentBatch]
    ops: Optional[OpsBatch] = None          # the ops path: runs + the inputs to build rows from
    amplicon: str = ""
    buf: Optional[np.ndarray] = None
    offsets: Optional[np.ndarray] = None

    def dataframe(self, name: str = "ref", just_score: bool = False,
                  index: Optional[pd.Index] = None) -> pd.DataFrame:
        """``index``: the ID index of another pass over the same reads, reused when this
        pass keeps the same reads (one Index object: pandas hashes it once, and joins
        two frames on it without a second hash table)."""
        if self.ops is not None:
            return ops_to_dataframe(self.ops, self.amplicon, self.buf, self.offsets, self.names, name, just_score,
                                    index=index)
        return batch_to_dataframe(self.batch, self.names, name, just_score)


def needle_pass(aligner: GpuAligner, amplicon: str, names: Sequence[str], buf: np.ndarray,
                offsets: np.ndarray, amplicon_id: str = "AMPL", outfile: Optional[str] = None,
                just_score: bool = False, packed=None, resident: bool = False) -> PassResult:
    """One ``needle -asequence=AMPL -bsequence=/dev/stdin`` run (CRISPRessoCORE.py:1797-1806).

    ``outfile`` (``needle_output_*.txt.gz``) is written only when given, as the
    reference keeps it only with --keep_intermediate/--dump (CRISPRessoCORE.py:3694-3697).
    ``just_score``: the caller reads only identities (the repair passes,
    CORE:1740-1741), so the alignment strings stay on the GPU unless a file is written.
    ``packed``: the same reads 2-bit packed in pinned memory (fastq.read_fastq_packed):
    the call uploads that (nw_align_ops_packed) instead of the text.  ``resident``: the
    reads are the batch this aligner's last pass uploaded (still in HBM; the HDR pass,
    CORE:1808-1828, re-streams the same FASTQ): nothing is uploaded.
    """
    from .aligner import default_output_mode

    use_ops = getattr(aligner, "ops_native", False) and default_output_mode() == "ops"
    try:
        if aligner.reference != amplicon:
            aligner.set_reference(amplicon)
        if use_ops and resident:
            ob = aligner.align_ops(None, offsets, resident=True, records_only=just_score and not outfile)
            res = PassResult(names if isinstance(names, (list, fastq.NameList)) else list(names), None, ob, amplicon, buf, offsets)
            batch = ob.expand(amplicon, buf, offsets) if outfile else None
        elif use_ops and packed is not None:
            ob = aligner.align_ops_packed(packed)
            res = PassResult(names if isinstance(names, (list, fastq.NameList)) else list(names), None, ob, amplicon, buf, offsets)
            batch = ob.expand(amplicon, buf, offsets) if outfile else None
        elif use_ops:
            ob = aligner.align_ops(buf, offsets, records_only=just_score and not outfile)
            res = PassResult(names if isinstance(names, (list, fastq.NameList)) else list(names), None, ob, amplicon, buf, offsets)
            batch = ob.expand(amplicon, buf, offsets) if outfile else None
        else:
            batch = aligner.align_packed(buf, offsets, strings=not just_score or bool(outfile))
            res = PassResult(names if isinstance(names, (list, fastq.NameList)) else list(names), batch)
    except (NeedleError, UnsupportedNeedleOption) as exc:
        raise NeedleException("Needle failed to run, please check the log file.") from exc
    if outfile:
        text = format_srspair(batch, amplicon_id, res.names, aligner.options)
        with gzip.open(outfile, "wt") as fh:
            fh.write(SRSPAIR_HEADER.format(a=amplicon_id))
            fh.write(text)
            fh.write(SRSPAIR_TRAILER)
    return res


@dataclass
class AlignArgs:
    """The fields of run_crispresso's argparse namespace the alignment step reads."""

    amplicon_seq: str
    expected_hdr_amplicon_seq: str = ""
    min_identity_score: float = 60.0
    needle_options_string: str = DEFAULT_NEEDLE_OPTIONS
    keep_intermediate: bool = False
    dump: bool = False
    # (--min_average_read_quality / --min_single_bp_quality act upstream of this step, on
    # the raw R1 / R2 before trimming and merging, CORE:1547-1583: fastq.filter_se_fastq_by_qual
    # / filter_pe_fastq_by_qual; processed_output_filename is already filtered)


def _dtypes_for_concat(df: pd.DataFrame, like: pd.DataFrame) -> pd.DataFrame:
    """`df` with its all-NA columns cast to `like`'s dtypes, so that pd.concat([like, df])
    (CRISPRessoCORE.py:1998) gives the dtypes it gives today -- pandas excludes all-NA
    columns when it picks a concatenation's dtypes (the RC-HDR quirk's NaN repair scores)
    and has deprecated that -- without depending on the pandas version."""
    cast = {c: like[c].dtype for c in df.columns
            if c in like.columns and df[c].dtype != like[c].dtype and df[c].isna().all()}
    return df.astype(cast) if cast else df


def align_reads(args: AlignArgs, processed_output_filename: str, aligner: Optional[GpuAligner] = None,
                output_dir: Optional[str] = None, database_id: str = "AMPL",
                rc_hdr_quirk: str = "reference", timings: Optional[dict] = None) -> pd.DataFrame:
    """CRISPRessoCORE.py:1788-2000 on the GPU: returns ``df_needle_alignment``.

    The result has the reference's columns (``score_ref, length, ref_seq,
    align_str, align_seq`` and, with an HDR amplicon, ``score_repaired,
    score_diff``) and index (read ids, ``_RC`` suffix for reverse-complement hits).

    Data path: the native ingest reads the FASTQ(.gz) and packs the reads 2 bits per base
    into pinned memory (fastq.read_fastq_packed); the forward pass uploads that batch once
    (nw_align_ops_packed) and the HDR pass re-aligns it where it lies in HBM
    (nw_align_ops_resident); records and runs come back into pinned memory, and the
    DataFrame is built from them and the text (ops_to_dataframe).  ``timings``, when a
    dict, receives the seconds of each stage (ingest, aligner calls, DataFrame, rest).
    """
    # CRISPRessoCORE.py:1283 and 1350 normalise the amplicons before anything else
    args.amplicon_seq = args.amplicon_seq.upper().strip().rstrip("\n")
    if args.expected_hdr_amplicon_seq:
        args.expected_hdr_amplicon_seq = args.expected_hdr_amplicon_seq.strip().upper()
    opts = NeedleOptions.parse(args.needle_options_string)
    own = aligner is None
    if own:
        aligner = GpuAligner(0, opts)
    keep_files = bool(output_dir) and (args.keep_intermediate or args.dump)
    _jp = (lambda f: os.path.join(output_dir, f)) if output_dir else (lambda f: f)
    import time

    tm = timings if timings is not None else {}
    clock = time.perf_counter
    t_start = clock()
    try:
        native = getattr(aligner, "ops_native", False) and hasattr(aligner, "align_ops_packed")
        t0 = clock()
        if native:
            names, buf, offsets, packed = fastq.read_fastq_packed(processed_output_filename, pinned=True)
        else:
            names, buf, offsets = fastq.read_fastq_as_fasta(processed_output_filename)
            packed = None
        tm["ingest_s"] = clock() - t0
        t0 = clock()
        # the HDR amplicon's copies among the reads take one alignment of it in the forward pass
        # (nw_set_known), the reference amplicon's copies in the resident HDR pass (automatic)
        # both passes in one call (nw_align_dual_ops_packed_lens: one upload, the HDR pass's chunks
        # interleaved with the forward pass's) when no needle file is kept
        dual = (native and bool(args.expected_hdr_amplicon_seq) and not keep_files and packed is not None
                and getattr(packed, "lens", None) is not None and hasattr(aligner, "align_dual_packed")
                and default_output_mode() == "ops" and _lib.has_symbol("nw_align_dual_ops_packed_lens"))
        known = args.expected_hdr_amplicon_seq if native and not dual and hasattr(aligner, "set_known") else None
        rep = None
        if dual:
            if aligner.reference != args.amplicon_seq:
                aligner.set_reference(args.amplicon_seq)
            try:
                ob1, ob2 = aligner.align_dual_packed(packed, args.expected_hdr_amplicon_seq, records_only2=True)
            except NeedleError as exc:
                raise NeedleException("Needle failed to run, please check the log file.") from exc
            nl = names if isinstance(names, (list, fastq.NameList)) else list(names)
            fwd = PassResult(nl, None, ob1, args.amplicon_seq, buf, offsets)
            rep = PassResult(nl, None, ob2, args.expected_hdr_amplicon_seq, buf, offsets)
        else:
            if known:
                aligner.set_known(known)
            try:
                fwd = needle_pass(aligner, args.amplicon_seq, names, buf, offsets, database_id,
                                  _jp(f"needle_output_{database_id}.txt.gz") if keep_files else None, packed=packed)
            finally:
                if known:
                    aligner.set_known(None)
        tm["align_s"] = clock() - t0
        if args.expected_hdr_amplicon_seq:
            t0 = clock()
            if rep is None:
                rep = needle_pass(aligner, args.expected_hdr_amplicon_seq, names, buf, offsets, database_id,
                                  _jp(f"needle_output_repair_{database_id}.txt.gz") if keep_files else None,
                                  just_score=True, resident=native)
            tm["align_hdr_s"] = clock() - t0
            t0 = clock()
            df_database = fwd.dataframe("ref")
            # same reads, same (non-empty) rows: the repair frame shares the ID index
            df_database_repair = rep.dataframe("repaired", just_score=True, index=df_database.index)
            df_database_and_repair = df_database.join(df_database_repair)
            # the reference's masks (CORE:1842-1851) as numpy arrays: a boolean Series would be
            # aligned on the 1M-entry object index first (~0.06 s per mask, same rows)
            sr_not_aligned = df_database_and_repair.loc[
                ((df_database_and_repair.score_ref < args.min_identity_score)
                 & (df_database_and_repair.score_ref < args.min_identity_score)).to_numpy()
            ].align_seq.apply(lambda x: x.replace("_", ""))
            df_database_and_repair = df_database_and_repair.loc[
                ((df_database_and_repair.score_ref > args.min_identity_score)
                 | (df_database_and_repair.score_repaired > args.min_identity_score)).to_numpy()
            ].copy()
            df_database_and_repair["score_diff"] = (
                df_database_and_repair.score_ref - df_database_and_repair.score_repaired
            )
            df_needle_alignment = df_database_and_repair
            tm["dataframe_s"] = clock() - t0
        else:
            t0 = clock()
            df_needle_alignment = fwd.dataframe("ref")
            tm["dataframe_s"] = clock() - t0
            sr_not_aligned = df_needle_alignment.loc[
                (df_needle_alignment.score_ref < args.min_identity_score).to_numpy()
            ].align_seq.apply(lambda x: x.replace("_", ""))
            df_needle_alignment = df_needle_alignment.loc[
                (df_needle_alignment.score_ref > args.min_identity_score).to_numpy()]

        if sr_not_aligned.count():
            fasta_text = "".join(f">{x0}\n{x1}\n" for x0, x1 in sr_not_aligned.items())
            if keep_files:
                with gzip.open(_jp("not_aligned_amplicon_forward.fa.gz"), "wt") as fh:
                    fh.write(fasta_text)
            rc_names, rc_buf, rc_off = fastq.parse_fasta_text(fasta_text)
            rc_amp = reverse_complement(args.amplicon_seq)
            rc = needle_pass(aligner, rc_amp, rc_names, rc_buf, rc_off, database_id,
                             _jp(f"needle_output_rc_{database_id}.txt.gz") if keep_files else None)
            if args.expected_hdr_amplicon_seq:
                if rc_hdr_quirk == "reference":
                    # CRISPRessoCORE.py:1924-1936: needle gets the literal text
                    # "args.needle_options_string" and aligns nothing; the empty output
                    # parses to an empty table (CORE:1776-1777)
                    df_repair_rc = pd.DataFrame([], columns=["ID", "score_repaired"]).set_index("ID")
                    if keep_files:
                        with gzip.open(_jp(f"needle_output_repair_rc_{database_id}.txt.gz"), "wt"):
                            pass
                else:
                    rc_rep = needle_pass(aligner, reverse_complement(args.expected_hdr_amplicon_seq), rc_names,
                                         rc_buf, rc_off, database_id,
                                         _jp(f"needle_output_repair_rc_{database_id}.txt.gz") if keep_files
                                         else None, just_score=True)
                    df_repair_rc = rc_rep.dataframe("repaired", just_score=True)
                df_database_and_repair_rc = rc.dataframe("ref").join(df_repair_rc)
                df_database_and_repair_rc = df_database_and_repair_rc.loc[
                    ((df_database_and_repair_rc.score_ref > args.min_identity_score)
                     | (df_database_and_repair_rc.score_repaired > args.min_identity_score)).to_numpy()
                ].copy()
                df_database_and_repair_rc["score_diff"] = (
                    df_database_and_repair_rc.score_ref - df_database_and_repair_rc.score_repaired
                )
                df_needle_alignment_rc = df_database_and_repair_rc
            else:
                df_needle_alignment_rc = rc.dataframe("ref")
                df_needle_alignment_rc = df_needle_alignment_rc.loc[
                    (df_needle_alignment_rc.score_ref > args.min_identity_score).to_numpy()
                ].copy()
            df_needle_alignment_rc["ref_seq"] = df_needle_alignment_rc["ref_seq"].apply(reverse_complement)
            df_needle_alignment_rc["align_seq"] = df_needle_alignment_rc["align_seq"].apply(reverse_complement)
            df_needle_alignment_rc["align_str"] = df_needle_alignment_rc["align_str"].apply(lambda x: x[::-1])
            df_needle_alignment_rc.index = map(lambda x: "_".join([x, "RC"]), df_needle_alignment_rc.index)
            df_needle_alignment = pd.concat([df_needle_alignment, _dtypes_for_concat(df_needle_alignment_rc,
                                                                                    df_needle_alignment)])
        tm["total_s"] = clock() - t_start
        return df_needle_alignment
    finally:
        if own:
            aligner.close()
