"""Host-side logic around the aligner (CPU only): needle options, the
FASTQ->FASTA semantics of the reference pipeline, the srspair writer, the
DataFrame fast path vs the restated parser, and the reference helpers."""
import gzip

import numpy as np
import pandas as pd
import pytest

from crispresso_amd import fastq, synth
from crispresso_amd.aligner import format_srspair, pack_reads, printed_percent
from crispresso_amd.needle import batch_to_dataframe, find_wrong_nt, parse_needle_output, reverse_complement
from crispresso_amd.needle_options import DEFAULT_NEEDLE_OPTIONS, NeedleOptions, UnsupportedNeedleOption
from tests.helpers import oracle_batch


def test_default_needle_options():
    o = NeedleOptions.parse(DEFAULT_NEEDLE_OPTIONS)
    assert (o.gap_open, o.gap_extend, o.awidth, o.end_weight, o.matrix) == (10.0, 0.5, 5000, False, "EDNAFULL")


@pytest.mark.parametrize("text,expect", [
    ("-gapopen 12 -gapextend=1", (12.0, 1.0)),
    ("-gapopen=5.5 -gapextend 0.25 -noendweight", (5.5, 0.25)),
    ("-auto -gapopen=10 -gapextend=0.5 -awidth3=60 -aformat3 srspair", (10.0, 0.5)),
])
def test_needle_option_forms(text, expect):
    o = NeedleOptions.parse(text)
    assert (o.gap_open, o.gap_extend) == expect


def test_endweight_options():
    o = NeedleOptions.parse("-gapopen=10 -gapextend=0.5 -endweight -endopen=3 -endextend 1.5")
    assert (o.end_weight, o.end_open, o.end_extend) == (True, 3.0, 1.5)
    o = NeedleOptions.parse("-endweight=N -endopen=3")
    assert not o.end_weight
    o = NeedleOptions.parse("-endweight=Y")
    assert (o.end_weight, o.end_open, o.end_extend) == (True, 10.0, 0.5)   # EMBOSS defaults


@pytest.mark.parametrize("text", ["-datafile=EBLOSUM62", "-bogus 3", "stray", "-endweight -endopen=-1"])
def test_unsupported_needle_options_raise(text):
    with pytest.raises(UnsupportedNeedleOption):
        NeedleOptions.parse(text)


def test_reference_helpers():
    # tests/crispresso_tests.py:99-101 of the reference
    assert reverse_complement("ACTGGT") == "ACCAGT"
    assert reverse_complement("ac-gN_") == "_NC-GT"
    with pytest.raises(KeyError):
        reverse_complement("ACR")
    # the reference test at :93-96 compares None == None; this is the intended check
    assert sorted(find_wrong_nt("ACBTGCNGRCCACTGFNNC")) == ["B", "F", "R"]


def test_fastq_to_fasta_semantics():
    data = (b"@M1:2:AB-C:1 1:N:0:1\nACGTN\n+\nIIIII\n"
            b"@r_2 desc\nac.gt-*x1\n+\nIIIIIIIII\n"
            b"@empty\n\n+\n\n")
    names, buf, off = fastq.fastq_bytes_as_fasta(data)
    # awk keeps '@' and the whole header; sed turns every ':' into '_'; EMBOSS keeps the first word
    assert names == ["@M1_2_AB-C_1", "@r_2", "@empty"]
    seqs = synth.unpack(buf, off)
    # EMBOSS keeps letters and *.~?#+- ; digits are dropped
    assert seqs == ["ACGTN", "ac.gt-*x", ""]
    # parse_needle_output turns '_' back into ':' (real underscores too)
    assert names[1].split()[-1].replace("_", ":") == "@r:2"


def test_fastq_file_counts(tmp_path):
    p = tmp_path / "r.fastq.gz"
    recs = b"".join(b"@id%d\nACGT\n+\nIIII\n" % i for i in range(25))
    p.write_bytes(gzip.compress(recs))
    names, buf, off = fastq.read_fastq_as_fasta(str(p))
    assert len(names) == 25 == fastq.count_reads(str(p))


def _batch(amp, reads, awidth=5000):
    buf, off = pack_reads(reads)
    return oracle_batch(amp, buf, off, awidth)


def test_cpp_writer_matches_oracle_writer(oracle):
    amp = synth.random_amplicon(120, 9)
    buf, off = synth.reads_from(amp, 60, 10, synth.PARITY_MIX)
    reads = synth.unpack(buf, off)
    batch = oracle_batch(amp, buf, off)
    names = [f"@M1_2_{k}" for k in range(len(reads))]
    text = format_srspair(batch, "AMPL", names, NeedleOptions())
    expect = ""
    for k, r in enumerate(reads):
        res, ra, mk, rb = oracle.align(amp, r)
        expect += oracle.srspair("AMPL", names[k], res, ra, mk, rb)
    assert text == expect


@pytest.mark.parametrize("awidth", [5000, 60])
def test_dataframe_fast_path_equals_text_parse(tmp_path, awidth):
    amp = synth.random_amplicon(150, 11)
    buf, off = synth.reads_from(amp, 200, 12, synth.PARITY_MIX)
    reads = synth.unpack(buf, off) + ["", "ACGT-ACGT"]
    buf, off = pack_reads(reads)
    batch = oracle_batch(amp, buf, off, awidth)
    names = [f"@M0_1_{k}" for k in range(len(reads))]
    o = NeedleOptions(awidth=awidth)
    p = tmp_path / "needle.txt.gz"
    with gzip.open(p, "wt") as fh:
        fh.write("# header\n\n" + format_srspair(batch, "AMPL", names, o) + "#---\n")
    for name, js in (("ref", False), ("repaired", True)):
        parsed = parse_needle_output(str(p), name, just_score=js)
        fast = batch_to_dataframe(batch, names, name, just_score=js)
        pd.testing.assert_frame_equal(parsed, fast)
    assert len(parsed) == len(reads) - 1        # needle skips the empty read


def test_printed_percent_is_printf_rounding():
    for num, den in [(151, 280), (1, 8), (1, 400), (3, 400), (100, 100), (0, 7)]:
        assert printed_percent(num, den) == float("%.1f" % (100.0 * num / den))


def test_needle_cli_argument_split():
    from crispresso_amd.needle_cli import split_args

    a, b, out, rest = split_args(["-asequence=A.fa", "-bsequence", "/dev/stdin", "-outfile=/dev/stdout",
                                  "-gapopen=10", "-gapextend=0.5", "-awidth3=5000"])
    assert (a, b, out) == ("A.fa", "/dev/stdin", "/dev/stdout")
    assert NeedleOptions.parse(rest).awidth == 5000


def test_needle_cli_rejects_bad_options(capsys):
    from crispresso_amd.needle_cli import main

    assert main(["-asequence=a", "-bsequence=b", "-datafile=EBLOSUM62"]) == 1
    assert "EDNAFULL" in capsys.readouterr().err


def test_ops_to_dataframe_equals_rows_dataframe():
    """The ops-path DataFrame (shared strings for reads identical to the amplicon,
    rows expanded only for the others) equals batch_to_dataframe's, column by column."""
    import numpy as np

    from crispresso_amd import synth
    from crispresso_amd.aligner import pack_reads
    from crispresso_amd.needle import batch_to_dataframe, ops_to_dataframe
    from tests.helpers import OracleAligner, ops_from_batch

    amp = synth.random_amplicon(230, 8)
    buf0, off0 = synth.reads_from(amp, 600, 9)
    reads = synth.unpack(buf0, off0) + ["", amp.lower(), amp, amp[:-1], "NNNN"]
    buf, off = pack_reads(reads)
    names = [f"@r_{i}" for i in range(len(reads))]
    al = OracleAligner()
    al.set_reference(amp)
    rows = al.align_packed(buf, off)
    ob = ops_from_batch(rows)
    want = batch_to_dataframe(rows, names, "ref")
    got = ops_to_dataframe(ob, amp, buf, off, names, "ref")
    assert list(got.columns) == list(want.columns) and list(got.index) == list(want.index)
    for c in want.columns:
        assert got[c].tolist() == want[c].tolist(), c
    assert got["score_ref"].dtype == want["score_ref"].dtype
    js = ops_to_dataframe(ob, amp, buf, off, names, "repaired", just_score=True)
    assert js.equals(batch_to_dataframe(rows, names, "repaired", just_score=True))
    assert int((np.asarray(got["ref_seq"].tolist(), dtype=object) == amp).sum()) >= 300
    # names as the native FASTQ reader returns them (IDs built from the byte block), and
    # rows cut at a narrow -awidth3: still the same frame, dtypes included
    import pandas as pd

    from crispresso_amd.fastq import NameList
    raw = np.frombuffer(("\n".join(names) + "\n").encode(), np.uint8).copy()
    for awidth in (5000, 100):
        rows.awidth = awidth
        ob.awidth = awidth
        want = batch_to_dataframe(rows, names, "ref")
        got = ops_to_dataframe(ob, amp, buf, off, NameList(names, raw), "ref")
        pd.testing.assert_frame_equal(got, want)
        assert got.index.tolist()[:2] == ["@r:0", "@r:1"]


def test_read_lengths16():
    """nw_read_lengths16 (the lengths nw_align_ops_packed_lens uploads instead of the offsets):
    np.diff of the offsets as uint16, threads over contiguous ranges; None past 65535 bases."""
    from crispresso_amd.aligner import pack_2bit, read_lengths16

    rng = np.random.Generator(np.random.PCG64(3))
    lens = rng.integers(0, 700, 300_000)
    off = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    off += 123   # a batch that starts mid-buffer
    got = read_lengths16(off)
    assert got.dtype == np.uint16 and np.array_equal(got, lens)
    out = np.empty(len(lens), np.uint16)
    assert read_lengths16(off, out) is not None and np.array_equal(out, lens)
    big = off.copy()
    big[1000:] += 70_000   # read 999 is 70k bases long
    assert read_lengths16(big) is None
    assert len(read_lengths16(np.zeros(1, np.int64))) == 0
    buf, o2 = synth.reads_from(synth.random_amplicon(120, 4), 50, 5)
    assert np.array_equal(pack_2bit(buf, o2).lens, np.diff(o2))


def test_reads_first_copy():
    """nw_reads_first_copy (the DataFrame hand-off builds each distinct read's strings once):
    the first index with the same bytes, over all reads and over an index subset; reads that
    differ only in length or case are distinct."""
    from crispresso_amd import _lib

    lib = _lib.load()
    rng = np.random.Generator(np.random.PCG64(11))
    pool = ["".join(rng.choice(list("ACGT"), int(rng.integers(0, 40)))) for _ in range(300)]
    pool += ["ACGT", "ACG", "acgt", ""]
    reads = [pool[int(k)] for k in rng.integers(0, len(pool), 50_000)]
    buf, off = pack_reads(reads)
    for idx in (None, np.sort(rng.choice(len(reads), 20_000, replace=False)).astype(np.int64)):
        sel = list(range(len(reads))) if idx is None else idx.tolist()
        seen, want = {}, []
        for q, r in enumerate(sel):
            want.append(seen.setdefault(reads[r], q))
        rep = np.empty(len(sel), np.int64)
        nd = lib.nw_reads_first_copy(_lib.ptr(buf), _lib.ptr(off), None if idx is None else _lib.ptr(idx), len(sel),
                                     _lib.ptr(rep), 0)
        assert nd == len(seen) and rep.tolist() == want


def test_names_to_ids():
    """nw_names_to_ids: CORE:1725's split()[-1].replace('_', ':') of each name, for names
    without whitespace (the reader keeps the header's first word); a name with whitespace,
    a non-ASCII byte or a count mismatch is left to Python."""
    from crispresso_amd import _lib

    lib = _lib.load()
    rng = np.random.Generator(np.random.PCG64(12))
    names = [f"@M0_{k}_{'x' * int(rng.integers(0, 30))}_1" if k % 7 else "" for k in range(200_000)]
    raw = np.frombuffer(("\n".join(names) + "\n").encode(), np.uint8).copy()   # > 1 MB: the parallel path
    ids = np.empty(len(raw), np.uint8)
    off = np.empty(len(names) + 1, np.int64)
    assert lib.nw_names_to_ids(_lib.ptr(raw), len(raw), len(names), _lib.ptr(ids), _lib.ptr(off)) == _lib.NW_OK
    got = [ids[off[i]:off[i + 1]].tobytes().decode() for i in range(len(names))]
    assert got == [nm.replace("_", ":") for nm in names]
    for bad in (b"@a b\n@c\n", "@é\n@c\n".encode()):
        r = np.frombuffer(bad, np.uint8).copy()
        assert lib.nw_names_to_ids(_lib.ptr(r), len(r), 2, _lib.ptr(ids), _lib.ptr(off)) == _lib.NW_E_UNSUPPORTED
    r = np.frombuffer(b"@a\n@c\n", np.uint8).copy()
    assert lib.nw_names_to_ids(_lib.ptr(r), len(r), 3, _lib.ptr(ids), _lib.ptr(off)) == _lib.NW_E_UNSUPPORTED
