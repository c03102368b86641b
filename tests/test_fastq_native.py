"""Native FASTQ ingest (nw_fastq_read) == the Python restatement of the reference's
gunzip | awk | sed stage and EMBOSS's reader (fastq.fastq_bytes_as_fasta), on the
reference's test reads, the golden fixtures and edge cases (no trailing newline, a
header without its sequence line, CRLF, ':' and digits in sequences, lower case,
whitespace-led headers, chunk-boundary-sized lines).  The reader has two decoders --
libdeflate into one buffer parsed by several threads in parts cut at record boundaries,
and zlib gzread (CRISPR_NW_FASTQ_ZLIB=1) -- held to the same outputs."""
import gzip
import os

import numpy as np
import pytest

from crispresso_amd import fastq

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _same(path):
    n1, b1, o1 = fastq.read_fastq_as_fasta(path)
    n2, b2, o2 = fastq.read_fastq_as_fasta_py(path)
    assert n1 == n2
    assert np.array_equal(o1, o2)
    assert np.array_equal(b1, b2)
    return n1


@pytest.mark.parametrize("name", [f for f in sorted(os.listdir(GOLDEN)) if f.endswith(".fastq.gz")])
def test_golden_fastq_files(name):
    assert len(_same(os.path.join(GOLDEN, name))) > 0


@pytest.mark.parametrize("gz", [False, True])
@pytest.mark.parametrize("text", [
    b"@r1:a b\nACGT\n+\nIIII\n@r2\nAC:GT\n+\nIIII\n",
    b"@r1\nACGT\n+\nIIII\n@r2\nACGT\n+\nIIII",            # no trailing newline
    b"@r1\nACGT\n+\nIIII\n@r2\n",                          # a header without its sequence line
    b"@r1\nACGT\n+\nIIII\n@r2",                            # ... and without a newline
    b"@r1 x\r\nAC gt\r\n+\r\nIIII\r\n",                    # CRLF, spaces, lower case
    b"  @r1\tname\nN-*.~?#+-12acgtRY_:\n+\n!!!!\n",        # whitespace before the name, odd bytes
    b"\n\n\n\n@r2\nAC\n+\nII\n",                           # an empty header line
    b"",
    b"@only\n",
])
def test_edge_cases(tmp_path, gz, text):
    p = tmp_path / ("x.fastq.gz" if gz else "x.fastq")
    if gz:
        with gzip.open(p, "wb") as f:
            f.write(text)
    else:
        p.write_bytes(text)
    _same(str(p))


def test_long_lines_across_read_chunks(tmp_path):
    """Lines longer than zlib's buffer and the reader's chunks cross chunk boundaries."""
    rng = np.random.Generator(np.random.PCG64(5))
    parts = []
    for k in range(3):
        seq = rng.choice(np.frombuffer(b"ACGTNacgt:1", np.uint8), 3_000_000 + k).tobytes()
        parts.append(b"@long%d x:y\n" % k + seq + b"\n+\n" + b"I" * len(seq) + b"\n")
    p = tmp_path / "long.fastq.gz"
    with gzip.open(p, "wb", compresslevel=1) as f:
        f.write(b"".join(parts))
    assert len(_same(str(p))) == 3


# ---- read quality filter (CORE:162-308, applied at 1547-1583) ----------------------------

R1 = os.path.join(GOLDEN, "test_L001_R1_001.fastq.gz")   # the reference's own test data
R2 = os.path.join(GOLDEN, "test_L001_R2_001.fastq.gz")


def test_ids_reads_to_remove_known_answers():
    """The reference's test_get_ids_reads_to_remove (tests/crispresso_tests.py:77-88)."""
    assert fastq.get_ids_reads_to_remove(R1, 23) == {"M06879:15:000000000-DFF22:1:1101:25894:23776",
                                                      "M06879:15:000000000-DFF22:1:1101:24046:20708"}
    assert fastq.get_ids_reads_to_remove(R2, 15) == {"M06879:15:000000000-DFF22:1:1102:22078:15849"}


@pytest.mark.parametrize("q", [(20, 0), (23, 0), (30, 0), (30, 10), (35, 20), (0, 15), (41, 0)])
@pytest.mark.parametrize("path", [R1, R2])
def test_native_quality_filter_matches_restatement(path, q):
    """nw_fastq_read_filtered keeps exactly the records filter_se_fastq_by_qual keeps
    (Python restatement of CORE:296-305), names and bases."""
    got = fastq.read_fastq_as_fasta(path, *q)
    want = fastq.read_fastq_as_fasta_py(path, *q)
    assert list(got[0]) == list(want[0])
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[2], want[2])
    # the dropped records are the ones get_ids_reads_to_remove names (SE test = PE test per file)
    allnames = fastq.read_fastq_as_fasta(path)[0]
    dropped = set(allnames) - set(got[0])
    ids = {("@" + i).split()[0].replace(":", "_") for i in fastq.get_ids_reads_to_remove(path, *q)}
    assert dropped == ids


def test_quality_filter_edge_cases(tmp_path):
    """Empty quality line (NaN mean: dropped), a record cut before its quality line,
    CRLF line ends, a quality exactly at the threshold (kept: mean >= q)."""
    text = (b"@a\nACGT\n+\nIIII\n"      # Q40
            b"@b\nACGT\n+\n\n"          # no qualities
            b"@c\r\nACGT\r\n+\r\n5555\r\n"   # Q20 exactly
            b"@d\nACGT\n+\n5554\n"      # mean 19.75
            b"@e\nAC\n+\n!I\n"           # min 0, mean 20
            b"@f\nACGTAC\n")             # truncated
    p = tmp_path / "q.fastq"
    p.write_bytes(text)
    for q in [(20, 0), (20, 1), (1, 0), (0, 1)]:
        got = fastq.read_fastq_as_fasta(str(p), *q)
        want = fastq.read_fastq_as_fasta_py(str(p), *q)
        assert list(got[0]) == list(want[0]), q
        assert np.array_equal(got[2], want[2])
    assert list(fastq.read_fastq_as_fasta(str(p), 20, 0)[0]) == ["@a", "@c", "@e"]


def test_filter_se_pe_files(tmp_path):
    """The reference's file-writing filters: outputs re-read to the same reads the
    in-memory filter gives; the PE pair drops a read from both files when either mate fails."""
    out = fastq.filter_se_fastq_by_qual(R1, str(tmp_path / "se.fastq.gz"), min_bp_quality=30)
    assert list(fastq.read_fastq_as_fasta(out)[0]) == list(fastq.read_fastq_as_fasta(R1, 30)[0])
    o1, o2 = fastq.filter_pe_fastq_by_qual(R1, R2, str(tmp_path / "r1.fastq.gz"), str(tmp_path / "r2.fastq.gz"),
                                           min_bp_quality=30)
    n1, n2 = fastq.read_fastq_as_fasta(o1)[0], fastq.read_fastq_as_fasta(o2)[0]
    drop = fastq.get_ids_reads_to_remove(R1, 30) | fastq.get_ids_reads_to_remove(R2, 30)
    assert len(n1) == len(n2) == len(fastq.read_fastq_as_fasta(R1)[0]) - len(drop)
    assert fastq.filter_se_fastq_by_qual.__defaults__[1:] == (20, 0)   # the reference's defaults


def _native(path, q=0, qs=0):
    n, b, o = fastq.read_fastq_as_fasta(path, q, qs)
    return list(n), b, o


def _random_fastq(rng, n, odd=True):
    """Records with the edge cases of test_edge_cases mixed in: '@' / '+' leading quality
    lines, CRLF, empty sequence lines, long lines, ':' and spaces."""
    alpha = np.frombuffer(b"ACGTNacgt:-*", np.uint8)
    out = []
    for i in range(n):
        L = int(rng.integers(0, 40)) if odd and i % 97 == 5 else int(rng.integers(60, 300))
        seq = rng.choice(alpha, L).tobytes()
        qual = rng.integers(33, 75, L).astype(np.uint8).tobytes()
        if odd and i % 13 == 0 and L:
            qual = b"@" + qual[1:]                 # a quality line that starts like a header
        if odd and i % 17 == 0 and L:
            qual = b"+" + qual[1:]
        eol = b"\r\n" if odd and i % 31 == 0 else b"\n"
        out.append(b"@read:%d extra%s" % (i, eol) + seq + eol + b"+" + eol + qual + eol)
    return b"".join(out)


@pytest.mark.parametrize("gz", [False, True])
@pytest.mark.parametrize("q", [(0, 0), (30, 0), (25, 10)])
@pytest.mark.parametrize("tail", [b"", b"@last\nACGT\n+\nII", b"@last\nACG", b"@last\n"])
def test_parallel_parse_equals_serial(tmp_path, monkeypatch, gz, q, tail):
    """Small files forced through the parallel parse (CRISPR_NW_FASTQ_PAR_MIN): parts cut
    at record boundaries anywhere, the last part's open record or line carried on; equal
    to the zlib streaming path and to the Python restatement, with and without the quality
    filter."""
    rng = np.random.Generator(np.random.PCG64(11 + len(tail)))
    text = _random_fastq(rng, 3000) + tail
    p = tmp_path / ("x.fastq.gz" if gz else "x.fastq")
    if gz:
        with gzip.open(p, "wb") as f:
            f.write(text)
    else:
        p.write_bytes(text)
    monkeypatch.setenv("CRISPR_NW_FASTQ_PAR_MIN", "1")
    par = _native(str(p), *q)
    monkeypatch.setenv("CRISPR_NW_FASTQ_ZLIB", "1")
    ser = _native(str(p), *q)
    py = fastq.read_fastq_as_fasta_py(str(p), *q)
    for a in (ser, py):
        assert par[0] == list(a[0])
        assert np.array_equal(par[1], a[1]) and np.array_equal(par[2], a[2])


def test_multi_member_gzip(tmp_path, monkeypatch):
    """Concatenated gzip members (each its own libdeflate call) and trailing garbage after
    the last member (ignored, as gzread does)."""
    rng = np.random.Generator(np.random.PCG64(3))
    p = tmp_path / "multi.fastq.gz"
    blobs = [_random_fastq(rng, 500, odd=False) for _ in range(3)]
    with open(p, "wb") as f:
        for b in blobs:
            f.write(gzip.compress(b))
    fast = _native(str(p))
    monkeypatch.setenv("CRISPR_NW_FASTQ_ZLIB", "1")
    slow = _native(str(p))
    assert fast[0] == slow[0] and len(fast[0]) == 1500
    assert np.array_equal(fast[1], slow[1]) and np.array_equal(fast[2], slow[2])


def _read_in_child(path, q):
    n, b, o = fastq.read_fastq_as_fasta(path)
    q.put((len(n), int(b.sum()), int(o[-1])))


@pytest.mark.timeout(120)
def test_host_pool_threads_and_fork(tmp_path, monkeypatch):
    """The parallel parse's host pool: callers on several Python threads at once (one
    job at a time: the others parse inline) and a forked child (the parked threads stay
    in the parent: the child parses inline instead of waiting for them)."""
    import multiprocessing as mp
    import threading

    rng = np.random.Generator(np.random.PCG64(29))
    p = tmp_path / "t.fastq.gz"
    with gzip.open(p, "wb") as f:
        f.write(_random_fastq(rng, 4000))
    monkeypatch.setenv("CRISPR_NW_FASTQ_PAR_MIN", "1")
    ref = _native(str(p))
    out = [None] * 6

    def run(i):
        out[i] = _native(str(p))

    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(out))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for r in out:
        assert r[0] == ref[0] and np.array_equal(r[1], ref[1]) and np.array_equal(r[2], ref[2])
    q = mp.get_context("fork").Queue()
    child = mp.get_context("fork").Process(target=_read_in_child, args=(str(p), q))
    child.start()
    got = q.get(timeout=60)
    child.join(timeout=60)
    assert child.exitcode == 0
    assert got == (len(ref[0]), int(ref[1].sum()), int(ref[2][-1]))


def test_packed_ingest_matches_text_and_pack_reads(tmp_path):
    """nw_fastq_pack: the aligner's packed input straight from the ingest (pageable here; pinned
    on a GPU box) equals nw_pack_reads of the text; text and offsets are the same reads the
    text reader returns (N and IUPAC bytes go to the exception list)."""
    import gzip

    from crispresso_amd.aligner import pack_2bit

    recs = []
    rng = np.random.Generator(np.random.PCG64(5))
    for k in range(3000):
        L = int(rng.integers(0, 300))
        seq = "".join(rng.choice(list("ACGTACGTACGTNacgtRY"), L))
        recs.append(f"@r:{k} x\n{seq}\n+\n{'I' * L}\n")
    p = tmp_path / "r.fastq.gz"
    with gzip.open(p, "wt") as f:
        f.write("".join(recs))
    names, text, off, pk = fastq.read_fastq_packed(str(p), pinned=False)
    n2, b2, o2 = fastq.read_fastq_as_fasta(str(p))
    assert list(names) == list(n2) and np.array_equal(off, o2) and np.array_equal(text, b2)
    want = pack_2bit(b2, o2)
    nb = (int(o2[-1]) + 3) // 4
    assert np.array_equal(pk.packed[:nb], want.packed[:nb])
    assert np.array_equal(pk.exc_pos, want.exc_pos) and np.array_equal(pk.exc_byte, want.exc_byte)
    assert len(pk.exc_pos) > 0 and pk.offsets is off
    assert pk.lens is not None and np.array_equal(pk.lens, np.diff(o2))   # nw_fastq_lens
