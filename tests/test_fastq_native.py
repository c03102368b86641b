"""Native FASTQ ingest (nw_fastq_read) == the Python restatement of the reference's
gunzip | awk | sed stage and EMBOSS's reader (fastq.fastq_bytes_as_fasta), on the
reference's test reads, the golden fixtures and edge cases (no trailing newline, a
header without its sequence line, CRLF, ':' and digits in sequences, lower case,
whitespace-led headers, chunk-boundary-sized lines)."""
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
