"""The FASTQ ingest's parallel gzip decoder (crispresso_amd/csrc/gz_inflate.cpp, exported as
nw_gunzip_parallel): when it takes an image, its bytes are zlib's; it refuses (and the
ingest decodes on one thread) what it cannot prove -- several members, damaged data, data
with no dynamic-Huffman block it can start from.  Streams with stored blocks (sync flushes,
incompressible stretches), fixed-Huffman blocks and every zlib level are covered, and the
ingest end to end (nw_fastq_read) on a file large enough to take the parallel path."""
import ctypes
import gzip
import os
import zlib

import numpy as np
import pytest

from crispresso_amd import _lib, fastq

THREADS = 8
MULTI = (os.cpu_count() or 1) >= 2


def _fastq_text(n, seed, amplicon_like=False):
    rng = np.random.Generator(np.random.PCG64(seed))
    amp = "".join(rng.choice(list("ACGT"), 250))
    out = []
    for r in range(n):
        if amplicon_like:
            s = amp if r % 3 else amp[: int(rng.integers(100, 250))] + "A" * int(rng.integers(0, 5))
            q = "I" * len(s)
        else:
            L = int(rng.integers(50, 300))
            s = "".join(rng.choice(list("ACGTN"), L))
            q = "".join(chr(33 + int(x)) for x in rng.integers(2, 41, L))
        out.append(f"@M0:{r}:FC:1 1:N:0\n{s}\n+\n{q}\n")
    return "".join(out).encode()


def _gzip(data, level=6, flush_every=0):
    co = zlib.compressobj(level, zlib.DEFLATED, 31)
    parts = []
    step = flush_every or len(data)
    for lo in range(0, len(data), step):
        parts.append(co.compress(data[lo:lo + step]))
        if flush_every:
            parts.append(co.flush(zlib.Z_SYNC_FLUSH))
    parts.append(co.flush())
    return b"".join(parts)


def _gunzip(gz):
    lib = _lib.load()
    src = np.frombuffer(gz, np.uint8)
    need = ctypes.c_int64()
    rc = lib.nw_gunzip_parallel(_lib.ptr(src), len(src), THREADS, None, 0, ctypes.byref(need))
    if rc != _lib.NW_E_CAPACITY:
        return rc, None
    out = np.empty(need.value, np.uint8)
    rc = lib.nw_gunzip_parallel(_lib.ptr(src), len(src), THREADS, _lib.ptr(out), len(out), ctypes.byref(need))
    return rc, out.tobytes()


@pytest.fixture(scope="module")
def text():
    return _fastq_text(60_000, 1)


@pytest.mark.parametrize("level", [1, 6, 9])
def test_levels(text, level):
    gz = _gzip(text, level)
    assert len(gz) >= 4 << 20
    rc, out = _gunzip(gz)
    if MULTI:
        assert rc == _lib.NW_OK
    if rc == _lib.NW_OK:
        assert out == text


def test_repetitive_amplicon_reads():
    """Amplicon-like reads with one quality: back-references reach to the first bytes of
    every range (the first pass's markers never run out)."""
    data = _fastq_text(400_000, 2, amplicon_like=True)
    gz = _gzip(data, 1)
    if len(gz) < 4 << 20:
        data = data * (((4 << 20) // len(gz)) + 1)
        gz = _gzip(data, 1)
    rc, out = _gunzip(gz)
    if MULTI:
        assert rc == _lib.NW_OK
    if rc == _lib.NW_OK:
        assert out == data


def test_stored_and_fixed_blocks(text):
    """Sync flushes every 20 kB (an empty stored block each, and short blocks zlib may code
    with the fixed table) and incompressible stretches (stored blocks) inside the text."""
    rng = np.random.Generator(np.random.PCG64(3))
    noise = [rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes() for _ in range(4)]
    q = len(text) // 5
    data = b"".join(text[k * q:(k + 1) * q] + (noise[k] if k < 4 else b"") for k in range(5))
    gz = _gzip(data, 6, flush_every=20_000)
    rc, out = _gunzip(gz)
    if MULTI:
        assert rc == _lib.NW_OK
    if rc == _lib.NW_OK:
        assert out == data


def test_refuses_what_it_cannot_prove(text):
    gz = _gzip(text, 1)
    bad = bytearray(gz)
    bad[len(bad) // 2] ^= 0x55   # damaged in the middle
    assert _gunzip(bytes(bad))[0] != _lib.NW_OK
    crc = bytearray(gz)
    crc[-6] ^= 1                  # a wrong CRC-32
    assert _gunzip(bytes(crc))[0] != _lib.NW_OK
    two = gz + _gzip(text[:1000], 1)   # two members
    assert _gunzip(two)[0] == _lib.NW_E_UNSUPPORTED
    rng = np.random.Generator(np.random.PCG64(4))
    binary = rng.integers(0, 256, 6 << 20, dtype=np.uint8).tobytes()
    assert _gunzip(_gzip(binary, 6))[0] == _lib.NW_E_UNSUPPORTED   # no text blocks to start from
    assert _gunzip(gzip.compress(text[:100_000]))[0] == _lib.NW_E_UNSUPPORTED   # small: one thread


def test_ingest_through_parallel_path(tmp_path, text):
    p = tmp_path / "big.fastq.gz"
    gz = _gzip(text, 1)
    p.write_bytes(gz)
    n1, b1, o1 = fastq.read_fastq_as_fasta(str(p))
    n2, b2, o2 = fastq.read_fastq_as_fasta_py(str(p))
    assert n1 == n2 and np.array_equal(o1, o2) and np.array_equal(b1, b2)
    assert len(n1) == 60_000
