"""nw_expand_ops on the host (no GPU): runs derived from the oracle's alignments
expand to the oracle's three rows, byte for byte; malformed runs are refused."""
import numpy as np

from crispresso_amd import _lib, synth
from crispresso_amd.aligner import OpsBatch, pack_reads


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


def test_expand_matches_oracle_rows(oracle):
    amp = synth.random_amplicon(250, 1)
    buf, off = synth.reads_from(amp, 1500, 3, synth.PARITY_MIX)
    reads = [r.replace("-", "") for r in synth.unpack(buf, off)]
    reads += ["", amp.lower(), amp[:50] + "RYKMNN" + amp[50:], "acgtNNNNtttgacca"]
    buf, off = pack_reads(reads)
    res, aln = oracle.align_batch(amp, buf, off, nthreads=8)
    n = len(off) - 1
    ops, ops_off = [], [0]
    for i in range(n):
        L = int(res["aln_len"][i])
        if off[i + 1] > off[i]:
            ops += runs_from_rows(aln[i, 0, :L].tobytes(), aln[i, 2, :L].tobytes())
        ops_off.append(len(ops))
    stats = np.zeros(n, dtype=_lib.STAT_DTYPE)
    for f in ("aln_len", "n_ident", "n_sim", "n_gaps", "score", "end_i", "end_j"):
        stats[f] = res[f]
    ob = OpsBatch(stats, np.array(ops, np.uint32), np.array(ops_off, np.int64), np.diff(off), 2)
    for nt in (1, 4):
        rows = ob.expand(amp, buf, off, nthreads=nt)
        for i in range(n):
            L = int(res["aln_len"][i])
            if off[i + 1] > off[i]:
                assert rows.aln[i, :, :L].tobytes() == aln[i, :, :L].tobytes(), i


def test_expand_rejects_runs_that_do_not_cover_the_read():
    lib = _lib.load()
    amp = b"ACGTACGT"
    buf, off = pack_reads(["ACGTACGT"])
    rows = np.zeros((1, 3, 32), np.uint8)
    for bad in ([(0 << 28) | 7], [(0 << 28) | 9], [(1 << 28) | 8], [(3 << 28) | 8]):
        ops = np.array(bad, np.uint32)
        oo = np.array([0, len(bad)], np.int64)
        assert lib.nw_expand_ops(amp, 8, _lib.ptr(buf), _lib.ptr(off), 1, _lib.ptr(ops), _lib.ptr(oo),
                                 _lib.ptr(rows), 32, 1) == _lib.NW_E_INVALID
    ops = np.array([(0 << 28) | 8], np.uint32)
    oo = np.array([0, 1], np.int64)
    assert lib.nw_expand_ops(amp, 8, _lib.ptr(buf), _lib.ptr(off), 1, _lib.ptr(ops), _lib.ptr(oo),
                             _lib.ptr(rows), 32, 1) == _lib.NW_OK
    assert rows[0, 1, :8].tobytes() == b"||||||||"


def test_pack_2bit_codes_and_exceptions():
    """nw_pack_reads: A C T G = 0 1 2 3 (case folded), everything else an exception with
    its byte, positions ascending; offsets need not start at 0; any thread count."""
    from crispresso_amd.aligner import pack_2bit

    rng = np.random.Generator(np.random.PCG64(3))
    alphabet = np.frombuffer(b"ACGTacgtNnRU-y", np.uint8)
    p = np.array([0.2, 0.2, 0.2, 0.2, 0.04, 0.04, 0.04, 0.04, 0.01, 0.01, 0.01, 0.01, 0.01, 0.01])
    for n, start in ((1, 0), (7, 3), (5000, 13)):
        lens = rng.integers(0, 300, n)
        off = np.zeros(n + 1, np.int64)
        off[0] = start
        off[1:] = start + np.cumsum(lens)
        buf = np.zeros(int(off[-1]) + 8, np.uint8)
        buf[start:off[-1]] = rng.choice(alphabet, int(off[-1] - start), p=p / p.sum())
        for nt in (1, 3, 0):
            pr = pack_2bit(buf, off, nthreads=nt)
            seg = buf[start:off[-1]]
            fold = seg & 0xDF
            acgt = np.isin(fold, np.frombuffer(b"ACGT", np.uint8))
            want_pos = np.flatnonzero(~acgt) + start
            assert np.array_equal(pr.exc_pos, want_pos)
            assert np.array_equal(pr.exc_byte, seg[~acgt])
            pos = np.arange(start, off[-1])
            codes = (pr.packed[pos // 4] >> (2 * (pos % 4))) & 3
            assert np.array_equal(codes[acgt], ((seg >> 1) & 3)[acgt])
