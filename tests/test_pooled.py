"""Pooled amplicons (crispresso_amd.pooled): host plumbing on CPU with the oracle-backed aligner."""
import numpy as np

from crispresso_amd import synth
from crispresso_amd.pooled import align_pooled
from tests.helpers import OracleAligner, oracle_batch


def _pooled_case(seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    amps = [synth.random_amplicon(int(L), seed * 31 + g) for g, L in enumerate(rng.integers(150, 301, 5))]
    reads = []
    for g, a in enumerate(amps):
        k = int(rng.integers(0, 40)) if g != 2 else 0          # one amplicon without reads
        buf, off = synth.reads_from(a, k, seed * 7 + g, synth.PARITY_MIX) if k else (np.zeros(0, np.uint8),
                                                                                   np.zeros(1, np.int64))
        reads.append((buf, off))
    return amps, reads


def test_pooled_matches_per_amplicon_oracle():
    amps, reads = _pooled_case(3)
    got = align_pooled(amps, reads, OracleAligner())
    for g, (a, (buf, off)) in enumerate(zip(amps, reads)):
        want = oracle_batch(a, buf, off)
        assert len(got[g]) == len(off) - 1
        assert np.array_equal(got[g].stats, want.stats)
        for i in range(len(want)):
            L = int(want.stats["aln_len"][i])
            assert np.array_equal(got[g].aln[i, :, :L], want.aln[i, :, :L])


def test_pooled_accepts_string_lists():
    amps = [synth.random_amplicon(120, 1), synth.random_amplicon(200, 2)]
    reads = [[amps[0][10:100], amps[0]], [amps[1][:150]]]
    got = align_pooled(amps, reads, OracleAligner())
    assert [len(b) for b in got] == [2, 1]
    assert got[1].ref_seq(0).replace("-", "") == amps[1]
