"""Every read of the benchmark workloads against the CPU oracle, through the exact paths
bench.py times (not a sample): the alignment of CRISPRessoCORE.py:1797-1806 (forward
pass) and 1812-1828 (HDR pass).

* C2: the headline's 1M-read batch (seed 2) through nw_align_ops_packed_lens (2-bit
  reads + lengths in, records + runs out);
* C3: the C3 reads against the amplicon (the same packed call) and, still resident in
  HBM, against the HDR amplicon (nw_align_ops_resident, with runs and records-only); and
  both passes of the dual call (nw_align_dual_ops_packed_lens, the bench's C3 step);
* C5: 96 amplicons x 10k reads in one nw_align_multi_ops_packed_lens call;
* C4: a 1M-read slice of the C4 generator (native, seed 10: rank 0's shard).

Every read's record (length, identity, similarity, gaps, score, start cell, flags) and
the three rows expanded from its runs equal the oracle's (tests/every_read.py: the
oracle runs once per distinct read; duplicates must carry the same GPU output).  These
cover round 3's certificate paths (one- and two-substitution reads finished in
classify, the walk's single-diagonal and plain-read records, the
128-diagonal wide level) on the workloads that exercise them.
"""
import os

import numpy as np
import pytest

from crispresso_amd import _lib, synth
from crispresso_amd.aligner import GpuAligner, pack_2bit
from tests.every_read import every_read, every_read_multi, every_read_records

pytestmark = pytest.mark.gpu

AMPLICON_LEN = 250          # bench.AMPLICON_LEN
READS = 1_000_000           # bench.READS_PER_GPU
THREADS = min(16, os.cpu_count() or 1)


def _pinned_out(n):
    bufs = (_lib.PinnedBuffer(n, _lib.STAT_DTYPE), _lib.PinnedBuffer(4 * n + 4096, np.uint32),
            _lib.PinnedBuffer(n + 1, np.int64))
    return bufs, tuple(b.array for b in bufs)


def _packed(buf, off):
    pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
    pp = _lib.PinnedBuffer((int(off[-1]) + 3) // 4 + 16, np.uint8)
    pl = _lib.PinnedBuffer(max(len(off) - 1, 1), np.uint16)
    pr = pack_2bit(pb.array, po.array, packed=pp.array, lens=pl.array)
    assert pr.lens is not None   # the lengths path (nw_align_ops_packed_lens), as in the bench
    return pr, (pb, po, pp, pl)


def _close(*groups):
    for g in groups:
        for b in g:
            b.close()


@pytest.fixture(scope="module")
def al():
    a = GpuAligner(0)
    yield a
    a.close()


def _assert_clean(res, what):
    assert res["mismatches"] == 0, f"{what}: {res}"
    assert res["reads"] > 0


def test_c2_every_read(al):
    amp = synth.random_amplicon(AMPLICON_LEN, 1)
    buf, off = synth.reads_from(amp, READS, 2)
    pr, keep = _packed(buf, off)
    outs, out = _pinned_out(len(off) - 1)
    al.set_reference(amp)
    ob = al.align_ops_packed(pr, out=out)
    counts = al.path_counts()
    res = every_read(amp, buf, off, ob, THREADS)
    _assert_clean(res, "C2")
    # the batch exercises the certificate paths this test is for
    assert counts["exact_copies"] > 700_000 and counts["band16"] > 0 and counts["band_fallback"] > 0
    _close(keep, outs)


def test_first_level_skip_every_read(al, monkeypatch):
    """KernelArgs::l1_skip (round 6): a launch of >= 65536 reads whose sort finds few DP reads sends
    them all to the wide level, past the 16-diagonal level.  A 200k-read C2-shaped batch as one resident
    pass (one launch: the skip) and as the pipelined call (its chunks take the skip too), every read
    against the oracle, and against the same reads with the skip off (CRISPR_NW_L1SKIP=0)."""
    amp = synth.random_amplicon(AMPLICON_LEN, 1)
    buf, off = synth.reads_from(amp, 200_000, 21)
    pr, keep = _packed(buf, off)
    n = len(off) - 1
    outs1, out1 = _pinned_out(n)
    outs2, out2 = _pinned_out(n)
    al.set_reference(amp)
    ob = al.align_ops_packed(pr, out=out1)
    _assert_clean(every_read(amp, buf, off, ob, THREADS), "call, first level skipped")
    res = al.align_ops(None, pr.offsets, out=out2, resident=True)
    c = al.path_counts()
    assert every_read_records(res.stats, ob.stats) == 0 and np.array_equal(res.ops_off, ob.ops_off)
    assert np.array_equal(res.ops[:int(res.ops_off[n])], ob.ops[:int(ob.ops_off[n])])
    monkeypatch.setenv("CRISPR_NW_L1SKIP", "0")
    res0 = al.align_ops(None, pr.offsets, out=out2, resident=True)
    c0 = al.path_counts()
    # with the skip the chunks' DP reads went to the wide level; without it the first level certified most
    assert c["band16"] == c0["band16"] > 0 and c["band_fallback"] > 2 * c0["band_fallback"]
    assert every_read_records(res0.stats, ob.stats) == 0 and np.array_equal(res0.ops_off, ob.ops_off)
    assert np.array_equal(res0.ops[:int(res0.ops_off[n])], ob.ops[:int(ob.ops_off[n])])
    _close(keep, outs1, outs2)


def test_c3_both_passes_every_read(al):
    amp, hdr, buf, off = synth.c3_workload(READS)
    pr, keep = _packed(buf, off)
    n = len(off) - 1
    outs1, out1 = _pinned_out(n)
    outs2, out2 = _pinned_out(n)
    outs3, out3 = _pinned_out(n)
    al.set_reference(amp)
    al.set_known(hdr)   # the bench's and align_reads' form: the HDR amplicon's copies from one alignment
    ob1 = al.align_ops_packed(pr, out=out1)
    al.set_known(None)
    _assert_clean(every_read(amp, buf, off, ob1, THREADS), "C3 amplicon pass (HDR copies known)")
    s1, oo1 = ob1.stats.copy(), ob1.ops_off.copy()
    al.set_reference(hdr)   # the reference amplicon's copies from one alignment (known copies)
    ob2 = al.align_ops(None, pr.offsets, out=out2, resident=True)
    _assert_clean(every_read(hdr, buf, off, ob2, THREADS), "C3 HDR pass (resident, runs)")
    # the bench's form of the HDR pass: records only, resident (right after the packed call)
    al.set_reference(amp)
    ob1b = al.align_ops_packed(pr, out=out1)   # no known sequence: the same records and runs
    assert every_read_records(ob1b.stats, s1) == 0 and np.array_equal(ob1b.ops_off, oo1)
    al.set_reference(hdr)
    ob3 = al.align_ops(None, pr.offsets, out=(out3[0], None, out3[2]), resident=True, records_only=True)
    assert every_read_records(ob3.stats, ob2.stats) == 0
    _close(keep, outs1, outs2, outs3)


def test_c3_dual_call_every_read(al):
    """The dual call (nw_align_dual_ops_packed_lens: one upload, the HDR pass's chunks interleaved
    with the amplicon pass's) against the oracle on every read of both passes, and its records-only
    form (the bench's C3 step) against the runs form."""
    amp, hdr, buf, off = synth.c3_workload(READS)
    pr, keep = _packed(buf, off)
    n = len(off) - 1
    outs1, out1 = _pinned_out(n)
    outs2, out2 = _pinned_out(n)
    outs3, out3 = _pinned_out(n)
    outs4, out4 = _pinned_out(n)
    al.set_reference(amp)
    ob1, ob2 = al.align_dual_packed(pr, hdr, out=out1, out2=out2)
    assert al.reference == amp
    _assert_clean(every_read(amp, buf, off, ob1, THREADS), "C3 dual call, amplicon pass")
    _assert_clean(every_read(hdr, buf, off, ob2, THREADS), "C3 dual call, HDR pass")
    ob3, ob4 = al.align_dual_packed(pr, hdr, out=out3, out2=(out4[0], None, out4[2]), records_only2=True)
    assert every_read_records(ob3.stats, ob1.stats) == 0 and np.array_equal(ob3.ops_off, ob1.ops_off)
    assert np.array_equal(ob3.ops, ob1.ops)
    assert every_read_records(ob4.stats, ob2.stats) == 0 and np.array_equal(ob4.ops_off, ob2.ops_off)
    assert not ob4.has_runs
    _close(keep, outs1, outs2, outs3, outs4)


def test_dual_call_small_and_odd_reads(al):
    """A one-chunk dual call with N bytes (exceptions of the packed stream) and reads that equal
    either amplicon: every read of both passes against the oracle."""
    amp, hdr, buf, off = synth.c3_workload(3000, seed=7)
    reads = [bytes(buf[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    reads[17] = reads[17][:40] + b"N" + reads[17][41:]
    reads[23] = reads[23][:100] + b"NN" + reads[23][102:]
    reads[31] = amp.encode()
    reads[37] = hdr.encode()
    lens = np.array([len(r) for r in reads], np.int64)
    off2 = np.zeros(len(reads) + 1, np.int64)
    np.cumsum(lens, out=off2[1:])
    buf2 = np.frombuffer(b"".join(reads), np.uint8).copy()
    pr, keep = _packed(buf2, off2)
    outs1, out1 = _pinned_out(len(reads))
    outs2, out2 = _pinned_out(len(reads))
    al.set_reference(amp)
    ob1, ob2 = al.align_dual_packed(pr, hdr, out=out1, out2=out2)
    _assert_clean(every_read(amp, buf2, off2, ob1, THREADS), "dual call (small), amplicon pass")
    _assert_clean(every_read(hdr, buf2, off2, ob2, THREADS), "dual call (small), HDR pass")
    _close(keep, outs1, outs2)


def test_c5_pooled_every_read(al):
    from bench import pooled_workload

    amps, buf, off, which = pooled_workload(96, 10_000)
    pr, keep = _packed(buf, off)
    pw = _lib.pinned_copy(which)
    outs, out = _pinned_out(len(off) - 1)
    ob = al.align_multi_ops(amps, pr, None, pw.array, out=out)
    res = every_read_multi(amps, buf, off, which, ob, THREADS)
    _assert_clean(res, "C5")
    _close(keep, outs, (pw,))


def test_c4_slice_every_read(al):
    amp = synth.random_amplicon(AMPLICON_LEN, 1)
    buf, off = synth.native_reads(amp, READS, 10)
    pr, keep = _packed(buf, off)
    outs, out = _pinned_out(len(off) - 1)
    al.set_reference(amp)
    ob = al.align_ops_packed(pr, out=out)
    _assert_clean(every_read(amp, buf, off, ob, THREADS), "C4 slice (seed 10)")
    _close(keep, outs)


def test_c1_shape_every_read(al):
    """The reference's own read shape (151 bp reads, 280 bp amplicon: tests/crispresso_tests.py:145-155)
    at the offsets bench.py's c1_shape leg uses (synth.c1_shape_workload), 200k reads: the window
    certificates and the seeded band (its reads through the wide level's band centred on their 16-mer
    hits, certified per read) against the oracle on every read."""
    amp, buf, off = synth.c1_shape_workload(200_000)
    pr, keep = _packed(buf, off)
    outs, out = _pinned_out(len(off) - 1)
    al.set_reference(amp)
    ob = al.align_ops_packed(pr, out=out)
    counts = al.path_counts()
    _assert_clean(every_read(amp, buf, off, ob, THREADS), "C1 shape")
    # the seeded band takes most reads no window certificate took: the second level
    # (32 diagonals centred on the hits) certifies most of them, the wide level most of the rest
    # (the refined certificate: insertions too), very few reach the exact kernel
    dp = len(off) - 1 - counts["exact_copies"]
    assert counts["band32"] > 0.5 * dp and counts["exact_kernel"] < 0.01 * dp, counts
    assert counts["band32"] + counts["wide128"] > 0.8 * dp, counts
    _close(keep, outs)
