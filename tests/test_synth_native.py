"""The native synthetic read generator (include/crispr_synth.h) and the pinned output pool's
lease logic (no GPU: a fake allocator stands in for hipHostMalloc)."""
import gc

import numpy as np

from crispresso_amd import _lib, synth


def test_native_reads_mix_and_determinism():
    amp = synth.random_amplicon(250, 1)
    buf, off = synth.native_reads(amp, 200_000, 10)
    lens = np.diff(off)
    assert (lens >= 220).all() and (lens <= 260).all()
    seqs = [bytes(buf[off[i]:off[i + 1]]) for i in range(0, 200_000, 7)]
    exact = np.mean([s == amp.encode() for s in seqs])
    assert abs(exact - 0.60) < 0.01
    assert abs(np.mean(lens < 250) - 0.10) < 0.01 and abs(np.mean(lens > 250) - 0.05) < 0.01
    assert set(np.unique(buf).tolist()) <= set(b"ACGT")
    b2, o2 = synth.native_reads(amp, 200_000, 10)
    assert np.array_equal(buf, b2) and np.array_equal(off, o2)
    b3, o3 = synth.native_reads(amp, 1000, 11)
    assert not np.array_equal(b3[:50000], buf[:len(b3[:50000])])


def test_native_reads_ranges_are_independent():
    amp = synth.random_amplicon(180, 3)
    buf, off = synth.native_reads(amp, 5000, 7)
    for first, n in ((0, 1), (1234, 2000), (4999, 1)):
        b, o = synth.native_reads(amp, n, 7, first=first)
        assert np.array_equal(b, buf[off[first]:off[first + n]])
        assert np.array_equal(np.diff(o), np.diff(off)[first:first + n])
    assert np.array_equal(synth.native_offsets(amp, 5000, 7), off)


class _FakePinned:
    def __init__(self, n, dt):
        self.mem = np.zeros(n, np.uint8)
        self._p = self.mem.ctypes.data

    def close(self):
        self.mem = None


def test_pinned_pool_leases(monkeypatch):
    monkeypatch.setattr(_lib, "PinnedBuffer", _FakePinned)
    pool = _lib.PinnedPool(keep_bytes=1 << 20)
    a = pool.array(1000, np.int64)
    a[:] = 7
    addr = a.ctypes.data
    b = pool.array((10, 3), np.int32)
    assert b.shape == (10, 3) and pool.free_bytes() == 0
    v = a[10:20]
    del a
    gc.collect()
    assert pool.free_bytes() == 0        # a view keeps the block leased
    del v
    gc.collect()
    assert pool.free_bytes() >= 8000
    c = pool.array(900, np.int64)
    assert c.ctypes.data == addr         # reused
    big = pool.array(1 << 19, np.uint8)
    del big, c, b
    gc.collect()
    assert pool.free_bytes() <= 1 << 20  # past keep_bytes the biggest free blocks are dropped
