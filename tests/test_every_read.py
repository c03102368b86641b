"""CPU test of the every-read checker (tests/every_read.py) itself: an oracle-made ops
batch passes; a changed record, a changed run of a duplicate read and a changed run of
a distinct read are each caught."""
import numpy as np

from crispresso_amd import synth
from tests.every_read import every_read, every_read_multi, first_occurrence
from tests.helpers import OracleAligner


def _batch(n=600, seed=5):
    amp = synth.random_amplicon(120, seed)
    buf, off = synth.reads_from(amp, n, seed, synth.PARITY_MIX)
    al = OracleAligner()
    al.set_reference(amp)
    return amp, buf, off, al.align_ops(buf, off)


def test_first_occurrence():
    amp = "ACGT"
    buf = np.frombuffer(b"ACGTACGTAC", np.uint8)
    off = np.array([0, 4, 8, 8, 10, 10], np.int64)
    assert first_occurrence(buf, off).tolist() == [0, 0, 2, 3, 2]
    del amp


def test_clean_batch_passes():
    amp, buf, off, ob = _batch()
    res = every_read(amp, buf, off, ob, threads=4)
    assert res["mismatches"] == 0 and res["reads"] == 600 and res["distinct"] < 600


def test_changes_are_caught():
    amp, buf, off, ob = _batch()
    rep = first_occurrence(buf, off)
    dup = int(np.flatnonzero((rep != np.arange(len(rep))) & (np.diff(ob.ops_off) > 0))[0])
    uniq = int(np.flatnonzero((rep == np.arange(len(rep))) & (np.diff(ob.ops_off) > 1))[0])
    # a record of a duplicate
    s = ob.stats.copy()
    s["score"][dup] += 1
    ob.stats, keep = s, ob.stats
    res = every_read(amp, buf, off, ob, threads=4)
    assert dup in res["first_bad"] and res["mismatches"] == 1
    ob.stats = keep
    # a run of a duplicate (same length: only the run compare sees it)
    ops = ob.ops.copy()
    ops[ob.ops_off[dup]] ^= 1 << 28
    ob.ops, keep = ops, ob.ops
    res = every_read(amp, buf, off, ob, threads=4)
    assert res["first_bad"] == [dup]
    ob.ops = keep
    # a run of a distinct read: the oracle compare sees it, and its duplicates fail with it
    ops = ob.ops.copy()
    a, b = ob.ops_off[uniq], ob.ops_off[uniq + 1]
    ops[a:b] = ops[a:b][::-1]
    ob.ops = ops
    res = every_read(amp, buf, off, ob, threads=4)
    assert uniq in res["first_bad"] and res["mismatches"] == int((rep == uniq).sum())


def test_multi():
    amps = [synth.random_amplicon(100, 7), synth.random_amplicon(140, 8)]
    parts = [synth.reads_from(a, 150, 9 + g, synth.PARITY_MIX) for g, a in enumerate(amps)]
    buf = np.concatenate([p[0] for p in parts])
    off = np.concatenate([[0], np.cumsum(np.concatenate([np.diff(p[1]) for p in parts]))]).astype(np.int64)
    which = np.repeat(np.arange(2, dtype=np.int32), 150)
    ob = OracleAligner().align_multi_ops(amps, buf, off, which)
    assert every_read_multi(amps, buf, off, which, ob, threads=4)["mismatches"] == 0
    ob.stats["n_ident"][200] += 1
    res = every_read_multi(amps, buf, off, which, ob, threads=4)
    assert 200 in res["first_bad"]
