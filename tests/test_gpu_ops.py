"""GPU parity of the call-level ops path (nw_align_ops): records + traceback runs
cross PCIe, the rows are rebuilt on the host (nw_expand_ops).  Bit-exact against
the CPU oracle: chunk boundaries of the pipeline, slot spills, the device-resident
ops mode, pinned buffers, the capacity protocol and its errors."""
import numpy as np
import pytest

from crispresso_amd import _lib, synth
from crispresso_amd.aligner import NeedleError, pack_reads
from tests.test_gpu_parity import FIELDS, assert_same

pytestmark = pytest.mark.gpu


def _reads(amp, seed):
    buf0, off0 = synth.reads_from(amp, 1500, seed, synth.PARITY_MIX)
    reads = synth.unpack(buf0, off0)
    rng = np.random.Generator(np.random.PCG64(seed))
    # reads with many gap runs (slot spills), empty reads, junk, exact copies
    for k in range(40):
        r = list(amp)
        for _ in range(int(rng.integers(5, 40))):
            p = int(rng.integers(1, len(r) - 1))
            if rng.random() < 0.5:
                del r[p]
            else:
                r.insert(p, "ACGT"[int(rng.integers(0, 4))])
        reads.append("".join(r))
    reads += ["", amp, amp.lower(), synth.random_amplicon(250, seed + 5), amp[:10], "-" + amp[1:]]
    return reads


@pytest.mark.parametrize("chunk", ["1", "613", "100000"])
@pytest.mark.parametrize("slot", ["1", "3", "64"])
def test_align_ops_chunks_and_spills(gpu_aligner_factory, oracle, monkeypatch, chunk, slot):
    monkeypatch.setenv("CRISPR_NW_CHUNK", chunk if chunk != "1" else "257")
    monkeypatch.setenv("CRISPR_NW_OPS_SLOT", slot)
    amp = synth.random_amplicon(250, 61)
    buf, off = pack_reads(_reads(amp, 62))
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops(buf, off)
    assert ob.ops_off[0] == 0 and np.all(np.diff(ob.ops_off) >= 0)
    lens = np.diff(off)
    assert np.all((np.diff(ob.ops_off) == 0) == (lens == 0))
    assert_same(oracle, amp, buf, off, ob.expand(amp, buf, off), f"ops chunk={chunk} slot={slot}")
    t = a.ops_times()
    assert t["h2d_bytes"] >= int(off[-1]) and t["compute_ms"] > 0


def test_exact_copy_is_one_run(gpu_aligner_factory):
    amp = synth.random_amplicon(230, 3)
    buf, off = pack_reads([amp, amp.lower(), amp[:-1], ""])
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops(buf, off)
    assert ob.runs(0) == [(_lib.NW_RUN_M, 230)] and ob.runs(1) == [(_lib.NW_RUN_M, 230)]
    assert ob.runs(3) == []
    assert ob.stats["flags"][3] & _lib.NW_FLAG_EMPTY


def test_ops_pinned_buffers_and_capacity(gpu_aligner_factory, oracle):
    """Pinned inputs/outputs (the bench's setup); an ops buffer that is too small
    returns NW_E_CAPACITY with the size needed in ops_off[n]."""
    amp = synth.random_amplicon(250, 1)
    buf, off = synth.reads_from(amp, 5000, 2)
    n = len(off) - 1
    a = gpu_aligner_factory()
    a.set_reference(amp)
    pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
    stats = _lib.PinnedBuffer(n, _lib.STAT_DTYPE)
    ops_off = _lib.PinnedBuffer(n + 1, np.int64)
    small = np.empty(10, np.uint32)
    rc = a.lib.nw_align_ops(a._h, _lib.ptr(pb.array), _lib.ptr(po.array), n, _lib.ptr(small), len(small),
                            _lib.ptr(ops_off.array), _lib.ptr(stats.array))
    assert rc == _lib.NW_E_CAPACITY
    need = int(ops_off.array[n])
    assert need > 10
    ops = _lib.PinnedBuffer(need, np.uint32)
    ob = a.align_ops(pb.array, po.array, out=(stats.array, ops.array, ops_off.array))
    assert int(ob.ops_off[n]) == need
    assert_same(oracle, amp, buf, off, ob.expand(amp, buf, off), "pinned")
    for b in (pb, po, stats, ops_off, ops):
        b.close()


def test_spill_area_full_raises(gpu_aligner_factory, monkeypatch):
    monkeypatch.setenv("CRISPR_NW_OPS_SLOT", "1")
    monkeypatch.setenv("CRISPR_NW_SPILL_WORDS", "8")
    amp = synth.random_amplicon(250, 61)
    buf, off = pack_reads(_reads(amp, 63))
    a = gpu_aligner_factory()
    a.set_reference(amp)
    with pytest.raises(NeedleError, match="spill area full"):
        a.align_ops(buf, off)
    monkeypatch.delenv("CRISPR_NW_SPILL_WORDS")
    monkeypatch.delenv("CRISPR_NW_OPS_SLOT")
    a.align_ops(buf, off)   # the context recovers


def test_device_resident_ops_mode(gpu_aligner_factory, oracle):
    """nw_batch_set_output(NW_OUT_OPS) + upload/run/download_ops: the bench's
    kernel-resident pass is the same kernels + compaction as the call."""
    amp = synth.random_amplicon(250, 1)
    buf, off = pack_reads(_reads(amp, 64))
    a = gpu_aligner_factory()
    a.set_reference(amp)
    a.set_output("ops")
    a.upload(buf, off)
    for _ in range(2):
        a.run_async()
        assert a.sync() > 0
    ob = a.download_ops(len(off) - 1)
    assert_same(oracle, amp, buf, off, ob.expand(amp, buf, off), "resident-ops")
    with pytest.raises(NeedleError):
        a.download(len(off) - 1, 300)           # rows are not produced in ops mode
    a.set_output("rows")
    a.upload(buf, off)
    a.run_async()
    a.sync()
    rows = a.download(len(off) - 1, int(np.diff(off).max()))
    for f in FIELDS:
        assert np.array_equal(rows.stats[f], ob.stats[f])


def test_rows_api_unaffected_by_ops_mode(gpu_aligner_factory, oracle):
    """nw_align_batch / nw_align_multi always produce rows, whatever the upload mode."""
    amp = synth.random_amplicon(200, 5)
    buf, off = synth.reads_from(amp, 700, 6, synth.PARITY_MIX)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    a.set_output("ops")
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off, mode="rows"), "rows-after-ops")


def test_resident_second_pass_hdr(gpu_aligner_factory, oracle):
    """The HDR pass over the same reads (nw_align_ops_resident): no upload, records
    equal to a fresh call against the HDR amplicon; a different batch is refused."""
    from crispresso_amd import synth as sy

    amp, hdr, buf, off = sy.c3_workload(3000)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    first = a.align_ops(buf, off)
    assert_same(oracle, amp, buf, off, first.expand(amp, buf, off), "c3-amp")
    a.set_reference(hdr)
    again = a.align_ops(None, off, resident=True)
    assert a.ops_times()["h2d_bytes"] == 0
    assert_same(oracle, hdr, buf, off, again.expand(hdr, buf, off), "c3-hdr-resident")
    rec = a.align_ops(None, off, resident=True, records_only=True)
    for f in FIELDS:
        assert np.array_equal(rec.stats[f], again.stats[f])
    with pytest.raises(NeedleError):
        a.align_ops(None, off[:101], resident=True)


@pytest.mark.parametrize("grouped", [True, False])
def test_multi_ops_96_amplicons(gpu_aligner_factory, oracle, grouped):
    """nw_align_multi_ops on the C5 shape scaled down: 96 amplicons of 150-300 bp,
    ~50 reads each (some empty groups, one group over a chunk boundary), grouped or
    interleaved read order; every read bit-exact against the oracle with its amplicon."""
    from crispresso_amd import synth as sy

    amps = sy.pooled_amplicons(96, 5)
    rng = np.random.Generator(np.random.PCG64(96))
    bufs, offs, which = [], [], []
    for g, amp in enumerate(amps):
        k = 0 if g % 31 == 7 else (400 if g == 50 else int(rng.integers(20, 80)))
        if k:
            b, o = sy.reads_from(amp, k, 1000 + g, sy.PARITY_MIX)
            bufs.append(b)
            offs.append(o)
            which += [g] * k
    reads = []
    for b, o in zip(bufs, offs):
        reads += sy.unpack(b, o)
    which = np.array(which, np.int32)
    if not grouped:
        perm = rng.permutation(len(reads))
        reads = [reads[i] for i in perm]
        which = which[perm]
    buf, off = pack_reads(reads)
    import os
    os.environ["CRISPR_NW_CHUNK"] = "300"
    try:
        a = gpu_aligner_factory()
        ob = a.align_multi_ops(amps, buf, off, which)
        # the same batch 2-bit packed (nw_align_multi_ops_packed): grouped reads only
        from crispresso_amd.aligner import pack_2bit
        pr = pack_2bit(buf, off)
        if grouped:
            assert pr.lens is not None
            for lens in (pr.lens, None):   # nw_align_multi_ops_packed_lens, then nw_align_multi_ops_packed
                pr.lens = lens
                pk = a.align_multi_ops(amps, pr, None, which)
                for f in FIELDS + ("flags",):
                    assert np.array_equal(pk.stats[f], ob.stats[f])
                assert np.array_equal(pk.ops, ob.ops) and np.array_equal(pk.ops_off, ob.ops_off)
        else:
            with pytest.raises(NeedleError):
                a.align_multi_ops(amps, pr, None, which)
    finally:
        del os.environ["CRISPR_NW_CHUNK"]
    assert a.reference is None
    for g, amp in enumerate(amps):
        sel = np.flatnonzero(which == g)
        if not len(sel):
            continue
        gb, go = pack_reads([reads[i] for i in sel])
        runs = [ob.ops[ob.ops_off[i]:ob.ops_off[i + 1]] for i in sel]
        goo = np.zeros(len(sel) + 1, np.int64)
        goo[1:] = np.cumsum([len(r) for r in runs])
        from crispresso_amd.aligner import OpsBatch
        sub = OpsBatch(ob.stats[sel], np.concatenate(runs), goo, np.diff(go), ob.scale)
        assert_same(oracle, amp, gb, go, sub.expand(amp, gb, go), f"multi g={g}")
    amp = amps[3]
    a.set_reference(amp)
    b, o = sy.reads_from(amp, 300, 7, sy.PARITY_MIX)
    assert_same(oracle, amp, b, o, a.align_packed(b, o), "after-multi-ops")


def test_multi_gpu_aligner_threads_on_one_device(oracle):
    """MultiGpuAligner with two contexts on device 0 (threads, shards in parallel):
    single-amplicon and pooled (cell-count partition) results equal one context's."""
    from crispresso_amd import synth as sy
    from crispresso_amd.aligner import GpuAligner
    from crispresso_amd.distributed import MultiGpuAligner

    amp = sy.random_amplicon(250, 1)
    buf, off = sy.reads_from(amp, 5001, 2, sy.PARITY_MIX)
    multi = MultiGpuAligner([0, 0])
    multi.set_reference(amp)
    got = multi.align_ops(buf, off)
    assert_same(oracle, amp, buf, off, got.expand(amp, buf, off), "multi-threads")
    amps = sy.pooled_amplicons(12, 5)
    parts = [sy.reads_from(a, 200, 30 + g) for g, a in enumerate(amps)]
    reads = []
    for b, o in parts:
        reads += sy.unpack(b, o)
    which = np.repeat(np.arange(12, dtype=np.int32), 200)
    pbuf, poff = pack_reads(reads)
    one = GpuAligner(0)
    want = one.align_multi_ops(amps, pbuf, poff, which)
    got = multi.align_multi_ops(amps, pbuf, poff, which)
    for f in FIELDS:
        assert np.array_equal(got.stats[f], want.stats[f])
    assert np.array_equal(got.ops, want.ops) and np.array_equal(got.ops_off, want.ops_off)
    one.close()
    multi.close()


@pytest.mark.parametrize("lens", [True, False])
@pytest.mark.parametrize("chunk", ["97", "1500", "100000"])
def test_packed_input_parity(gpu_aligner_factory, oracle, monkeypatch, chunk, lens):
    """nw_align_ops_packed: 2-bit bases + exceptions (N, IUPAC, U, '-', lower case) give
    the same records and runs as the text path and the oracle; a batch whose offsets
    start mid-buffer; chunk edges inside packed bytes and inside 1024-read length groups
    (lens: nw_align_ops_packed_lens, the offsets rebuilt on the device); the resident
    second pass after it."""
    from crispresso_amd.aligner import pack_2bit

    monkeypatch.setenv("CRISPR_NW_CHUNK", chunk)
    amp = synth.random_amplicon(250, 61)
    reads = _reads(amp, 65)
    reads += ["acgtNNNNtttgacca", "T-C-A", "ACGTRYKMSWBDHVNU", amp.lower()[:77] + "u" + amp[78:], "n" * 30]
    full, foff = pack_reads(["PREFIX"] + reads)
    off = foff[1:]                       # offsets start at 6: the batch is a slice of a bigger buffer
    buf, off0 = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    pr = pack_2bit(full, off)
    assert pr.lens is not None and np.array_equal(pr.lens, np.diff(off))
    if not lens:
        pr.lens = None
    ob = a.align_ops_packed(pr)
    assert a.ops_times()["h2d_bytes"] < (int(off[-1]) - int(off[0])) // 2
    assert_same(oracle, amp, buf, off0, ob.expand(amp, full, off), f"packed chunk={chunk}")
    text = a.align_ops(buf, off0)
    for f in FIELDS + ("flags",):
        assert np.array_equal(ob.stats[f], text.stats[f])
    assert np.array_equal(ob.ops, text.ops) and np.array_equal(ob.ops_off, text.ops_off)
    # resident pass after a packed upload
    a.align_ops_packed(pr)
    hdr = synth.hdr_amplicon(amp, 4)
    a.set_reference(hdr)
    again = a.align_ops(None, off, resident=True)
    assert_same(oracle, hdr, buf, off0, again.expand(hdr, full, off), "packed-resident")


def test_packed_lens_must_match_offsets(gpu_aligner_factory, oracle):
    """nw_align_ops_packed_lens checks every length against its offsets before any kernel
    runs: a mismatch is NW_E_INVALID (also one that keeps its 1024-read group's sum), and the
    context still works."""
    from crispresso_amd.aligner import NeedleError, pack_2bit

    amp = synth.random_amplicon(200, 71)
    buf, off = synth.reads_from(amp, 5000, 72)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    pr = pack_2bit(buf, off)
    pr.lens = pr.lens.copy()
    pr.lens[3000] += 1
    with pytest.raises(NeedleError, match="lens differ from the offsets"):
        a.align_ops_packed(pr)
    pr.lens[3001] -= 1   # same group sum, two wrong lengths
    with pytest.raises(NeedleError, match="lens differ from the offsets"):
        a.align_ops_packed(pr)
    pr.lens[3000] -= 1
    pr.lens[3001] += 1
    assert_same(oracle, amp, buf, off, a.align_ops_packed(pr).expand(amp, buf, off), "lens-after-error")


def test_adaptive_first_level_hdr_pass(gpu_aligner_factory, oracle, monkeypatch):
    """The HDR pass (most DP reads need the 32-diagonal level): after the first chunks
    the pipeline skips the 16-diagonal level; records and runs are unchanged (same as
    with both levels on every chunk, CRISPR_NW_ADAPT=0) and bit-identical to the oracle."""
    amp, hdr, buf, off = synth.c3_workload(24000)
    monkeypatch.setenv("CRISPR_NW_CHUNK", "2048")
    a = gpu_aligner_factory()
    a.set_reference(hdr)
    ob = a.align_ops(buf, off)
    paths = a.path_counts()
    assert paths["band32"] > paths["band16"] // 2   # the skipped chunks count their DP reads on level 2
    monkeypatch.setenv("CRISPR_NW_ADAPT", "0")
    both = a.align_ops(buf, off)
    for f in FIELDS + ("flags",):
        assert np.array_equal(ob.stats[f], both.stats[f])
    assert np.array_equal(ob.ops, both.ops) and np.array_equal(ob.ops_off, both.ops_off)
    sel = np.arange(0, len(off) - 1, 7)
    sb, so = pack_reads([bytes(buf[off[i]:off[i + 1]]).decode() for i in sel])
    runs = [ob.ops[ob.ops_off[i]:ob.ops_off[i + 1]] for i in sel]
    roff = np.zeros(len(sel) + 1, np.int64)
    roff[1:] = np.cumsum([len(r) for r in runs])
    from crispresso_amd.aligner import OpsBatch
    sub = OpsBatch(ob.stats[sel], np.concatenate(runs), roff, np.diff(so), ob.scale)
    assert_same(oracle, hdr, sb, so, sub.expand(hdr, sb, so), "adaptive-hdr")


def test_adaptive_levels_sorted_input(gpu_aligner_factory, monkeypatch):
    """Reads whose character changes part-way (synth.c3_workload puts the HDR reads last):
    the adaptive level choice, made from finished chunks, must not send the late chunks'
    second-level reads to the exact kernel (a rule that did measured 15 -> 24 ms per C3
    step)."""
    amp, _, buf, off = synth.c3_workload(100000)
    monkeypatch.setenv("CRISPR_NW_CHUNK", "16384")
    a = gpu_aligner_factory()
    a.set_reference(amp)
    a.align_ops(buf, off)
    paths = a.path_counts()
    assert paths["band32"] > 5000                       # the HDR reads took the second level
    # the exact kernel: the rare uncertified reads, plus the few (~0.3 %) first-level
    # give-ups of the reference-like chunks (KernelArgs::redo_direct); the HDR chunks'
    # tens of thousands stay on the second level
    assert paths["exact_kernel"] < 0.01 * (len(off) - 1)



def test_set_params_endweight_through_ctypes(oracle):
    """The ABI contract of include/crispr_nw.h for -endweight: nw_set_params(end_weight=1,
    end_open, end_extend) called straight through ctypes returns NW_OK, and an alignment
    with a leading overhang then pays the end gap as the oracle's restatement
     says -- not the free-end-gap answer."""
    import ctypes

    from crispresso_amd import _lib

    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.nw_create(0, ctypes.byref(h)) == _lib.NW_OK
    try:
        assert lib.nw_set_params(h, 10.0, 0.5, 1, 3.0, 1.0, b"EDNAFULL", _lib.NW_TIE_EMBOSS) == _lib.NW_OK
        assert lib.nw_score_scale(h) == 2
        # an end penalty not on the 1/16 grid is refused, as the header says
        assert lib.nw_set_params(h, 10.0, 0.5, 1, 0.03, 1.0, b"EDNAFULL", _lib.NW_TIE_EMBOSS) == _lib.NW_E_INEXACT
        assert lib.nw_set_params(h, 10.0, 0.5, 1, 3.0, 1.0, b"EDNAFULL", _lib.NW_TIE_EMBOSS) == _lib.NW_OK
        amp = synth.random_amplicon(200, 808)
        reads = [amp[40:], amp[:150] + "ACGT", amp]
        buf, off = pack_reads(reads)
        assert lib.nw_set_reference(h, amp.encode(), len(amp)) == _lib.NW_OK
        stride = int(lib.nw_required_stride(h, int(np.diff(off).max())))
        stats = np.zeros(len(reads), _lib.STAT_DTYPE)
        aln = np.zeros((len(reads), 3, stride), np.uint8)
        assert lib.nw_align_batch(h, _lib.ptr(buf), _lib.ptr(off), len(reads), _lib.ptr(aln), stride,
                                  _lib.ptr(stats)) == _lib.NW_OK
        p = oracle.params(10.0, 0.5, True, 3.0, 1.0)
        res, want = oracle.align_batch(amp, buf, off, p, nthreads=1)
        for f in FIELDS:
            assert np.array_equal(stats[f], res[f]), f
        for i in range(len(reads)):
            L = int(res["aln_len"][i])
            assert aln[i, :, :L].tobytes() == want[i, :, :L].tobytes()
        free, _ = oracle.align_batch(amp, buf, off, oracle.params(10.0, 0.5), nthreads=1)
        assert stats["score"][0] != free["score"][0]   # the overhang's end gap is charged
    finally:
        lib.nw_destroy(h)


def test_multi_gpu_aligner_c4_and_pooled_vs_oracle(oracle):
    """MultiGpuAligner with two contexts on device 0 (one host thread each): a batch of the
    C4 generator (native, seed 10: bench's C4 shards) through the pinned 2-bit path and the
    resident HDR pass, and a 96-amplicon pooled batch split by DP cells -- every read's
    record and runs equal to the oracle's."""
    from crispresso_amd import synth as sy
    from crispresso_amd.aligner import OpsBatch, PackedReads, pack_2bit
    from crispresso_amd.distributed import MultiGpuAligner

    amp = sy.random_amplicon(250, 1)
    buf, off = sy.native_reads(amp, 20001, 10)
    multi = MultiGpuAligner([0, 0])
    try:
        multi.set_reference(amp)
        pr = pack_2bit(buf, off)
        got = multi.align_ops_packed(pr)
        assert_same(oracle, amp, buf, off, got.expand(amp, buf, off), "multi-c4")
        hdr = sy.hdr_amplicon(amp, 4)
        multi.set_reference(hdr)
        rec = multi.align_ops(None, off, resident=True, records_only=True)
        res, _ = oracle.align_batch(hdr, buf, off, nthreads=8)
        for f in FIELDS:
            assert np.array_equal(rec.stats[f], res[f]), f
        # pooled: 96 amplicons, ~60 reads each from the native generator, grouped by amplicon
        amps = sy.pooled_amplicons(96, 5)
        parts = [sy.native_reads(a, 40 + (g % 5) * 10, 100 + g) for g, a in enumerate(amps)]
        reads = []
        for b, o in parts:
            reads += sy.unpack(b, o)
        which = np.repeat(np.arange(96, dtype=np.int32), [len(o) - 1 for _, o in parts])
        pbuf, poff = pack_reads(reads)
        ob = multi.align_multi_ops(amps, pbuf, poff, which)
        assert multi.reference is None
        for g, a in enumerate(amps):
            sel = np.flatnonzero(which == g)
            gb, go = pack_reads([reads[i] for i in sel])
            runs = [ob.ops[ob.ops_off[i]:ob.ops_off[i + 1]] for i in sel]
            goo = np.zeros(len(sel) + 1, np.int64)
            goo[1:] = np.cumsum([len(r) for r in runs])
            sub = OpsBatch(ob.stats[sel], np.concatenate(runs), goo, np.diff(go), ob.scale)
            assert_same(oracle, a, gb, go, sub.expand(a, gb, go), f"multi-pooled g={g}")
        # a single-amplicon pass after the pooled call sets its amplicon again
        multi.set_reference(amp)
        again = multi.align_ops_packed(pr)
        assert np.array_equal(again.stats, got.stats) and np.array_equal(again.ops, got.ops)
    finally:
        multi.close()


def test_pinned_pool_outputs_are_reused_and_kept(gpu_aligner_factory, oracle):
    """Outputs leased from the pinned pool: a batch the caller keeps is never overwritten by
    the next call; a dropped one's block is reused."""
    import gc

    from crispresso_amd import _lib

    amp = synth.random_amplicon(250, 71)
    buf, off = synth.reads_from(amp, 3000, 72, synth.PARITY_MIX)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    first = a.align_ops(buf, off)
    keep = (first.stats.copy(), first.ops.copy(), first.ops_off.copy())
    buf2, off2 = synth.reads_from(amp, 3000, 73, synth.PARITY_MIX)
    second = a.align_ops(buf2, off2)
    assert first.stats.ctypes.data != second.stats.ctypes.data
    assert np.array_equal(first.stats, keep[0]) and np.array_equal(first.ops, keep[1])
    pool = _lib.pinned_pool()
    free0 = pool.free_bytes()
    del first
    gc.collect()
    freed = pool.free_bytes() - free0
    assert freed > 0                            # the dropped batch's blocks went back to the pool
    third = a.align_ops(buf, off)
    assert pool.free_bytes() <= free0 + freed - freed // 2   # ... and the next call leased from it
    assert np.array_equal(third.stats, keep[0]) and np.array_equal(third.ops_off, keep[2])
    assert_same(oracle, amp, buf2, off2, second.expand(amp, buf2, off2), "pool")


def test_outputs_fully_written_over_stale_memory(gpu_aligner_factory):
    """The pinned pool hands out blocks without zeroing them (aligner._outputs): every call
    must write every record and run offset itself (empty reads included).  Outputs filled
    with junk first give the same results as zeroed ones, for the text, packed, resident
    and records-only calls."""
    from crispresso_amd.aligner import pack_2bit

    amp = synth.random_amplicon(250, 81)
    buf, off = pack_reads(_reads(amp, 82))
    n = len(off) - 1

    def outs(fill):
        st = np.zeros(n, _lib.STAT_DTYPE)
        ops = np.zeros(4 * n + 4096, np.uint32)
        oo = np.zeros(n + 1, np.int64)
        for x in (st, ops, oo):
            x.view(np.uint8)[...] = fill
        return st, ops, oo

    a = gpu_aligner_factory()
    a.set_reference(amp)
    pr = pack_2bit(buf, off)
    for call in ("text", "packed", "resident", "records"):
        res = []
        for fill in (0, 0x5A):
            st, ops, oo = outs(fill)
            if call == "text":
                ob = a.align_ops(buf, off, out=(st, ops, oo))
            elif call == "packed":
                ob = a.align_ops_packed(pr, out=(st, ops, oo))
            else:
                a.align_ops(buf, off)
                ob = a.align_ops(None, off, out=(st, None if call == "records" else ops, oo), resident=True,
                                 records_only=call == "records")
            res.append((ob.stats.copy(), ob.ops_off.copy(), ob.ops.copy()))
        (s0, o0, r0), (s1, o1, r1) = res
        assert np.array_equal(s0, s1) and np.array_equal(o0, o1) and np.array_equal(r0, r1), call


def test_packed_batch_upload_runs_the_call_kernels(gpu_aligner_factory, oracle):
    """nw_batch_upload_packed: the resident pass over a packed batch (classify decodes the
    2-bit reads, rebuilds the offsets from the lengths, writes only the DP reads' bytes) gives
    the oracle's records and runs, run after run; nw_batch_device_ops then holds every read's
    bytes (the quantification reads them)."""
    from crispresso_amd.aligner import pack_2bit

    amp = synth.random_amplicon(250, 91)
    reads = _reads(amp, 92) + ["N" * 250, amp[:100] + "NNN" + amp[103:]]
    buf, off = pack_reads(reads)
    n = len(off) - 1
    # the batch mid-buffer (offsets not starting at 0 or a multiple of 16)
    full = np.concatenate([np.frombuffer(b"ACGTACG", np.uint8), buf])
    off7 = off + 7
    pr = pack_2bit(full, off7)
    assert len(pr.exc_pos) > 0 and pr.lens is not None
    a = gpu_aligner_factory()
    a.set_reference(amp)
    a.upload_packed(pr)
    for _ in range(2):
        a.run_async()
        a.sync()
        ob = a.download_ops(n)
        assert_same(oracle, amp, buf, off, ob.expand(amp, full, off7), "packed batch upload")
    from crispresso_amd.devmem import _D2H, hip

    dev = a.device_ops()
    got = np.zeros(int(off7[-1] - off7[0]), np.uint8)
    assert hip().hipMemcpy(got.ctypes.data, dev["reads"] + int(off7[0]) - dev["reads_bias"], got.nbytes, _D2H) == 0
    assert got.tobytes() == bytes(buf).upper()   # the kernels' bytes: upper case, every read


@pytest.mark.parametrize("kind", ["c2", "repeats"])
def test_lane_walk_resident_pass_matches_call_and_oracle(gpu_aligner_factory, oracle, kind):
    """A resident pass of 400k reads with the lane walk on (nw_batch_set_lane_walk: the first
    level's nw_band_walk<16, true> and its fill's stop summary), and one without (the call's own
    kernels in one launch each), give the same records and runs as the pipelined call over the
    same batch (the wave-per-read walk), every read; and every read of the lane-walk pass against
    the oracle.
    "repeats": homopolymer and tandem-repeat runs in the amplicon (gap placement among equal
    scores, "M < max" bits off the path) and the parity mix (more indels, N codes)."""
    from crispresso_amd.aligner import pack_2bit

    if kind == "c2":
        amp = synth.random_amplicon(250, 1)
        buf, off = synth.reads_from(amp, 400_000, 7)
    else:
        rnd = synth.random_amplicon(250, 3)
        amp = (rnd[:40] + "AAAAAAAA" + rnd[40:70] + "CAGCAGCAGCAGCAG" + rnd[70:120] + "TTTTTTGGGGGG" +
               rnd[120:160] + "ATATATATAT" + rnd[160:])[:250]
        buf, off = synth.reads_from(amp, 400_000, 8, synth.PARITY_MIX)
    n = len(off) - 1
    pr = pack_2bit(buf, off)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    call = a.align_ops_packed(pr)
    c_stats, c_off = call.stats.copy(), call.ops_off.copy()
    c_ops = call.ops[:int(c_off[n])].copy()
    a.upload_packed(pr)
    for lane_walk in (False, True):
        a.set_lane_walk(lane_walk)
        a.run_async()
        a.sync()
        res = a.download_ops(n)
        assert int(res.ops_off[n]) == int(c_off[n])
        np.testing.assert_array_equal(res.ops_off, c_off)
        for f in FIELDS:
            np.testing.assert_array_equal(res.stats[f], c_stats[f], err_msg=f)
        np.testing.assert_array_equal(res.ops[:int(c_off[n])], c_ops)
    a.set_lane_walk(False)
    # every read of the resident pass (the one the bench's roofline is quoted on) against the
    # oracle: once per distinct read, duplicates against their first copy (tests/every_read.py)
    from tests.every_read import every_read

    chk = every_read(amp, buf, off, res, threads=16)
    assert chk["mismatches"] == 0, chk


@pytest.mark.parametrize("hdr_kind", ["block", "one_sub", "two_sub", "longer"])
def test_known_copies_resident_pass(gpu_aligner_factory, hdr_kind):
    """The HDR pass's copies of the reference amplicon (known copies): a resident pass
    against a new amplicon takes the reads equal to the batch's previous amplicon (upper or lower
    case) from one exact-kernel alignment of it.  Every read against the oracle, for an HDR amplicon
    10 bases apart (the C3 shape), 1 and 2 substitutions apart (the classify certificates take those
    reads first) and of another length (no known copies)."""
    from crispresso_amd.aligner import pack_2bit
    from tests.every_read import every_read

    amp = synth.random_amplicon(250, 21)
    if hdr_kind == "block":
        hdr = synth.hdr_amplicon(amp, 4)
    elif hdr_kind == "one_sub":
        hdr = amp[:100] + ("A" if amp[100] != "A" else "C") + amp[101:]
    elif hdr_kind == "two_sub":
        hdr = amp[:60] + ("G" if amp[60] != "G" else "T") + amp[61:180] + ("A" if amp[180] != "A" else "C") + amp[181:]
    else:
        hdr = amp[:120] + "ACGTA" + amp[120:]
    rng = np.random.Generator(np.random.PCG64(22))
    b1, o1 = synth.reads_from(amp, 30000, 23, synth.PARITY_MIX)
    seqs = synth.unpack(b1, o1)
    for k in rng.choice(len(seqs), 3000, replace=False):   # lower-case copies of the amplicon
        seqs[k] = amp.lower() if k % 2 else amp[:50] + amp[50:].lower()
    b2, o2 = synth.reads_from(hdr, 5000, 24)
    seqs += synth.unpack(b2, o2)
    buf, off = pack_reads(seqs)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    pr = pack_2bit(buf, off)
    ob1 = a.align_ops_packed(pr)
    chk1 = every_read(amp, buf, off, ob1, threads=16)
    assert chk1["mismatches"] == 0, chk1
    a.set_reference(hdr)
    ob2 = a.align_ops(None, off, resident=True)
    chk2 = every_read(hdr, buf, off, ob2, threads=16)
    assert chk2["mismatches"] == 0, chk2
    # the records-only pass (the HDR pass CRISPResso runs, CORE:1740-1741) gives the same records
    ob3 = a.align_ops(None, off, resident=True, records_only=True)
    for f in FIELDS:
        np.testing.assert_array_equal(ob3.stats[f], ob2.stats[f], err_msg=f)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["hdr", "parity", "long_indels"])
def test_lane_walk_resident_pass_hard_inputs(gpu_aligner_factory, oracle, kind):
    """A resident pass with the first level's lane walk (the kernels bench.py times) against the same
    pass with the wave walk, every read, and every read against the oracle, on inputs that load the
    levels after the first: "hdr" (reads against the HDR amplicon: most DP reads need the second
    level, no direct hand-off), "parity" (N codes, IUPAC bytes: the wave path inside the lane walk),
    "long_indels" (length changes of >= 10 bases, four times over: the wide level)."""
    from crispresso_amd.aligner import pack_2bit
    from tests.every_read import every_read

    n = 200_000
    if kind == "hdr":
        amp, hdr, buf, off = synth.c3_workload(n)
        ref = hdr
    elif kind == "parity":
        ref = synth.random_amplicon(250, 11)
        buf, off = synth.reads_from(ref, n, 12, synth.PARITY_MIX)
    else:
        ref = synth.random_amplicon(250, 13)
        buf, off = synth.reads_from(ref, n, 14)
        lens = np.diff(off)
        idx = np.flatnonzero(np.abs(lens - 250) >= 10)
        keep = np.concatenate([np.arange(len(lens))[: n // 2], np.tile(idx, 4)])
        parts = [buf[off[i]:off[i + 1]] for i in keep]
        buf = np.concatenate(parts)
        off = np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.int64)
    n = len(off) - 1
    pr = pack_2bit(buf, off)
    a = gpu_aligner_factory()
    a.set_reference(ref)
    a.upload_packed(pr)
    res = {}
    for lane_walk in (True, False):
        a.set_lane_walk(lane_walk)
        a.run_async()
        a.sync()
        res[lane_walk] = a.download_ops(n)
    a.set_lane_walk(False)
    on, off_ = res[True], res[False]
    np.testing.assert_array_equal(on.ops_off, off_.ops_off)
    for f in FIELDS:
        np.testing.assert_array_equal(on.stats[f], off_.stats[f], err_msg=f)
    np.testing.assert_array_equal(on.ops[:int(on.ops_off[n])], off_.ops[:int(off_.ops_off[n])])
    chk = every_read(ref, buf, off, on, threads=16)
    assert chk["mismatches"] == 0, chk
