"""GPU parity: the HIP kernel (through the C ABI) vs the CPU oracle, bit for bit.

Compared per read: the three alignment strings (aligned amplicon, markup,
aligned read), alignment length, identity/similarity/gap counts, score and the
traceback start cell.  Integer/byte work, so the bar is exact equality.
"""
import numpy as np
import pytest

from crispresso_amd import synth
from crispresso_amd.aligner import pack_2bit, pack_reads

pytestmark = pytest.mark.gpu

# The kernel families production selects: "diag" = the certified band
# levels + the exact kernel on what they hand on (the default); "full" = the exact
# int32 kernel on every read (what runs when the band does not apply: -endweight,
# penalties outside the band's int16 range).
KERNELS = ["diag", "full"]


@pytest.fixture(params=[f"{k}/{m}" for k in KERNELS for m in ("ops", "rows")])
def kernel(request, monkeypatch):
    """Run a test once per kernel family (CRISPR_NW_KERNEL selects it) and output
    mode (ops: runs over PCIe + host expansion, the default; rows: the kernels write
    the three strings)."""
    fam, mode = request.param.split("/")
    monkeypatch.setenv("CRISPR_NW_KERNEL", fam)
    monkeypatch.setenv("CRISPR_NW_OUTPUT", mode)
    return request.param

FIELDS = ("aln_len", "n_ident", "n_sim", "n_gaps", "score", "end_i", "end_j")


def assert_same(oracle, amplicon, buf, offsets, batch, label="", params=None):
    res, aln = oracle.align_batch(amplicon, buf, offsets, params, nthreads=8)
    n = len(offsets) - 1
    assert len(batch) == n
    lens = np.diff(offsets)
    bad = []
    for f in FIELDS:
        g = batch.stats[f].astype(np.int64)
        o = res[f].astype(np.int64)
        mism = np.flatnonzero((g != o) & (lens > 0))
        if mism.size:
            bad.append((f, mism[:5].tolist(), g[mism[:5]].tolist(), o[mism[:5]].tolist()))
    assert not bad, f"{label} stat mismatches: {bad}"
    for i in range(n):
        if lens[i] == 0:
            assert batch.empty(i)
            continue
        L = int(res["aln_len"][i])
        for k in range(3):
            g = batch.aln[i, k, :L].tobytes()
            o = aln[i, k, :L].tobytes()
            assert g == o, f"{label} read {i} string {k}:\n gpu {g!r}\n cpu {o!r}"


def test_hand_cases(gpu_aligner_factory, oracle, kernel):
    amp = "ACGTACGTTTGACCA"
    reads = ["ACGTACGTGACCA", "ACGTACGTTTGACCAGG", "TTGACC", "A", "ACGTACGTTTGACCA", "", "acgtNNNNtttgacca",
             "GGGGGGGGGGGGGGGGGGGGGGGGGGGGGG", "T-C-A", "ACGTRYKMSWBDHVNU"]
    a = gpu_aligner_factory()
    a.set_reference(amp)
    buf, off = pack_reads(reads)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), "hand")


def test_c2_mix(gpu_aligner_factory, oracle, kernel):
    amp = synth.random_amplicon(250, 1)
    buf, off = synth.reads_from(amp, 3000, 2)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), "c2")


def test_parity_mix(gpu_aligner_factory, oracle, kernel):
    amp = synth.random_amplicon(250, 1)
    buf, off = synth.reads_from(amp, 3000, 3, synth.PARITY_MIX)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), "parity")


@pytest.mark.parametrize("La", [1, 2, 7, 63, 64, 65, 128, 129, 192, 250, 257, 320, 384, 448, 512, 513, 640, 768,
                                 896, 1024])
def test_amplicon_lengths(gpu_aligner_factory, oracle, kernel, La):
    amp = synth.random_amplicon(La, 100 + La)
    rng = np.random.Generator(np.random.PCG64(La))
    reads = []
    for L in [1, 2, 5, max(1, La - 3), La, La + 7, 60, 130, 300]:
        if rng.random() < 0.5 and L <= La:
            s = rng.integers(0, La - L + 1)
            reads.append(amp[s:s + L])
        else:
            reads.append(synth.random_amplicon(L, int(rng.integers(1 << 30))))
    sub, soff = synth.reads_from(amp, 40, La + 7)
    reads += synth.unpack(sub, soff)
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), f"La={La}")


def test_global_traceback_slab(gpu_aligner_factory, oracle):
    """Reads long enough that the traceback bits leave LDS for a global slab."""
    amp = synth.random_amplicon(250, 1)
    rng = np.random.Generator(np.random.PCG64(9))
    reads = [synth.random_amplicon(1400, 11), amp[:100] + synth.random_amplicon(1250, 12) + amp[100:]]
    reads += [amp] * 3 + [amp[5:200]]
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert a.fallbacks() >= 2
    assert_same(oracle, amp, buf, off, batch, "global-tb")


def test_repeated_batches_reuse_context(gpu_aligner_factory, oracle, kernel):
    amp = synth.random_amplicon(180, 21)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    for seed in (1, 2, 3):
        buf, off = synth.reads_from(amp, 500 + 100 * seed, seed)
        assert_same(oracle, amp, buf, off, a.align_packed(buf, off), f"rep{seed}")
    amp2 = synth.random_amplicon(300, 22)
    a.set_reference(amp2)
    buf, off = synth.reads_from(amp2, 700, 5)
    assert_same(oracle, amp2, buf, off, a.align_packed(buf, off), "switch-ref")


def test_band_fallbacks_exact(gpu_aligner_factory, oracle):
    """Reads whose traceback leaves the diagonal band (large indels, shifted
    reads) are re-run with full storage; results stay bit-identical."""
    amp = synth.random_amplicon(250, 1)
    rng = np.random.Generator(np.random.PCG64(33))
    reads = []
    for d in (40, 60, 100, 150):
        p = int(rng.integers(20, 250 - d - 20))
        reads.append(amp[:p] + amp[p + d:])                                 # big deletion
    for k in (40, 80):
        reads.append(amp[:125] + synth.random_amplicon(k, 50 + k) + amp[125:])  # big insertion
    reads += [amp[100:], amp[:90], amp[60:200], synth.random_amplicon(250, 77)]  # shifted / unrelated
    buf0, off0 = synth.reads_from(amp, 400, 8, synth.PARITY_MIX)
    reads += synth.unpack(buf0, off0)
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert a.geometry()["tb_mode"] == "diag-int16"
    assert a.fallbacks() >= 6
    assert_same(oracle, amp, buf, off, batch, "band-fallback")


@pytest.mark.parametrize("exact", ["multi", "split", "wave"])
@pytest.mark.parametrize("La", [1, 5, 63, 64, 65, 200, 250, 333, 600, 1000, 1024])
def test_exact_kernel_work_list(gpu_aligner_factory, oracle, monkeypatch, La, exact):
    """Every read through the exact int32 kernels (CRISPR_NW_KERNEL=full): the multi-wave kernel (nw_exact.hip: one row per lane, up
    to 16 waves, LDS ring hand-off between waves), the one-wave kernel, and the two
    splitting one list (the multi-wave kernel takes the first grid entries) give the
    oracle's alignments -- IUPAC, '-' and lower-case reads, reads longer and shorter
    than the amplicon, big indels."""
    monkeypatch.setenv("CRISPR_NW_KERNEL", "full")
    if exact != "wave":
        # split: 7 reads to the multi-wave kernel, the rest to the one-wave kernel
        monkeypatch.setenv("CRISPR_NW_EXACT", "multi:7" if exact == "split" else "multi")
    amp = synth.random_amplicon(La, 500 + La)
    rng = np.random.Generator(np.random.PCG64(La))
    reads = [amp, amp.lower(), amp[: max(1, La // 2)], "ACGTRYKMSWBDHVNU", "T-C-A" * 3, "N" * 9]
    for L in (1, 3, La + 40, 2 * La + 5):
        reads.append(synth.random_amplicon(L, int(rng.integers(1 << 30))))
    if La > 60:
        d = La // 5
        reads += [amp[:La // 3] + amp[La // 3 + d:], amp[:La // 2] + synth.random_amplicon(d, 7) + amp[La // 2:]]
    sub, soff = synth.reads_from(amp, 60, La + 3, synth.PARITY_MIX)
    reads += synth.unpack(sub, soff)
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert_same(oracle, amp, buf, off, batch, f"exact-{exact} La={La}")
    assert a.geometry()["tb_mode"] in ("full-lds", "full-global")


@pytest.mark.parametrize("mode", ["ops", "rows"])
@pytest.mark.parametrize("La", [1025, 1500, 2100, 4100])
def test_long_amplicons(gpu_aligner_factory, oracle, monkeypatch, La, mode):
    """Amplicons past the band / one-wave kernels' 1024 bp: every read through the
    multi-wave exact kernel (R = 2 / 4 / 8 rows per lane, up to 16 waves), traceback in
    an HBM slab -- bit-identical to the oracle, rows and ops output."""
    monkeypatch.setenv("CRISPR_NW_OUTPUT", mode)
    amp = synth.random_amplicon(La, 900 + La)
    rng = np.random.Generator(np.random.PCG64(La))
    reads = [amp, amp[: La // 3], amp[La // 2:], amp[:100] + amp[400:], "ACGTRYKMSWBDHVNU", "",
             amp[:La // 2] + synth.random_amplicon(60, 3) + amp[La // 2:], synth.random_amplicon(300, 5)]
    for _ in range(6):
        r = bytearray(amp.encode())
        for p in rng.integers(0, La, 12):
            r[p] = ord("ACGT"[int(rng.integers(4))])
        reads.append(r.decode())
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), f"long La={La}")


@pytest.mark.parametrize("mode", ["ops", "rows"])
@pytest.mark.parametrize("ends", [(10.0, 0.5), (3.0, 1.0), (0.5, 0.25), (40.0, 0.0)])
@pytest.mark.parametrize("La", [60, 250, 1100])
def test_endweight(gpu_aligner_factory, oracle, monkeypatch, La, ends, mode):
    """needle -endweight -endopen -endextend: end gaps cost endopen +
    (k-1) endextend; every read through the exact kernels (one-wave, and the multi-wave
    kernel for an amplicon over 1024 bp) -- bit-identical to the oracle's restatement.
    Parity vs EMBOSS itself is unpinned (CRISPResso never sets these options)."""
    from crispresso_amd.needle_options import NeedleOptions

    monkeypatch.setenv("CRISPR_NW_OUTPUT", mode)
    eo, ee = ends
    opts = NeedleOptions.parse(f"-gapopen=10 -gapextend=0.5 -endweight -endopen={eo} -endextend={ee}")
    amp = synth.random_amplicon(La, 700 + La)
    reads = [amp, amp[La // 4:], amp[: 3 * La // 4], "ACGTACGT" + amp, amp + "TTGCA", amp[10:-10],
             amp[:La // 2] + amp[La // 2 + 7:], "ACGTRYKMSWBDHVNU", "A"]
    sub, soff = synth.reads_from(amp, 80, La + 11, synth.PARITY_MIX)
    reads += synth.unpack(sub, soff)
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory(opts)
    a.set_reference(amp)
    p = oracle.params(10.0, 0.5, True, eo, ee)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), f"endweight {ends} La={La}", params=p)
    # and the free-end-gap answer differs for an overhanging read (the option is applied)
    free = oracle.align(amp, amp[La // 4:])[0]
    assert free["score"] != oracle.align(amp, amp[La // 4:], p)[0]["score"]


def test_pairs_with_unequal_and_empty_reads(gpu_aligner_factory, oracle):
    """Band pairs: partners of different lengths, empty partners, odd batch size."""
    amp = synth.random_amplicon(230, 41)
    rng = np.random.Generator(np.random.PCG64(41))
    reads = []
    for k in range(301):
        L = int(rng.integers(0, 260)) if k % 7 else 0
        s = int(rng.integers(0, max(1, 230 - L)))
        r = amp[s:s + L] if rng.random() < 0.7 else synth.random_amplicon(max(L, 1), k)[:L]
        reads.append(r)
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert a.geometry()["tb_mode"] == "diag-int16"
    assert_same(oracle, amp, buf, off, batch, "pairs")


def _mixed_lengths(amp, n, seed):
    """Reads of every length class: tiny,
    short, full, longer than the amplicon, empty; exact copies and variants."""
    rng = np.random.Generator(np.random.PCG64(seed))
    La = len(amp)
    reads = []
    for k in range(n):
        u = rng.random()
        if u < 0.15:
            L = int(rng.integers(1, 16))
        elif u < 0.25:
            L = 0
        elif u < 0.6:
            L = int(rng.integers(16, La))
        else:
            L = int(rng.integers(La - 5, La + 40))
        s = int(rng.integers(0, max(1, La - L)))
        r = amp[s:s + L] if rng.random() < 0.6 else synth.random_amplicon(max(L, 1), seed * 7919 + k)[:L]
        reads.append(r)
    return reads


@pytest.mark.parametrize("La", [31, 100, 250, 500])
def test_mixed_lengths(gpu_aligner_factory, oracle, La):
    """Every length class (tiny, short, full, longer than the amplicon, empty) on the
    band path: pairs of unequal lengths, reads past the band's length cap."""
    amp = synth.random_amplicon(La, 300 + La)
    reads = _mixed_lengths(amp, 400, La)
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), f"mixed La={La}")


def test_rare_codes_go_exact(gpu_aligner_factory, oracle):
    """Reads with IUPAC codes outside A C G T N are flagged by the band fill and
    re-aligned by the exact kernel; their pair partners are not."""
    amp = synth.random_amplicon(240, 17)
    buf0, off0 = synth.reads_from(amp, 600, 18, synth.PARITY_MIX)
    reads = synth.unpack(buf0, off0)
    rng = np.random.Generator(np.random.PCG64(19))
    rare = "RYKMSWBDHVU"
    bad = set()
    for k in rng.choice(len(reads), 25, replace=False):
        r = list(reads[int(k)])
        if not r:
            continue
        r[int(rng.integers(0, len(r)))] = rare[int(rng.integers(0, len(rare)))]
        reads[int(k)] = "".join(r)
        bad.add(int(k))
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert a.fallbacks() >= len(bad)
    assert_same(oracle, amp, buf, off, batch, "rare-codes")


def test_band_multiple_passes(gpu_aligner_factory, oracle, monkeypatch):
    """A region budget smaller than the batch splits the band levels into several
    fill + walk passes."""
    monkeypatch.setenv("CRISPR_NW_REGION_MB", "2")
    amp = synth.random_amplicon(250, 8)
    buf, off = synth.reads_from(amp, 3001, 9, synth.PARITY_MIX)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off, mode="rows")   # kernel_times describe an upload/run pass
    assert_same(oracle, amp, buf, off, batch, "passes")
    t = a.kernel_times()
    assert t["fill_ms"] > 0 and t["walk_ms"] > 0 and t["rest_ms"] >= 0


def test_needle_cli_matches_oracle_cli(tmp_path, oracle):
    """The GPU `needle` shim and the oracle CLI print the same srspair blocks."""
    import subprocess
    import sys

    amp = synth.random_amplicon(180, 61)
    buf, off = synth.reads_from(amp, 200, 62, synth.PARITY_MIX)
    reads = synth.unpack(buf, off)
    (tmp_path / "a.fa").write_text(f">AMPL\n{amp}\n")
    fasta = "".join(f">@M0_1_{k} 1_N\n{r}\n" for k, r in enumerate(reads))
    args = [f"-asequence={tmp_path / 'a.fa'}", "-bsequence=/dev/stdin", "-outfile=/dev/stdout",
            "-gapopen=10", "-gapextend=0.5", "-awidth3=5000"]
    import os
    shim = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "crispresso_amd", "bin", "needle")
    gpu = subprocess.run([sys.executable, shim] + args, input=fasta, capture_output=True, text=True, check=True).stdout
    cpu = subprocess.run([oracle.CLI] + args, input=fasta, capture_output=True, text=True, check=True).stdout
    strip = lambda t: t[t.index("#=="): t.rindex("#---------------------------------------\n#---")]  # noqa: E731
    assert strip(gpu) == strip(cpu)


def test_pooled_multi_amplicon(gpu_aligner_factory, oracle):
    """nw_align_multi: many amplicons in one call (pair-table, profile and int32
    kernel paths by amplicon length), empty and one-read groups, read order kept;
    the context aligns single-amplicon batches correctly afterwards."""
    from crispresso_amd.pooled import align_pooled
    from tests.helpers import OracleAligner

    rng = np.random.Generator(np.random.PCG64(77))
    lengths = [150, 180, 64, 231, 256, 257, 300, 420, 199]
    amps = [synth.random_amplicon(L, 900 + g) for g, L in enumerate(lengths)]
    reads = []
    for g, a in enumerate(amps):
        k = [120, 0, 1, 333, 64, 91, 150, 40, 257][g]
        reads.append(synth.reads_from(a, k, 950 + g, synth.PARITY_MIX) if k else [])
    al = gpu_aligner_factory()
    got = align_pooled(amps, reads, al)
    want = align_pooled(amps, reads, OracleAligner())
    for g in range(len(amps)):
        assert len(got[g]) == len(want[g])
        for f in FIELDS:
            assert np.array_equal(got[g].stats[f], want[g].stats[f]), (g, f)
        for i in range(len(want[g])):
            L = int(want[g].stats["aln_len"][i])
            assert np.array_equal(got[g].aln[i, :, :L], want[g].aln[i, :, :L]), (g, i)
    amp = amps[3]
    buf, off = synth.reads_from(amp, 500, 999, synth.PARITY_MIX)
    al.set_reference(amp)
    assert_same(oracle, amp, buf, off, al.align_packed(buf, off), "after-multi")


# ---------------------------------------------------------------- certified band (nw_band.hip)

@pytest.mark.parametrize("direct", ["0", None])
def test_diag_is_default_and_certifies_c2(gpu_aligner_factory, oracle, monkeypatch, direct):
    """The default path is the certified diagonal band; on the C2 mix almost every
    read is certified (no fallback) and all are bit-identical to the oracle.  With the
    second level always run (CRISPR_NW_DIRECT=0) only the rare read neither band
    certifies reaches the exact kernel; by default the first level's few give-ups
    (~0.3 %) go there directly (KernelArgs::redo_direct)."""
    if direct is not None:
        monkeypatch.setenv("CRISPR_NW_DIRECT", direct)
    amp = synth.random_amplicon(250, 1)
    buf, off = synth.reads_from(amp, 4001, 2)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert a.geometry()["tb_mode"] == "diag-int16"
    paths = a.path_counts()
    if direct == "0":
        assert a.fallbacks() <= 4 and paths["band32"] > 0
    else:
        assert paths["band32"] == 0 and 0 < a.fallbacks() <= 0.01 * (len(off) - 1)
    assert a.fallbacks() == paths["band_fallback"] and paths["exact_kernel"] <= paths["band_fallback"]
    assert_same(oracle, amp, buf, off, batch, "diag-c2")


def test_diag_certificate_failures_fall_back(gpu_aligner_factory, oracle):
    """Reads the band cannot certify -- chimeras, shifted or unrelated reads, length
    differences beyond the band, IUPAC codes -- go to the exact kernel."""
    amp = synth.random_amplicon(250, 3)
    rng = np.random.Generator(np.random.PCG64(5))
    reads = [amp[:60] + synth.random_amplicon(70, 6) + amp[130:],          # junk block, same length
             amp[:100] + amp[140:], amp[:125] + synth.random_amplicon(35, 7) + amp[125:],  # |Lb - La| > 31
             amp[40:] + amp[:40], synth.random_amplicon(250, 8), amp[::-1],
             amp[:80] + "R" + amp[81:], amp[:20] + "-" + amp[21:]]
    reads += [amp] * 7 + [amp[:100] + amp[101:]] * 5
    buf0, off0 = synth.reads_from(amp, 300, 9, synth.PARITY_MIX)
    reads += synth.unpack(buf0, off0)
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert a.fallbacks() >= 6
    assert_same(oracle, amp, buf, off, batch, "diag-fallback")


def test_diag_multiple_passes_and_odd_counts(gpu_aligner_factory, oracle, monkeypatch):
    """Region budget below the batch: several fill + walk passes over the sorted
    pairs; an odd read count leaves the last sorted read without a partner."""
    monkeypatch.setenv("CRISPR_NW_REGION_MB", "1")
    amp = synth.random_amplicon(250, 8)
    buf, off = synth.reads_from(amp, 1003, 9, synth.PARITY_MIX)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off, mode="rows")   # kernel_times describe an upload/run pass
    assert a.geometry()["tb_mode"] == "diag-int16"
    assert_same(oracle, amp, buf, off, batch, "diag-passes")
    t = a.kernel_times()
    assert t["fill_ms"] > 0 and t["walk_ms"] > 0
    ob = a.align_ops(buf, off)
    assert_same(oracle, amp, buf, off, ob.expand(amp, buf, off), "diag-passes-ops")


@pytest.mark.parametrize("La", [40, 150, 333, 700, 1024])
def test_diag_lengths_around_the_band(gpu_aligner_factory, oracle, La):
    """Read lengths from La - 40 to La + 40 (inside and outside the band's reach),
    empty reads, and single reads of a length."""
    amp = synth.random_amplicon(La, 500 + La)
    rng = np.random.Generator(np.random.PCG64(La))
    reads = []
    for k in range(240):
        D = int(rng.integers(-40, 41))
        L = max(0, La + D)
        if k % 17 == 0:
            L = 0
        base = amp if D <= 0 else amp + synth.random_amplicon(D, k)
        s = int(rng.integers(0, len(base) - L + 1)) if L < len(base) else 0
        r = list(base[s:s + L])
        for _ in range(int(rng.integers(0, 4))):
            if r:
                r[int(rng.integers(0, len(r)))] = "ACGT"[int(rng.integers(0, 4))]
        reads.append("".join(r))
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), f"diag La={La}")


def test_diag_homopolymer_ties(gpu_aligner_factory, oracle):
    """Indels inside homopolymer runs and tandem repeats: co-optimal placements,
    decided by the tie rules -- the band must reproduce them."""
    unit = "ACGTTTTTGCAAAAACGCGCGTCA"
    amp = (unit * 11)[:250]
    rng = np.random.Generator(np.random.PCG64(13))
    reads = []
    for k in range(400):
        r = list(amp)
        for _ in range(int(rng.integers(1, 4))):
            p = int(rng.integers(1, len(r) - 1))
            op = rng.integers(0, 3)
            if op == 0:
                del r[p]
            elif op == 1:
                r.insert(p, r[p])
            else:
                r[p] = "ACGT"[int(rng.integers(0, 4))]
        reads.append("".join(r))
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    assert_same(oracle, amp, buf, off, a.align_packed(buf, off), "diag-homopolymer")


def test_diag_exact_copies(gpu_aligner_factory, oracle):
    """Reads identical to the amplicon (any case) take the no-DP path; near-copies
    (one N, one substitution, U for T, one base short) and an amplicon with N do not."""
    amp = synth.random_amplicon(200, 31)
    reads = [amp, amp.lower(), amp[:50].lower() + amp[50:], amp] * 5
    reads += [amp[:70] + "N" + amp[71:], amp[:70] + ("A" if amp[70] != "A" else "C") + amp[71:],
              amp.replace("T", "U"), amp[:-1], amp[1:], amp + "A", ""]
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert_same(oracle, amp, buf, off, batch, "exact")
    amp_n = amp[:100] + "N" + amp[101:]
    a.set_reference(amp_n)
    buf, off = pack_reads([amp_n, amp_n.lower(), amp] * 3)
    assert_same(oracle, amp_n, buf, off, a.align_packed(buf, off), "exact-N")


@pytest.mark.parametrize("levels", ["16+32", "32", "16+32 direct", "16+32 direct-small"])
def test_diag_band_levels(gpu_aligner_factory, oracle, monkeypatch, levels):
    """The 16-diagonal first level hands what it cannot certify (indels of 8+,
    noisy and junk reads) to the 32-diagonal level, which hands the rest to the
    exact kernel; with the first level off the 32-diagonal level sees every read.
    "direct": the second level skips itself on the device and the exact kernel takes
    the first level's give-ups after its own list (threshold above / below the batch's
    give-ups: both branches of KernelArgs::redo_direct)."""
    if levels == "32":
        monkeypatch.setenv("CRISPR_NW_KERNEL", "diag32")
    monkeypatch.setenv("CRISPR_NW_DIRECT", {"16+32 direct": "100000", "16+32 direct-small": "1"}.get(levels, "0"))
    amp = synth.random_amplicon(250, 44)
    rng = np.random.Generator(np.random.PCG64(45))
    reads = synth.unpack(*synth.reads_from(amp, 1500, 46, synth.PARITY_MIX))
    for g in (6, 9, 14, 17, 24, 29, 35):      # deletions around both bands' reach
        p = int(rng.integers(30, 200))
        reads += [amp[:p] + amp[p + g:]] * 3
        reads += [amp[:p] + synth.random_amplicon(g, g) + amp[p:]] * 2
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert a.geometry()["tb_mode"] == "diag-int16"
    paths = a.path_counts()
    if levels == "16+32 direct":
        assert paths["band32"] == 0 and paths["band_fallback"] > 1
    elif levels.startswith("16+32"):
        assert paths["band32"] > 1
    assert_same(oracle, amp, buf, off, batch, f"levels={levels}")
    if levels == "16+32 direct":   # ops output too (the chunked pipeline's counts)
        ob = a.align_ops(buf, off)
        assert a.path_counts()["band32"] == 0
        assert_same(oracle, amp, buf, off, ob.expand(amp, buf, off), "levels=direct ops")


@pytest.mark.parametrize("levels", ["16+32", "32"])
def test_diag_iupac_in_every_pair_slot(gpu_aligner_factory, oracle, monkeypatch, levels):
    """Reads with codes outside the band's score table (IUPAC, '-') in every pair
    slot of the fill's wavefronts: each must leave the band for the exact kernel
    (the per-pair flag is taken by a ballot that every lane must see)."""
    if levels == "32":
        monkeypatch.setenv("CRISPR_NW_KERNEL", "diag32")
    amp = synth.random_amplicon(250, 7)
    rng = np.random.Generator(np.random.PCG64(71))
    reads = []
    for k in range(512):
        L = int(rng.integers(20, 250))
        s = int(rng.integers(0, 250 - L + 1))
        r = list(amp[s:s + L])
        if k % 3 == 0:
            for _ in range(int(rng.integers(1, 3))):
                r[int(rng.integers(0, L))] = "RYKMSWBDHV-"[int(rng.integers(0, 11))]
        elif k % 3 == 1:
            r[int(rng.integers(0, L))] = "ACGT"[int(rng.integers(0, 4))]
        reads.append("".join(r))
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert a.fallbacks() >= 512 // 3
    assert_same(oracle, amp, buf, off, batch, f"diag-iupac {levels}")


@pytest.mark.parametrize("block", [6, 10, 12, 20])
def test_diag_refined_certificate_clustered_mismatches(gpu_aligner_factory, oracle, monkeypatch, block):
    """Reads with a block of mismatches (the HDR pass of CRISPResso: reference-derived
    reads against the HDR amplicon, CORE:1808-1828) fail the plain certificate; the
    refined one (gapped escapes pay the gap open, single diagonals scored exactly)
    keeps most of them on the band.  Bit-exact either way.  (Both levels always run:
    the counts below are the certificate's, not KernelArgs::redo_direct's.)"""
    monkeypatch.setenv("CRISPR_NW_DIRECT", "0")
    amp = synth.random_amplicon(250, 4)
    hdr = synth.hdr_amplicon(amp, 4, 120, block)
    buf, off = synth.reads_from(amp, 1200, 5)
    a = gpu_aligner_factory()
    a.set_reference(hdr)
    ob = a.align_ops(buf, off)
    assert_same(oracle, hdr, buf, off, ob.expand(hdr, buf, off), f"hdr-block{block}")
    counts = a.path_counts()
    if block <= 10:
        assert counts["exact_kernel"] < 0.05 * (len(off) - 1), counts


@pytest.mark.parametrize("ops", [False, True])
def test_iupac_amplicon_band_path(gpu_aligner_factory, oracle, monkeypatch, ops):
    """An amplicon with IUPAC codes (and a byte outside EDNAFULL) keeps the certified
    band path: its rows score from the table's EDNAFULL rows.  Reads from it (ACGT at
    the IUPAC positions, the parity mix of edits) equal the oracle, and few (~4 %) need
    the exact kernel (both levels always run: the certificate's count)."""
    monkeypatch.setenv("CRISPR_NW_DIRECT", "0")
    base = synth.random_amplicon(250, 23)
    amp = list(base)
    for pos, code in zip((10, 57, 120, 121, 200, 233), "RYNKMS"):
        amp[pos] = code
    amp = "".join(amp)
    reads = synth.unpack(*synth.reads_from(base, 3000, 24, synth.PARITY_MIX))
    reads += [amp, amp.replace("N", "A"), base, "ACGTRYKMSWBDHVNU", ""]
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    if ops:
        ob = a.align_ops(buf, off)
        batch = ob.expand(amp, buf, off)
    else:
        batch = a.align_packed(buf, off)
    paths = a.path_counts()
    assert_same(oracle, amp, buf, off, batch, f"iupac-amplicon ops={ops}")
    assert paths["band16"] > 1000 and paths["exact_kernel"] < 0.1 * len(reads)


# ---------------------------------------------------------------- the wide level (128 diagonals)

def _wide_reads(amp, seed, n_bulk=300):
    """Reads the 16 / 32-diagonal levels cannot certify but 128 diagonals can (deletions and
    insertions of 26-60 bp, two separated indels), reads no band certifies (chimeras,
    unrelated, reversed, IUPAC codes), and a bulk of parity-mix reads."""
    La = len(amp)
    rng = np.random.Generator(np.random.PCG64(seed))
    reads = []
    for d in (26, 28, 30, 34, 40, 50, 60):
        if d <= La // 2:
            p = int(rng.integers(La // 8, La - d - La // 8))
            reads.append(amp[:p] + amp[p + d:])
    for k in (26, 33, 45, 60):
        p = int(rng.integers(La // 8, La - La // 8))
        reads.append(amp[:p] + synth.random_amplicon(k, 90 + k) + amp[p:])
    if La >= 200:
        p, q = La // 4, 2 * La // 3
        reads.append(amp[:p] + amp[p + 20:q] + synth.random_amplicon(25, 5) + amp[q:])   # -20 then +25
        reads.append(amp[:p] + amp[p + 30:q] + amp[q + 12:])                              # two deletions
    reads += [amp[:60] + synth.random_amplicon(90, 6) + amp[150:], synth.random_amplicon(La, 8), amp[::-1],
              amp[40:] + amp[:40], amp[:80] + "R" + amp[81:]]
    buf0, off0 = synth.reads_from(amp, n_bulk, seed + 1, synth.PARITY_MIX)
    reads += synth.unpack(buf0, off0)
    return reads


@pytest.mark.parametrize("wide", [None, "0"])
@pytest.mark.parametrize("La", [250, 96, 600])
def test_wide_level(gpu_aligner_factory, oracle, monkeypatch, kernel, wide, La):
    """The 128-diagonal wide level takes what the 16 / 32 levels give up on (the exact
    kernel's list before it): large indels are certified there, the rest reaches the
    exact kernel; bit-identical either way (CRISPR_NW_WIDE=0: no wide level)."""
    if wide is not None:
        monkeypatch.setenv("CRISPR_NW_WIDE", wide)
    amp = synth.random_amplicon(La, 40 + La)
    reads = _wide_reads(amp, La)
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    batch = a.align_packed(buf, off)
    assert_same(oracle, amp, buf, off, batch, f"wide={wide} La={La}")
    if kernel.startswith("diag"):
        fb, ex = a.fallbacks(), a.exact_reads()
        assert fb >= 10
        if wide is None:
            assert 4 <= ex < fb - 5, (fb, ex)   # the large indels certified on the wide level
        else:
            assert ex == fb


def test_wide_level_capacity(gpu_aligner_factory, oracle, monkeypatch):
    """More reads for the wide level than its region holds (2048 pairs per chunk): the
    list's tail goes straight to the exact kernel."""
    amp = synth.random_amplicon(150, 61)
    rng = np.random.Generator(np.random.PCG64(62))
    reads = []
    for i in range(4700):
        d = int(rng.integers(30, 70))
        p = int(rng.integers(10, 150 - d - 10))
        reads.append(amp[:p] + amp[p + d:] if i % 3 else amp[:p] + synth.random_amplicon(d, i) + amp[p:])
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pack_2bit(buf, off))
    assert a.fallbacks() > 4096
    assert_same(oracle, amp, buf, off, ob.expand(amp, buf, off), "wide-capacity")


@pytest.mark.parametrize("kind", ["random", "homopolymer", "all-A", "dinucleotide", "La256", "La257"])
def test_one_substitution_certificate(gpu_aligner_factory, oracle, kind):
    """Reads of the amplicon's length with one or two A C G T substitutions are finished by
    the classify kernel (no DP) when no shifted diagonal or one-gap alignment can reach the
    main one; repeats, N, three substitutions and amplicons over 256 bp go through the band.
    Bit-identical."""
    La = {"La256": 256, "La257": 257}.get(kind, 250)
    rng = np.random.Generator(np.random.PCG64(91))
    if kind == "homopolymer":
        amp = "".join(b * int(rng.integers(1, 9)) for b in rng.choice(list("ACGT"), 80))[:La]
    elif kind == "all-A":
        amp = "A" * La
    elif kind == "dinucleotide":
        amp = ("AC" * La)[:La]
    else:
        amp = synth.random_amplicon(La, 92)
    La = len(amp)
    sub = {"A": "C", "C": "G", "G": "T", "T": "A"}
    reads = []
    for p in sorted({0, 1, 2, La // 3, La // 2, La - 3, La - 2, La - 1} | set(rng.integers(0, La, 40).tolist())):
        reads.append(amp[:p] + sub[amp[p]] + amp[p + 1:])
    reads.append(amp[:10].lower() + sub[amp[10]].lower() + amp[11:])
    reads.append(amp[:50] + "N" + amp[51:])
    # two substitutions: apart, adjacent, in one dword, at both ends, near the ends
    for p, q in [(50, 90), (0, La - 1), (0, 1), (La - 2, La - 1), (1, 2), (3, 4), (4, 5), (7, 8), (100, 101),
                 (100, 102), (30, La - 30), (2, La - 3)] + [tuple(sorted(rng.choice(La, 2, replace=False).tolist()))
                                                            for _ in range(30)]:
        reads.append(amp[:p] + sub[amp[p]] + amp[p + 1:q] + sub[amp[q]] + amp[q + 1:])
    reads.append(amp[:60] + sub[amp[60]] + amp[61:70] + sub[amp[70]] + amp[71:80] + sub[amp[80]] + amp[81:])
    reads.append(amp[:60] + "N" + amp[61:70] + sub[amp[70]] + amp[71:])
    reads += [amp] * 3
    buf, off = pack_reads(reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pack_2bit(buf, off))
    assert_same(oracle, amp, buf, off, ob.expand(amp, buf, off), f"sub1 {kind}")
    if kind in ("random", "La256"):
        # no DP but for N, the triple substitution and the few double substitutions whose bases leave a
        # one-gap alignment possible (adjacent or end positions: the certificate cannot exclude it)
        assert a.path_counts()["exact_copies"] >= len(reads) - 12
