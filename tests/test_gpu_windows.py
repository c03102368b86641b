"""Window reads (reads shorter than the amplicon, the reference's own test shape: 151 bp
reads against its 280 bp amplicon, tests/crispresso_tests.py:145-155) through the packed
call, whose classify certifies exact windows and one-substitution windows without a DP
("Window reads"): every read against the CPU oracle, including the cases the
certificate's argument turns on -- windows inside repeats (the largest offset wins the
start-cell scan), a substitution among the first or the last 16 bases (the other seed),
substitutions next to a shifted copy (a second diagonal with one mismatch: no certificate),
reads of 16 bases and of La - 1, windows at both ends, N and lower case."""
import numpy as np
import pytest

from crispresso_amd import synth
from crispresso_amd.aligner import pack_2bit, pack_reads
from tests.every_read import every_read

pytestmark = pytest.mark.gpu

SUB = {"A": "C", "C": "G", "G": "T", "T": "A"}


def _sub(s, p):
    return s[:p] + SUB[s[p]] + s[p + 1:]


def _window_reads(amp, rng, n):
    La = len(amp)
    out = []
    for _ in range(n):
        Lb = int(rng.integers(16, La))
        s = int(rng.integers(0, La - Lb + 1))
        r = amp[s:s + Lb]
        kind = int(rng.integers(0, 6))
        if kind == 1:
            r = _sub(r, int(rng.integers(0, Lb)))
        elif kind == 2:   # substitution among the first 16 bases
            r = _sub(r, int(rng.integers(0, min(16, Lb))))
        elif kind == 3:   # among the last 16
            r = _sub(r, Lb - 1 - int(rng.integers(0, min(16, Lb))))
        elif kind == 4:   # two substitutions (the DP)
            r = _sub(_sub(r, int(rng.integers(0, Lb))), int(rng.integers(0, Lb)))
        elif kind == 5 and Lb > 30:   # a deletion (the DP)
            p = int(rng.integers(5, Lb - 10))
            r = r[:p] + r[p + 3:]
        out.append(r)
    return out


def _run(amp, reads):
    buf, off = pack_reads(reads)
    pr = pack_2bit(buf, off)
    assert pr.lens is not None
    return buf, off, pr


@pytest.mark.parametrize("La", [40, 151, 280, 600, 1024])
def test_window_reads_random_amplicon(gpu_aligner_factory, La):
    amp = synth.random_amplicon(La, 700 + La)
    rng = np.random.Generator(np.random.PCG64(La))
    reads = _window_reads(amp, rng, 3000)
    reads += [amp[:16], amp[-16:], amp[:-1], amp[1:], amp[: La // 2].lower(), "N" + amp[1:20], amp[3:40] + "N"]
    buf, off, pr = _run(amp, reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pr)
    res = every_read(amp, buf, off, ob, threads=8)
    assert res["mismatches"] == 0, res
    assert a.path_counts()["exact_copies"] > 500   # the windows left the DP


def test_window_reads_in_repeats(gpu_aligner_factory):
    """An amplicon made of repeated blocks (tandem repeats, a shifted copy one base off): exact
    windows appear at several offsets (the largest wins), and one-substitution windows often
    have a second diagonal with one or no mismatch (then the DP decides)."""
    rng = np.random.Generator(np.random.PCG64(5))
    unit = synth.random_amplicon(37, 6)
    amp = synth.random_amplicon(20, 7) + unit * 4 + synth.random_amplicon(30, 8) + unit[1:] + unit + "ACGTTGCA" * 3
    La = len(amp)
    reads = _window_reads(amp, rng, 4000)
    for s in range(0, La - 60, 7):   # every offset: windows that lie inside the repeats
        reads += [amp[s:s + 60], _sub(amp[s:s + 60], 30), _sub(amp[s:s + 60], 3), _sub(amp[s:s + 60], 57)]
    reads += [unit * 2, unit, (unit * 3)[5:70]]
    buf, off, pr = _run(amp, reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pr)
    res = every_read(amp, buf, off, ob, threads=8)
    assert res["mismatches"] == 0, res


def test_window_homopolymer_amplicon(gpu_aligner_factory):
    """A low-complexity amplicon: every 16-mer occurs many times (more than the seed loop
    tries): certified or not, every read must equal the oracle's."""
    amp = "A" * 60 + "C" * 50 + "AC" * 40 + "G" * 45
    rng = np.random.Generator(np.random.PCG64(9))
    reads = _window_reads(amp, rng, 1500)
    buf, off, pr = _run(amp, reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pr)
    res = every_read(amp, buf, off, ob, threads=8)
    assert res["mismatches"] == 0, res


def test_window_c1_shape_resident_hdr(gpu_aligner_factory):
    """The packed batch still resident, against a second amplicon (the HDR pass's form)."""
    amp, buf, off = synth.c1_shape_workload(20_000)
    hdr = synth.hdr_amplicon(amp, 4, 140, 10)
    pr = pack_2bit(buf, off)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pr)
    assert every_read(amp, buf, off, ob, threads=8)["mismatches"] == 0
    a.set_reference(hdr)
    ob2 = a.align_ops(None, pr.offsets, resident=True)
    assert every_read(hdr, buf, off, ob2, threads=8)["mismatches"] == 0


def _seeded_mix(amp, seed):
    """Full-length reads with the parity mix (the 16-diagonal level and its redo list) and window
    reads (the seeded list): edits the 32-diagonal seeded band certifies, and ones it leaves to the
    wide level (deletions of 20-40 bases: hits too far apart; insertions of 12-15: the certificate)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    La = len(amp)
    b1, o1 = synth.reads_from(amp, 5000, seed, synth.PARITY_MIX)
    reads = [bytes(b1[o1[i]:o1[i + 1]]).decode() for i in range(len(o1) - 1)]
    b2, o2 = synth.window_reads(amp, 6000, seed + 1)
    reads += [bytes(b2[o2[i]:o2[i + 1]]).decode() for i in range(len(o2) - 1)]
    for _ in range(1500):
        Lb = int(rng.integers(100, La - 60))
        s = int(rng.integers(0, La - Lb - 40))
        r = amp[s:s + Lb + 40]
        kind = int(rng.integers(0, 4))
        p = int(rng.integers(30, Lb - 30))
        if kind == 0:
            r = r[:p] + r[p + int(rng.integers(20, 41)):]
        elif kind == 1:
            r = r[:p] + "".join(rng.choice(list("ACGT"), int(rng.integers(12, 16)))) + r[p:Lb]
        elif kind == 2:   # two indels far apart
            q = min(p + 50, len(r) - 10)
            r = r[:p] + r[p + 4:q] + "GATTACA" + r[q:Lb]
        else:
            r = _sub(_sub(_sub(r[:Lb], 10), Lb // 2), Lb - 20)
        reads.append(r)
    order = rng.permutation(len(reads))
    return [reads[i] for i in order]


@pytest.mark.parametrize("env", [{}, {"CRISPR_NW_DIRECT": "0"}, {"CRISPR_NW_CHUNK": "3001"},
                                 {"CRISPR_NW_ADAPT": "0", "CRISPR_NW_CHUNK": "4097"}, {"CRISPR_NW_SEED32": "0"}])
def test_seeded_levels_mixed_lists(gpu_aligner_factory, monkeypatch, env):
    """The seeded list through the 32-diagonal level: after that level's own list (the
    redo list, or as the only level the sorted DP list) from an even position -- an odd count leaves a
    hole --, padded to even per sort segment, its leftovers compacted as whole pairs for the wide level;
    chunks of odd sizes, both levels forced, the direct hand-off: every read against the oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    amp = synth.random_amplicon(280, 31)
    reads = _seeded_mix(amp, 32)
    buf, off, pr = _run(amp, reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pr)
    counts = a.path_counts()
    res = every_read(amp, buf, off, ob, threads=8)
    assert res["mismatches"] == 0, (res, counts)
    assert counts["wide128"] > 0, counts


@pytest.mark.parametrize("n", [8193, 4097 * 3])
def test_all_seeded_odd_batch(gpu_aligner_factory, n):
    """Every read of an odd-sized batch on the seeded list (151-base windows of a 280-base amplicon with
    a deletion and a substitution: no window certificate, and the 16-diagonal band cannot hold them), so
    every sort segment with an odd count pads its last pair past n entries: the seeded list, its flags
    and their compaction are reserved for that (n + n/4096 + 2 entries).  One-chunk call and a resident
    pass of the same batch: every read against the oracle, and the path counters leave the padding out
    (no read is a certified copy: n minus the DP reads is 0, not minus the padding entries)."""
    amp = synth.random_amplicon(280, 77)
    rng = np.random.Generator(np.random.PCG64(n))
    reads = []
    for _ in range(n):
        s = int(rng.integers(0, 280 - 155))
        r = amp[s:s + 154]
        p = int(rng.integers(40, 110))
        r = r[:p] + r[p + 3:]
        reads.append(_sub(r, int(rng.integers(120, 150))))
    buf, off, pr = _run(amp, reads)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pr)
    counts = a.path_counts()
    assert every_read(amp, buf, off, ob, threads=8)["mismatches"] == 0
    assert counts["exact_copies"] == 0, counts
    assert all(0 <= v <= n for v in counts.values()), counts
    ob2 = a.align_ops(None, pr.offsets, resident=True)
    assert every_read(amp, buf, off, ob2, threads=8)["mismatches"] == 0
