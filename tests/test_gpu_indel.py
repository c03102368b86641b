"""Classify's one-indel certificate ("One indel"): a read equal to the amplicon with one
gap of k <= 10 residues (a deletion: the read is La - k long; an insertion: La + k) is aligned without
any DP -- runs M q, the gap, M the rest, with the gap placed where the traceback's tie rules put it
(left-most among equal placements).  Every read is checked against the CPU oracle (records and rows),
on the inputs the certificate's argument turns on: gaps in homopolymers and tandem repeats (the gap
slides), next to substitutions (not one-indel reads: the DP), near both ends (where an end gap or a
shifted diagonal competes), inserted copies of the neighbouring bases, k at and past the bound, the
amplicon of the reference's own test (its repeats), packed batches with N; and the path counters
show that the certificate took the one-indel reads."""
import numpy as np
import pytest

from crispresso_amd import synth
from crispresso_amd.aligner import pack_2bit, pack_reads
from tests.every_read import every_read

pytestmark = pytest.mark.gpu

REF_AMPLICON = (   # tests/crispresso_tests.py:145-155 (the reference's e2e amplicon)
    "GTCGCCCCTCAAATCTTACAGCTGCTCACTCCCCTGCAGGGCAACGCCCAGGGACCAAGTTAGCCCCTTAAGCCTAGGCAAAAGAATCCCGCCCATAATCGAG"
    "AAGCGACTCGACATGGAGGCGATGACGAGATCACGCGAGGAGGAAAGGAGGGAGGGCTTCTTCCAGGCCCAGGGCGGTCCTTACAAGACGGGAGGCAGCAGA"
    "GAACTCCCATAAAGGTATTGCGGCACTCCCCTCCCCCTGCCCAGAAGGGTGCGGCCTTCTCTCCACCTCCTCCAC"
)
SUB = {"A": "C", "C": "G", "G": "T", "T": "A"}


def repeat_amplicon(La: int, seed: int) -> str:
    """Random sequence laced with homopolymers and tandem repeats (units of 2-4 bases)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    while sum(map(len, out)) < La:
        kind = int(rng.integers(0, 4))
        if kind == 0:
            out.append("".join(rng.choice(list("ACGT"), int(rng.integers(4, 12)))))
        elif kind == 1:
            out.append(str(rng.choice(list("ACGT"))) * int(rng.integers(3, 9)))
        else:
            unit = "".join(rng.choice(list("ACGT"), int(rng.integers(2, 5))))
            out.append(unit * int(rng.integers(2, 6)))
    return "".join(out)[:La]


def indel_reads(amp: str, n: int, seed: int, kmax: int = 12) -> list:
    rng = np.random.Generator(np.random.PCG64(seed))
    La = len(amp)
    reads = []
    for _ in range(n):
        k = int(rng.integers(1, kmax + 1))
        where = int(rng.integers(0, 5))
        if where == 0:     # near the start
            p = int(rng.integers(1, 8))
        elif where == 1:   # near the end
            p = La - k - int(rng.integers(1, 8))
        else:
            p = int(rng.integers(1, La - k - 1))
        p = max(1, min(p, La - k - 1))
        kind = int(rng.integers(0, 6))
        if kind <= 1:      # deletion
            r = amp[:p] + amp[p + k:]
        elif kind == 2:    # insertion of random bases
            r = amp[:p] + "".join(rng.choice(list("ACGT"), k)) + amp[p:]
        elif kind == 3:    # insertion copying the bases before p (a tandem duplication: slides)
            r = amp[:p] + amp[max(0, p - k):p].rjust(k, amp[0]) + amp[p:]
        elif kind == 4:    # insertion copying the bases after p
            r = amp[:p] + amp[p:p + k].ljust(k, amp[-1]) + amp[p:]
        else:              # deletion plus a substitution (no certificate: the DP)
            r = amp[:p] + amp[p + k:]
            q = int(rng.integers(0, len(r)))
            r = r[:q] + SUB[r[q]] + r[q + 1:]
        reads.append(r)
    return reads


def run_every_read(gpu_aligner_factory, amp: str, reads: list):
    buf, off = pack_reads(reads)
    pr = pack_2bit(buf, off)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pr)
    counts = a.path_counts()
    res = every_read(amp, buf, off, ob, threads=8)
    assert res["mismatches"] == 0, (res, counts)
    return a, pr, buf, off, counts


@pytest.mark.parametrize("La,seed", [(250, 1), (151, 7), (256, 9), (40, 3)])
def test_indel_reads_random_amplicon(gpu_aligner_factory, La, seed):
    amp = synth.random_amplicon(La, seed)
    reads = indel_reads(amp, 4000, seed + 100)
    _, _, _, _, counts = run_every_read(gpu_aligner_factory, amp, reads)
    # one-indel reads of k <= 10 (about 5 in 6 of the batch) mostly take the certificate
    assert counts["exact_copies"] > len(reads) // 2, counts


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_indel_reads_repeat_amplicon(gpu_aligner_factory, seed):
    """Homopolymers and tandem repeats: the gap slides over a range of equal placements."""
    amp = repeat_amplicon(240, seed)
    reads = indel_reads(amp, 4000, seed + 200)
    # every deletion / insertion inside each homopolymer and repeat run, 1..4 units
    for p in range(1, len(amp) - 12, 3):
        for k in (1, 2, 3, 4):
            reads.append(amp[:p] + amp[p + k:])
            reads.append(amp[:p] + amp[p:p + k] + amp[p:])
    run_every_read(gpu_aligner_factory, amp, reads)


def test_indel_reads_reference_amplicon(gpu_aligner_factory):
    """The reference's own amplicon (its CCCC / GGAGG repeats) with every deletion of 1..10 at every
    fourth position and insertions of the neighbouring bases."""
    amp = REF_AMPLICON
    reads = []
    for p in range(1, len(amp) - 11, 4):
        for k in range(1, 11):
            reads.append(amp[:p] + amp[p + k:])
            reads.append(amp[:p] + amp[p - min(p, k):p] + amp[p:])
    run_every_read(gpu_aligner_factory, amp, reads)


def test_indel_reads_c2_mix_resident(gpu_aligner_factory):
    """The C2 mix (its deletion and insertion classes) with N in some reads: the call, then a resident
    pass of the same packed batch; every read against the oracle, both times."""
    amp = synth.random_amplicon(250, 1)
    buf, off = synth.reads_from(amp, 20000, 5, synth.PARITY_MIX)
    pr = pack_2bit(buf, off)
    a = gpu_aligner_factory()
    a.set_reference(amp)
    ob = a.align_ops_packed(pr)
    assert every_read(amp, buf, off, ob, threads=8)["mismatches"] == 0
    ob2 = a.align_ops(None, pr.offsets, resident=True)
    assert every_read(amp, buf, off, ob2, threads=8)["mismatches"] == 0


def sub_reads(amp: str, n: int, seed: int, k: int = 3) -> list:
    """Reads of the amplicon's length with k substitutions: uniform, clustered (adjacent or two apart),
    near the ends, and one copying the neighbouring base (a shifted diagonal then matches locally)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    La = len(amp)
    reads = []
    for _ in range(n):
        kind = int(rng.integers(0, 5))
        if kind == 0:
            pos = sorted(rng.choice(La, k, replace=False).tolist())
        elif kind == 1:
            p = int(rng.integers(0, La - 2 * k))
            pos = [p + i * int(rng.integers(1, 3)) for i in range(k)]
        elif kind == 2:
            pos = sorted(rng.choice(list(range(4)) + list(range(La - 4, La)), k, replace=False).tolist())
        else:
            pos = sorted(rng.choice(La, k, replace=False).tolist())
        r = list(amp)
        for p in pos:
            if kind == 4 and 0 < p < La - 1 and amp[p - 1] != amp[p]:
                r[p] = amp[p - 1]   # copies its left neighbour
            else:
                r[p] = SUB[amp[p]] if rng.integers(0, 2) else {"A": "G", "C": "T", "G": "A", "T": "C"}[amp[p]]
        reads.append("".join(r))
    return reads


@pytest.mark.parametrize("maker,seed", [("random", 21), ("repeat", 22), ("repeat", 23), ("reference", 24)])
def test_three_substitution_reads(gpu_aligner_factory, maker, seed):
    """Classify's three-substitution certificate: every read against the oracle, on random,
    repeat-laced and the reference's own amplicon (jogs through a neighbouring diagonal and one-gap
    alternatives are possible there), with 2- and 4-substitution reads mixed in."""
    amp = {"random": synth.random_amplicon(250, seed), "repeat": repeat_amplicon(250, seed),
           "reference": REF_AMPLICON}[maker]
    reads = sub_reads(amp, 3000, seed) + sub_reads(amp, 500, seed + 1, 2) + sub_reads(amp, 500, seed + 2, 4)
    _, _, _, _, counts = run_every_read(gpu_aligner_factory, amp, reads)
    if maker == "random":   # most 3-substitution reads leave the DP
        assert counts["exact_copies"] > 2500, counts


def clean_indel_reads(amp: str, n: int, seed: int) -> list:
    """One deletion or one insertion of random bases, 1..10 residues, away from the ends."""
    rng = np.random.Generator(np.random.PCG64(seed))
    La = len(amp)
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 11))
        p = int(rng.integers(20, La - 30))
        if rng.integers(0, 2):
            out.append(amp[:p] + amp[p + k:])
        else:
            out.append(amp[:p] + "".join(rng.choice(list("ACGT"), k)) + amp[p:])
    return out


def test_cert_queue_layouts(gpu_aligner_factory):
    """nw_band_cert's queues ("Where the two checks run"): classify wavefronts whose 64 reads are
    all three-substitution candidates (the front of the wavefront's 64 entries full), all one-indel candidates
    (the back full), both kinds alternating, none (exact copies), a run of 1024 mixed candidates (one cert
    block's 16 wavefronts, both lists long) and a partial last wavefront -- every read against the oracle, in
    the call and in a resident pass of the same batch."""
    amp = synth.random_amplicon(250, 31)
    s3 = sub_reads(amp, 64 * 3 + 512 + 37, 32)
    ind = clean_indel_reads(amp, 64 * 3 + 512, 33)
    reads = s3[:64] + ind[:64]
    reads += [x for pair in zip(s3[64:96], ind[64:96]) for x in pair]   # alternating
    reads += [amp] * 64
    mixed = s3[192:704] + ind[192:704]
    rng = np.random.Generator(np.random.PCG64(34))
    reads += [mixed[i] for i in rng.permutation(len(mixed))]
    reads += s3[704:]   # a partial last wavefront (37 reads)
    a, pr, buf, off, counts = run_every_read(gpu_aligner_factory, amp, reads)
    # most candidates leave the DP (sub_reads' clustered and neighbour-copying reads may not)
    assert counts["exact_copies"] > 64 + 0.6 * (len(reads) - 64), counts
    res = a.align_ops(None, pr.offsets, resident=True)
    assert every_read(amp, buf, off, res, threads=8)["mismatches"] == 0
