"""CPU restatement of classify's three-substitution certificate, checked against the
oracle: every read the checks accept must be aligned by the oracle as the main diagonal with its three
mismatches (record La, La - 3, La - 3, 0, D at the corner).  The kernel runs the same checks (a more
conservative jog test: one 16-base word after f) and tests/test_gpu_indel.py holds it to the oracle on
every read; this model pins the argument itself on CPU, on random, repeat-laced, tandem-repeat and the
reference's amplicons with substitutions chosen to open jogs and one-gap splits."""
import numpy as np

from crispresso_amd import synth
from oracle import oracle_py

M, X, O, E = 10, 8, 20, 1   # EDNAFULL 5 / -4, gapopen 10, gapextend 0.5, scaled by 2
D3 = 3 * (M + X)
SUB = {"A": "C", "C": "G", "G": "T", "T": "A"}


def diag_info(amp, r, d):
    La = len(amp)
    pos = [j for j in range(La) if 0 <= j - d < La and r[j] != amp[j - d]]
    f1 = pos[0] if pos else La
    f2 = pos[1] if len(pos) > 1 else La
    g1 = pos[-1] + 1 if pos else 0
    g2 = pos[-2] + 1 if len(pos) > 1 else 0
    return min(len(pos), 3), f1, f2, g1, g2, pos


def certified(amp, r):
    La = len(amp)
    if len(r) != La:
        return False
    info = {d: diag_info(amp, r, d) for d in range(-5, 6)}
    pos0 = info[0][5]
    if len(pos0) != 3:
        return False
    f, l = pos0[0], pos0[-1]
    for d in range(-5, 6):
        if d and not M * abs(d) + (M + X) * info[d][0] > D3:
            return False
    for d1 in range(-3, 4):
        for d2 in range(-3, 4):
            if d1 == d2:
                continue
            g = abs(d2 - d1)
            U = (-d1 if d1 < 0 else 0) + (d2 if d2 > 0 else 0) + (d1 - d2 if d1 > d2 else 0)
            slack = D3 - M * U - O - (g - 1) * E
            if slack < 0:
                continue
            wmax = slack // (M + X)
            gb = max(0, d2 - d1)
            a1, a2 = info[d1][1], info[d1][2]
            b1, b2 = info[d2][3], info[d2][4]
            exists = b1 - gb <= a1 or (wmax >= 1 and (b2 - gb <= a1 or b1 - gb <= a2)) or wmax >= 2
            if exists:
                return False
    if l - f < 2:
        return False
    return all(any(f + 1 <= p <= l - 1 for p in info[d][5]) for d in (-1, 1))


def three_sub_reads(amp, n, rng):
    La = len(amp)
    out = []
    for _ in range(n):
        r = list(amp)
        for p in sorted(rng.choice(La, 3, replace=False)):
            if 0 < p and amp[p - 1] != amp[p] and rng.integers(0, 2):
                r[p] = amp[p - 1]        # copies its neighbour: a shifted diagonal matches locally
            elif p < La - 1 and amp[p + 1] != amp[p] and rng.integers(0, 2):
                r[p] = amp[p + 1]
            else:
                r[p] = SUB[amp[p]]
        out.append("".join(r))
    return out


def test_three_substitution_certificate_model_against_oracle():
    rng = np.random.Generator(np.random.PCG64(5))
    amps = [synth.random_amplicon(120, 3)]
    for _ in range(6):   # tandem repeats and homopolymers in random flanks
        unit = "".join(rng.choice(list("ACGT"), int(rng.integers(1, 4))))
        amps.append("".join(rng.choice(list("ACGT"), 25)) + unit * int(rng.integers(5, 15)) +
                    "".join(rng.choice(list("ACGT"), 25)))
    accepted = bad = 0
    for amp in amps:
        sel = [r for r in three_sub_reads(amp, 150, rng) if certified(amp, r)]
        accepted += len(sel)
        if not sel:
            continue
        buf = np.frombuffer("".join(sel).encode(), np.uint8)
        off = np.zeros(len(sel) + 1, np.int64)
        off[1:] = np.cumsum([len(s) for s in sel])
        res, _ = oracle_py.align_batch(amp, buf, off, nthreads=4)
        La = len(amp)
        ok = ((res["aln_len"] == La) & (res["n_ident"] == La - 3) & (res["n_gaps"] == 0) &
              (res["score"] == M * La - D3) & (res["end_i"] == La) & (res["end_j"] == La))
        bad += int((~ok).sum())
    assert accepted > 300
    assert bad == 0
