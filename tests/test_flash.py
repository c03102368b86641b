"""GPU paired-end merge (crispresso_amd/flash.py, csrc/flash_merge.hip) against the
FLASH 1.2.11 restatement (oracle/flash_oracle.py) on the reference's own paired-end
test reads (tests/golden/flash_pairs.json.gz, made by make_flash_golden.py) and on
seeded synthetic pairs (innies, outies, N / lowercase bases, unequal lengths)."""
import gzip
import json
import os
import sys

import numpy as np
import pytest

from crispresso_amd import _lib
from crispresso_amd.flash import FlashError, FlashOptions, merge_pairs, run_flash

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import flash_oracle  # noqa: E402

GOLDEN = os.path.join(HERE, "golden", "flash_pairs.json.gz")


def load_golden():
    with gzip.open(GOLDEN, "rt") as f:
        return json.load(f)


def test_flash_symbols_exported():
    syms = _lib.exported_symbols()
    assert all(syms[s] for s in _lib.FLASH_EXPORTS)


def test_flash_header_declares_the_exports():
    with open(os.path.join(os.path.dirname(HERE), "include", "crispr_flash.h")) as f:
        text = f.read()
    for s in _lib.FLASH_EXPORTS:
        assert f" {s}(" in text


def test_max_overlap_default_formula():
    # FLASH: -M = 2r - f + 2.5 s when not given
    assert FlashOptions.max_overlap_for(150, 250, 25) == 112


def test_mismatched_inputs_raise():
    with pytest.raises(FlashError):
        merge_pairs([b"ACGT"], [b"III"], [b"ACGT"], [b"IIII"])


def test_golden_is_the_oracle():
    """The fixture's expected merges are what the restatement computes (first 100 pairs)."""
    g = load_golden()
    for name, e in g["expected"].items():
        m = flash_oracle.Merger(**e["options"])
        for (s1, q1, s2, q2), exp in list(zip(g["pairs"], e["merged"]))[:100]:
            res = m.merge_pair(s1.encode(), q1.encode(), s2.encode(), q2.encode())
            got = None if res is None else [res[0].decode(), res[1].decode(), bool(res[2])]
            assert got == exp, name


def synth_pairs(n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    s1, q1, s2, q2 = [], [], [], []
    comp = bytes.maketrans(b"ACGTN", b"TGCAN")
    for k in range(n):
        frag_len = int(rng.integers(40, 320))
        frag = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), frag_len))
        la, lb = int(rng.integers(20, 160)), int(rng.integers(20, 160))
        r1 = bytearray(frag[:la])
        r2 = bytearray(frag[::-1].translate(comp)[:lb])
        if k % 5 == 1:   # reads run past a short fragment into adapter: an outie
            frag = frag[:int(rng.integers(25, 60))]
            r1 = bytearray(frag + bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), int(rng.integers(5, 40)))))
            r2 = bytearray(frag[::-1].translate(comp) + bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8),
                                                                         int(rng.integers(5, 40)))))
        for r in (r1, r2):   # sequencing errors, N, lowercase
            for _ in range(int(rng.integers(0, 4))):
                if len(r):
                    r[int(rng.integers(0, len(r)))] = b"ACGTNacgtn"[int(rng.integers(0, 10))]
        if k % 7 == 0:   # unrelated mates
            r2 = bytearray(rng.choice(np.frombuffer(b"ACGT", np.uint8), lb))
        s1.append(bytes(r1))
        s2.append(bytes(r2))
        q1.append(bytes(rng.integers(35, 75, len(r1)).astype(np.uint8)))
        q2.append(bytes(rng.integers(35, 75, len(r2)).astype(np.uint8)))
    return s1, q1, s2, q2


@pytest.mark.gpu
@pytest.mark.parametrize("setting", ["crispresso", "flash_defaults"])
def test_gpu_merge_matches_golden(setting):
    g = load_golden()
    e = g["expected"][setting]
    pairs = g["pairs"]
    opts = FlashOptions(**e["options"])
    res = merge_pairs([p[0].encode() for p in pairs], [p[1].encode() for p in pairs],
                      [p[2].encode() for p in pairs], [p[3].encode() for p in pairs], opts)
    for i, exp in enumerate(e["merged"]):
        got = res.merged(i)
        got = None if got is None else [got[0].decode(), got[1].decode(), got[2]]
        assert got == exp, f"{setting} pair {i}"


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(min_overlap=4, max_overlap=100, allow_outies=True),
                                dict(min_overlap=10, max_overlap=65, allow_outies=False),
                                dict(min_overlap=6, max_overlap=30, allow_outies=True, cap_mismatch_quals=True,
                                     max_mismatch_density=0.1)])
def test_gpu_merge_matches_oracle_synthetic(kw):
    s1, q1, s2, q2 = synth_pairs(600, 11)
    res = merge_pairs(s1, q1, s2, q2, FlashOptions(**kw))
    m = flash_oracle.Merger(**kw)
    n_comb = n_out = 0
    for i in range(len(s1)):
        exp = m.merge_pair(s1[i], q1[i], s2[i], q2[i])
        got = res.merged(i)
        assert got == exp, f"pair {i}"
        n_comb += exp is not None
        n_out += exp is not None and exp[2]
    assert n_comb > 150
    if kw.get("allow_outies"):
        assert n_out > 10


@pytest.mark.gpu
def test_gpu_run_flash_files_match_oracle(tmp_path):
    s1, q1, s2, q2 = synth_pairs(300, 5)
    for name, seqs, quals in (("r1.fastq", s1, q1), ("r2.fastq", s2, q2)):
        with open(tmp_path / name, "wb") as f:
            for i, (s, q) in enumerate(zip(seqs, quals)):
                f.write(b"@read%d/%s\n%s\n+\n%s\n" % (i, name[1].encode(), s, q))
    kw = dict(min_overlap=4, max_overlap=100, allow_outies=True)
    st_gpu = run_flash(str(tmp_path / "r1.fastq"), str(tmp_path / "r2.fastq"), str(tmp_path / "gpu"),
                       options=FlashOptions(**kw))
    st_cpu = flash_oracle.run_flash(str(tmp_path / "r1.fastq"), str(tmp_path / "r2.fastq"), str(tmp_path / "cpu"),
                                    **kw)
    assert st_gpu == st_cpu
    for fn in ("out.extendedFrags.fastq.gz", "out.notCombined_1.fastq.gz", "out.notCombined_2.fastq.gz"):
        with gzip.open(tmp_path / "gpu" / fn) as a, gzip.open(tmp_path / "cpu" / fn) as b:
            assert a.read() == b.read(), fn
    for fn in ("out.hist", "out.histogram"):
        assert (tmp_path / "gpu" / fn).read_text() == (tmp_path / "cpu" / fn).read_text()
