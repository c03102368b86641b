"""The reference's own end-to-end assertions, reproduced.

tests/crispresso_tests.py (the reference) runs CRISPResso on its paired-end test data twice and
asserts 14 values each time ("ground truth values are from the original CRISPResso Docker": real
Trimmomatic 0.33 + FLASH 1.2.11 + EMBOSS needle 6.6.0): aligned / unmodified / NHEJ counts, the
indel, insertion, deletion and substitution histograms and the four most frequent alleles.  Those
values depend on every merged read and on the gap placement of every alignment, so they are the
offline check of this build's alignments against EMBOSS.

* ``test`` (crispresso_tests.py:125-195): test_L001, 7,058 aligned reads, almost no indels.
* ``test1`` (crispresso_tests.py:198-272): test1_L001 with --trim_sequences (Trimmomatic
  ILLUMINACLIP/MINLEN), --min_identity_score 30, --window_around_sgrna 23: 4,039 aligned reads,
  680 NHEJ deletions and 49 insertions -- the reference's only record of EMBOSS gap placement on
  indel-rich reads.  It pinned the X-vs-Y traceback tie.

tests/golden/make_e2e_golden.py ran the reference's own run_crispresso here with `java` =
oracle/trimmomatic_oracle.py, `flash` = oracle/flash_oracle.py and `needle` = the CPU oracle and
recorded the merged reads, the DataFrame its parse_needle_output built and the 14 values: all 14
match for ``test``; for ``test1`` 9 match and the other 5 (n_total, n_modified and the three NHEJ
counts) are each exactly one short -- one modified read (with insertions, deletions and
substitutions) that the Trimmomatic / FLASH restatements do not produce; no tie rule of the
aligner changes them.

Here the same merged reads go through this build's path -- crispresso_amd.needle.align_reads
(CORE:1788-2000), the quantification (CORE:2014-2067, 428-753) and
crispresso_amd.quantify.run_summary (CORE:2866-2953, 3751-3904) -- with the oracle on CPU and with
the HIP kernels on the GPU, and must give the reference's DataFrame and its values.
"""
import gzip
import json
import os
import types

import numpy as np
import pytest

from crispresso_amd import quantify
from crispresso_amd.needle import AlignArgs, align_reads

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_TEST_DATA = "/root/reference/tests/test_data"

CASES = {
    "test": dict(fixture="e2e_test_data.json.gz", prefix="test", window=1, min_identity=60.0, pairs=8906,
                 merged=8092, trim=None, known_upstream={}),
    # CORE:4113-4117 (the default --trimmomatic_options_string), with the adapters as a fixture
    "test1": dict(fixture="e2e_test1_data.json.gz", prefix="test1", window=23, min_identity=30.0, pairs=4941,
                  merged=4093, trim=["ILLUMINACLIP:" + os.path.join(HERE, "NexteraPE-PE.fa") + ":0:90:10:0:true",
                                     "MINLEN:40"],
                  known_upstream={"n_total": (4038, 4039), "n_modified": (1391, 1392), "nhej_inserted": (48, 49),
                                  "nhej_deleted": (679, 680), "nhej_mutated": (889, 890)}),
}


@pytest.fixture(scope="module", params=sorted(CASES))
def case(request):
    c = dict(CASES[request.param], name=request.param)
    with gzip.open(os.path.join(HERE, c["fixture"]), "rt") as f:
        c["fx"] = json.load(f)
    return c


@pytest.fixture(scope="module")
def fixture(case):
    return case["fx"]


@pytest.fixture(scope="module")
def merged_fastq(case, tmp_path_factory):
    p = tmp_path_factory.mktemp("e2e_" + case["name"]) / "out.extendedFrags.fastq.gz"
    with gzip.open(p, "wt") as f:
        for name, seq in case["fx"]["merged_reads"]:
            f.write(f"@{name}\n{seq}\n+\n{'I' * len(seq)}\n")
    return str(p)


def quant_args(fx, case):
    """The run's CRISPResso args (reference defaults, CORE:3995-4284; the test's guides and window)."""
    return types.SimpleNamespace(
        amplicon_seq=fx["amplicon_seq"].upper(), guide_seq=fx["guide_seq"], cleavage_offset=-3,
        window_around_sgrna=case["window"], exclude_bp_from_left=15, exclude_bp_from_right=15, coding_seq=None,
        ignore_substitutions=False, ignore_insertions=False, ignore_deletions=False,
        hide_mutations_outside_window_NHEJ=False, expected_hdr_amplicon_seq=None,
        hdr_perfect_alignment_threshold=98.0)


def summary_values(s):
    return {
        "n_total": s["n_total"], "n_unmodified": s["n_unmodified"], "n_mixed_hdr_nhej": s["n_mixed_hdr_nhej"],
        "n_modified": s["n_modified"], "n_repaired": s["n_repaired"], "nhej_inserted": s["nhej_inserted"],
        "nhej_deleted": s["nhej_deleted"], "nhej_mutated": s["nhej_mutated"],
        "df_indels_fq4": [int(x) for x in s["df_indels"]["fq"].values[:4]],
        "df_insertion_fq4": [int(x) for x in s["df_insertion"]["fq"].values[:4]],
        "df_deletion_fq4": [int(x) for x in s["df_deletion"]["fq"].values[:4]],
        "df_substitution_fq4": [int(x) for x in s["df_substitution"]["fq"].values[:4]],
        "df_alleles_reads4": [int(x) for x in s["df_alleles"]["#Reads"].values[:4]],
    }


def expected(fx):
    """The values the reference's pipeline gave on the fixture's merged reads (== the reference test's
    assertions except the known upstream differences, checked in test_fixture_records_a_match)."""
    e = dict(fx["reference_aggregates"])
    e.pop("n_reads_input")     # FASTQ record count of R1, upstream of the merge
    return e


def check_rows(df, fx):
    rows = fx["df_needle_alignment"]
    assert df.shape[0] == len(rows)
    assert list(df.index) == [r["ID"] for r in rows]
    for c in ("ref_seq", "align_str", "align_seq", "length"):
        got = df[c].tolist()
        want = [r[c] for r in rows]
        bad = [i for i in range(len(rows)) if got[i] != want[i]]
        assert not bad, (c, len(bad), rows[bad[0]]["ID"])
    np.testing.assert_array_equal(df["score_ref"].to_numpy(), np.array([r["score_ref"] for r in rows]))


def test_fixture_records_a_match(case):
    """The generator's own verdict: the reference's pipeline, fed by the restatements, reproduced
    every asserted value (test1: all but one read's worth, listed in known_upstream)."""
    fx = case["fx"]
    assert {k: tuple(v) for k, v in fx["mismatches"].items()} == case["known_upstream"]
    assert len(fx["merged_reads"]) == fx["n_reads_after_preprocessing"] == case["merged"]
    agg, want = fx["reference_aggregates"], fx["expected_by_reference_test"]
    matched = [k for k in want if agg[k] == want[k]]
    assert len(matched) == 14 - len(case["known_upstream"])


def test_e2e_pin_oracle_backend(case, merged_fastq):
    """CPU: this build's host path over the oracle aligner and the quantification
    restatement reproduces the reference's DataFrame and its asserted values."""
    from oracle import quant_oracle as qo
    from tests.helpers import OracleAligner

    fixture = case["fx"]
    args = quant_args(fixture, case)
    df = align_reads(AlignArgs(amplicon_seq=fixture["amplicon_seq"], min_identity_score=case["min_identity"]),
                     merged_fastq, aligner=OracleAligner())
    check_rows(df, fixture)
    amp = args.amplicon_seq
    cuts = qo.cut_points(amp, args.guide_seq)
    prm = qo.QuantParams(len_amplicon=len(amp),
                         include_idxs=frozenset(qo.include_idxs(len(amp), cuts, case["window"], 15, 15)))
    um = (df["score_ref"] == 100).to_numpy()
    res = qo.process_rows(df["ref_seq"].tolist(), df["align_str"].tolist(), df["align_seq"].tolist(), um,
                          None, None, prm)
    for k, v in qo.class_flags(res["cls"], um).items():
        df[k] = v
    for k in ("n_mutated", "n_inserted", "n_deleted"):
        df[k] = np.where(res["cls"] == 0, 0, res[k])
    assert summary_values(quantify.run_summary(df, len(amp), cuts)) == expected(fixture)


def gpu_summary(case, merged, aligner):
    fixture = case["fx"]
    args = quant_args(fixture, case)
    df = align_reads(AlignArgs(amplicon_seq=fixture["amplicon_seq"], min_identity_score=case["min_identity"]),
                     merged, aligner=aligner)
    check_rows(df, fixture)
    g = quantify.globals_from_args(args)
    quantify.quantify_alignments(df, args, globals_=g)
    cuts = quantify.compute_cut_points(args.amplicon_seq, args.guide_seq)
    return summary_values(quantify.run_summary(df, g.LEN_AMPLICON, cuts))


@pytest.mark.gpu
def test_e2e_pin_gpu(case, merged_fastq, gpu_aligner_factory):
    """GPU: HIP aligner + HIP quantification give the reference's DataFrame and
    its asserted values."""
    assert gpu_summary(case, merged_fastq, gpu_aligner_factory()) == expected(case["fx"])


@pytest.mark.skipif(not os.path.isdir(REF_TEST_DATA), reason="needs the reference's test data (this container only)")
def test_golden_inputs_are_the_references(case):
    """tests/golden/<prefix>_L001_R{1,2}_001.fastq.gz are the reference's own test data, byte for byte."""
    for r in (1, 2):
        name = f"{case['prefix']}_L001_R{r}_001.fastq.gz"
        with open(os.path.join(HERE, name), "rb") as a, open(os.path.join(REF_TEST_DATA, name), "rb") as b:
            assert a.read() == b.read()


def restated_merge(case, tmp_path):
    """Trimmomatic (test1) and FLASH restatements over the golden raw pairs (CORE:1620-1677)."""
    from oracle import flash_oracle, trimmomatic_oracle

    r1 = os.path.join(HERE, f"{case['prefix']}_L001_R1_001.fastq.gz")
    r2 = os.path.join(HERE, f"{case['prefix']}_L001_R2_001.fastq.gz")
    if case["trim"]:
        outs = [str(tmp_path / f"{n}.fq.gz") for n in ("fp", "fu", "rp", "ru")]
        st = trimmomatic_oracle.run_pe(r1, r2, outs, case["trim"])
        assert st["pairs"] == case["pairs"]
        r1, r2 = outs[0], outs[2]
    return r1, r2


def test_merge_restatements_reproduce_fixture(case, tmp_path):
    """The merged reads in the fixture are what the restatements make of the reference's test
    pairs with CRISPResso's options (CORE:1620-1640, 1655-1664)."""
    from oracle import flash_oracle

    r1, r2 = restated_merge(case, tmp_path)
    out = tmp_path / "flash"
    st = flash_oracle.run_flash(r1, r2, str(out), min_overlap=4, max_overlap=100, allow_outies=True)
    assert st["combined"] == len(case["fx"]["merged_reads"]) == case["merged"]
    got = [(n, s) for n, s, _ in flash_oracle.read_fastq(str(out / "out.extendedFrags.fastq.gz"))]
    assert [tuple(x) for x in case["fx"]["merged_reads"]] == [(n, s.decode()) for n, s in got]


@pytest.mark.gpu
def test_e2e_pin_gpu_from_raw_pairs(case, tmp_path, gpu_aligner_factory):
    """The reference's pinned paired-end runs from the raw reads: (test1: the Trimmomatic
    restatement, test infrastructure) the FLASH merge on the GPU (CORE:1655-1677) with
    CRISPResso's options, the alignment of the merged reads (CORE:1788-2000), the
    quantification (CORE:2014-2067, 428-753) and the summary: the asserted values."""
    from crispresso_amd.flash import FlashOptions, run_flash

    r1, r2 = restated_merge(case, tmp_path)
    st = run_flash(r1, r2, str(tmp_path), options=FlashOptions(min_overlap=4, max_overlap=100, allow_outies=True))
    assert st["combined"] == len(case["fx"]["merged_reads"]) == case["merged"]
    merged = str(tmp_path / "out.extendedFrags.fastq.gz")
    assert gpu_summary(case, merged, gpu_aligner_factory()) == expected(case["fx"])
