"""The reference's own end-to-end assertions, reproduced.

tests/crispresso_tests.py:125-195 (the reference) runs CRISPResso on its
paired-end test data and asserts 14 values ("ground truth values are from the
original CRISPResso Docker": real FLASH 1.2.11 + real EMBOSS needle 6.6.0):
aligned / unmodified / NHEJ counts, the indel, insertion, deletion and
substitution histograms and the four most frequent alleles.  Those values
depend on every merged read and on the gap placement of every alignment, so
they are the one offline check of this build's alignments against EMBOSS.

tests/golden/make_e2e_golden.py ran the reference's own run_crispresso here
with `flash` = oracle/flash_oracle.py and `needle` = the CPU oracle and
recorded the FLASH-merged reads, the DataFrame its parse_needle_output built
and the 14 values: all 14 match the reference test's assertions.

Here the same merged reads go through this build's path --
crispresso_amd.needle.align_reads (CORE:1788-2000), the quantification
(CORE:2014-2067, 428-753) and crispresso_amd.quantify.run_summary
(CORE:2866-2953, 3751-3904) -- with the oracle on CPU and with the HIP kernels
on the GPU, and must give the reference's DataFrame and its 14 asserted values.
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


@pytest.fixture(scope="module")
def fixture():
    with gzip.open(os.path.join(HERE, "e2e_test_data.json.gz"), "rt") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def merged_fastq(fixture, tmp_path_factory):
    p = tmp_path_factory.mktemp("e2e") / "out.extendedFrags.fastq.gz"
    with gzip.open(p, "wt") as f:
        for name, seq in fixture["merged_reads"]:
            f.write(f"@{name}\n{seq}\n+\n{'I' * len(seq)}\n")
    return str(p)


def quant_args(fx):
    """The run's CRISPResso args (reference defaults, CORE:3995-4284; guides of the test)."""
    return types.SimpleNamespace(
        amplicon_seq=fx["amplicon_seq"].upper(), guide_seq=fx["guide_seq"], cleavage_offset=-3,
        window_around_sgrna=1, exclude_bp_from_left=15, exclude_bp_from_right=15, coding_seq=None,
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
    e = dict(fx["expected_by_reference_test"])
    e.pop("n_reads_input")     # FASTQ record count of R1 (8906), upstream of the merge
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


def test_fixture_records_a_match(fixture):
    """The generator's own verdict: the reference's pipeline, fed by the two
    restatements, reproduced every asserted value."""
    assert fixture["mismatches"] == {}
    assert fixture["reference_aggregates"]["n_total"] == fixture["expected_by_reference_test"]["n_total"]
    assert len(fixture["merged_reads"]) == fixture["n_reads_after_preprocessing"] == 8092


def test_e2e_pin_oracle_backend(fixture, merged_fastq):
    """CPU: this build's host path over the oracle aligner and the quantification
    restatement reproduces the reference's DataFrame and its 14 asserted values."""
    from oracle import quant_oracle as qo
    from tests.helpers import OracleAligner

    args = quant_args(fixture)
    df = align_reads(AlignArgs(amplicon_seq=fixture["amplicon_seq"]), merged_fastq, aligner=OracleAligner())
    check_rows(df, fixture)
    amp = args.amplicon_seq
    cuts = qo.cut_points(amp, args.guide_seq)
    prm = qo.QuantParams(len_amplicon=len(amp), include_idxs=frozenset(qo.include_idxs(len(amp), cuts, 1, 15, 15)))
    um = (df["score_ref"] == 100).to_numpy()
    res = qo.process_rows(df["ref_seq"].tolist(), df["align_str"].tolist(), df["align_seq"].tolist(), um,
                          None, None, prm)
    for k, v in qo.class_flags(res["cls"], um).items():
        df[k] = v
    for k in ("n_mutated", "n_inserted", "n_deleted"):
        df[k] = np.where(res["cls"] == 0, 0, res[k])
    assert summary_values(quantify.run_summary(df, len(amp), cuts)) == expected(fixture)


@pytest.mark.gpu
def test_e2e_pin_gpu(fixture, merged_fastq, gpu_aligner_factory):
    """GPU: HIP aligner + HIP quantification give the reference's DataFrame and
    its 14 asserted values."""
    args = quant_args(fixture)
    df = align_reads(AlignArgs(amplicon_seq=fixture["amplicon_seq"]), merged_fastq, aligner=gpu_aligner_factory())
    check_rows(df, fixture)
    g = quantify.globals_from_args(args)
    quantify.quantify_alignments(df, args, globals_=g)
    cuts = quantify.compute_cut_points(args.amplicon_seq, args.guide_seq)
    assert summary_values(quantify.run_summary(df, g.LEN_AMPLICON, cuts)) == expected(fixture)


@pytest.mark.skipif(not os.path.isdir(REF_TEST_DATA), reason="needs the reference's test data (this container only)")
def test_flash_restatement_reproduces_fixture(fixture, tmp_path):
    """The merged reads in the fixture are what oracle/flash_oracle.py makes of
    the reference's test pairs with CRISPResso's FLASH options (CORE:1655-1664)."""
    from oracle import flash_oracle

    st = flash_oracle.run_flash(os.path.join(REF_TEST_DATA, "test_L001_R1_001.fastq.gz"),
                                os.path.join(REF_TEST_DATA, "test_L001_R2_001.fastq.gz"), str(tmp_path),
                                min_overlap=4, max_overlap=100, allow_outies=True)
    assert st["pairs"] == 8906 and st["combined"] == len(fixture["merged_reads"])
    got = [(n, s) for n, s, _ in flash_oracle.read_fastq(str(tmp_path / "out.extendedFrags.fastq.gz"))]
    assert [tuple(x) for x in fixture["merged_reads"]] == [(n, s.decode()) for n, s in got]


@pytest.mark.gpu
def test_e2e_pin_gpu_from_raw_pairs(fixture, tmp_path, gpu_aligner_factory):
    """The reference's pinned paired-end run (tests/crispresso_tests.py:131-195) from the raw
    reads, every stage on the GPU: the FLASH merge (CORE:1655-1677) of
    tests/golden/test_L001_R{1,2}_001.fastq.gz (the reference's own test data) with
    CRISPResso's options, the alignment of the merged reads (CORE:1788-2000), the
    quantification (CORE:2014-2067, 428-753) and the summary: the 14 asserted values."""
    from crispresso_amd.flash import FlashOptions, run_flash

    st = run_flash(os.path.join(HERE, "test_L001_R1_001.fastq.gz"), os.path.join(HERE, "test_L001_R2_001.fastq.gz"),
                   str(tmp_path), options=FlashOptions(min_overlap=4, max_overlap=100, allow_outies=True))
    assert st["pairs"] == 8906 and st["combined"] == len(fixture["merged_reads"]) == 8092
    merged = str(tmp_path / "out.extendedFrags.fastq.gz")
    args = quant_args(fixture)
    df = align_reads(AlignArgs(amplicon_seq=fixture["amplicon_seq"]), merged, aligner=gpu_aligner_factory())
    check_rows(df, fixture)
    g = quantify.globals_from_args(args)
    quantify.quantify_alignments(df, args, globals_=g)
    cuts = quantify.compute_cut_points(args.amplicon_seq, args.guide_seq)
    assert summary_values(quantify.run_summary(df, g.LEN_AMPLICON, cuts)) == expected(fixture)
