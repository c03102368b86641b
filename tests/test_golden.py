"""Golden fixtures produced by the reference's own run_crispresso (tests/golden/make_golden.py).

Each case pins the whole alignment block of CRISPRessoCORE.py:1788-2000 as the
reference executes it -- FASTQ->FASTA shell stage, needle text output read by
its parse_needle_output, the HDR join, the min_identity_score filters, the
reverse-complement retry with its quirks -- against crispresso_amd.needle.align_reads.
The CPU test drives align_reads with the oracle-backed aligner (the same
arithmetic the fixtures were made with); the GPU test drives it with the HIP
aligner, which must give the identical DataFrame.
"""
import gzip
import json
import math
import os

import pytest

from crispresso_amd.needle import AlignArgs, align_reads

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["c1_plumbing", "syn_rc", "syn_hdr", "syn_hdr_rcfail"]


def load(case):
    with gzip.open(os.path.join(HERE, f"{case}.json.gz"), "rt") as f:
        return json.load(f)


def args_for(rec):
    inp = rec["inputs"]
    a = AlignArgs(amplicon_seq=inp["amplicon_seq"])
    extra = inp["extra_args"]
    for k in range(0, len(extra), 2):
        if extra[k] == "--min_identity_score":
            a.min_identity_score = float(extra[k + 1])
        elif extra[k] == "--expected_hdr_amplicon_seq":
            a.expected_hdr_amplicon_seq = extra[k + 1]
    return a


def same(a, b):
    if isinstance(a, float) and math.isnan(a):
        return b is None
    return a == b


def check(case, aligner):
    rec = load(case)
    df = align_reads(args_for(rec), os.path.join(HERE, rec["inputs"]["fastq"]), aligner=aligner)
    rows = rec["df_needle_alignment"]
    assert list(df.index) == [r["ID"] for r in rows]
    cols = ["score_ref", "length", "ref_seq", "align_str", "align_seq"]
    if "score_repaired" in rows[0]:
        cols += ["score_repaired", "score_diff"]
    assert list(df.columns) == cols
    # the dtypes CORE:1998's pd.concat gives the reference (pandas 2.x: all-NA repair scores
    # of the RC-HDR quirk do not turn the column into object)
    for c in ("score_ref", "score_repaired", "score_diff"):
        if c in cols:
            assert str(df[c].dtype) == "float64", (case, c, df[c].dtype)
    for (idx, got), want in zip(df.iterrows(), rows):
        for c in cols:
            assert same(got[c], want[c]), (case, idx, c, got[c], want[c])


@pytest.mark.parametrize("case", CASES)
def test_golden_with_oracle_backend(case):
    from tests.helpers import OracleAligner

    check(case, OracleAligner())


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_golden_on_gpu(case, gpu_aligner_factory):
    check(case, gpu_aligner_factory())


def test_fixture_sanity():
    rc = load("syn_rc")
    assert any(r["ID"].endswith("_RC") for r in rc["df_needle_alignment"])
    fail = load("syn_hdr_rcfail")
    rc_rows = [r for r in fail["df_needle_alignment"] if r["ID"].endswith("_RC")]
    assert rc_rows and all(r["score_repaired"] is None for r in rc_rows)
    c1 = load("c1_plumbing")
    assert c1["exception"] is None and len(c1["df_needle_alignment"]) > 1500
