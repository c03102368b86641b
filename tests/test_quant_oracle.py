"""The quantification oracle (oracle/quant_oracle.py) against the reference's
own process_df_chunk outputs (tests/golden/quant_*.json.gz, make_quant_golden.py)
and against the end-to-end captures of make_golden.py."""
from __future__ import annotations

import gzip
import json
import math
import os

import numpy as np
import pytest

from oracle import quant_oracle as qo

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
QUANT_SETS = ("quant_a200", "quant_n180")


def load(name):
    with gzip.open(os.path.join(GOLDEN, f"{name}.json.gz"), "rt") as f:
        return json.load(f)


def params_from(case, amp):
    p = case["params"]
    g = case["globals"]
    return qo.QuantParams(
        len_amplicon=len(amp), include_idxs=frozenset(g["INCLUDE_IDXS"]),
        exon_positions=None if g["EXON_POSITIONS"] is None else frozenset(g["EXON_POSITIONS"]),
        splicing_positions=None if g["SPLICING_POSITIONS"] is None else frozenset(g["SPLICING_POSITIONS"]),
        ignore_substitutions=p["ignore_substitutions"], ignore_insertions=p["ignore_insertions"],
        ignore_deletions=p["ignore_deletions"], window_around_sgrna=p["window_around_sgrna"],
        hide_mutations_outside_window_NHEJ=p["hide_mutations_outside_window_NHEJ"],
        expected_hdr=p["expected_hdr"], hdr_perfect_alignment_threshold=p["hdr_perfect_alignment_threshold"])


def golden_cases():
    for name in QUANT_SETS:
        rec = load(name)
        for cname in rec["cases"]:
            yield name, cname


def case_inputs(rec, case):
    rows = rec["rows"]
    sr = np.array([math.nan if x is None else x for x in rec["score_repaired"]])
    score = np.array([r["score_ref"] for r in rows])
    return ([r["ref_seq"] for r in rows], case["rows_in"]["align_str"], [r["align_seq"] for r in rows],
            case["rows_in"]["UNMODIFIED"], score - sr, sr)


def check_against_case(out, case, unmodified_in):
    flags = qo.class_flags(out["cls"], unmodified_in)
    for k in ("UNMODIFIED", "NHEJ", "HDR", "MIXED"):
        assert flags[k].astype(int).tolist() == case["rows_out"][k], k
    for k in ("n_mutated", "n_inserted", "n_deleted"):
        assert out[k].tolist() == case["rows_out"][k], k
    for k in qo.VECTORS:
        assert out["vectors"][k].astype(float).tolist() == case["vectors"][k], k
    assert sorted(map(list, out["hist_inframe"].items())) == case["hist_inframe"]
    assert sorted(map(list, out["hist_frameshift"].items())) == case["hist_frameshift"]
    assert out["counters"] == case["counters"]


@pytest.mark.parametrize("name,cname", list(golden_cases()))
def test_oracle_matches_reference_process_df_chunk(name, cname):
    rec = load(name)
    case = rec["cases"][cname]
    prm = params_from(case, rec["amplicon"])
    R, M, S, um, sd, sr = case_inputs(rec, case)
    out = qo.process_rows(R, M, S, um, sd, sr, prm)
    check_against_case(out, case, um)


@pytest.mark.parametrize("name", QUANT_SETS)
def test_globals_and_n_rule(name):
    rec = load(name)
    amp = rec["amplicon"]
    for cname, case in rec["cases"].items():
        p = case["params"]
        cuts = qo.cut_points(amp, p["guide_seq"], p["cleavage_offset"])
        assert cuts == case["globals"]["cut_points"]
    case = rec["cases"]["defaults"]
    for r, mk, um in zip(rec["rows"], case["rows_in"]["align_str"], case["rows_in"]["UNMODIFIED"]):
        m2, u2 = (qo.ignore_n_in_alignment(r["ref_seq"], r["align_str"], r["score_ref"] == 100)
                  if "N" in amp else (r["align_str"], r["score_ref"] == 100))
        assert (m2, u2) == (mk, um)


def test_ref_positions_quirks():
    assert qo.compute_ref_positions("--AC-G--") == [-1, -1, 0, 1, -2, 2, -3, -3]
    assert qo.include_idxs(10, [4], 1, 0, 0) == frozenset({4, 5})
    assert qo.include_idxs(10, [], 1, 2, 3) == frozenset(range(2, 7))


def test_e2e_captures_consistent_with_oracle():
    """make_golden.py's end-to-end captures: the DataFrame the reference handed to
    process_df_chunk and the aggregates it returned (no guides: INCLUDE_IDXS is
    range(LEN) minus 15 bp each side, CORE:2740-2762)."""
    for name in ("c1_plumbing", "syn_rc", "syn_hdr"):
        rec = load(name)
        if "quantification" not in rec:
            continue
        amp = rec["inputs"]["amplicon_seq"].upper()
        rows = rec["df_needle_alignment"]
        hdr = "--expected_hdr_amplicon_seq" in rec["inputs"]["extra_args"]
        prm = qo.QuantParams(len_amplicon=len(amp), include_idxs=qo.include_idxs(len(amp), [], 1, 15, 15),
                             expected_hdr=hdr)
        um = [r["score_ref"] == 100 for r in rows]
        nanv = lambda x: math.nan if x is None else x  # noqa: E731
        sd = [nanv(r.get("score_diff")) for r in rows]
        sr = [nanv(r.get("score_repaired")) for r in rows]
        out = qo.process_rows([r["ref_seq"] for r in rows], [r["align_str"] for r in rows],
                              [r["align_seq"] for r in rows], um, sd, sr, prm)
        q = rec["quantification"]
        flags = qo.class_flags(out["cls"], um)
        assert int(flags["UNMODIFIED"].sum()) == q["n_unmodified"], name
        assert int(flags["NHEJ"].sum()) == q["n_nhej"], name
        assert int(flags["HDR"].sum()) == q["n_hdr"], name
        assert int(flags["MIXED"].sum()) == q["n_mixed"], name
        for k in ("effect_vector_insertion", "effect_vector_deletion", "effect_vector_mutation",
                  "effect_vector_any"):
            assert out["vectors"][k].astype(float).tolist() == q[k], (name, k)
