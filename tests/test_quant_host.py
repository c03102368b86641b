"""Host-side logic of crispresso_amd.quantify (no GPU): the run_crispresso globals
against the reference's values recorded in the golden fixtures, packing, input
flags, and the C ABI symbols."""
from __future__ import annotations

import math

import numpy as np
import pytest

from crispresso_amd import _lib, quantify
from tests.test_quant_oracle import QUANT_SETS, load


@pytest.mark.parametrize("name", QUANT_SETS)
def test_globals_match_fixture(name):
    rec = load(name)
    amp = rec["amplicon"]
    for cname, case in rec["cases"].items():
        p = case["params"]
        cuts = quantify.compute_cut_points(amp, p["guide_seq"], p["cleavage_offset"])
        assert cuts == case["globals"]["cut_points"], cname
        inc = quantify.compute_include_idxs(len(amp), cuts, p["window_around_sgrna"], p["exclude_bp_from_left"],
                                            p["exclude_bp_from_right"])
        assert sorted(inc) == case["globals"]["INCLUDE_IDXS"], cname
        exon, spl = quantify.compute_exon_positions(amp, p["coding_seq"])
        assert exon == case["globals"]["EXON_POSITIONS"], cname
        assert (None if spl is None else sorted(spl)) == case["globals"]["SPLICING_POSITIONS"], cname


def test_pack_rows_layout():
    aln, lens = quantify.pack_rows(["AC-GT", "A"], ["|. ||", "|"], ["AT-GT"[:5], "A"])
    assert aln.shape == (2, 3, 16) and aln.dtype == np.uint8
    assert lens.tolist() == [5, 1]
    assert aln[0, 0, :5].tobytes() == b"AC-GT" and aln[0, 1, :5].tobytes() == b"|. ||"
    assert not aln[0, :, 5:].any() and not aln[1, :, 1:].any()


def test_pre_flags_nan_and_threshold():
    um = [True, False, False, False, False]
    sd = [0.0, -1.0, -1.0, math.nan, 2.0]
    sr = [100.0, 98.0, 97.9, math.nan, 90.0]
    pre = quantify.pre_flags(um, sd, sr, 98.0)
    assert pre.tolist() == [1, 2, 4, 0, 0]
    assert quantify.pre_flags(um).tolist() == [1, 0, 0, 0, 0]


def test_quant_symbols_exported():
    syms = _lib.exported_symbols()
    missing = [s for s in _lib.QUANT_EXPORTS + ("nw_batch_device_output",) if not syms.get(s)]
    assert not missing


def test_product_path_has_no_cpu_fallback(monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libcrispr_nw.so")
    quantify._DEFAULT.clear()
    with pytest.raises(_lib.NativeLibraryError):
        quantify.GpuQuantifier(0)
