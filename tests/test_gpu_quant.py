"""GPU quantification (crispresso_amd/csrc/nw_quant.hip through include/crispr_quant.h)
against the reference's own process_df_chunk outputs (golden fixtures) and the
CPU oracle (oracle/quant_oracle.py) on seeded synthetic alignments.  Bit-exact:
every per-row class and count, every vector entry, histogram and counter."""
from __future__ import annotations

import functools
import math

import numpy as np
import pandas as pd
import pytest

from crispresso_amd import _lib, quantify, synth
from crispresso_amd.devmem import DeviceBuffer
from oracle import oracle_py
from oracle import quant_oracle as qo
from tests.test_quant_oracle import QUANT_SETS, case_inputs, golden_cases, load, params_from

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gq():
    q = quantify.GpuQuantifier(0)
    yield q
    q.close()


class _Args:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def args_for(prm: qo.QuantParams, coding: bool):
    return _Args(ignore_substitutions=prm.ignore_substitutions, ignore_insertions=prm.ignore_insertions,
                 ignore_deletions=prm.ignore_deletions, window_around_sgrna=prm.window_around_sgrna,
                 hide_mutations_outside_window_NHEJ=prm.hide_mutations_outside_window_NHEJ,
                 coding_seq="X" if coding else None,
                 expected_hdr_amplicon_seq="HDR" if prm.expected_hdr else "",
                 hdr_perfect_alignment_threshold=prm.hdr_perfect_alignment_threshold)


def globals_for(prm: qo.QuantParams):
    return quantify.QuantGlobals(prm.len_amplicon, set(prm.include_idxs),
                                 None if prm.exon_positions is None else sorted(prm.exon_positions),
                                 None if prm.splicing_positions is None else set(prm.splicing_positions))


def gpu_quant(gq, prm, R, M, S, um, sd, sr, n_rule=False):
    gq.set_params(globals_for(prm), args_for(prm, prm.exon_positions is not None), amplicon_has_n=n_rule)
    aln, lens = quantify.pack_rows(R, M, S)
    pre = quantify.pre_flags(um, sd if prm.expected_hdr else None, sr if prm.expected_hdr else None,
                             prm.hdr_perfect_alignment_threshold)
    reads, totals = gq.run(aln, lens, pre)
    return reads, gq.unpack_totals(totals, aln.shape[2]), aln, lens


def assert_matches_oracle(reads, tot, ref, um):
    assert (reads["cls"] >= 0).all()
    flags = qo.class_flags(ref["cls"], um)
    got = qo.class_flags(reads["cls"].astype(np.int8), um)
    for k in flags:
        assert np.array_equal(got[k], flags[k]), k
    for k in ("n_mutated", "n_inserted", "n_deleted"):
        assert np.array_equal(reads[k].astype(np.int64), ref[k]), k
    for k in qo.VECTORS:
        assert np.array_equal(tot["vectors"][k], ref["vectors"][k]), k
    assert tot["counters"] == ref["counters"]
    assert tot["hist_inframe"] == ref["hist_inframe"]
    assert tot["hist_frameshift"] == ref["hist_frameshift"]


@pytest.mark.parametrize("name,cname", list(golden_cases()))
def test_golden_process_df_chunk(gq, name, cname):
    """The reference's process_df_chunk outputs, recorded in this container."""
    rec = load(name)
    case = rec["cases"][cname]
    prm = params_from(case, rec["amplicon"])
    R, M, S, um, sd, sr = case_inputs(rec, case)
    reads, tot, _, _ = gpu_quant(gq, prm, R, M, S, um, sd, sr)
    got = qo.class_flags(reads["cls"].astype(np.int8), um)
    for k in ("UNMODIFIED", "NHEJ", "HDR", "MIXED"):
        assert got[k].astype(int).tolist() == case["rows_out"][k], k
    for k in ("n_mutated", "n_inserted", "n_deleted"):
        assert reads[k].tolist() == case["rows_out"][k], k
    for k in qo.VECTORS:
        assert tot["vectors"][k].astype(float).tolist() == case["vectors"][k], k
    assert sorted(map(list, tot["hist_inframe"].items())) == case["hist_inframe"]
    assert sorted(map(list, tot["hist_frameshift"].items())) == case["hist_frameshift"]
    assert tot["counters"] == case["counters"]


def test_golden_n_rule_in_kernel(gq):
    """ignore_n_in_alignment (CORE:2031-2046) done by the kernel on the raw aligner rows."""
    rec = load("quant_n180")
    for cname in ("defaults", "guide_w20_hide", "coding_guide_w10"):
        case = rec["cases"][cname]
        prm = params_from(case, rec["amplicon"])
        rows = rec["rows"]
        R = [r["ref_seq"] for r in rows]
        M = [r["align_str"] for r in rows]
        S = [r["align_seq"] for r in rows]
        um = [r["score_ref"] == 100 for r in rows]
        sr = np.array([math.nan if x is None else x for x in rec["score_repaired"]])
        sd = np.array([r["score_ref"] for r in rows]) - sr
        reads, tot, aln, lens = gpu_quant(gq, prm, R, M, S, um, sd, sr, n_rule=True)
        fixed = [aln[i, 1, :lens[i]].tobytes().decode() for i in range(len(rows))]
        assert fixed == case["rows_in"]["align_str"]
        got = qo.class_flags(reads["cls"].astype(np.int8), um)
        assert got["UNMODIFIED"].astype(int).tolist() == case["rows_out"]["UNMODIFIED"]
        assert got["NHEJ"].astype(int).tolist() == case["rows_out"]["NHEJ"]
        for k in qo.VECTORS:
            assert tot["vectors"][k].astype(float).tolist() == case["vectors"][k], (cname, k)


@functools.lru_cache(maxsize=None)
def synthetic_rows(La, n, seed, pad=0):
    mix = synth.PARITY_MIX
    amp = synth.random_amplicon(La, seed)
    buf, off = synth.reads_from(amp, n, seed + 1, mix)
    if pad:   # overhangs on both sides: leading / trailing insertions, end deletions
        rng = np.random.Generator(np.random.PCG64(seed + 2))
        seqs = synth.unpack(buf, off)
        for k in rng.choice(n, n // 10, replace=False):
            s = seqs[k]
            m = int(rng.integers(0, 4))
            if m == 0:
                s = "".join(rng.choice(list("ACGT"), pad)) + s
            elif m == 1:
                s = s + "".join(rng.choice(list("ACGT"), pad))
            elif m == 2:
                s = s[pad:]
            else:
                s = s[: len(s) - pad]
            seqs[k] = s
        buf = np.frombuffer("".join(seqs).encode(), np.uint8).copy()
        off = np.r_[0, np.cumsum([len(s) for s in seqs])].astype(np.int64)
    res, aln = oracle_py.align_batch(amp, buf, off, nthreads=8)
    lens = res["aln_len"]
    R = [aln[i, 0, :lens[i]].tobytes().decode() for i in range(n)]
    M = [aln[i, 1, :lens[i]].tobytes().decode() for i in range(n)]
    S = [aln[i, 2, :lens[i]].tobytes().decode() for i in range(n)]
    score = np.array([float("%.1f" % (100.0 * a / b)) for a, b in zip(res["n_ident"], lens)])
    return amp, R, M, S, score


PARAMS = {
    "defaults": dict(),
    "guide_w4": dict(guide=True, window=4),
    "guide_w30_hide": dict(guide=True, window=30, hide=True),
    "coding_guide": dict(guide=True, window=12, coding=True),
    "coding_nowin_hdr": dict(coding=True, window=0, hdr=True),
    "ignore_all_but_del": dict(ign_sub=True, ign_ins=True),
}


def make_params(amp, spec):
    L = len(amp)
    cuts = qo.cut_points(amp, amp[L // 2 - 20:L // 2]) if spec.get("guide") else []
    win = spec.get("window", 1)
    inc = qo.include_idxs(L, cuts, win, 15, 15)
    exon, spl = qo.exon_splicing_positions(amp, amp[L // 3:2 * L // 3]) if spec.get("coding") else (None, None)
    return qo.QuantParams(len_amplicon=L, include_idxs=inc, exon_positions=exon, splicing_positions=spl,
                          ignore_substitutions=spec.get("ign_sub", False), ignore_insertions=spec.get("ign_ins", False),
                          window_around_sgrna=win, hide_mutations_outside_window_NHEJ=spec.get("hide", False),
                          expected_hdr=spec.get("hdr", False))


@pytest.mark.parametrize("La,n,pad", [(250, 6000, 12), (97, 3000, 20), (700, 1500, 40)])
@pytest.mark.parametrize("pname", list(PARAMS))
def test_synthetic_vs_oracle(gq, La, n, pad, pname):
    """C2-style reads (and overhangs) at amplicon lengths below one 256-column step,
    at 250 and across several steps (700: runs straddling step boundaries)."""
    amp, R, M, S, score = synthetic_rows(La, n, 31 + La, pad=pad)
    prm = make_params(amp, PARAMS[pname])
    rng = np.random.Generator(np.random.PCG64(La))
    sr = rng.choice([100.0, 99.0, 97.0, 50.0, math.nan], size=n)
    sd = score - sr
    um = score == 100
    ref = qo.process_rows(R, M, S, um, sd, sr, prm)
    reads, tot, _, _ = gpu_quant(gq, prm, R, M, S, um, sd, sr)
    assert_matches_oracle(reads, tot, ref, um)


def test_edge_rows(gq):
    """Hand-made rows: leading/trailing insertions (wrapped flank positions),
    all-gap read, insertion runs one base apart, alignment exactly 256 columns,
    and a row that is not an alignment of the amplicon (cls -1)."""
    amp = synth.random_amplicon(256, 7)
    rows = [
        ("---" + amp, "   " + "|" * 256, "ACG" + amp),
        (amp + "--", "|" * 256 + "  ", amp + "TT"),
        ("-" + amp + "-", " " + "|" * 256 + " ", "A" + amp + "C"),
        (amp, " " * 256, "-" * 256),
        (amp[:100] + "-" + amp[100] + "--" + amp[101:], "|" * 100 + " | " + " " + "|" * 155,
         amp[:100] + "G" + amp[100] + "TT" + amp[101:]),
        (amp, "|" * 255 + ".", amp[:255] + ("A" if amp[255] != "A" else "C")),
    ]
    R, M, S = (list(x) for x in zip(*rows))
    um = [False] * len(rows)
    for spec in ({}, {"guide": True, "window": 300}, {"coding": True}):
        prm = make_params(amp, spec)
        ref = qo.process_rows(R, M, S, um, None, None, prm)
        reads, tot, _, _ = gpu_quant(gq, prm, R, M, S, um, None, None)
        assert_matches_oracle(reads, tot, ref, np.array(um))
    bad_R = R + [amp[:-1]]
    reads, _, _, _ = gpu_quant(gq, make_params(amp, {}), bad_R, M + ["|" * 255], S + [amp[:-1]], um + [False],
                               None, None)
    assert reads["cls"][-1] == -1 and (reads["cls"][:-1] >= 0).all()


def test_empty_batch(gq):
    prm = make_params(synth.random_amplicon(50, 3), {})
    reads, tot, _, _ = gpu_quant(gq, prm, [], [], [], [], None, None)
    assert len(reads) == 0 and not any(v.any() for v in tot["vectors"].values())


def test_process_df_chunk_dropin(gq):
    """crispresso_amd.quantify.process_df_chunk with the reference's calling convention."""
    rec = load("quant_a200")
    case = rec["cases"]["coding_guide_w10"]
    prm = params_from(case, rec["amplicon"])
    g = case["globals"]
    quantify.set_globals(len(rec["amplicon"]), g["INCLUDE_IDXS"], g["EXON_POSITIONS"], g["SPLICING_POSITIONS"])
    rows = rec["rows"]
    df = pd.DataFrame({"ref_seq": [r["ref_seq"] for r in rows], "align_str": case["rows_in"]["align_str"],
                       "align_seq": [r["align_seq"] for r in rows], "UNMODIFIED": case["rows_in"]["UNMODIFIED"]},
                      index=[f"r{i}" for i in range(len(rows))])
    out = quantify.process_df_chunk([df, args_for(prm, True)], quantifier=gq)
    assert len(out) == 22
    d = out[0]
    for k in ("UNMODIFIED", "NHEJ", "HDR", "MIXED", "n_mutated", "n_inserted", "n_deleted"):
        assert d[k].astype(int).tolist() == case["rows_out"][k], k
    names = list(qo.VECTORS[:13]) + ["hist_inframe", "hist_frameshift"] + list(qo.VECTORS[13:]) + list(qo.COUNTERS)
    res = dict(zip(names, out[1:]))
    for k in qo.VECTORS:
        assert res[k].dtype == np.float64 and res[k].tolist() == case["vectors"][k], k
    assert sorted(map(list, res["hist_inframe"].items())) == case["hist_inframe"]
    for k in qo.COUNTERS:
        assert res[k] == case["counters"][k]


def test_e2e_capture_quantify_alignments(gq):
    """quantify_alignments on the DataFrames the reference's run_crispresso handed to
    process_df_chunk (make_golden.py): same class counts and effect vectors."""
    for name in ("c1_plumbing", "syn_hdr"):
        rec = load(name)
        rows = rec["df_needle_alignment"]
        amp = rec["inputs"]["amplicon_seq"].upper()
        hdr = "--expected_hdr_amplicon_seq" in rec["inputs"]["extra_args"]
        df = pd.DataFrame({"score_ref": [r["score_ref"] for r in rows], "ref_seq": [r["ref_seq"] for r in rows],
                           "align_str": [r["align_str"] for r in rows], "align_seq": [r["align_seq"] for r in rows]},
                          index=[r["ID"] for r in rows])
        if hdr:
            df["score_repaired"] = [math.nan if r["score_repaired"] is None else r["score_repaired"] for r in rows]
            df["score_diff"] = [math.nan if r["score_diff"] is None else r["score_diff"] for r in rows]
        args = _Args(amplicon_seq=amp, expected_hdr_amplicon_seq="HDR" if hdr else None, guide_seq=None,
                     coding_seq=None, window_around_sgrna=1, exclude_bp_from_left=15, exclude_bp_from_right=15,
                     hdr_perfect_alignment_threshold=98.0)
        g = quantify.globals_from_args(args)
        out = quantify.quantify_alignments(df, args, quantifier=gq, globals_=g)
        q = rec["quantification"]
        d = out[0]
        assert int(d["UNMODIFIED"].sum()) == q["n_unmodified"] and int(d["NHEJ"].sum()) == q["n_nhej"]
        assert int(d["HDR"].sum()) == q["n_hdr"] and int(d["MIXED"].sum()) == q["n_mixed"]
        for i, k in enumerate(("effect_vector_insertion", "effect_vector_deletion", "effect_vector_mutation",
                               "effect_vector_any")):
            assert out[1 + i].tolist() == q[k], (name, k)


def test_device_resident_after_aligner(gpu_aligner_factory, gq):
    """Aligner output consumed in HBM (nw_batch_device_output -> nwq_run_device)
    gives what the oracle gives on the downloaded strings."""
    amp = synth.random_amplicon(250, 11)
    buf, off = synth.reads_from(amp, 20000, 12)
    al = gpu_aligner_factory()
    al.set_reference(amp)
    al.upload(buf, off)
    al.run_async()
    al.sync()
    d_aln, stride, d_stats = al.device_output()
    batch = al.download(len(off) - 1, int(np.diff(off).max()))
    n = len(off) - 1
    lens = batch.stats["aln_len"]
    score = np.array([float("%.1f" % (100.0 * a / b)) for a, b in zip(batch.stats["n_ident"], lens)])
    um = score == 100
    prm = make_params(amp, {"guide": True, "window": 10})
    gq.set_params(globals_for(prm), args_for(prm, False))
    with DeviceBuffer.from_array(quantify.pre_flags(um)) as d_pre, DeviceBuffer(16 * n) as d_out:
        tot_dev = gq.unpack_totals(gq.run_device(d_aln, stride, d_stats, 8, d_pre.ptr, n, d_out.ptr), stride)
        reads_dev = d_out.download(np.zeros((n, 4), np.int32))
    R = [batch.aln[i, 0, :lens[i]].tobytes().decode() for i in range(n)]
    M = [batch.aln[i, 1, :lens[i]].tobytes().decode() for i in range(n)]
    S = [batch.aln[i, 2, :lens[i]].tobytes().decode() for i in range(n)]
    ref = qo.process_rows(R, M, S, um, None, None, prm)
    assert np.array_equal(reads_dev[:, 0].astype(np.int8), ref["cls"])
    assert np.array_equal(reads_dev[:, 1], ref["n_mutated"])
    assert np.array_equal(reads_dev[:, 2], ref["n_inserted"])
    assert np.array_equal(reads_dev[:, 3], ref["n_deleted"])
    for k in qo.VECTORS:
        assert np.array_equal(tot_dev["vectors"][k], ref["vectors"][k]), k


@pytest.mark.parametrize("spec,with_n", [({"guide": True, "window": 10}, False), ({"guide": True, "window": 1}, True),
                                          ({"guide": True, "coding": True, "window": 5}, False)])
def test_device_resident_ops_after_aligner(gpu_aligner_factory, gq, spec, with_n):
    """The aligner's default OPS output consumed in HBM (nw_batch_device_ops ->
    nwq_run_device_ops: rows rebuilt on the device from the runs) gives what the oracle
    gives on the rows the host expands from the same runs -- every class, count, vector
    entry, histogram and counter.  An amplicon with N exercises the N rule (every read's
    rows expanded)."""
    amp = synth.random_amplicon(250, 11)
    if with_n:
        amp = amp[:60] + "N" + amp[61:180] + "N" + amp[181:]
    buf, off = synth.reads_from(amp.replace("N", "A"), 12000, 12, synth.PARITY_MIX)
    al = gpu_aligner_factory()
    al.set_reference(amp)
    al.set_output("ops")
    al.upload(buf, off)
    al.run_async()
    al.sync()
    dev = al.device_ops()
    n = len(off) - 1
    ob = al.download_ops(n)
    rows = ob.expand(amp, buf, off)
    lens = rows.stats["aln_len"]
    score = np.array([float("%.1f" % (100.0 * a / b)) if b else 0.0 for a, b in zip(rows.stats["n_ident"], lens)])
    um = score == 100
    prm = make_params(amp, spec)
    gq.set_params(globals_for(prm), args_for(prm, prm.exon_positions is not None), amplicon_has_n=with_n)
    stride = dev["max_cols"]
    with DeviceBuffer.from_array(quantify.pre_flags(um)) as d_pre, DeviceBuffer(16 * n) as d_out:
        tot_dev = gq.unpack_totals(gq.run_device_ops(amp, dev, d_pre.ptr, n, d_out.ptr), stride)
        reads_dev = d_out.download(np.zeros((n, 4), np.int32))
    keep = lens > 0
    R = [rows.aln[i, 0, :lens[i]].tobytes().decode() for i in range(n)]
    M = [rows.aln[i, 1, :lens[i]].tobytes().decode() for i in range(n)]
    S = [rows.aln[i, 2, :lens[i]].tobytes().decode() for i in range(n)]
    if with_n:   # the reference's ignore_n_in_alignment rewrite of align_str (CORE:2031-2046)
        M = ["".join("|" if r == "N" else m for r, m in zip(Rr, Mm)) for Rr, Mm in zip(R, M)]
        # ... and a row whose markup is then one character is UNMODIFIED (CORE:2047-2048)
        um = um | np.array([len(set(m)) == 1 for m in M])
    idx = np.flatnonzero(keep)
    ref = qo.process_rows([R[i] for i in idx], [M[i] for i in idx], [S[i] for i in idx], um[idx], None, None, prm)
    assert np.array_equal(reads_dev[idx, 0].astype(np.int8), ref["cls"])
    for c, k in ((1, "n_mutated"), (2, "n_inserted"), (3, "n_deleted")):
        assert np.array_equal(reads_dev[idx, c], ref[k]), k
    for k in qo.VECTORS:
        assert np.array_equal(tot_dev["vectors"][k], ref["vectors"][k]), k
    assert tot_dev["counters"] == ref["counters"]
    assert tot_dev["hist_inframe"] == ref["hist_inframe"]
    assert tot_dev["hist_frameshift"] == ref["hist_frameshift"]


@functools.lru_cache(maxsize=None)
def odd_reads(La, n, seed, pad):
    """C2 parity-mix reads with what the lane path must handle or hand to the row path:
    overhangs (leading / trailing insertions, end deletions), lowercase stretches, IUPAC codes,
    N, and '-' bytes (RC-retry input, CORE:1846: the lane path's fallback)."""
    amp = synth.random_amplicon(La, seed)
    buf, off = synth.reads_from(amp, n, seed + 1, synth.PARITY_MIX)
    rng = np.random.Generator(np.random.PCG64(seed + 2))
    seqs = synth.unpack(buf, off)
    for k in range(n):
        s = seqs[k]
        u = rng.random()
        if u < 0.04 and pad:
            m = int(rng.integers(0, 4))
            s = ("".join(rng.choice(list("ACGT"), pad)) + s if m == 0 else s + "".join(rng.choice(list("ACGT"), pad))
                 if m == 1 else s[pad:] if m == 2 else s[: len(s) - pad])
        elif u < 0.06 and len(s) > 20:
            a = int(rng.integers(0, len(s) - 10))
            s = s[:a] + s[a:a + 10].lower() + s[a + 10:]
        elif u < 0.08 and len(s) > 2:
            a = int(rng.integers(0, len(s)))
            s = s[:a] + str(rng.choice(list("RYKMSWN"))) + s[a + 1:]
        elif u < 0.09 and len(s) > 2:
            a = int(rng.integers(0, len(s)))
            s = s[:a] + "-" + s[a + 1:]
        seqs[k] = s
    buf = np.frombuffer("".join(seqs).encode(), np.uint8).copy()
    off = np.r_[0, np.cumsum([len(s) for s in seqs])].astype(np.int64)
    return amp, buf, off


@pytest.fixture(scope="module")
def gq_rows():
    """A quantifier that sends every read through the rows (CRISPR_NWQ_ROWS=1 at create)."""
    import os

    old = os.environ.get("CRISPR_NWQ_ROWS")
    os.environ["CRISPR_NWQ_ROWS"] = "1"
    try:
        q = quantify.GpuQuantifier(0)
    finally:
        if old is None:
            os.environ.pop("CRISPR_NWQ_ROWS", None)
        else:
            os.environ["CRISPR_NWQ_ROWS"] = old
    yield q
    q.close()


@pytest.mark.parametrize("La,n,pad", [(250, 8000, 12), (97, 3000, 20), (613, 2000, 40)])
@pytest.mark.parametrize("pname", list(PARAMS))
def test_device_ops_lane_path_vs_oracle(gpu_aligner_factory, gq, gq_rows, La, n, pad, pname):
    """quant_lanes (features straight from the runs; its fallback reads through the rows) on the
    aligner's resident ops output, against the oracle on the rows the host expands from the same
    runs, for every parameter set (windows, hide, coding, HDR / MIXED flags, ignore flags); the
    forced row path gives the same."""
    amp, buf, off = odd_reads(La, n, 90 + La, pad)
    al = gpu_aligner_factory()
    al.set_reference(amp)
    al.set_output("ops")
    al.upload(buf, off)
    al.run_async()
    al.sync()
    dev = al.device_ops()
    ob = al.download_ops(n)
    rows = ob.expand(amp, buf, off)
    lens = rows.stats["aln_len"]
    score = np.array([float("%.1f" % (100.0 * a / b)) if b else 0.0 for a, b in zip(rows.stats["n_ident"], lens)])
    R = [rows.aln[i, 0, :lens[i]].tobytes().decode("latin-1") for i in range(n)]
    M = [rows.aln[i, 1, :lens[i]].tobytes().decode("latin-1") for i in range(n)]
    S = [rows.aln[i, 2, :lens[i]].tobytes().decode("latin-1") for i in range(n)]
    # KNOWN DIVERGENCE: a '-' byte of the read aligned inside an insertion (ref '-'
    # and align_seq '-' in one column) is a deletion column whose reference position is negative
    # (compute_ref_positions, CORE:2055-2067) and lands, by numpy's wrap-around, on another
    # position; the row kernel indexes it at the amplicon position instead.  Such reads (only
    # RC-retry input has '-' bytes, CORE:1846) are left out here as UNMODIFIED rows.
    dash_ins = np.array([any(r == "-" and q == "-" for r, q in zip(Rr, Ss)) for Rr, Ss in zip(R, S)])
    um = (score == 100) | dash_ins
    prm = make_params(amp, PARAMS[pname])
    rng = np.random.Generator(np.random.PCG64(La + 5))
    sr = rng.choice([100.0, 99.0, 97.0, 50.0, math.nan], size=n)
    sd = score - sr
    pre = quantify.pre_flags(um, sd if prm.expected_hdr else None, sr if prm.expected_hdr else None,
                             prm.hdr_perfect_alignment_threshold)
    stride = dev["max_cols"]
    keep = lens > 0
    idx = np.flatnonzero(keep)
    ref = qo.process_rows([R[i] for i in idx], [M[i] for i in idx], [S[i] for i in idx], um[idx],
                          sd[idx] if prm.expected_hdr else None, sr[idx] if prm.expected_hdr else None, prm)
    for q in (gq, gq_rows):
        q.set_params(globals_for(prm), args_for(prm, prm.exon_positions is not None))
        with DeviceBuffer.from_array(pre) as d_pre, DeviceBuffer(16 * n) as d_out:
            tot_dev = q.unpack_totals(q.run_device_ops(amp, dev, d_pre.ptr, n, d_out.ptr), stride)
            reads_dev = d_out.download(np.zeros((n, 4), np.int32))
        assert np.array_equal(reads_dev[idx, 0].astype(np.int8), ref["cls"])
        for c, k in ((1, "n_mutated"), (2, "n_inserted"), (3, "n_deleted")):
            assert np.array_equal(reads_dev[idx, c], ref[k]), k
        for k in qo.VECTORS:
            assert np.array_equal(tot_dev["vectors"][k], ref["vectors"][k]), k
        assert tot_dev["counters"] == ref["counters"]
        assert tot_dev["hist_inframe"] == ref["hist_inframe"]
        assert tot_dev["hist_frameshift"] == ref["hist_frameshift"]
