#!/usr/bin/env python3
"""Golden vectors for the quantification step, from the REFERENCE's own code.

What runs: ``process_df_chunk`` (CRISPResso/CRISPRessoCORE.py:428-753) imported
from /root/reference, unchanged, on DataFrames built here, with the module
globals it reads (LEN_AMPLICON, INCLUDE_IDXS, EXON_POSITIONS,
SPLICING_POSITIONS -- set by run_crispresso at CORE:1261-1264) assigned
directly.  The rows are alignments of synthetic reads (and hand-made edge
cases: end overhangs, reads longer than the amplicon on either side, indels
one base apart, N in amplicon and reads) made by the CPU oracle aligner; the
parameter sets cover guides/windows, exclusion, hide_mutations_outside_window,
ignore_*, HDR classes (with NaN repair scores) and the frameshift analysis.

The globals are computed by oracle/quant_oracle.py's restatements (cut points,
INCLUDE_IDXS, exons); those restatements are pinned separately by the
end-to-end captures of make_golden.py, which record the reference's own
globals.  Output: tests/golden/quant_<dataset>.json.gz.
Run:  python tests/golden/make_quant_golden.py   (needs /root/reference; CPU only)
"""
from __future__ import annotations

import gzip
import json
import os
import sys
import tempfile
import types

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from crispresso_amd import synth  # noqa: E402
from oracle import oracle_py, quant_oracle as qo  # noqa: E402


def edge_reads(amp: str, rng) -> list:
    def rnd(k):
        return "".join(rng.choice(list("ACGT"), size=k))
    L = len(amp)
    m = L // 2
    out = [
        amp[20:], amp[:-25], amp[40:-40],                       # end deletions / short reads
        rnd(6) + amp, amp + rnd(7), rnd(4) + amp + rnd(5),      # leading / trailing insertions
        amp[:m] + rnd(3) + amp[m] + rnd(2) + amp[m + 1:],       # two insertions one base apart
        amp[:m] + amp[m + 4:m + 5] + amp[m + 9:],               # two deletions one base apart
        amp[:m] + rnd(1) + amp[m + 1:m + 30] + amp[m + 33:],    # substitution + deletion
        amp[:3] + amp[10:],                                      # deletion near the left edge
        amp[:L - 12] + amp[L - 5:],                              # deletion near the right edge
        rnd(3) + amp[8:m] + rnd(5) + amp[m:],                    # mixed left edge
        amp[:m] + "N" * 4 + amp[m + 4:],                         # N run in the read
    ]
    return out


def make_dataset(name: str, amp: str, seed: int, n_reads: int):
    rng = np.random.Generator(np.random.PCG64(seed))
    mix = synth.Mix(exact=0.15, subs=0.2, deletion=0.25, insertion=0.2, noise=0.2, n_rate=0.01,
                    homopolymer=True)
    buf, off = synth.reads_from(amp, n_reads, seed, mix)
    seqs = synth.unpack(buf, off) + edge_reads(amp, rng)
    rows = []
    for s in seqs:
        res, ra, mk, rb = oracle_py.align(amp, s)
        rows.append((ra, mk, rb, float("%.1f" % (100.0 * res["n_ident"] / res["aln_len"]))))
    # HDR scores: a mix of better / worse / equal / missing repair identities
    sr = rng.choice([100.0, 99.0, 98.0, 97.9, 95.0, 60.0, np.nan], size=len(rows))
    return {"name": name, "amplicon": amp, "rows": rows, "score_repaired": sr}


def param_sets(amp: str):
    L = len(amp)
    g_fw = amp[L // 2 - 20:L // 2]                         # a guide whose cut lands mid-amplicon
    g_rc = qo._rc(amp[L // 2 + 10:L // 2 + 30])
    exon = amp[L // 2 - 30:L // 2 + 31]
    ex2 = amp[30:60] + "," + amp[L - 70:L - 40]
    base = dict(guide_seq=None, cleavage_offset=-3, window_around_sgrna=1, exclude_bp_from_left=15,
                exclude_bp_from_right=15, coding_seq=None, ignore_substitutions=False, ignore_insertions=False,
                ignore_deletions=False, hide_mutations_outside_window_NHEJ=False, expected_hdr=False,
                hdr_perfect_alignment_threshold=98.0)
    sets = {
        "defaults": {},
        "guide_w1": dict(guide_seq=g_fw),
        "guide_w20_hide": dict(guide_seq=g_fw, window_around_sgrna=20, hide_mutations_outside_window_NHEJ=True),
        "two_guides_w6": dict(guide_seq=g_fw + "," + g_rc, window_around_sgrna=6),
        "w0_noexclude": dict(window_around_sgrna=0, exclude_bp_from_left=0, exclude_bp_from_right=0),
        "hide_noguide": dict(hide_mutations_outside_window_NHEJ=True, exclude_bp_from_left=40),
        "ignore_subs": dict(guide_seq=g_fw, window_around_sgrna=30, ignore_substitutions=True),
        "ignore_indels": dict(ignore_insertions=True, ignore_deletions=True),
        "coding_guide_w10": dict(guide_seq=g_fw, window_around_sgrna=10, coding_seq=exon),
        "coding_two_exons": dict(coding_seq=ex2, exclude_bp_from_left=0, exclude_bp_from_right=0),
        "hdr_guide": dict(guide_seq=g_fw, window_around_sgrna=8, expected_hdr=True),
        "hdr_coding_hide": dict(expected_hdr=True, hdr_perfect_alignment_threshold=99.0, coding_seq=exon,
                                hide_mutations_outside_window_NHEJ=True, window_around_sgrna=0),
    }
    return {k: {**base, **v} for k, v in sets.items()}


def globals_for(amp: str, p: dict):
    cuts = qo.cut_points(amp, p["guide_seq"], p["cleavage_offset"])
    inc = qo.include_idxs(len(amp), cuts, p["window_around_sgrna"], p["exclude_bp_from_left"],
                          p["exclude_bp_from_right"])
    exon, spl = qo.exon_splicing_positions(amp, p["coding_seq"])
    return cuts, inc, exon, spl


def run_reference(core, ds, p):
    amp = ds["amplicon"]
    cuts, inc, exon, spl = globals_for(amp, p)
    core.LEN_AMPLICON = len(amp)
    core.INCLUDE_IDXS = set(inc)
    if exon is not None:
        core.EXON_POSITIONS = sorted(exon)
        core.SPLICING_POSITIONS = set(spl)
    recs = []
    for i, (ra, mk, rb, score) in enumerate(ds["rows"]):
        um = score == 100
        if "N" in amp:
            mk, um = qo.ignore_n_in_alignment(ra, mk, um)
        rec = {"ref_seq": ra, "align_str": mk, "align_seq": rb, "score_ref": score, "UNMODIFIED": um,
               "MIXED": False, "HDR": False, "NHEJ": False, "n_mutated": 0, "n_inserted": 0, "n_deleted": 0}
        if p["expected_hdr"]:
            rec["score_repaired"] = float(ds["score_repaired"][i])
            rec["score_diff"] = score - rec["score_repaired"]
        recs.append(rec)
    df = pd.DataFrame(recs, index=[f"r{i}" for i in range(len(recs))])
    df["ref_positions"] = df["ref_seq"].apply(lambda s: np.array(qo.compute_ref_positions(s)))
    args = types.SimpleNamespace(
        coding_seq=p["coding_seq"], ignore_substitutions=p["ignore_substitutions"],
        ignore_insertions=p["ignore_insertions"], ignore_deletions=p["ignore_deletions"],
        expected_hdr_amplicon_seq="HDR" if p["expected_hdr"] else "",
        hdr_perfect_alignment_threshold=p["hdr_perfect_alignment_threshold"],
        hide_mutations_outside_window_NHEJ=p["hide_mutations_outside_window_NHEJ"],
        window_around_sgrna=p["window_around_sgrna"])
    out = core.process_df_chunk([df.copy(), args])
    d = out[0]
    names = ["df"] + list(qo.VECTORS[:13]) + ["hist_inframe", "hist_frameshift"] + list(qo.VECTORS[13:]) + \
        list(qo.COUNTERS)
    res = dict(zip(names, out))
    return {
        "params": p,
        "globals": {"cut_points": [int(c) for c in cuts], "INCLUDE_IDXS": sorted(int(x) for x in inc),
                    "EXON_POSITIONS": None if exon is None else sorted(int(x) for x in exon),
                    "SPLICING_POSITIONS": None if spl is None else sorted(int(x) for x in spl)},
        "rows_in": {"UNMODIFIED": [bool(r["UNMODIFIED"]) for r in recs],
                    "align_str": [r["align_str"] for r in recs]},
        "rows_out": {k: [int(x) for x in d[k].tolist()] for k in
                     ("UNMODIFIED", "NHEJ", "HDR", "MIXED", "n_mutated", "n_inserted", "n_deleted")},
        "vectors": {k: [float(x) for x in res[k]] for k in qo.VECTORS},
        "hist_inframe": sorted([int(k), int(v)] for k, v in res["hist_inframe"].items()),
        "hist_frameshift": sorted([int(k), int(v)] for k, v in res["hist_frameshift"].items()),
        "counters": {k: int(res[k]) for k in qo.COUNTERS},
    }


def main():
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference")
    os.system(f"make -s -C {os.path.join(ROOT, 'oracle')}")
    import make_golden  # stubs for Bio / seaborn (absent here)

    tmp = tempfile.mkdtemp(prefix="qgolden_")
    make_golden.install_stubs(tmp)
    sys.path.insert(0, REF)
    import CRISPResso.CRISPRessoCORE as core  # noqa: E402

    amp_a = synth.random_amplicon(200, 201)
    amp_n = list(synth.random_amplicon(180, 202))
    for k in (7, 60, 91, 150):
        amp_n[k] = "N"
    amp_n = "".join(amp_n)
    datasets = [make_dataset("a200", amp_a, 203, 400), make_dataset("n180", amp_n, 204, 250)]
    for ds in datasets:
        cases = {}
        for pname, p in param_sets(ds["amplicon"]).items():
            cases[pname] = run_reference(core, ds, p)
        rec = {"amplicon": ds["amplicon"],
               "rows": [{"ref_seq": r[0], "align_str": r[1], "align_seq": r[2], "score_ref": r[3]}
                        for r in ds["rows"]],
               "score_repaired": [None if np.isnan(x) else float(x) for x in ds["score_repaired"]],
               "cases": cases}
        with gzip.open(os.path.join(HERE, f"quant_{ds['name']}.json.gz"), "wt") as f:
            json.dump(rec, f)
        nh = {k: sum(v["rows_out"]["NHEJ"]) for k, v in cases.items()}
        print(f"quant_{ds['name']}: {len(ds['rows'])} rows; NHEJ per case {nh}")


if __name__ == "__main__":
    main()
