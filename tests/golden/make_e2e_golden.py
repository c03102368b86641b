#!/usr/bin/env python3
"""Run the REFERENCE's own run_crispresso end to end on its own paired-end test
data, with `flash` = oracle/flash_oracle.py (FLASH 1.2.11 restated) and
`needle` = oracle/_build/needle_oracle (EMBOSS needle restated), and compare
with the values the reference's test asserts (tests/crispresso_tests.py:
125-195, "ground truth values are from the original CRISPResso Docker", i.e.
real FLASH + real EMBOSS).

This is the only check of the two restatements against outputs of the real
programs that exists offline: the asserted counts and allele frequencies
depend on every merged read and every alignment's gap placement.

Writes tests/golden/e2e_test_data.json.gz: the FLASH-merged reads the
restatement produced (the input of the alignment stage), the DataFrame rows
the reference's parse_needle_output built from the oracle's srspair text, the
reference's own aggregates from run_crispresso, and the test's asserted values.
Run:  python tests/golden/make_e2e_golden.py   (needs /root/reference; CPU only)
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import stat
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden  # noqa: E402

AMPLICON = (
    "gtcgcccctcaaatcttacagctgctcactc" "ccctgcagggcaacgcccagggaccaagttag" "ccccttaagcctaggcaaaagaatcccgccca"
    "taatcgagaagcgactcgacatggaggcgatg" "acgagatcacgcgaggaggaaaggagggaggg" "cttcttccaggcccagggcggtccttacaaga"
    "cgggaggcagcagagaactcccataaaggtat" "tgcggcactcccctccccctgcccagaagggt" "gcggccttctctccacctcctccac"
)
GUIDES = "aatcgagaagcgactcgaca,taaggggctaacttggtccc"
# tests/crispresso_tests.py:181-195
EXPECTED = {
    "n_total": 7058, "n_reads_input": 8906, "n_unmodified": 6853, "n_mixed_hdr_nhej": 0, "n_modified": 205,
    "n_repaired": 0, "nhej_inserted": 0, "nhej_deleted": 12, "nhej_mutated": 193,
    "df_indels_fq4": [1, 0, 0, 0], "df_insertion_fq4": [7058, 0, 0, 0], "df_deletion_fq4": [7046, 0, 0, 0],
    "df_substitution_fq4": [6865, 188, 5, 0], "df_alleles_reads4": [1098, 346, 19, 17],
}
# tests/crispresso_tests.py:198-272 (test1_run_crispresso): the same amplicon, other guides,
# --min_identity_score 30 --window_around_sgrna 23 --trim_sequences (Trimmomatic 0.33 PE with the
# default ILLUMINACLIP:NexteraPE-PE.fa:0:90:10:0:true MINLEN:40, CORE:4113-4117, 1620-1640), p = 5.
GUIDES_TEST1 = "cgagaagcgactcgacatgg,aaggggctaacttggtccct"
EXPECTED_TEST1 = {
    "n_total": 4039, "n_reads_input": 4941, "n_unmodified": 2647, "n_mixed_hdr_nhej": 0, "n_modified": 1392,
    "n_repaired": 0, "nhej_inserted": 49, "nhej_deleted": 680, "nhej_mutated": 890,
    "df_indels_fq4": [2, 4, 5, 5], "df_insertion_fq4": [3990, 6, 1, 0], "df_deletion_fq4": [3359, 43, 3, 0],
    "df_substitution_fq4": [3149, 693, 105, 23], "df_alleles_reads4": [184, 68, 44, 26],
}
CASES = {
    "test": dict(prefix="test", guides=GUIDES, expected=EXPECTED, n_processes=1, trim=False, extra={},
                 out="e2e_test_data.json.gz"),
    "test1": dict(prefix="test1", guides=GUIDES_TEST1, expected=EXPECTED_TEST1, n_processes=5, trim=True,
                  extra={"window_around_sgrna": 23, "min_identity_score": 30.0}, out="e2e_test1_data.json.gz"),
}


def install_java(tmp):
    """`java -jar trimmomatic-0.33.jar PE ...` (CORE:1628-1634) -> oracle/trimmomatic_oracle.py (the
    vendored jar is never run)."""
    p = os.path.join(tmp, "bin", "java")
    with open(p, "w") as f:
        f.write(f'#!/bin/sh\nshift 2\nexec "{sys.executable}" "{os.path.join(ROOT, "oracle", "trimmomatic_oracle.py")}" "$@"\n')
    os.chmod(p, os.stat(p).st_mode | stat.S_IEXEC)


def install_flash(tmp):
    p = os.path.join(tmp, "bin", "flash")
    with open(p, "w") as f:
        f.write(f'#!/bin/sh\nexec "{sys.executable}" "{os.path.join(ROOT, "oracle", "flash_oracle.py")}" "$@"\n')
    os.chmod(p, os.stat(p).st_mode | stat.S_IEXEC)


def patch_plotting():
    import matplotlib
    matplotlib.use("Agg")
    from matplotlib.legend import Legend
    if not hasattr(Legend, "legendHandles"):      # removed in matplotlib 3.9 (CORE:2103)
        Legend.legendHandles = property(lambda self: self.legend_handles)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", choices=sorted(CASES), default="test")
    ap.add_argument("--no-trim", action="store_true", help="probe: run the case with --trim_sequences off")
    ap.add_argument("--pool", action="store_true",
                    help="probe: the test's own n_processes (a Pool; the DataFrame is then not captured)")
    opt = ap.parse_args(argv)
    case = CASES[opt.case]
    trim = case["trim"] and not opt.no_trim
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference")
    os.system(f"make -s -C {os.path.join(ROOT, 'oracle')}")
    tmp = tempfile.mkdtemp(prefix="e2e_")
    cwd = os.getcwd()
    try:
        make_golden.install_stubs(tmp)
        install_flash(tmp)
        if trim:
            install_java(tmp)
        patch_plotting()
        sys.path.insert(0, REF)
        import CRISPResso.CRISPRessoCORE as core  # noqa: E402
        import matplotlib.pyplot as plt

        record = {}
        real = core.process_df_chunk

        def capture(chunk_input):
            df = chunk_input[0]
            record["df_needle_alignment"] = [
                {"ID": idx, "score_ref": float(r.score_ref), "length": r.length, "ref_seq": r.ref_seq,
                 "align_str": r.align_str, "align_seq": r.align_seq} for idx, r in df.iterrows()]
            out = real(chunk_input)
            d = out[0]
            record["quantified_rows"] = {
                "NHEJ": d["NHEJ"].astype(bool).tolist(), "UNMODIFIED": d["UNMODIFIED"].astype(bool).tolist(),
                "n_inserted": d["n_inserted"].astype(int).tolist(), "n_deleted": d["n_deleted"].astype(int).tolist(),
                "n_mutated": d["n_mutated"].astype(int).tolist()}
            return out

        if not opt.pool:
            core.process_df_chunk = capture
        core.plot_alleles_table = lambda *a, **k: plt.figure()   # seaborn heatmap (absent); plots are out of scope
        os.chdir(os.path.join(REF, "tests"))
        out = os.path.join(tmp, "out")
        r1 = f"test_data/{case['prefix']}_L001_R1_001.fastq.gz"
        r2 = f"test_data/{case['prefix']}_L001_R2_001.fastq.gz"
        sys.argv = ["CRISPResso", "-r1", r1, "-r2", r2, "--amplicon_seq", AMPLICON, "--guide_seq", case["guides"],
                    "-o", out, "--keep_intermediate"]
        args = core.parse_args(sys.argv[1:])
        args.fastq_r1 = r1
        args.fastq_r2 = r2
        args.amplicon_seq = AMPLICON
        args.guide_seq = case["guides"]
        # process_df_chunk is captured in this process, so the quantification runs as one chunk; the test's
        # n_processes only splits the rows over a Pool and sums the chunks (CORE:2762-2864).
        args.n_processes = case["n_processes"] if opt.pool else 1
        args.keep_intermediate = True
        args.output_folder = out
        args.trim_sequences = trim
        for k, v in case["extra"].items():
            setattr(args, k, v)
        res = core.run_crispresso(args)
        os.chdir(cwd)
        core.process_df_chunk = real
        (n_total, n_reads_input, n_unmodified, n_mixed, n_modified, n_repaired, nhej_ins, nhej_del, nhej_mut,
         df_indels, df_insertion, df_deletion, df_substitution, df_alleles) = res
        got = {
            "n_total": int(n_total), "n_reads_input": int(n_reads_input), "n_unmodified": int(n_unmodified),
            "n_mixed_hdr_nhej": int(n_mixed), "n_modified": int(n_modified), "n_repaired": int(n_repaired),
            "nhej_inserted": int(nhej_ins), "nhej_deleted": int(nhej_del), "nhej_mutated": int(nhej_mut),
            "df_indels_fq4": [int(x) for x in df_indels["fq"].values[:4]],
            "df_insertion_fq4": [int(x) for x in df_insertion["fq"].values[:4]],
            "df_deletion_fq4": [int(x) for x in df_deletion["fq"].values[:4]],
            "df_substitution_fq4": [int(x) for x in df_substitution["fq"].values[:4]],
            "df_alleles_reads4": [int(x) for x in df_alleles["#Reads"].values[:4]],
        }
        dirs = [d for d in os.listdir(out) if d.startswith("CRISPResso_on")]
        rdir = os.path.join(out, dirs[0]) if dirs else out
        merged = []
        with gzip.open(os.path.join(rdir, "out.extendedFrags.fastq.gz"), "rt") as f:
            lines = f.read().split("\n")
        for k in range(0, len(lines) - 3, 4):
            merged.append([lines[k][1:], lines[k + 1]])
        expected = case["expected"]
        record.update({"case": opt.case, "trim_sequences": trim, "extra_args": case["extra"],
                       "amplicon_seq": AMPLICON, "guide_seq": case["guides"], "merged_reads": merged,
                       "reference_aggregates": got, "expected_by_reference_test": expected,
                       "n_reads_after_preprocessing": len(merged)})
        mism = {k: (got[k], expected[k]) for k in expected if got[k] != expected[k]}
        record["mismatches"] = mism
        with gzip.open(os.environ.get("E2E_OUT", os.path.join(HERE, case["out"])), "wt") as f:
            json.dump(record, f)
        print(json.dumps(got))
        print("MATCH" if not mism else f"MISMATCH {mism}")
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
