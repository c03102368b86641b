#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE's own code in this container.

What runs: CRISPResso/CRISPRessoCORE.py:run_crispresso from /root/reference,
unchanged -- its FASTQ->FASTA shell pipeline (CORE:1791-1797), its `needle`
calls (CORE:1797-1806, 1812-1828, 1910-1936), its parse_needle_output
(CORE:1707-1786) and its merge/filter/RC logic (CORE:1830-2000).  `needle` on
PATH is oracle/_build/needle_oracle (EMBOSS is not installed anywhere; see
oracle/nw_oracle.h), so these fixtures pin everything AROUND the aligner
arithmetic (text format compatibility, id handling, filters, RC transform,
quirks) -- not EMBOSS's arithmetic itself.

The reference needs Biopython and seaborn at import (CORE:36, 365-368), which
are absent; throw-away stubs are generated in a temp dir (SeqIO is unused on
these paths; pairwise2.align.globalxx is restated for the HDR-validation check
at CORE:1367).  `java`/`flash` shims only satisfy check_program (CORE:361-363).
The quantification step is intercepted: the DataFrame passed to
process_df_chunk (CORE:2864) is recorded, the real process_df_chunk is run on
it and its aggregate outputs recorded, then the run is stopped (plots are out
of scope).

Outputs (tests/golden/): <case>.json.gz with the inputs' description, args,
the DataFrame rows and the quantification aggregates; FASTQ inputs as .fastq.gz.
Run:  python tests/golden/make_golden.py   (needs /root/reference; CPU only)
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import stat
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)

from crispresso_amd import synth  # noqa: E402

C1_AMPLICON = (
    "gtcgcccctcaaatcttacagctgctcactcccctgcagggcaacgcccagggaccaagttagccccttaagcctaggcaaaagaatcccgcccataatcgag"
    "aagcgactcgacatggaggcgatgacgagatcacgcgaggaggaaaggagggagggcttcttccaggcccagggcggtccttacaagacgggaggcagcaga"
    "gaactcccataaaggtattgcggcactccccctccccctgcccagaagggtgcggccttctctccacctcctccac"
)


def globalxx(a, b):
    """Biopython pairwise2.align.globalxx restated: match 1, mismatch 0, no gap cost."""
    n, m = len(a), len(b)
    S = np.zeros((n + 1, m + 1), dtype=np.int32)
    for i in range(1, n + 1):
        for j in range(1, m + 1):
            S[i, j] = max(S[i - 1, j - 1] + (a[i - 1] == b[j - 1]), S[i - 1, j], S[i, j - 1])
    i, j, ra, rb = n, m, [], []
    while i > 0 or j > 0:
        if i > 0 and j > 0 and S[i, j] == S[i - 1, j - 1] + (a[i - 1] == b[j - 1]):
            ra.append(a[i - 1]); rb.append(b[j - 1]); i -= 1; j -= 1
        elif i > 0 and S[i, j] == S[i - 1, j]:
            ra.append(a[i - 1]); rb.append("-"); i -= 1
        else:
            ra.append("-"); rb.append(b[j - 1]); j -= 1
    return [("".join(reversed(ra)), "".join(reversed(rb)), float(S[n, m]), 0, len(ra))]


def install_stubs(tmp):
    bio = types.ModuleType("Bio")
    seqio = types.ModuleType("Bio.SeqIO")
    seqio.parse = lambda *a, **k: iter(())
    seqio.write = lambda *a, **k: 0
    pw2 = types.ModuleType("Bio.pairwise2")
    pw2.align = types.SimpleNamespace(globalxx=globalxx)
    bio.SeqIO, bio.pairwise2 = seqio, pw2
    sys.modules.update({"Bio": bio, "Bio.SeqIO": seqio, "Bio.pairwise2": pw2})
    sns = types.ModuleType("seaborn")
    sns.matrix = types.SimpleNamespace(_HeatMapper=object)
    sns.utils = types.SimpleNamespace()
    sns.set_context = sns.set = sns.set_style = lambda *a, **k: None
    sys.modules["seaborn"] = sns
    bindir = os.path.join(tmp, "bin")
    os.makedirs(bindir)
    shims = {
        "needle": f'#!/bin/sh\nexec "{os.path.join(ROOT, "oracle", "_build", "needle_oracle")}" "$@"\n',
        "flash": "#!/bin/sh\nexit 0\n",
        "java": "#!/bin/sh\nexit 0\n",
    }
    for name, body in shims.items():
        p = os.path.join(bindir, name)
        with open(p, "w") as f:
            f.write(body)
        os.chmod(p, os.stat(p).st_mode | stat.S_IEXEC)
    os.environ["PATH"] = bindir + os.pathsep + os.environ["PATH"]


class Captured(Exception):
    pass


def run_case(core, name, fastq_path, amplicon, extra, workdir):
    sys.argv = ["CRISPResso", "-r1", fastq_path, "--amplicon_seq", amplicon, "-o", workdir] + extra
    args = core.parse_args(sys.argv[1:])
    record = {}
    real = core.process_df_chunk

    def capture(chunk_input):
        df = chunk_input[0]
        rows = []
        for idx, r in df.iterrows():
            row = {"ID": idx, "score_ref": float(r.score_ref), "length": r.length, "ref_seq": r.ref_seq,
                   "align_str": r.align_str, "align_seq": r.align_seq}
            if "score_repaired" in df.columns:
                row["score_repaired"] = None if np.isnan(r.score_repaired) else float(r.score_repaired)
                row["score_diff"] = None if np.isnan(r.score_diff) else float(r.score_diff)
            rows.append(row)
        record["df_needle_alignment"] = rows
        out = real([df.copy(), chunk_input[1]])
        d = out[0]
        record["quantification"] = {
            "n_total": int(len(d)),
            "n_unmodified": int(d["UNMODIFIED"].sum()), "n_nhej": int(d["NHEJ"].sum()),
            "n_hdr": int(d["HDR"].sum()), "n_mixed": int(d["MIXED"].sum()),
            "effect_vector_insertion": out[1].tolist(), "effect_vector_deletion": out[2].tolist(),
            "effect_vector_mutation": out[3].tolist(), "effect_vector_any": out[4].tolist(),
        }
        raise Captured()

    core.process_df_chunk = capture
    try:
        core.run_crispresso(args)
        record["exception"] = None
    except Captured:
        record["exception"] = None
    except Exception as exc:  # the reference's own failure modes (e.g. NeedleException)
        record["exception"] = type(exc).__name__
    finally:
        core.process_df_chunk = real
    return record


def write_fastq(path, names, seqs):
    with gzip.open(path, "wt") as f:
        for n, s in zip(names, seqs):
            f.write(f"@{n}\n{s}\n+\n{'I' * len(s)}\n")


def main():
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference")
    os.system(f"make -s -C {os.path.join(ROOT, 'oracle')}")
    tmp = tempfile.mkdtemp(prefix="golden_")
    try:
        install_stubs(tmp)
        sys.path.insert(0, REF)
        import CRISPResso.CRISPRessoCORE as core  # noqa: E402

        cases = {}
        # C1 (plumbing config): the reference's own test reads vs its test amplicon,
        # --min_identity_score 30 (as tests/crispresso_tests.py:238), first 2000 reads.
        src = os.path.join(REF, "tests", "test_data", "test_L001_R1_001.fastq.gz")
        with gzip.open(src, "rt") as f:
            lines = f.read().split("\n")
        c1 = os.path.join(HERE, "c1_R1_2000.fastq.gz")
        with gzip.open(c1, "wt") as f:
            f.write("\n".join(lines[: 4 * 2000]) + "\n")
        cases["c1_plumbing"] = (c1, C1_AMPLICON, ["--min_identity_score", "30"])

        # synthetic with reverse-complemented and off-target reads: exercises the RC pass
        amp = synth.random_amplicon(200, 101)
        buf, off = synth.reads_from(amp, 300, 102, synth.PARITY_MIX)
        seqs = synth.unpack(buf, off)
        rng = np.random.Generator(np.random.PCG64(103))
        for k in rng.choice(len(seqs), 30, replace=False):
            seqs[k] = synth.reverse_complement_str(seqs[k]) if hasattr(synth, "reverse_complement_str") else \
                seqs[k][::-1].translate(str.maketrans("ACGTN", "TGCAN"))
        names = [f"SYN:1:FC{k % 3}:1:{1000 + k}:{2000 + k} 1:N:0:1" for k in range(len(seqs))]
        rc_fq = os.path.join(HERE, "syn_rc.fastq.gz")
        write_fastq(rc_fq, names, seqs)
        cases["syn_rc"] = (rc_fq, amp, [])

        # synthetic HDR without forward failures: dual alignment, join, score_diff
        hdr = synth.hdr_amplicon(amp, 104)
        b1, o1 = synth.reads_from(amp, 150, 105)
        b2, o2 = synth.reads_from(hdr, 50, 106)
        seqs = synth.unpack(b1, o1) + synth.unpack(b2, o2)
        names = [f"HDR:{k}" for k in range(len(seqs))]
        hdr_fq = os.path.join(HERE, "syn_hdr.fastq.gz")
        write_fastq(hdr_fq, names, seqs)
        cases["syn_hdr"] = (hdr_fq, amp, ["--expected_hdr_amplicon_seq", hdr, "--min_identity_score", "50"])

        # HDR + a forward failure: the RC-HDR needle call gets the literal
        # "args.needle_options_string" (CORE:1928), aligns nothing, and the pipeline's
        # exit status (gzip's) hides it: RC rows get NaN repair scores
        seqs2 = seqs[:20] + [seqs[0][::-1].translate(str.maketrans("ACGTN", "TGCAN"))]
        hdr_fail_fq = os.path.join(HERE, "syn_hdr_rcfail.fastq.gz")
        write_fastq(hdr_fail_fq, [f"F:{k}" for k in range(len(seqs2))], seqs2)
        cases["syn_hdr_rcfail"] = (hdr_fail_fq, amp, ["--expected_hdr_amplicon_seq", hdr])

        for name, (fq, amplicon, extra) in cases.items():
            work = os.path.join(tmp, name)
            rec = run_case(core, name, fq, amplicon, extra, work)
            rec["inputs"] = {"fastq": os.path.basename(fq), "amplicon_seq": amplicon, "extra_args": extra}
            with gzip.open(os.path.join(HERE, f"{name}.json.gz"), "wt") as f:
                json.dump(rec, f)
            n = len(rec.get("df_needle_alignment", []))
            print(f"{name}: {n} rows, exception={rec['exception']}")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
