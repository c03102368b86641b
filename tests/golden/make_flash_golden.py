#!/usr/bin/env python3
"""Golden vectors for the GPU paired-end merge (tests/test_flash.py).

Inputs: the first 1000 read pairs of the reference's own paired-end test data
(tests/test_data/test_L001_R1_001.fastq.gz / _R2_, the files of
tests/crispresso_tests.py:131-195).  Expected outputs: oracle/flash_oracle.py
(the FLASH 1.2.11 restatement, pinned end to end by the reference's e2e
assertions through make_e2e_golden.py) under CRISPResso's FLASH options
(--allow-outies --max-overlap 100 --min-overlap 4, CRISPRessoCORE.py:1657-1663,
defaults at 4119-4138) and under FLASH's own defaults (-m 10 -M 65, no outies).

Run here (the reference exists only in this container):
    python tests/golden/make_flash_golden.py
"""
import gzip
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import flash_oracle  # noqa: E402

REF = "/root/reference/tests/test_data"
N = 1000
SETTINGS = {
    "crispresso": dict(min_overlap=4, max_overlap=100, allow_outies=True),
    "flash_defaults": dict(min_overlap=10, max_overlap=65, allow_outies=False),
}


def main():
    r1 = list(flash_oracle.read_fastq(os.path.join(REF, "test_L001_R1_001.fastq.gz")))[:N]
    r2 = list(flash_oracle.read_fastq(os.path.join(REF, "test_L001_R2_001.fastq.gz")))[:N]
    out = {"source": "reference tests/test_data/test_L001_R{1,2}_001.fastq.gz, first %d pairs" % N,
           "pairs": [[a[1].decode(), a[2].decode(), b[1].decode(), b[2].decode()] for a, b in zip(r1, r2)],
           "expected": {}}
    for name, kw in SETTINGS.items():
        m = flash_oracle.Merger(**kw)
        exp = []
        for (_, s1, q1), (_, s2, q2) in zip(r1, r2):
            res = m.merge_pair(s1, q1, s2, q2)
            exp.append(None if res is None else [res[0].decode(), res[1].decode(), bool(res[2])])
        out["expected"][name] = {"options": kw, "merged": exp}
        print(name, sum(e is not None for e in exp), "of", len(exp), "combined")
    with gzip.open(os.path.join(ROOT, "tests", "golden", "flash_pairs.json.gz"), "wt") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
