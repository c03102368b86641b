#!/usr/bin/env python3
"""CPU restatement of FLASH 1.2.11's read-pair merge -- TEST INFRASTRUCTURE ONLY.

The reference merges paired-end reads with FLASH before alignment
(CRISPResso/CRISPRessoCORE.py:1655-1677):

    flash R1 R2 --allow-outies --max-overlap M --min-overlap m -f LEN -r AVG -s STD -z -d OUT

FLASH 1.2.11 (environment.yml:21, bioconda flash=1.2.11; setup.py:124-141
builds FLASH-1.2.11.tar.gz) is a third-party program that is NOT vendored in
/root/reference and not installed here.  Its published algorithm (Magoc &
Salzberg 2011, and the FLASH 1.2.11 manual), restated:

* read 2 is reverse-complemented (bases) and reversed (qualities);
* every overlap of at least ``min_overlap`` bases is scored by its mismatch
  density (mismatches / overlap length; an overlap longer than
  ``max_overlap`` is scored over ``max_overlap`` bases) -- "innies" (read 2
  starts at or after read 1's start, position i = 0, 1, ...) first, then, with
  --allow-outies, "outies" (read 2 starts before read 1);
* the lowest density wins, ties broken by the lower average quality at the
  mismatched positions (sum of min(q1, q2) over mismatches / overlap length),
  remaining ties by the first overlap tried; no overlap with density <=
  ``max_mismatch_density`` (0.25) leaves the pair not combined;
* the merged read is read 1's prefix, the overlap, and read 2's suffix (for an
  outie, read 2's prefix, the overlap, read 1's suffix); in the overlap equal
  bases keep the higher quality, unequal ones take the base of the higher
  quality read (read 2 on equal qualities) with quality max(|q1 - q2|, 2);
* the merged read keeps read 1's name.

Parity: FLASH itself cannot run here ("parity unpinned" for this file alone);
the restatement is pinned end to end by the reference's own e2e assertions
(tests/crispresso_tests.py:181-195) through tests/golden/make_e2e_golden.py.
Only tests/ and tests/golden/ scripts use this module.
"""
from __future__ import annotations

import argparse
import gzip
import os
import sys
from typing import Iterator, List, Optional, Tuple

import numpy as np

_CANON = np.full(256, ord("N"), dtype=np.uint8)
for _c in b"ACGT":
    _CANON[_c] = _c
    _CANON[ord(chr(_c).lower())] = _c
_COMP = np.full(256, ord("N"), dtype=np.uint8)
for _a, _b in zip(b"ACGTN", b"TGCAN"):
    _COMP[_a] = _b


def read_fastq(path: str) -> Iterator[Tuple[str, bytes, bytes]]:
    op = gzip.open if open(path, "rb").read(2) == b"\x1f\x8b" else open
    with op(path, "rb") as f:
        while True:
            h = f.readline()
            if not h:
                return
            s = f.readline().rstrip(b"\r\n")
            f.readline()
            q = f.readline().rstrip(b"\r\n")
            yield h.rstrip(b"\r\n")[1:].decode(), s, q


def _diag_sums(mat: np.ndarray, width: int) -> np.ndarray:
    """out[i] = sum_{k < min(width, ...)} mat[i + k, k] for i in [0, rows)."""
    r, c = mat.shape
    w = min(width, c)
    pad = np.zeros((r + w, c), dtype=mat.dtype)
    pad[:r] = mat
    sk = np.lib.stride_tricks.as_strided(pad, shape=(r, w), strides=(pad.strides[0], pad.strides[0] + pad.strides[1]))
    return sk.sum(axis=1)


class Merger:
    def __init__(self, min_overlap=10, max_overlap=65, max_mismatch_density=0.25, allow_outies=False,
                 phred_offset=33, cap_mismatch_quals=False):
        self.min_ov, self.max_ov = min_overlap, max_overlap
        self.max_density = max_mismatch_density
        self.allow_outies = allow_outies
        self.off = phred_offset
        self.cap = cap_mismatch_quals

    def _scan(self, a: np.ndarray, qa: np.ndarray, b: np.ndarray, qb: np.ndarray, first_pos: int):
        """Overlaps of b's start against a at positions i (b[0] under a[i]); returns
        (density, qual_score, i) arrays for i in [first_pos, len(a) - min_ov]."""
        na, nb = len(a), len(b)
        last = na - self.min_ov
        if last < first_pos or nb < self.min_ov:
            return None
        mis = a[:, None] != b[None, :]
        qm = np.where(mis, np.minimum(qa[:, None], qb[None, :]), 0).astype(np.int64)
        pos = np.arange(first_pos, last + 1)
        ov = np.minimum(na - pos, nb)
        mm = _diag_sums(mis.astype(np.int64), self.max_ov)[pos]
        qt = _diag_sums(qm, self.max_ov)[pos]
        eff = np.minimum(ov, self.max_ov).astype(np.float32)
        dens = mm.astype(np.float32) / eff
        qs = qt.astype(np.float32) / eff
        return dens, qs, pos, ov

    def align(self, r1, q1, r2, q2) -> Tuple[int, bool]:
        best_d = np.float32(self.max_density + 1.0)
        best_q = np.float32(0.0)
        best_pos, best_outie = -1, False
        scans = [(False, self._scan(r1, q1, r2, q2, 0))]
        if self.allow_outies:
            scans.append((True, self._scan(r2, q2, r1, q1, 1)))
        for outie, sc in scans:
            if sc is None:
                continue
            dens, qs, pos, ov = sc
            for k in range(len(pos)):
                d = dens[k]
                if d <= best_d and (d < best_d or qs[k] < best_q):
                    best_d, best_q, best_pos, best_outie = d, qs[k], int(pos[k]), outie
        if best_d > np.float32(self.max_density):
            return -1, False
        return best_pos, best_outie

    def combine(self, a, qa, b, qb, pos):
        ov = min(len(a) - pos, len(b))
        sa, sqa = a[pos:pos + ov], qa[pos:pos + ov]
        sb, sqb = b[:ov], qb[:ov]
        eq = sa == sb
        seq = np.where(eq, sa, np.where(sqa > sqb, sa, sb))
        diff = np.abs(sqa.astype(np.int32) - sqb.astype(np.int32))
        mq = np.maximum(diff, 2)
        if self.cap:
            mq = np.minimum(mq, 2)
        qual = np.where(eq, np.maximum(sqa, sqb), mq).astype(np.uint8)
        tail_s = b[ov:] if len(b) > ov else a[pos + ov:]
        tail_q = qb[ov:] if len(b) > ov else qa[pos + ov:]
        return (np.concatenate([a[:pos], seq, tail_s]), np.concatenate([qa[:pos], qual, tail_q]))

    def merge_pair(self, s1: bytes, qs1: bytes, s2: bytes, qs2: bytes):
        r1 = _CANON[np.frombuffer(s1, dtype=np.uint8)]
        q1 = np.frombuffer(qs1, dtype=np.uint8).astype(np.int32) - self.off
        r2 = _COMP[_CANON[np.frombuffer(s2, dtype=np.uint8)]][::-1]
        q2 = (np.frombuffer(qs2, dtype=np.uint8).astype(np.int32) - self.off)[::-1]
        pos, outie = self.align(r1, q1, r2, q2)
        if pos < 0:
            return None
        if outie:
            s, q = self.combine(r2, q2, r1, q1, pos)
        else:
            s, q = self.combine(r1, q1, r2, q2, pos)
        return s.tobytes(), (q + self.off).astype(np.uint8).tobytes(), outie


def run_flash(r1: str, r2: str, out_dir: str, prefix: str = "out", gz: bool = True, **kw) -> dict:
    m = Merger(**kw)
    os.makedirs(out_dir, exist_ok=True)
    op = (lambda p: gzip.open(p + ".gz", "wb", compresslevel=1)) if gz else (lambda p: open(p, "wb"))
    ext = op(os.path.join(out_dir, f"{prefix}.extendedFrags.fastq"))
    nc1 = op(os.path.join(out_dir, f"{prefix}.notCombined_1.fastq"))
    nc2 = op(os.path.join(out_dir, f"{prefix}.notCombined_2.fastq"))
    hist = {}
    stats = {"pairs": 0, "combined": 0, "innies": 0, "outies": 0}
    for (n1, s1, q1), (n2, s2, q2) in zip(read_fastq(r1), read_fastq(r2)):
        stats["pairs"] += 1
        res = m.merge_pair(s1, q1, s2, q2)
        if res is None:
            nc1.write(b"@%s\n%s\n+\n%s\n" % (n1.encode(), s1, q1))
            nc2.write(b"@%s\n%s\n+\n%s\n" % (n2.encode(), s2, q2))
            continue
        s, q, outie = res
        name = n1[:-2] if n1.endswith("/1") else n1
        ext.write(b"@%s\n%s\n+\n%s\n" % (name.encode(), s, q))
        stats["combined"] += 1
        stats["outies" if outie else "innies"] += 1
        hist[len(s)] = hist.get(len(s), 0) + 1
    for f in (ext, nc1, nc2):
        f.close()
    with open(os.path.join(out_dir, f"{prefix}.hist"), "w") as f:
        for k in sorted(hist):
            f.write(f"{k}\t{hist[k]}\n")
    with open(os.path.join(out_dir, f"{prefix}.histogram"), "w") as f:
        for k in sorted(hist):
            f.write(f"{k}\t{'*' * max(1, hist[k] * 80 // max(hist.values()))}\n")
    return stats


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="flash")
    ap.add_argument("r1")
    ap.add_argument("r2")
    ap.add_argument("-m", "--min-overlap", type=int, default=10)
    ap.add_argument("-M", "--max-overlap", type=int, default=None)
    ap.add_argument("-x", "--max-mismatch-density", type=float, default=0.25)
    ap.add_argument("-O", "--allow-outies", action="store_true")
    ap.add_argument("-p", "--phred-offset", type=int, default=33)
    ap.add_argument("-r", "--read-len", type=float, default=100)
    ap.add_argument("-f", "--fragment-len", type=float, default=180)
    ap.add_argument("-s", "--fragment-len-stddev", type=float, default=18)
    ap.add_argument("-c", "--cap-mismatch-quals", action="store_true")
    ap.add_argument("-z", "--compress", action="store_true")
    ap.add_argument("-d", "--output-directory", default=".")
    ap.add_argument("-o", "--output-prefix", default="out")
    a = ap.parse_args(argv)
    max_ov = a.max_overlap
    if max_ov is None:   # FLASH: 2r - f + 2.5 s when -M is not given
        max_ov = int(2 * a.read_len - a.fragment_len + 2.5 * a.fragment_len_stddev)
    st = run_flash(a.r1, a.r2, a.output_directory, a.output_prefix, a.compress, min_overlap=a.min_overlap,
                   max_overlap=max_ov, max_mismatch_density=a.max_mismatch_density,
                   allow_outies=a.allow_outies, phred_offset=a.phred_offset, cap_mismatch_quals=a.cap_mismatch_quals)
    sys.stderr.write(f"[FLASH restatement] pairs {st['pairs']} combined {st['combined']} "
                     f"(innies {st['innies']}, outies {st['outies']})\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
