#!/usr/bin/env python3
"""CPU restatement of Trimmomatic 0.33's ILLUMINACLIP + MINLEN -- TEST INFRASTRUCTURE ONLY.

The reference trims paired-end reads before FLASH when ``--trim_sequences`` is given
(CRISPResso/CRISPRessoCORE.py:1620-1640):

    java -jar trimmomatic-0.33.jar PE -phred33 R1 R2 out_fp out_fu out_rp out_ru <options>

with the default options ``ILLUMINACLIP:<data>/NexteraPE-PE.fa:0:90:10:0:true MINLEN:40``
(CORE:4113-4117).  Trimmomatic 0.33 is third-party Java; the reference ships it only as a prebuilt jar
(CRISPResso/data/trimmomatic-0.33.jar), which is never run here, and Java is absent anyway.  Its
published algorithm (Bolger, Lohse & Usadel, Bioinformatics 30:2114, 2014; the Trimmomatic 0.33
manual), restated:

* ``ILLUMINACLIP:<fasta>:<seed mismatches>:<palindrome threshold>:<simple threshold>[:<min adapter
  length>[:<keep both reads>]]``.  Adapter records whose name ends in ``/1`` clip read 1, ``/2`` read
  2, others both reads ("common"); a ``Prefix*/1`` + ``Prefix*/2`` pair is a palindrome prefix pair
  (both cut to the shorter one's length from their 3' ends).  Duplicate sequences are used once.
* Bases are compared as one-hot nibbles (A 1, T 2, C 4, G 8, anything else 0) packed 16 to a 64-bit
  word; a seed matches when the XOR of two words has at most ``2 * seed mismatches`` bits set.
* **Simple mode**, per read and adapter: the read's 16-mers at every position ``i`` (zero-padded past
  the read's end, masked to the bases present) are compared with the adapter's 16-mers at positions
  0, 4, 8, ... (``INTERLEAVE`` 4); a seed hit gives the alignment offset ``i - j``; the offsets are
  tried in increasing order, each scored over the overlap of read and adapter: +log10(4) per equal
  base, -q/10 per unequal base (q = the read base's phred quality), 0 where either base is N; the
  score is the best "maximum range" (alternating runs of positive and negative sums, merging a
  negative run into its neighbours while both exceed it, the largest sum left); the first offset
  scoring at least the simple threshold clips the read to ``offset`` bases.  Only reads positions
  with at least ``min(15, int(threshold / log10 4))`` bases left seed.
* **Palindrome mode**, per pair: ``prefix1 + read1`` against the reverse complement of
  ``prefix2 + read2``; the total overlap grows one base per step, the seed positions alternate
  between the two reads' packs around the middle of the overlap, and a seed hit is scored over the
  whole overlap (+log10 4 equal, -min(q1, q2)/10 unequal, 0 at N, prefix bases quality 100), summed;
  the first overlap scoring at least the palindrome threshold clips read 1 (and read 2 when "keep both
  reads", else read 2 is dropped) to ``overlap - 2 * prefix length`` bases.  The scan stops
  ``15 + min adapter length`` short of the longer read.
* The smallest length any test gives wins; a read clipped to 0 or less is dropped.
* ``MINLEN:n`` drops reads shorter than n.  A pair whose two reads survive goes to the paired outputs,
  a lone survivor to its unpaired output (outputs gzip-compressed when named ``*.gz``).

Parity: Trimmomatic cannot run here ("parity unpinned" for this file alone); the restatement is pinned
end to end by the reference's own second e2e assertions (tests/crispresso_tests.py:198-272, real
Trimmomatic 0.33 + FLASH 1.2.11 + EMBOSS 6.6.0 output) through tests/golden/make_e2e_golden.py --case
test1.  Only tests/ and tests/golden/ scripts use this module.
"""
from __future__ import annotations

import gzip
import sys
from typing import Dict, Iterator, List, Optional, Tuple

LOG10_4 = 0.60206          # float32 constant of the Java code; sums are formed in float32 below
INTERLEAVE = 4
_NIB = {"A": 0x1, "T": 0x2, "C": 0x4, "G": 0x8}
_NIB_RC = {"A": 0x2, "T": 0x1, "C": 0x8, "G": 0x4}
_COMP = {"A": "T", "T": "A", "C": "G", "G": "C"}
_MASK64 = (1 << 64) - 1

try:
    import numpy as _np

    def _f32(x: float) -> float:
        return float(_np.float32(x))
except ImportError:  # pragma: no cover
    def _f32(x: float) -> float:
        return x


LOG10_4 = _f32(LOG10_4)


def pack_internal(seq: str, reverse: bool) -> List[int]:
    """16-mers of seq (only complete ones): forward = first base in the top nibble; reverse = the
    reverse complement of the 16-mer, so forward(a) == reverse(b) iff seq_a[a:a+16] == rc(seq_b[b:b+16])."""
    out = []
    pack = 0
    for i, ch in enumerate(seq):
        if not reverse:
            pack = ((pack << 4) | _NIB.get(ch, 0)) & _MASK64
        else:
            pack = (pack >> 4) | (_NIB_RC.get(ch, 0) << 60)
        if i >= 15:
            out.append(pack)
    return out


def pack_external(seq: str) -> List[int]:
    """A 16-mer at every position of seq, zero nibbles past its end."""
    n = len(seq)
    out = []
    pack = 0
    off = 0
    for _ in range(15):
        pack = ((pack << 4) | (_NIB.get(seq[off], 0) if off < n else 0)) & _MASK64
        off += 1
    for _ in range(n):
        pack = ((pack << 4) | (_NIB.get(seq[off], 0) if off < n else 0)) & _MASK64
        out.append(pack)
        off += 1
    return out


def single_mask(length: int) -> int:
    m = _MASK64
    if length < 16:
        m = (m << ((16 - length) * 4)) & _MASK64
    return m


def maximum_range(vals: List[float]) -> float:
    """Trimmomatic's calculateMaximumRange: group into same-sign runs, then repeatedly merge a negative
    run with both neighbours while each neighbour exceeds its magnitude; the largest remaining sum."""
    merges: List[float] = []
    total = 0.0
    for v in vals:
        if (total > 0 and v < 0) or (total < 0 and v > 0):
            merges.append(total)
            total = v
        else:
            total = _f32(total + v)
    merges.append(total)
    again = True
    while merges and again:
        again = False
        k = 1
        while k < len(merges) - 1:
            v = merges[k]
            if v < 0:
                prev, nxt = merges[k - 1], merges[k + 1]
                if prev > -v and nxt > -v:
                    merges[k - 1:k + 2] = [_f32(_f32(prev + v) + nxt)]
                    again = True
                    continue          # the merged run is re-examined by the next pass's scan position
            k += 1
    best = 0.0
    for v in merges:
        if v > best:
            best = v
    return best


class ClipSeq:
    """One simple-mode adapter (IlluminaLongClippingSeq; the short / medium classes of the Java code
    differ only in how they seed adapters under 24 bases, which NexteraPE-PE.fa does not hold)."""

    def __init__(self, seq: str, seed_max: int, min_overlap: int, min_likelihood: float):
        self.seq = seq
        full = pack_internal(seq, False)
        self.pack = [full[i] for i in range(0, len(full), INTERLEAVE)]
        self.seed_max = seed_max
        self.min_overlap = min_overlap
        self.min_likelihood = min_likelihood
        self.index: Dict[int, List[int]] = {}
        for j, p in enumerate(self.pack):
            self.index.setdefault(p, []).append(j)

    def quality(self, seq: str, quals: List[int], overlap: int, offset: int) -> float:
        rp = offset if offset > 0 else 0
        cp = -offset if offset < 0 else 0
        vals = []
        for _ in range(overlap):
            a, b = seq[rp], self.seq[cp]
            if a == "N" or b == "N":
                vals.append(0.0)
            elif a != b:
                vals.append(_f32(-quals[rp] / 10.0))
            else:
                vals.append(LOG10_4)
            rp += 1
            cp += 1
        return maximum_range(vals)

    def compare(self, seq: str, quals: List[int]) -> int:
        prec = pack_external(seq)
        n = len(prec)
        offsets = set()
        for i in range(n - self.min_overlap):
            mask = single_mask(n - i)
            lrec = prec[i] & mask
            if self.seed_max == 0 and mask == _MASK64:
                for j in self.index.get(lrec, ()):
                    offsets.add(i - j * INTERLEAVE)
                continue
            for j, lclip in enumerate(self.pack):
                if bin((lrec ^ lclip) & mask).count("1") <= self.seed_max:
                    offsets.add(i - j * INTERLEAVE)
        for off in sorted(offsets):
            rec_len = len(seq) - off if off > 0 else len(seq)
            clip_len = len(self.seq) + off if off < 0 else len(self.seq)
            comp = min(rec_len, clip_len)
            if comp > self.min_overlap and self.quality(seq, quals, comp, off) >= self.min_likelihood:
                return off
        return sys.maxsize


class PrefixPair:
    def __init__(self, p1: str, p2: str, seed_max: int, min_likelihood: float, min_prefix: int):
        m = min(len(p1), len(p2))
        self.p1, self.p2 = p1[len(p1) - m:], p2[len(p2) - m:]
        self.seed_max = seed_max
        self.min_likelihood = min_likelihood
        self.min_prefix = min_prefix

    def quality(self, s1, q1, s2, q2, overlap, skip1, skip2) -> float:
        a = self.p1 + s1
        b = self.p2 + s2
        pl = len(self.p1)
        total = 0.0
        for i in range(overlap):
            o1 = i + skip1
            o2 = skip2 + overlap - i - 1
            c1 = a[o1]
            c2 = _COMP.get(b[o2], b[o2])
            qa = 100 if o1 < pl else q1[o1 - pl]
            qb = 100 if o2 < pl else q2[o2 - pl]
            if c1 == "N" or c2 == "N":
                v = 0.0
            elif c1 != c2:
                v = _f32(-min(qa, qb) / 10.0)
            else:
                v = LOG10_4
            total = _f32(total + v)
        return total

    def compare(self, s1, q1, s2, q2) -> int:
        pack1 = pack_internal(self.p1 + s1, False)
        pack2 = pack_internal(self.p2 + s2, True)
        pl = len(self.p1)
        test, ref = 0, pl
        if len(pack1) <= ref or len(pack2) <= ref:
            return sys.maxsize
        count = 0
        skip = pl - 16
        if skip > 0:
            test = count = skip
        len1, len2 = len(s1) + pl, len(s2) + pl
        max_count = max(len1, len2) - 15 - self.min_prefix
        while count < max_count:
            r1, r2 = pack1[ref], pack2[ref]
            if ((test < len(pack2) and bin(r1 ^ pack2[test]).count("1") <= self.seed_max)
                    or (test < len(pack1) and bin(r2 ^ pack1[test]).count("1") <= self.seed_max)):
                total = count + pl + 16
                skip1 = skip2 = 0
                if total > len1:
                    skip2 = total - len1
                if total > len2:
                    skip1 = total - len2
                actual = total - skip1 - skip2
                if self.quality(s1, q1, s2, q2, actual, skip1, skip2) >= self.min_likelihood:
                    return total - 2 * pl
            count += 1
            if (count & 1) == 0 and ref + 1 < len(pack1) and ref + 1 < len(pack2):
                ref += 1
            else:
                test += 1
        return sys.maxsize


def read_fasta(path: str) -> List[Tuple[str, str]]:
    recs: List[Tuple[str, str]] = []
    name, seq = None, []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith(">"):
                if name is not None:
                    recs.append((name, "".join(seq)))
                name, seq = line[1:].split()[0] if len(line) > 1 else "", []
            elif line:
                seq.append(line.upper())
    if name is not None:
        recs.append((name, "".join(seq)))
    return recs


class IlluminaClip:
    def __init__(self, spec: str):
        a = spec.split(":")
        seed_mm, pal, simple = int(a[0 + 1]), int(a[2]), int(a[3])
        min_prefix = int(a[4]) if len(a) > 4 else 8
        keep_both = (a[5].lower() == "true") if len(a) > 5 else False
        self.keep_both = keep_both
        seed_max = seed_mm * 2
        min_ov = min(15, int(simple / LOG10_4))
        fwd, rev, com = {}, {}, {}
        fpre, rpre = set(), set()
        for name, seq in read_fasta(a[0]):
            if name.endswith("/1"):
                fwd[name] = seq
                if name.startswith("Prefix"):
                    fpre.add(name[:-2])
            elif name.endswith("/2"):
                rev[name] = seq
                if name.startswith("Prefix"):
                    rpre.add(name[:-2])
            else:
                com[name] = seq
        self.pairs = []
        for p in sorted(fpre & rpre):
            self.pairs.append(PrefixPair(fwd.pop(p + "/1"), rev.pop(p + "/2"), seed_max, pal, min_prefix))

        def clipset(d):
            seen, out = set(), []
            for s in d.values():
                if s not in seen:
                    seen.add(s)
                    out.append(ClipSeq(s, seed_max, min_ov, simple))
            return out
        self.fwd, self.rev, self.com = clipset(fwd), clipset(rev), clipset(com)

    def process(self, r1, r2):
        """r = (name, seq, qual-string) or None; returns the clipped records (None = dropped)."""
        keep1 = keep2 = sys.maxsize
        if r1 is not None and r2 is not None:
            q1 = [ord(c) - 33 for c in r1[2]]
            q2 = [ord(c) - 33 for c in r2[2]]
            for pp in self.pairs:
                k = pp.compare(r1[1], q1, r2[1], q2)
                if k < keep1:
                    keep1 = k
                    keep2 = k if self.keep_both else 0
        if r1 is not None:
            q = [ord(c) - 33 for c in r1[2]]
            for cs in self.fwd + self.com:
                keep1 = min(keep1, cs.compare(r1[1], q))
        if r2 is not None:
            q = [ord(c) - 33 for c in r2[2]]
            for cs in self.rev + self.com:
                keep2 = min(keep2, cs.compare(r2[1], q))
        return _cut(r1, keep1), _cut(r2, keep2)


def _cut(r, keep):
    if r is None or keep >= len(r[1]):
        return r
    if keep <= 0:
        return None
    return (r[0], r[1][:keep], r[2][:keep])


def read_fastq(path: str) -> Iterator[Tuple[str, str, str]]:
    op = gzip.open if open(path, "rb").read(2) == b"\x1f\x8b" else open
    with op(path, "rt") as f:
        while True:
            h = f.readline()
            if not h:
                return
            s = f.readline().rstrip("\n")
            f.readline()
            q = f.readline().rstrip("\n")
            yield h.rstrip("\n")[1:], s, q


def _open_out(path: str):
    return gzip.open(path, "wt", compresslevel=1) if path.endswith(".gz") else open(path, "w")


def _write(f, r):
    f.write(f"@{r[0]}\n{r[1]}\n+\n{r[2]}\n")


def run_pe(r1: str, r2: str, outs: List[str], steps: List[str]) -> Dict[str, int]:
    clip: Optional[IlluminaClip] = None
    minlen = 0
    for st in steps:
        if st.startswith("ILLUMINACLIP:"):
            clip = IlluminaClip(st[len("ILLUMINACLIP:"):])
        elif st.startswith("MINLEN:"):
            minlen = int(st.split(":")[1])
        else:
            raise SystemExit(f"trimmomatic restatement: step {st!r} not restated")
    fp, fu, rp, ru = (_open_out(p) for p in outs)
    st = {"pairs": 0, "both": 0, "fwd_only": 0, "rev_only": 0, "dropped": 0}
    for a, b in zip(read_fastq(r1), read_fastq(r2)):
        st["pairs"] += 1
        if clip is not None:
            a, b = clip.process(a, b)
        if a is not None and len(a[1]) < minlen:
            a = None
        if b is not None and len(b[1]) < minlen:
            b = None
        if a is not None and b is not None:
            _write(fp, a)
            _write(rp, b)
            st["both"] += 1
        elif a is not None:
            _write(fu, a)
            st["fwd_only"] += 1
        elif b is not None:
            _write(ru, b)
            st["rev_only"] += 1
        else:
            st["dropped"] += 1
    for f in (fp, fu, rp, ru):
        f.close()
    return st


def main(argv: Optional[List[str]] = None) -> int:
    """`trimmomatic PE [-phred33] R1 R2 fp fu rp ru STEP...` (the jar's argument order)."""
    a = list(sys.argv[1:] if argv is None else argv)
    if not a or a[0] != "PE":
        raise SystemExit("trimmomatic restatement: only PE mode is restated")
    a = [x for x in a[1:] if x not in ("-phred33",)]
    files, steps = a[:6], a[6:]
    st = run_pe(files[0], files[1], files[2:6], steps)
    sys.stderr.write(f"[Trimmomatic restatement] Input Read Pairs: {st['pairs']} Both Surviving: {st['both']} "
                     f"Forward Only Surviving: {st['fwd_only']} Reverse Only Surviving: {st['rev_only']} "
                     f"Dropped: {st['dropped']}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
