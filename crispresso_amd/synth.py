"""Synthetic amplicon-sequencing workloads, vectorised numpy.

Used by bench.py and the tests; seeds and mixes follow SURVEY.md 8(d):

* C2: 250 bp amplicon (seed 1), reads (seed 2): 60% exact, 20% with 1-3
  substitutions, 10% one deletion (length ~ Geom(0.3) truncated to 1-30,
  start in 125 +/- 10), 5% one insertion of 1-10 random bases (125 +/- 10),
  5% with 1%-per-base substitution noise.
* parity mix (seed 3): the same plus 0.5%-per-base N, 2% reverse-complemented
  reads, and indels placed inside homopolymer runs (co-optimal gap placement).
* C3: HDR amplicon = amplicon with bases 120-129 replaced (seed 4); 15% of the
  reads are drawn from the HDR amplicon.
* C5: 96 amplicons of length U[150, 300] (seed 5).

All generators return (buf uint8, offsets int64) packed batches; reads are
bytes over ``ACGTN``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTN-", b"TGCAN-"):
    _COMP[_a] = _b


def random_amplicon(length: int, seed: int) -> str:
    rng = np.random.Generator(np.random.PCG64(seed))
    return BASES[rng.integers(0, 4, size=length)].tobytes().decode()


def hdr_amplicon(amplicon: str, seed: int = 4, start: int = 120, length: int = 10) -> str:
    rng = np.random.Generator(np.random.PCG64(seed))
    a = np.frombuffer(amplicon.encode(), dtype=np.uint8).copy()
    codes = np.searchsorted(BASES, a[start:start + length])
    a[start:start + length] = BASES[(codes + rng.integers(1, 4, size=length)) % 4]
    return a.tobytes().decode()


def _pack(mat: np.ndarray, lens: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    mask = np.arange(mat.shape[1])[None, :] < lens[:, None]
    return np.ascontiguousarray(mat[mask]), offsets


@dataclass
class Mix:
    exact: float = 0.60
    subs: float = 0.20
    deletion: float = 0.10
    insertion: float = 0.05
    noise: float = 0.05
    n_rate: float = 0.0         # per-base probability of N
    rc_frac: float = 0.0        # fraction reverse-complemented
    homopolymer: bool = False   # place indels inside homopolymer runs when possible


C2_MIX = Mix()
PARITY_MIX = Mix(exact=0.50, subs=0.20, deletion=0.12, insertion=0.08, noise=0.10, n_rate=0.005,
                 rc_frac=0.02, homopolymer=True)


def _homopolymer_starts(amp: np.ndarray) -> np.ndarray:
    run_start = np.r_[True, amp[1:] != amp[:-1]]
    starts = np.flatnonzero(run_start)
    lens = np.diff(np.r_[starts, len(amp)])
    return starts[lens >= 2]


def reads_from(amplicon: str, n: int, seed: int, mix: Mix = C2_MIX) -> Tuple[np.ndarray, np.ndarray]:
    """n reads derived from `amplicon` with the SURVEY 8d mutation mix."""
    rng = np.random.Generator(np.random.PCG64(seed))
    amp = np.frombuffer(amplicon.encode(), dtype=np.uint8)
    La = len(amp)
    probs = np.array([mix.exact, mix.subs, mix.deletion, mix.insertion, mix.noise], dtype=np.float64)
    kind = rng.choice(5, size=n, p=probs / probs.sum())
    width = La + 12
    idx = np.arange(width)[None, :]
    src = np.broadcast_to(idx, (n, width)).copy()     # source position in amp, -1 = random base
    lens = np.full(n, La, dtype=np.int64)
    centre = La // 2
    hp = _homopolymer_starts(amp) if mix.homopolymer else np.zeros(0, np.int64)

    def positions(sel: np.ndarray) -> np.ndarray:
        p = centre + rng.integers(-10, 11, size=sel.size)
        if hp.size and mix.homopolymer:
            use = rng.random(sel.size) < 0.5
            p = np.where(use, hp[rng.integers(0, hp.size, size=sel.size)], p)
        return np.clip(p, 1, La - 1)

    d_sel = np.flatnonzero(kind == 2)
    if d_sel.size:
        d = np.minimum(rng.geometric(0.3, size=d_sel.size), 30)
        p = positions(d_sel)
        d = np.minimum(d, La - p - 1)
        rows = src[d_sel]
        src[d_sel] = np.where(rows < p[:, None], rows, rows + d[:, None])
        lens[d_sel] = La - d
    i_sel = np.flatnonzero(kind == 3)
    if i_sel.size:
        k = rng.integers(1, 11, size=i_sel.size)
        p = positions(i_sel)
        rows = src[i_sel]
        src[i_sel] = np.where(rows < p[:, None], rows, np.where(rows < (p + k)[:, None], -1, rows - k[:, None]))
        lens[i_sel] = La + k
    valid = idx < lens[:, None]
    src = np.where(valid & (src >= La), La - 1, src)
    mat = np.where(src >= 0, amp[np.clip(src, 0, La - 1)], BASES[rng.integers(0, 4, size=src.shape)])
    mat = mat.astype(np.uint8)

    def substitute(rows: np.ndarray, mask: np.ndarray) -> None:
        cur = mat[rows]
        codes = np.searchsorted(BASES, cur)
        shifted = BASES[(np.clip(codes, 0, 3) + rng.integers(1, 4, size=cur.shape)) % 4]
        mat[rows] = np.where(mask, shifted, cur)

    s_sel = np.flatnonzero(kind == 1)
    if s_sel.size:
        nsub = rng.integers(1, 4, size=s_sel.size)
        keys = rng.random((s_sel.size, width))
        keys[:, La:] = 2.0
        thr = np.sort(keys, axis=1)[np.arange(s_sel.size), nsub - 1]
        substitute(s_sel, keys <= thr[:, None])
    z_sel = np.flatnonzero(kind == 4)
    if z_sel.size:
        substitute(z_sel, rng.random((z_sel.size, width)) < 0.01)
    if mix.n_rate > 0:
        mat = np.where(rng.random(mat.shape) < mix.n_rate, np.uint8(ord("N")), mat)
    if mix.rc_frac > 0:
        rc = np.flatnonzero(rng.random(n) < mix.rc_frac)
        for r in rc:
            L = lens[r]
            mat[r, :L] = _COMP[mat[r, :L][::-1]]
    return _pack(mat, lens)


def c2_workload(n: int = 1_000_000, seed: int = 2) -> Tuple[str, np.ndarray, np.ndarray]:
    amp = random_amplicon(250, 1)
    buf, off = reads_from(amp, n, seed)
    return amp, buf, off


def c3_workload(n: int = 1_000_000, seed: int = 2) -> Tuple[str, str, np.ndarray, np.ndarray]:
    amp = random_amplicon(250, 1)
    hdr = hdr_amplicon(amp, 4)
    n_hdr = int(round(0.15 * n))
    b1, o1 = reads_from(amp, n - n_hdr, seed)
    b2, o2 = reads_from(hdr, n_hdr, seed + 1000)
    buf = np.concatenate([b1, b2])
    off = np.concatenate([o1, o2[1:] + o1[-1]])
    return amp, hdr, buf, off


def window_reads(amplicon: str, n: int, seed: int, read_len: int = 151, mix: Mix = C2_MIX
                 ) -> Tuple[np.ndarray, np.ndarray]:
    """Reads shorter than the amplicon (the reference's own test shape: 151 bp reads against the
    280 bp amplicon, tests/crispresso_tests.py:145-155): read r covers amplicon[s : s + read_len]
    for an offset s drawn uniformly from 0 .. La - read_len, with the `mix` edits applied to that
    window (indels at its centre).  Reads of all offsets interleaved (seeded permutation)."""
    La = len(amplicon)
    span = La - read_len + 1
    if span < 1:
        raise ValueError("read_len exceeds the amplicon")
    rng = np.random.Generator(np.random.PCG64(seed))
    s_of = rng.integers(0, span, size=n)
    counts = np.bincount(s_of, minlength=span)
    parts = []
    for s_off in range(span):
        if counts[s_off]:
            parts.append(reads_from(amplicon[s_off:s_off + read_len], int(counts[s_off]), seed * 1000 + s_off, mix))
    lens = np.concatenate([np.diff(o) for _, o in parts])
    starts = np.concatenate([o[:-1] + base for (_, o), base in
                             zip(parts, np.cumsum([0] + [len(b) for b, _ in parts[:-1]]))])
    allbuf = np.concatenate([b for b, _ in parts])
    perm = rng.permutation(n)
    lens_p = lens[perm]
    off = np.zeros(n + 1, np.int64)
    np.cumsum(lens_p, out=off[1:])
    src = np.repeat(starts[perm], lens_p) + (np.arange(int(off[-1]), dtype=np.int64) - np.repeat(off[:-1], lens_p))
    return np.ascontiguousarray(allbuf[src]), off


def c1_shape_workload(n: int = 1_000_000, seed: int = 6) -> Tuple[str, np.ndarray, np.ndarray]:
    """C1 at volume: 151 bp windows of a 280 bp amplicon (seed 6) with the C2 edit mix."""
    amp = random_amplicon(280, seed)
    buf, off = window_reads(amp, n, seed + 1)
    return amp, buf, off


def pooled_amplicons(k: int = 96, seed: int = 5) -> list:
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = rng.integers(150, 301, size=k)
    return [random_amplicon(int(L), seed * 1000 + i) for i, L in enumerate(lens)]


def unpack(buf: np.ndarray, offsets: np.ndarray) -> list:
    b = buf.tobytes()
    return [b[offsets[i]:offsets[i + 1]].decode() for i in range(len(offsets) - 1)]


def native_reads(amplicon: str, n: int, seed: int, mix: Mix = C2_MIX, nthreads: int = 0,
                 buf: Optional[np.ndarray] = None, first: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """n reads of the C2 / C4 mix from the native generator (include/crispr_synth.h):
    the same mutation kinds and rates as :func:`reads_from` (no N, RC or homopolymer
    options), a counter-based RNG instead of numpy's PCG64, ~30x faster.  Used for the
    large sets (C4 shards of 12.5M reads).  ``first``: reads first .. first + n - 1 of
    the set (any range is generated on its own).  ``buf``: a preallocated uint8 array
    (e.g. pinned) of at least the range's bytes."""
    from . import _lib

    if mix.n_rate or mix.rc_frac or mix.homopolymer:
        raise ValueError("native_reads: the N / RC / homopolymer options are numpy-only (reads_from)")
    lib = _lib.load()
    amp = amplicon.encode("ascii")
    w = np.array([mix.exact, mix.subs, mix.deletion, mix.insertion, mix.noise], dtype=np.float64)
    off = np.empty(n + 1, np.int64)
    total = lib.nw_synth_offsets(amp, len(amp), first, n, seed, _lib.ptr(w), _lib.ptr(off), nthreads)
    if total < 0:
        raise ValueError("nw_synth_offsets: bad arguments")
    if buf is None:
        buf = np.empty(max(int(total), 1), np.uint8)
    elif len(buf) < total:
        raise ValueError(f"buffer of {len(buf)} bytes < {total}")
    if lib.nw_synth_reads(amp, len(amp), first, n, seed, _lib.ptr(w), _lib.ptr(off), _lib.ptr(buf), nthreads) != 0:
        raise ValueError("nw_synth_reads failed")
    return buf[: int(total)], off


def native_offsets(amplicon: str, n: int, seed: int, mix: Mix = C2_MIX, first: int = 0) -> np.ndarray:
    """Only the offsets of :func:`native_reads` (lengths without the bytes: cheap)."""
    from . import _lib

    lib = _lib.load()
    amp = amplicon.encode("ascii")
    w = np.array([mix.exact, mix.subs, mix.deletion, mix.insertion, mix.noise], dtype=np.float64)
    off = np.empty(n + 1, np.int64)
    if lib.nw_synth_offsets(amp, len(amp), first, n, seed, _lib.ptr(w), _lib.ptr(off), 0) < 0:
        raise ValueError("nw_synth_offsets: bad arguments")
    return off
