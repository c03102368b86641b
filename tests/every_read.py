"""Every-read parity of an ops batch (records + runs) against the CPU oracle.

TEST INFRASTRUCTURE ONLY (the oracle is the checker).  Identical reads have identical
oracle results (oracle/nw_oracle.c is a pure function of amplicon and read), so the
oracle runs once per distinct read: each distinct read's GPU record and the three rows
expanded from its GPU runs are compared with the oracle's, and every other read's GPU
record and runs must equal those of the first read with the same bytes.  Together that
is the comparison of every read with the oracle at a fraction of the oracle time (60 %
of a C2 batch are exact copies of the amplicon).
"""
from __future__ import annotations

import numpy as np

from crispresso_amd.aligner import OpsBatch
from oracle import oracle_py

FIELDS = ("aln_len", "n_ident", "n_sim", "n_gaps", "score", "end_i", "end_j")


def first_occurrence(buf: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    """rep[r] = the first read with read r's bytes (rep[r] == r for a distinct read)."""
    n = len(offsets) - 1
    mv = memoryview(np.ascontiguousarray(buf, dtype=np.uint8))
    off = offsets.tolist()
    seen: dict = {}
    rep = np.empty(n, np.int64)
    for r in range(n):
        rep[r] = seen.setdefault(mv[off[r]:off[r + 1]].tobytes(), r)
    return rep


def _same_runs(ops: np.ndarray, ops_off: np.ndarray, rep: np.ndarray) -> np.ndarray:
    """bad[r]: read r's run count or runs differ from those of rep[r]."""
    cnt = np.diff(ops_off)
    bad = cnt != cnt[rep]
    sel = np.flatnonzero(~bad & (rep != np.arange(len(rep))) & (cnt > 0))
    if not len(sel):
        return bad
    c = cnt[sel]
    starts = np.zeros(len(sel), np.int64)
    np.cumsum(c[:-1], out=starts[1:])
    ramp = np.arange(int(c.sum()), dtype=np.int64) - np.repeat(starts, c)
    a = ops[np.repeat(ops_off[sel], c) + ramp]
    b = ops[np.repeat(ops_off[rep[sel]], c) + ramp]
    diff = a != b
    if diff.any():
        owner = np.repeat(np.arange(len(sel)), c)
        bad[sel[np.unique(owner[diff])]] = True
    return bad


def check_subset(amplicon: str, buf: np.ndarray, offsets: np.ndarray, ob: OpsBatch, idx: np.ndarray,
                 threads: int, oracle_params=None) -> np.ndarray:
    """bad[q] for reads idx[q]: record and expanded rows vs the oracle."""
    lens = (offsets[idx + 1] - offsets[idx]).astype(np.int64)
    soff = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(lens, out=soff[1:])
    sbuf = np.empty(max(int(soff[-1]), 1), np.uint8)
    for q, r in enumerate(idx.tolist()):
        sbuf[soff[q]:soff[q + 1]] = buf[offsets[r]:offsets[r + 1]]
    cnt = ob.ops_off[idx + 1] - ob.ops_off[idx]
    sops_off = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(cnt, out=sops_off[1:])
    total = int(sops_off[-1])
    starts = np.repeat(ob.ops_off[idx], cnt) + (np.arange(total, dtype=np.int64) - np.repeat(sops_off[:-1], cnt))
    sub = OpsBatch(ob.stats[idx], ob.ops[starts], sops_off, lens, ob.scale)
    got = sub.expand(amplicon, sbuf, soff, nthreads=threads)
    res, aln = oracle_py.align_batch(amplicon, sbuf, soff, oracle_params, nthreads=threads)
    bad = np.zeros(len(idx), bool)
    for f in FIELDS:
        bad |= got.stats[f] != res[f]
    for q in np.flatnonzero(~bad).tolist():
        L = int(res["aln_len"][q])
        bad[q] = got.aln[q, :, :L].tobytes() != aln[q, :, :L].tobytes()
    return bad


def every_read(amplicon: str, buf: np.ndarray, offsets: np.ndarray, ob: OpsBatch, threads: int = 16,
               chunk: int = 100_000, oracle_params=None) -> dict:
    """Every read of `ob` (an ops batch of the reads buf/offsets against `amplicon`) vs the
    oracle.  -> {"reads": n, "distinct": d, "mismatches": k, "first_bad": [...]}."""
    offsets = np.asarray(offsets, dtype=np.int64)
    n = len(offsets) - 1
    rep = first_occurrence(buf, offsets)
    bad = np.zeros(n, bool)
    for f in FIELDS + ("flags",):
        col = ob.stats[f]
        bad |= col != col[rep]
    bad |= _same_runs(ob.ops, ob.ops_off, rep)
    uniq = np.flatnonzero(rep == np.arange(n))
    for lo in range(0, len(uniq), chunk):
        idx = uniq[lo:lo + chunk]
        bad[idx] |= check_subset(amplicon, buf, offsets, ob, idx, threads, oracle_params)
    bad |= bad[rep]   # a duplicate of a wrong distinct read is wrong too
    where = np.flatnonzero(bad)
    return {"reads": int(n), "distinct": int(len(uniq)), "mismatches": int(len(where)),
            "first_bad": where[:10].tolist()}


def every_read_records(stats: np.ndarray, ref: np.ndarray) -> int:
    """Reads whose records differ between two batches (e.g. a records-only pass vs the same
    pass with runs)."""
    bad = np.zeros(len(stats), bool)
    for f in FIELDS + ("flags",):
        bad |= stats[f] != ref[f]
    return int(bad.sum())


def every_read_multi(amplicons, buf, offsets, which, ob: OpsBatch, threads: int = 16) -> dict:
    """every_read over a pooled batch grouped by amplicon (which non-decreasing)."""
    offsets = np.asarray(offsets, dtype=np.int64)
    out = {"reads": 0, "distinct": 0, "mismatches": 0, "first_bad": []}
    bounds = np.searchsorted(which, np.arange(len(amplicons) + 1))
    for g, amp in enumerate(amplicons):
        lo, hi = int(bounds[g]), int(bounds[g + 1])
        if lo == hi:
            continue
        sub_off = offsets[lo:hi + 1] - offsets[lo]
        r0, r1 = int(ob.ops_off[lo]), int(ob.ops_off[hi])
        sub = OpsBatch(ob.stats[lo:hi], ob.ops[r0:r1], ob.ops_off[lo:hi + 1] - r0, np.diff(sub_off), ob.scale)
        res = every_read(amp, buf[offsets[lo]:offsets[hi]], sub_off, sub, threads)
        out["reads"] += res["reads"]
        out["distinct"] += res["distinct"]
        out["mismatches"] += res["mismatches"]
        out["first_bad"] += [lo + b for b in res["first_bad"]][: 10 - len(out["first_bad"])]
    return out

