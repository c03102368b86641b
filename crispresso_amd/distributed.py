"""Read sharding across GPUs: reads are independent, so N GPUs
take N contiguous read ranges and results are concatenated in read order.
There is no collective on the data path.

* :class:`MultiGpuAligner` -- one process, one host thread and one C-ABI
  context per device (ctypes releases the GIL during the GPU calls).  This is
  what the CRISPResso host uses on an 8-GPU node: a single run aligns its reads
  on every GPU.
* :func:`align_sharded` / :func:`align_pooled_sharded` -- one process per GPU
  under torch.distributed (``torchrun``; the host-side process group is gloo:
  the data never touches a collective, only the compact results are gathered):
  each rank aligns its shard, rank 0 gathers the records and traceback runs
  (about 45 B per read, not the rows) in read order.

Balance: single-amplicon batches split into equal read counts; pooled batches
(C5: 96 amplicons of 150-300 bp) split by DP cells, ``len(amplicon) * len(read)``
per read (:func:`cell_partition`), contiguous in the grouped read order so each
device aligns whole amplicon groups plus at most two partial ones.

All entry points take an aligner (or a factory) so tests can run the sharding on
CPU with the oracle-backed stand-in.
"""
from __future__ import annotations

import concurrent.futures as cf
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .aligner import AlignmentBatch, OpsBatch


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of n reads for `rank` of `world` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def cell_partition(costs: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) ranges of the reads whose summed costs are as equal as a
    contiguous split allows: boundaries where the running cost crosses k / world of the
    total (each part is within one read's cost of the ideal share)."""
    costs = np.asarray(costs, dtype=np.float64)
    n = len(costs)
    if n == 0 or world == 1:
        return [shard_range(n, world, r) for r in range(world)]
    cum = np.cumsum(costs)
    total = cum[-1]
    cuts = [0]
    for k in range(1, world):
        cuts.append(max(cuts[-1], int(np.searchsorted(cum, total * k / world, side="left")) + 1))
    cuts.append(n)
    cuts = [min(c, n) for c in cuts]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def pooled_costs(amplicons: Sequence[str], offsets: np.ndarray, amplicon_of_read: np.ndarray) -> np.ndarray:
    """DP cells of every read of a pooled batch: len(its amplicon) x len(read)."""
    amp_len = np.array([len(a) for a in amplicons], dtype=np.int64)
    return amp_len[np.asarray(amplicon_of_read)] * np.diff(np.asarray(offsets, dtype=np.int64))


def slice_batch(buf: np.ndarray, offsets: np.ndarray, lo: int, hi: int) -> Tuple[np.ndarray, np.ndarray]:
    sub = offsets[lo:hi + 1]
    return buf[sub[0]:sub[-1]], sub - sub[0]


def concat_batches(parts: Sequence[AlignmentBatch]) -> AlignmentBatch:
    parts = [p for p in parts if len(p)] or list(parts[:1])
    stride = max(p.aln.shape[2] for p in parts)
    aln = np.zeros((sum(len(p) for p in parts), 3, stride), dtype=np.uint8)
    r = 0
    for p in parts:
        aln[r:r + len(p), :, : p.aln.shape[2]] = p.aln
        r += len(p)
    return AlignmentBatch(np.concatenate([p.stats for p in parts]), aln,
                          np.concatenate([p.read_lens for p in parts]), parts[0].scale, parts[0].awidth)


def concat_ops(parts: Sequence[OpsBatch]) -> OpsBatch:
    """Shards' records and runs in read order (run offsets rebased)."""
    parts = list(parts)
    offs, base = [np.zeros(1, np.int64)], 0
    for p in parts:
        offs.append(p.ops_off[1:] - p.ops_off[0] + base)
        base += int(p.ops_off[-1] - p.ops_off[0])
    return OpsBatch(np.concatenate([p.stats for p in parts]),
                    np.concatenate([p.ops for p in parts]) if parts else np.zeros(0, np.uint32),
                    np.concatenate(offs), np.concatenate([p.read_lens for p in parts]),
                    parts[0].scale, parts[0].awidth, has_runs=all(getattr(p, "has_runs", True) for p in parts))


class MultiGpuAligner:
    """Aligns one batch on several devices at once (contiguous shards, one thread each).

    Drop-in for :class:`~crispresso_amd.aligner.GpuAligner` in ``needle.align_reads``:
    ``align_ops_packed`` takes the pinned 2-bit batch of the native ingest (each device
    uploads only its shard's packed bytes), ``align_ops(..., resident=True)`` re-aligns
    every device's last shard where it lies in HBM (the HDR pass)."""

    ops_native = True

    def __init__(self, devices: Sequence[int], factory: Optional[Callable] = None, options=None):
        if factory is None:
            from .aligner import GpuAligner

            factory = GpuAligner
        self.devices = list(devices)
        self.aligners = [factory(d, options) for d in self.devices]
        self.options = self.aligners[0].options
        self.scale = self.aligners[0].scale
        self.reference: Optional[str] = None
        self._pool = cf.ThreadPoolExecutor(max_workers=len(self.devices))
        self._resident = None   # (n, per-device shard offsets) of the last upload

    def set_reference(self, seq: str) -> None:
        for a in self.aligners:
            a.set_reference(seq)
        self.reference = seq

    def _shards(self, n: int, costs: Optional[np.ndarray] = None):
        world = len(self.aligners)
        return cell_partition(costs, world) if costs is not None else [shard_range(n, world, r) for r in range(world)]

    def align_packed(self, buf: np.ndarray, offsets: np.ndarray, strings: bool = True) -> AlignmentBatch:
        jobs = []
        for al, (lo, hi) in zip(self.aligners, self._shards(len(offsets) - 1)):
            b, o = slice_batch(buf, offsets, lo, hi)
            jobs.append(self._pool.submit(al.align_packed, b, o, strings))
        return concat_batches([j.result() for j in jobs])

    def align_ops(self, buf: Optional[np.ndarray], offsets: np.ndarray, resident: bool = False,
                  records_only: bool = False) -> OpsBatch:
        """Records + runs of every read (nw_align_ops per device, shards in parallel).
        ``resident``: every device re-aligns the shard its last call uploaded (against the
        current amplicon; ``offsets`` must be that batch's)."""
        from .aligner import NeedleError

        n = len(offsets) - 1
        jobs = []
        if resident:
            if self._resident is None or self._resident[0] != n:
                raise NeedleError(f"no resident batch of these {n} reads on the devices")
            for al, o in zip(self.aligners, self._resident[1]):
                jobs.append(self._pool.submit(al.align_ops, None, o, None, True, records_only))
            return concat_ops([j.result() for j in jobs])
        shard_offs = []
        for al, (lo, hi) in zip(self.aligners, self._shards(n)):
            b, o = slice_batch(buf, offsets, lo, hi)
            shard_offs.append(o)
            jobs.append(self._pool.submit(al.align_ops, b, o, None, False, records_only))
        out = concat_ops([j.result() for j in jobs])
        self._resident = (n, shard_offs)
        return out

    def align_ops_packed(self, pr) -> OpsBatch:
        """The pinned 2-bit batch (aligner.PackedReads) over the devices: device k's call
        takes reads [lo, hi) -- its slice of the offsets (batch positions unchanged), the
        same packed bytes (it uploads only its own), the exceptions inside its range."""
        from .aligner import PackedReads

        n = len(pr.offsets) - 1
        jobs, shard_offs = [], []
        for al, (lo, hi) in zip(self.aligners, self._shards(n)):
            o = pr.offsets[lo:hi + 1]
            e0, e1 = np.searchsorted(pr.exc_pos, [o[0], o[-1]]) if len(pr.exc_pos) else (0, 0)
            sub = PackedReads(pr.packed, o, pr.exc_pos[e0:e1], pr.exc_byte[e0:e1],
                              pr.lens[lo:hi] if pr.lens is not None else None)
            shard_offs.append(o)
            jobs.append(self._pool.submit(al.align_ops_packed, sub))
        out = concat_ops([j.result() for j in jobs])
        self._resident = (n, shard_offs)
        return out

    def align_multi_ops(self, amplicons: Sequence[str], buf: np.ndarray, offsets: np.ndarray,
                        amplicon_of_read: np.ndarray) -> OpsBatch:
        """Pooled batch over the devices, split by DP cells."""
        which = np.asarray(amplicon_of_read, dtype=np.int32)
        jobs = []
        for al, (lo, hi) in zip(self.aligners, self._shards(len(offsets) - 1,
                                                             pooled_costs(amplicons, offsets, which))):
            b, o = slice_batch(buf, offsets, lo, hi)
            jobs.append(self._pool.submit(al.align_multi_ops, list(amplicons), b, o, which[lo:hi]))
        out = concat_ops([j.result() for j in jobs])
        # as GpuAligner: every context is left without an amplicon (set_reference before the next pass)
        self.reference = None
        self._resident = None
        return out

    def close(self) -> None:
        for a in self.aligners:
            a.close()
        self._pool.shutdown()


def _populate(mm, lo: int, hi: int) -> None:
    """Fault in bytes [lo, hi) of a shared mapping in one call (MADV_POPULATE_WRITE, Linux 5.14+;
    without it the first writes fault page by page)."""
    if hi <= lo:
        return
    page = 4096
    a, b = lo - lo % page, min(len(mm), hi + (-hi) % page)
    try:
        mm.madvise(23, a, b - a)
    except (OSError, ValueError, AttributeError):
        pass


def _gather_ops(mine: OpsBatch, dist, rank: int, world: int, method: str = "auto") -> Optional[OpsBatch]:
    """Rank 0 receives every rank's records + runs in rank order (others get None) -- no pickling
    (round 5 sent them through ``gather_object``: pickled objects over gloo TCP, ~4.5 GB into rank 0
    for C4).  The part sizes go first (one ``all_gather`` of four int64 per rank), then ``method``:

    * ``"shm"`` -- ranks on one host (torchrun's LOCAL_WORLD_SIZE == WORLD_SIZE: the 8-GPU node of
      SURVEY 8e): rank 0 creates one shared-memory segment laid out as the joined arrays (records 32 B
      per read, runs uint32, run offsets int64, read lengths int64); every rank faults in and writes
      its own slices in parallel (its run offsets already rebased); rank 0's result is views of the
      segment (unlinked at once: it lives as long as the returned batch) -- no copy on rank 0;
    * ``"p2p"`` -- otherwise: each rank sends its arrays as tensors (``isend``; records as bytes, runs
      as int32) and rank 0 receives them into the joined arrays' slices (every ``irecv`` in flight);
    * ``"auto"`` -- shm when the ranks share the host, else p2p.
    """
    import mmap
    import os

    import torch

    if method == "auto":
        local = int(os.environ.get("LOCAL_WORLD_SIZE", "0") or 0)
        method = "shm" if local == world else "p2p"
    n = len(mine)
    off0 = int(mine.ops_off[0]) if len(mine.ops_off) else 0
    has = bool(mine.has_runs)
    nr = int(mine.ops_off[-1]) - off0 if (len(mine.ops_off) and has) else 0
    ops = np.ascontiguousarray(mine.ops[off0:off0 + nr]) if has else np.zeros(0, np.uint32)
    stats = np.ascontiguousarray(mine.stats)
    lens = np.ascontiguousarray(mine.read_lens, dtype=np.int64)
    offs = np.ascontiguousarray(mine.ops_off, dtype=np.int64)
    mine_sz = torch.tensor([n, nr, int(has), os.getpid()], dtype=torch.int64)
    allsz = [torch.zeros(4, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allsz, mine_sz)
    szs = [tuple(int(v) for v in t.tolist()) for t in allsz]
    N = sum(z[0] for z in szs)
    all_runs = all(z[2] for z in szs)
    R = sum(z[1] for z in szs) if all_runs else 0
    lo = sum(z[0] for z in szs[:rank])
    rbase = sum(z[1] for z in szs[:rank])
    sb = stats.dtype.itemsize
    if method == "shm":
        # layout: records | runs | run offsets | read lengths (8-byte aligned sections)
        o_stats = 0
        o_ops = N * sb
        o_off = o_ops + 4 * R + (-(4 * R)) % 8
        o_lens = o_off + 8 * (N + 1)
        total = max(o_lens + 8 * N, 1)
        path = f"/dev/shm/crispr_gather_{os.environ.get('MASTER_PORT', '0')}_{szs[0][3]}"
        if rank == 0:
            fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
            os.ftruncate(fd, total)
        dist.barrier()
        if rank != 0:
            fd = os.open(path, os.O_RDWR)
        mm = mmap.mmap(fd, total)
        os.close(fd)
        view = np.ndarray(total, np.uint8, buffer=mm)
        out_stats = view[o_stats:o_stats + N * sb].view(stats.dtype)
        out_ops = view[o_ops:o_ops + 4 * R].view(np.uint32)
        out_off = view[o_off:o_off + 8 * (N + 1)].view(np.int64)
        out_lens = view[o_lens:o_lens + 8 * N].view(np.int64)
        for a_, b_ in ((o_stats + lo * sb, o_stats + (lo + n) * sb), (o_ops + 4 * rbase, o_ops + 4 * (rbase + nr)),
                       (o_off + 8 * lo, o_off + 8 * (lo + n + 1)), (o_lens + 8 * lo, o_lens + 8 * (lo + n))):
            _populate(mm, a_, b_)
        out_stats[lo:lo + n].view(np.uint8)[...] = stats.view(np.uint8)   # bytes: a structured copy is 10x slower
        if all_runs:
            out_ops[rbase:rbase + nr] = ops
        if n:
            np.subtract(offs[1:], offs[0] - rbase, out=out_off[lo + 1:lo + n + 1])
        if rank == 0:
            out_off[0] = 0
        out_lens[lo:lo + n] = lens
        dist.barrier()   # every part written
        if rank != 0:
            del view, out_stats, out_ops, out_off, out_lens
            mm.close()
            return None
        os.unlink(path)   # the mapping stays until the batch is freed
        res = OpsBatch(out_stats, out_ops, out_off, out_lens, mine.scale, mine.awidth, has_runs=all_runs)
        res._shm = mm
        return res
    parts = [(stats.view(np.uint8), 0), (ops.view(np.int32), 1), (offs, 2), (lens, 3)]
    if rank != 0:
        reqs = [dist.isend(torch.from_numpy(x.reshape(-1)), dst=0, tag=k) for x, k in parts if x.size]
        for q in reqs:
            q.wait()
        return None
    out_stats = np.empty(N, dtype=stats.dtype)
    out_ops = np.empty(R, dtype=np.uint32)
    out_off = np.zeros(N + 1, dtype=np.int64)
    out_lens = np.empty(N, dtype=np.int64)
    reqs, part_offs = [], []
    plo = pr = 0
    for r, (pn, pnr, _, _) in enumerate(szs):
        dst = [out_stats[plo:plo + pn].view(np.uint8), out_ops[pr:pr + pnr].view(np.int32) if all_runs else None,
               np.empty(pn + 1, np.int64), out_lens[plo:plo + pn]]
        if r == 0:
            for d, (x, _) in zip(dst, parts):
                if d is not None and x.size:
                    d[...] = x
        else:
            for k, d in enumerate(dst):
                if d is not None and d.size:
                    reqs.append(dist.irecv(torch.from_numpy(d.reshape(-1)), src=r, tag=k))
        part_offs.append((dst[2], plo, pn, pr))
        plo, pr = plo + pn, pr + pnr
    for q in reqs:
        q.wait()
    for po, plo, pn, pr in part_offs:
        if pn:
            np.subtract(po[1:], po[0] - pr, out=out_off[plo + 1:plo + pn + 1])
    return OpsBatch(out_stats, out_ops, out_off, out_lens, mine.scale, mine.awidth, has_runs=all_runs)


def align_sharded(amplicon: str, buf: np.ndarray, offsets: np.ndarray, aligner, dist=None,
                  gather: bool = True):
    """One rank's share of a torch.distributed alignment job.

    Every rank holds the same (buf, offsets) description of the job (or at
    least its own slice), aligns reads [lo, hi) with its local aligner and, if
    `gather`, rank 0 receives all shards in read order (others get None): an
    :class:`OpsBatch` (records + runs; ``.expand`` builds the rows) when the aligner
    has the ops path, else an :class:`AlignmentBatch`.
    """
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    lo, hi = shard_range(len(offsets) - 1, world, rank)
    b, o = slice_batch(buf, offsets, lo, hi)
    if aligner.reference != amplicon:
        aligner.set_reference(amplicon)
    ops = hasattr(aligner, "align_ops")
    mine = aligner.align_ops(b, o) if ops else aligner.align_packed(b, o)
    if dist is None or world == 1 or not gather:
        return mine
    if ops:
        return _gather_ops(mine, dist, rank, world)
    payload = (mine.stats, mine.aln, mine.read_lens)
    got: List = [None] * world if rank == 0 else None
    dist.gather_object(payload, got, dst=0)
    if rank != 0:
        return None
    return concat_batches([AlignmentBatch(s, a, l, mine.scale, mine.awidth) for s, a, l in got])


def align_pooled_sharded(amplicons: Sequence[str], buf: np.ndarray, offsets: np.ndarray,
                         amplicon_of_read: np.ndarray, aligner, dist=None, gather: bool = True) -> Optional[OpsBatch]:
    """One rank's share of a pooled job (C5): reads split by DP cells
    (:func:`cell_partition`), each rank aligns its range with one
    ``align_multi_ops`` call, rank 0 gathers records + runs in read order."""
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    which = np.asarray(amplicon_of_read, dtype=np.int32)
    lo, hi = cell_partition(pooled_costs(amplicons, offsets, which), world)[rank]
    b, o = slice_batch(buf, offsets, lo, hi)
    mine = aligner.align_multi_ops(list(amplicons), b, o, which[lo:hi])
    if dist is None or world == 1 or not gather:
        return mine
    return _gather_ops(mine, dist, rank, world)
