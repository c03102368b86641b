"""Read sharding across GPUs: reads are independent, so N GPUs
take N contiguous read ranges and results are concatenated in read order.
There is no collective on the data path.

* :class:`MultiGpuAligner` -- one process, one host thread and one C-ABI
  context per device (ctypes releases the GIL during the GPU calls).  This is
  what the CRISPResso host uses on an 8-GPU node: a single run aligns its reads
  on every GPU.
* :func:`align_sharded` -- one process per GPU under torch.distributed
  (``torchrun``; RCCL on GPUs, gloo on CPU): each rank aligns its shard, rank 0
  gathers the records in read order.  Used when the host pipeline itself is
  run per rank.

Both take an aligner factory so tests can run the sharding on CPU with the
oracle-backed stand-in.
"""
from __future__ import annotations

import concurrent.futures as cf
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .aligner import AlignmentBatch


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of n reads for `rank` of `world` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


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


class MultiGpuAligner:
    """Aligns one batch on several devices at once (contiguous shards, one thread each)."""

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

    def set_reference(self, seq: str) -> None:
        for a in self.aligners:
            a.set_reference(seq)
        self.reference = seq

    def align_packed(self, buf: np.ndarray, offsets: np.ndarray, strings: bool = True) -> AlignmentBatch:
        n = len(offsets) - 1
        world = len(self.aligners)
        jobs = []
        for rank, al in enumerate(self.aligners):
            lo, hi = shard_range(n, world, rank)
            b, o = slice_batch(buf, offsets, lo, hi)
            jobs.append(self._pool.submit(al.align_packed, b, o, strings))
        return concat_batches([j.result() for j in jobs])

    def close(self) -> None:
        for a in self.aligners:
            a.close()
        self._pool.shutdown()


def align_sharded(amplicon: str, buf: np.ndarray, offsets: np.ndarray, aligner, dist=None,
                  gather: bool = True) -> Optional[AlignmentBatch]:
    """One rank's share of a torch.distributed alignment job.

    Every rank holds the same (buf, offsets) description of the job (or at
    least its own slice), aligns reads [lo, hi) with its local aligner and, if
    `gather`, rank 0 receives all shards in read order (others get None).
    """
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    lo, hi = shard_range(len(offsets) - 1, world, rank)
    b, o = slice_batch(buf, offsets, lo, hi)
    if aligner.reference != amplicon:
        aligner.set_reference(amplicon)
    mine = aligner.align_packed(b, o)
    if dist is None or world == 1:
        return mine
    if not gather:
        return mine
    payload = (mine.stats, mine.aln, mine.read_lens)
    got: List = [None] * world if rank == 0 else None
    dist.gather_object(payload, got, dst=0)
    if rank != 0:
        return None
    return concat_batches([AlignmentBatch(s, a, l, mine.scale, mine.awidth) for s, a, l in got])
