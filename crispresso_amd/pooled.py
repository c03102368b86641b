"""Pooled amplicons in one GPU call (third row).

CRISPRessoPooled demultiplexes reads to amplicons (bowtie2,
CRISPRessoPooled.py:844-878, unchanged upstream) and then runs one CRISPResso
process per amplicon (CRISPRessoPooled.py:882-908), each spawning its own
`needle` pipelines.  Here the demultiplexed reads of every amplicon go to the
aligner at once: ``nw_align_multi`` uploads them grouped by amplicon, queues
each group's kernels back to back on one stream and returns all alignments in
the callers' order, so a 96-amplicon run is one host call instead of 96
process start-ups, 96 FASTA round trips and 96 single-threaded aligners.

With the ops output (the default, ``CRISPR_NW_OUTPUT``) the call is
``nw_align_multi_ops``: every amplicon's tables uploaded once, the reads (already
grouped by amplicon) pipelined over PCIe in chunks of one amplicon each, runs
back; each amplicon's rows are rebuilt on the host (``nw_expand_ops``).
"""
from __future__ import annotations

from typing import List, Sequence, Union

import numpy as np

from .aligner import AlignmentBatch, OpsBatch, default_output_mode, pack_reads

Reads = Union[Sequence[str], tuple]


def _packed(reads: Reads):
    if isinstance(reads, tuple) and len(reads) == 2 and isinstance(reads[0], np.ndarray):
        return reads
    return pack_reads(list(reads))


def align_pooled(amplicons: Sequence[str], reads_per_amplicon: Sequence[Reads], aligner) -> List[AlignmentBatch]:
    """Align each amplicon's reads against it, all in one aligner call.

    `reads_per_amplicon[g]` are the reads demultiplexed to `amplicons[g]`
    (a list of strings or a packed ``(buf, offsets)`` pair).  Returns one
    AlignmentBatch per amplicon, rows in that amplicon's read order.
    """
    if len(amplicons) != len(reads_per_amplicon):
        raise ValueError(f"{len(amplicons)} amplicons but {len(reads_per_amplicon)} read sets")
    parts = [_packed(r) for r in reads_per_amplicon]
    counts = [len(off) - 1 for _, off in parts]
    bufs, offs, base = [], [np.zeros(1, dtype=np.int64)], 0
    for buf, off in parts:
        bufs.append(np.asarray(buf, dtype=np.uint8)[off[0]:off[-1]])
        offs.append(np.asarray(off[1:], dtype=np.int64) - off[0] + base)
        base += int(off[-1] - off[0])
    buf = np.concatenate(bufs) if bufs else np.zeros(0, dtype=np.uint8)
    offsets = np.concatenate(offs)
    which = np.repeat(np.arange(len(amplicons), dtype=np.int32), counts)
    if hasattr(aligner, "align_multi_ops") and default_output_mode() == "ops":
        ob = aligner.align_multi_ops(list(amplicons), buf, offsets, which)
        out, lo = [], 0
        for g, k in enumerate(counts):
            o0, o1 = int(ob.ops_off[lo]), int(ob.ops_off[lo + k])
            sub = OpsBatch(ob.stats[lo:lo + k].copy(), ob.ops[o0:o1], ob.ops_off[lo:lo + k + 1] - o0,
                           ob.read_lens[lo:lo + k], ob.scale, ob.awidth)
            gbuf, goff = parts[g]
            out.append(sub.expand(amplicons[g], np.asarray(gbuf, dtype=np.uint8), np.asarray(goff, dtype=np.int64)))
            lo += k
        return out
    whole = aligner.align_multi(list(amplicons), buf, offsets, which)
    out, lo = [], 0
    for g, k in enumerate(counts):
        sl = slice(lo, lo + k)
        width = len(amplicons[g]) + (int(np.diff(parts[g][1]).max()) if k else 1)
        stride = max(16, ((width + 15) // 16) * 16)
        out.append(AlignmentBatch(whole.stats[sl].copy(), whole.aln[sl, :, :stride].copy(), whole.read_lens[sl].copy(),
                                  whole.scale, whole.awidth))
        lo += k
    return out
