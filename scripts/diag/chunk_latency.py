"""Latency of one pipelined call on the first S reads of the C2 batch (one chunk when S <= the
chunk size): how long a chunk's chain takes from its upload to its records in host memory, by
size.  Usage: chunk_latency.py [sizes, comma-separated] [calls]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import _lib, synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner, PackedReads, pack_2bit  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4096,16384,65536,262144").split(",")]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 30
nr = max(sizes)
amplicon = synth.random_amplicon(bench.AMPLICON_LEN, 1)
buf, off = synth.reads_from(amplicon, nr, 2)
pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
p_packed = _lib.PinnedBuffer((int(off[-1]) + 3) // 4 + 16, np.uint8)
p_lens = _lib.PinnedBuffer(max(nr, 1), np.uint16)
pr = pack_2bit(pb.array, po.array, packed=p_packed.array, lens=p_lens.array)
stats = _lib.PinnedBuffer(nr, _lib.STAT_DTYPE)
ops_off = _lib.PinnedBuffer(nr + 1, np.int64)
ops = _lib.PinnedBuffer(4 * nr + 4096, np.uint32)
al = GpuAligner(0)
al.set_reference(amplicon)
for s in sizes:
    sub = PackedReads(pr.packed, po.array[: s + 1], pr.exc_pos, pr.exc_byte, pr.lens[:s])
    out = (stats.array[:s], ops.array, ops_off.array[: s + 1])
    for _ in range(5):
        al.align_ops_packed(sub, out=out)
    t = []
    for _ in range(calls):
        t0 = time.perf_counter()
        al.align_ops_packed(sub, out=out)
        t.append((time.perf_counter() - t0) * 1e3)
    t = np.array(t)
    print(f"S={s:7d}: call median {np.median(t):.3f} ms min {t.min():.3f}  path_counts {al.path_counts()}  "
          f"ops_times {al.ops_times()}", flush=True)
al.close()
