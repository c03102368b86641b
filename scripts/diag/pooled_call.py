"""Warm nw_align_multi_ops_packed calls on the C5 shape (bench.py pooled_workload), for
rocprofv3 traces of the pooled pipeline: python pooled_call.py [amplicons] [reads_per_amplicon].
python pooled_call.py single [reads]: the headline's nw_align_ops_packed call (C2) instead."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import _lib  # noqa: E402
from crispresso_amd.aligner import GpuAligner, pack_2bit  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] == "single":
    from crispresso_amd import synth
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else bench.READS_PER_GPU
    amplicon = synth.random_amplicon(bench.AMPLICON_LEN, 1)
    buf, off = synth.reads_from(amplicon, nr, 2)
    pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
    stats = _lib.PinnedBuffer(nr, _lib.STAT_DTYPE)
    ops_off = _lib.PinnedBuffer(nr + 1, np.int64)
    ops = _lib.PinnedBuffer(4 * nr + 4096, np.uint32)
    p_packed = _lib.PinnedBuffer((int(off[-1]) + 3) // 4 + 1, np.uint8)
    pr = pack_2bit(pb.array, po.array, packed=p_packed.array)
    al = GpuAligner(0)
    al.set_reference(amplicon)
    for i in range(4):
        t0 = time.perf_counter()
        al.align_ops_packed(pr, out=(stats.array, ops.array, ops_off.array))
        print(f"call {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
        time.sleep(0.05)
    al.close()
    sys.exit(0)
na = int(sys.argv[1]) if len(sys.argv) > 1 else 96
rpa = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
amps, buf, off, which = bench.pooled_workload(na, rpa)
n = len(off) - 1
pb, po, pw = _lib.pinned_copy(buf), _lib.pinned_copy(off), _lib.pinned_copy(which)
stats = _lib.PinnedBuffer(n, _lib.STAT_DTYPE)
ops_off = _lib.PinnedBuffer(n + 1, np.int64)
ops = _lib.PinnedBuffer(4 * n + 4096, np.uint32)
p_packed = _lib.PinnedBuffer((int(off[-1]) + 3) // 4 + 1, np.uint8)
pr = pack_2bit(pb.array, po.array, packed=p_packed.array)
al = GpuAligner(0)
out = (stats.array, ops.array, ops_off.array)
for i in range(3):
    t0 = time.perf_counter()
    al.align_multi_ops(amps, pr, None, pw.array, out=out)
    print(f"call {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
    time.sleep(0.05)   # an idle gap > 100 us marks the last call in the trace
al.close()
