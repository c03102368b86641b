"""Diagnostics: per-call ms of the pooled (C5) call and the C4-shard call, in a given order,
to find where warm-up / state effects come from."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import _lib, synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner  # noqa: E402


def main():
    al = GpuAligner(0)
    amp = synth.random_amplicon(250, 1)
    amps = synth.pooled_amplicons(96, 5)
    _, buf, off, which = bench.pooled_workload(96, 100_000)
    ppr, keep1 = bench.pack_pinned(buf, off, 16)
    pw = _lib.pinned_copy(which)
    n = len(off) - 1
    pout = (_lib.PinnedBuffer(n, _lib.STAT_DTYPE).array, _lib.PinnedBuffer(4 * n + 4096, np.uint32).array,
            _lib.PinnedBuffer(n + 1, np.int64).array)
    t, o = synth.native_reads(amp, 12_500_000, 10)
    cpr, keep2 = bench.pack_pinned(t, o, 16)
    m = len(o) - 1
    cout = (_lib.PinnedBuffer(m, _lib.STAT_DTYPE).array, _lib.PinnedBuffer(2 * m + 4096, np.uint32).array,
            _lib.PinnedBuffer(m + 1, np.int64).array)
    t2, o2 = synth.reads_from(amp, 1_000_000, 2)
    hpr, keep3 = bench.pack_pinned(t2, o2, 16)
    k = len(o2) - 1
    hout = (_lib.PinnedBuffer(k, _lib.STAT_DTYPE).array, _lib.PinnedBuffer(2 * k + 4096, np.uint32).array,
            _lib.PinnedBuffer(k + 1, np.int64).array)
    for what in sys.argv[1:]:
        name, reps = what.split(":")
        ms = []
        for _ in range(int(reps)):
            t0 = time.perf_counter()
            if name == "pooled":
                al.align_multi_ops(amps, ppr, None, pw.array, out=pout)
            elif name == "c4":
                al.set_reference(amp)
                al.align_ops_packed(cpr, out=cout)
            else:
                al.set_reference(amp)
                al.align_ops_packed(hpr, out=hout)
            ms.append((time.perf_counter() - t0) * 1e3)
        print(name, " ".join(f"{x:.2f}" for x in ms), flush=True)
    al.close()


if __name__ == "__main__":
    main()
