"""Where the C3 dual-alignment step goes (BASELINE configs[2], CORE:1808-1828): each piece of
bench.dual_leg's step timed on its own (set_reference of the amplicon, the packed amplicon pass,
set_reference of the HDR amplicon, the resident records-only HDR pass), with each pass's path
counts and upload / compute spans.  Usage: c3_probe.py [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import _lib, synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner, pack_2bit  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
amp, hdr, buf, off = synth.c3_workload(bench.READS_PER_GPU)
n = len(off) - 1
pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
stats = _lib.PinnedBuffer(n, _lib.STAT_DTYPE)
stats2 = _lib.PinnedBuffer(n, _lib.STAT_DTYPE)
ops_off = _lib.PinnedBuffer(n + 1, np.int64)
ops_off2 = _lib.PinnedBuffer(n + 1, np.int64)
ops = _lib.PinnedBuffer(4 * n + 4096, np.uint32)
p_packed = _lib.PinnedBuffer((int(off[-1]) + 3) // 4 + 1, np.uint8)
p_lens = _lib.PinnedBuffer(max(n, 1), np.uint16)
pr = pack_2bit(pb.array, po.array, packed=p_packed.array, lens=p_lens.array)
al = GpuAligner(0)
names = ("set_amp", "amp_pass", "set_hdr", "hdr_pass")
t = {k: [] for k in names}
info = {}
for i in range(rounds + 3):
    marks = [time.perf_counter()]
    al.set_reference(amp)
    al.set_known(hdr)
    marks.append(time.perf_counter())
    al.align_ops_packed(pr, out=(stats.array, ops.array, ops_off.array))
    al.set_known(None)
    marks.append(time.perf_counter())
    info["amp_pass"] = (al.path_counts(), al.ops_times())
    al.set_reference(hdr)
    marks.append(time.perf_counter())
    al.align_ops(None, po.array, out=(stats2.array, None, ops_off2.array), resident=True, records_only=True)
    marks.append(time.perf_counter())
    info["hdr_pass"] = (al.path_counts(), al.ops_times())
    if i >= 3:
        for k, a, b in zip(names, marks, marks[1:]):
            t[k].append((b - a) * 1e3)
tot = sum(np.median(t[k]) for k in names)
for k in names:
    print(f"{k:9s} median {np.median(t[k]):7.3f} ms  min {np.min(t[k]):7.3f}")
print(f"sum of medians {tot:.3f} ms")
for k, (pc, ot) in info.items():
    print(k, "path_counts", pc, "ops_times", {a: round(b, 3) if isinstance(b, float) else b for a, b in ot.items()})
al.close()
