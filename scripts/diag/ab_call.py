"""In-process A/B of the headline call (nw_align_ops_packed, C2 1M reads) under two settings
of env knobs the library reads per call: calls alternate A, B, A, B ... so that box-level
drift (PCIe, host load) hits both alike.
Usage: ab_call.py "VAR=v,VAR2=w" "VAR=u" [rounds] [pooled]   (an empty string = defaults;
c1: the C1-shape call (151 bp windows x 280 bp amplicon); pooled: the C5 call, nw_align_multi_ops_packed over 96 amplicons x 100k reads; c3: the dual
alignment step, packed amplicon pass + resident HDR pass records-only; dual: A = that step, B = the
one-call dual alignment, nw_align_dual_ops_packed_lens; dualonly: the dual call alone; resident: the bench value's pass over the C2 batch held in HBM,
nw_batch_run_async + nw_batch_sync with the lane walk, as bench.py times it)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import _lib, synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner, pack_2bit  # noqa: E402


def parse(spec):
    return dict(kv.split("=", 1) for kv in spec.split(",") if kv)


A, B = parse(sys.argv[1]), parse(sys.argv[2])
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 40
pooled = len(sys.argv) > 4 and sys.argv[4] == "pooled"
c3 = len(sys.argv) > 4 and sys.argv[4] == "c3"
c4 = len(sys.argv) > 4 and sys.argv[4] == "c4"
c1 = len(sys.argv) > 4 and sys.argv[4] == "c1"
resident = len(sys.argv) > 4 and sys.argv[4] == "resident"
# dual: A = the two-call C3 step, B = the dual call (the env specs still apply); dualonly: the dual call
dual = len(sys.argv) > 4 and sys.argv[4] in ("dual", "dualonly")
dualonly = len(sys.argv) > 4 and sys.argv[4] == "dualonly"
c3 = c3 or dual
if c1:   # the C1 shape: 151 bp windows of a 280 bp amplicon
    amplicon, buf, off = synth.c1_shape_workload(bench.READS_PER_GPU)
    nr = len(off) - 1
elif c4:   # the C4 shard: 12.5M reads of the native generator in one call
    amplicon = synth.random_amplicon(bench.AMPLICON_LEN, 1)
    buf, off = synth.native_reads(amplicon, bench.C4_CALL_READS, 10)
    nr = len(off) - 1
elif c3:
    amplicon, hdr, buf, off = synth.c3_workload(bench.READS_PER_GPU)
    nr = len(off) - 1
elif pooled:
    amps, buf, off, which = bench.pooled_workload(96, 100_000)
    pw = _lib.pinned_copy(which)
    nr = len(off) - 1
else:
    nr = bench.READS_PER_GPU
    amplicon = synth.random_amplicon(bench.AMPLICON_LEN, 1)
    buf, off = synth.reads_from(amplicon, nr, 2)
pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
stats = _lib.PinnedBuffer(nr, _lib.STAT_DTYPE)
ops_off = _lib.PinnedBuffer(nr + 1, np.int64)
ops = _lib.PinnedBuffer((2 if c4 else 4) * nr + 4096, np.uint32)
p_packed = _lib.PinnedBuffer((int(off[-1]) + 3) // 4 + 1, np.uint8)
p_lens = _lib.PinnedBuffer(max(nr, 1), np.uint16)
pr = pack_2bit(pb.array, po.array, packed=p_packed.array, lens=p_lens.array)
al = GpuAligner(0)
stats2 = _lib.PinnedBuffer(nr, _lib.STAT_DTYPE)
ops_off2 = _lib.PinnedBuffer(nr + 1, np.int64)
if not pooled:
    al.set_reference(amplicon)
if resident:
    al.upload_packed(pr)
    al.set_lane_walk(True)
    al.set_phase_events(False)
keys = set(A) | set(B)
times = {"A": [], "B": []}
counts = {}
ref = None
for i in range(2 * rounds + 4):
    which = "A" if i % 2 == 0 else "B"
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update(A if which == "A" else B)
    t0 = time.perf_counter()
    if resident:
        al.run_async()
        al.sync()
    elif pooled:
        al.align_multi_ops(amps, pr, None, pw.array, out=(stats.array, ops.array, ops_off.array))
    elif dual and (which == "B" or dualonly):
        al.set_reference(amplicon)
        al.align_dual_packed(pr, hdr, out=(stats.array, ops.array, ops_off.array),
                             out2=(stats2.array, None, ops_off2.array), records_only2=True)
    elif c3:
        al.set_reference(amplicon)
        al.set_known(hdr)
        al.align_ops_packed(pr, out=(stats.array, ops.array, ops_off.array))
        al.set_known(None)
        al.set_reference(hdr)
        al.align_ops(None, po.array, out=(stats2.array, None, ops_off2.array), resident=True, records_only=True)
    else:
        al.align_ops_packed(pr, out=(stats.array, ops.array, ops_off.array))
    dt = time.perf_counter() - t0
    if i >= 4:
        times[which].append(dt * 1e3)
    if os.environ.get("AB_COUNTS"):
        counts[which] = al.path_counts()
    if resident:
        r = al.download_ops(nr)
        out = (r.stats.tobytes(), r.ops_off.tobytes(), r.ops[:int(r.ops_off[nr])].tobytes())
    else:
        out = (stats.array.tobytes(), ops_off.array.tobytes(), ops.array[:int(ops_off.array[-1])].tobytes(),
               stats2.array.tobytes() if c3 else b"")
    if ref is None:
        ref = out
    elif out != ref and not os.environ.get("AB_NOCHECK"):
        print("OUTPUT DIFFERS at call", i, which)
        sys.exit(1)
if os.environ.get("AB_COUNTS"):
    print("path_counts A", counts.get("A"), "B", counts.get("B"), "ops_times", al.ops_times())
for w, spec in (("A", sys.argv[1]), ("B", sys.argv[2])):
    t = np.array(times[w])
    print(f"{w} [{spec}]: median {np.median(t):.3f} ms  min {t.min():.3f}  p90 {np.percentile(t, 90):.3f}  "
          f"-> {nr / np.median(t) / 1e3:.1f} M reads/s (median)")
al.close()
