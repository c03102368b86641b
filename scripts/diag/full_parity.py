"""Every read of the benchmark workloads against the CPU oracle (not a sample): C2 (1M reads,
the headline's packed call), C3 (the same reads against the HDR amplicon, resident pass) and
C5 (96 amplicons x 10k reads, one pooled call).  Records and the rows expanded from the runs.
Usage: full_parity.py [out.json]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import _lib, synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner, pack_2bit  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/full_parity.json"
threads = 16
res = {}
al = GpuAligner(0)


def pinned_outputs(n):
    st = _lib.PinnedBuffer(n, _lib.STAT_DTYPE)
    oo = _lib.PinnedBuffer(n + 1, np.int64)
    ops = _lib.PinnedBuffer(4 * n + 4096, np.uint32)
    return st, oo, ops


# C2: the headline batch (seed 2), packed call
t0 = time.time()
amp = synth.random_amplicon(bench.AMPLICON_LEN, 1)
buf, off = synth.reads_from(amp, bench.READS_PER_GPU, 2)
pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
st, oo, ops = pinned_outputs(len(off) - 1)
pr = pack_2bit(pb.array, po.array)
al.set_reference(amp)
ob = al.align_ops_packed(pr, out=(st.array, ops.array, oo.array))
res["C2"] = bench.sample_check(amp, buf, off, ob, 1, threads)
print("C2", res["C2"]["sample_mismatches"], f"{time.time() - t0:.1f}s", flush=True)

# C3: the C3 reads against the amplicon (packed call) and the HDR amplicon (resident pass)
t0 = time.time()
amp3, hdr, buf3, off3 = synth.c3_workload(bench.READS_PER_GPU)
pb3, po3 = _lib.pinned_copy(buf3), _lib.pinned_copy(off3)
st3, oo3, ops3 = pinned_outputs(len(off3) - 1)
pr3 = pack_2bit(pb3.array, po3.array)
al.set_reference(amp3)
ob3 = al.align_ops_packed(pr3, out=(st3.array, ops3.array, oo3.array))
res["C3_ref"] = bench.sample_check(amp3, buf3, off3, ob3, 1, threads)
al.set_reference(hdr)
st4, oo4, ops4 = pinned_outputs(len(off3) - 1)
ob4 = al.align_ops(None, po3.array, out=(st4.array, ops4.array, oo4.array), resident=True)
res["C3_hdr"] = bench.sample_check(hdr, buf3, off3, ob4, 1, threads)
print("C3", res["C3_ref"]["sample_mismatches"], res["C3_hdr"]["sample_mismatches"], f"{time.time() - t0:.1f}s",
      flush=True)

# C5: 96 amplicons x 10k reads in one pooled call, each amplicon's reads checked against it
t0 = time.time()
amps, buf5, off5, which = bench.pooled_workload(96, 10_000)
pb5, po5, pw5 = _lib.pinned_copy(buf5), _lib.pinned_copy(off5), _lib.pinned_copy(which)
st5, oo5, ops5 = pinned_outputs(len(off5) - 1)
pr5 = pack_2bit(pb5.array, po5.array)
ob5 = al.align_multi_ops(amps, pr5, None, pw5.array, out=(st5.array, ops5.array, oo5.array))
from crispresso_amd.aligner import OpsBatch  # noqa: E402

bad = 0
for g, a in enumerate(amps):
    idx = np.flatnonzero(which == g)
    lo, hi = int(idx[0]), int(idx[-1]) + 1
    sub_off = off5[lo:hi + 1] - off5[lo]
    sub_buf = buf5[off5[lo]:off5[hi]]
    runs0, runs1 = int(ob5.ops_off[lo]), int(ob5.ops_off[hi])
    sub = OpsBatch(ob5.stats[lo:hi], ob5.ops[runs0:runs1], ob5.ops_off[lo:hi + 1] - runs0, np.diff(sub_off), ob5.scale)
    bad += bench.sample_check(a, sub_buf, sub_off, sub, 1, threads)["sample_mismatches"]
res["C5"] = {"reads_checked": int(len(off5) - 1), "amplicons": 96, "sample_mismatches": int(bad)}
print("C5", bad, f"{time.time() - t0:.1f}s", flush=True)
al.close()
res["what"] = ("every read: record (length, identity, similarity, gaps, score, start cell) and the three rows "
               "expanded from the runs, vs oracle/nw_oracle.c")
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps({k: v.get("sample_mismatches") for k, v in res.items() if isinstance(v, dict)}))
