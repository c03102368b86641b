"""Kernel-resident pass of the C2 batch: text upload (byte classify) vs packed upload (packed
classify), alternating; prints the phase times (classify + sort, fills, walk, rest).
Usage: classify_ab.py [rounds] [c1]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner, pack_2bit  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
if len(sys.argv) > 2 and sys.argv[2] == "c1":   # the C1-shape leg's reads (151 bp windows of 280 bp)
    amp, buf, off = synth.c1_shape_workload(1_000_000)
else:
    amp = synth.random_amplicon(bench.AMPLICON_LEN, 1)
    buf, off = synth.reads_from(amp, bench.READS_PER_GPU, 2)
pr = pack_2bit(buf, off)
al = GpuAligner(0)
al.set_reference(amp)
res = {"text": [], "packed": []}
for r in range(rounds):
    for mode in ("text", "packed"):
        if mode == "text":
            al.set_output("ops")
            al.upload(buf, off)
        else:
            al.upload_packed(pr)
        for _ in range(3):
            al.run_async()
            al.sync()
        ph = []
        for _ in range(5):
            al.run_async()
            ms = al.sync()
            ph.append((ms, al.phase_times()))
        res[mode].append((float(np.median([p[0] for p in ph])),
                          {k: float(np.median([p[1][k] for p in ph])) for k in ph[0][1]}))
for mode, v in res.items():
    print(mode, "kernel_ms", round(float(np.median([x[0] for x in v])), 4),
          {k: round(float(np.median([x[1][k] for x in v])), 4) for k in v[0][1]})
al.close()
