"""The C1-shape leg (1M 151 bp windows of a 280 bp amplicon, synth.c1_shape_workload) under two
settings of the library's env switches, alternating calls; prints median call times.
Usage: c1_ab.py "VAR=v" "VAR=u" [rounds]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import time  # noqa: E402

import numpy as np  # noqa: E402

from crispresso_amd import synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner, pack_2bit  # noqa: E402


def parse(spec):
    return dict(kv.split("=", 1) for kv in spec.split(",") if kv)


A, B = parse(sys.argv[1]), parse(sys.argv[2])
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
amp, buf, off = synth.c1_shape_workload(1_000_000)
pr = pack_2bit(buf, off)
al = GpuAligner(0)
al.set_reference(amp)
times = {"A": [], "B": []}
for r in range(rounds + 1):
    for name, env in (("A", A), ("B", B)):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        t0 = time.perf_counter()
        al.align_ops_packed(pr)
        dt = time.perf_counter() - t0
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        if r:
            times[name].append(dt * 1e3)
for name, env in (("A", A), ("B", B)):
    print(name, env, "median ms", round(float(np.median(times[name])), 3), "paths", al.path_counts())
al.close()
