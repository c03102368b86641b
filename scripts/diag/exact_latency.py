"""Latency of the one-wave exact kernel on a handful of C2 reads (CRISPR_NW_KERNEL=full),
for rocprofv3 --kernel-trace --stats; CRISPR_NW_DEBUG_MODE=1 stops after the fill and the
start cell, 2 after the traceback walk (phase split).  Usage: exact_latency.py [reads]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
os.environ.setdefault("CRISPR_NW_KERNEL", "full")
from crispresso_amd import synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
amp = synth.random_amplicon(250, 1)
buf, off = synth.reads_from(amp, n, 9)
al = GpuAligner(0)
al.set_reference(amp)
for _ in range(20):
    al.align_ops(buf, off)
al.close()
print("ok")
