"""C3's second pass (reads vs the HDR amplicon, batch resident): path counts and phase times.
Usage: python scripts/diag/hdr_pass.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from crispresso_amd import synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner  # noqa: E402

amp, hdr, buf, off = synth.c3_workload(1_000_000)
al = GpuAligner(0)
out = {}
for name, ref in (("amplicon", amp), ("hdr", hdr)):
    al.set_reference(ref)
    al.align_ops(buf, off)
    t = time.perf_counter()
    ob = al.align_ops(buf, off)
    out[name] = {"call_ms": (time.perf_counter() - t) * 1e3, "paths": al.path_counts(), "pcie": al.ops_times()}
    al.align_ops(None, off, resident=True)
    t = time.perf_counter()
    al.align_ops(None, off, resident=True, records_only=True)
    out[name]["resident_records_ms"] = (time.perf_counter() - t) * 1e3
    out[name]["resident_paths"] = al.path_counts()
    al.set_output("ops")
    al.upload(buf, off)
    for _ in range(2):
        al.run_async()
        ms = al.sync()
    out[name]["kernel_ms"] = ms
    out[name]["phases"] = al.phase_times()
    out[name]["kernel_paths"] = al.path_counts()
print(json.dumps(out, indent=1))
