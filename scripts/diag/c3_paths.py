"""C3 diagnostic: path counts and timings of the two passes (amplicon, HDR amplicon)."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from crispresso_amd import synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner  # noqa: E402

amp, hdr, buf, off = synth.c3_workload(1_000_000)
for name, ref in (("amplicon", amp), ("hdr", hdr)):
    a = GpuAligner(0)
    a.set_reference(ref)
    a.align_ops(buf, off)
    t0 = time.perf_counter()
    a.align_ops(buf, off)
    dt = time.perf_counter() - t0
    print(name, f"call {dt * 1e3:.2f} ms", a.path_counts(), a.ops_times())
    a.set_output("ops")
    a.upload(buf, off)
    a.run_async()
    print(name, "resident", a.sync(), a.phase_times(), a.path_counts())
    a.close()
