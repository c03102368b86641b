"""Diagnostics: the C5 pooled leg on its own, then after the C4 shard leg, 5 timed calls each
(per-call ms), and one call with CRISPR_NW_HOST_TIMING=1 (per-chunk upload / start / end)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner  # noqa: E402


def main():
    al = GpuAligner(0)
    amp = synth.random_amplicon(250, 1)
    al.set_reference(amp)
    order = sys.argv[1:] or ["pooled", "c4", "pooled"]
    for what in order:
        if what == "pooled":
            r = bench.pooled_leg(al, 0, 1, None, 96, 100_000, 5, 2, 16, text_too=False)
            print("pooled ms", r["ms_per_step"], r["path_counts"], r["pcie"], flush=True)
        elif what == "c4":
            al.set_reference(amp)
            r = bench.c4_leg(al, amp, 0, 1, None, 16, 3, 1, 0)
            print("c4 ms", r["ms_per_pass"], flush=True)
        elif what == "timing":
            os.environ["CRISPR_NW_HOST_TIMING"] = "1"
            r = bench.pooled_leg(al, 0, 1, None, 96, 100_000, 1, 1, 16, text_too=False)
            del os.environ["CRISPR_NW_HOST_TIMING"]
            print("pooled (timed host) ms", r["ms_per_step"], flush=True)
    al.close()


if __name__ == "__main__":
    main()
