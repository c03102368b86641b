"""cProfile of align_reads on N synthetic reads (e2e_timing.py's workload): where the host
time of the CRISPResso-level call goes.  Usage: profile_align_reads.py [n_reads] [hdr]"""
import cProfile
import os
import pstats
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import e2e_timing  # noqa: E402
from crispresso_amd import synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner  # noqa: E402
from crispresso_amd.needle import AlignArgs, align_reads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
hdr_pass = len(sys.argv) > 2 and sys.argv[2] == "hdr"
amp, hdr, buf, off = synth.c3_workload(n)
with tempfile.TemporaryDirectory() as td:
    fq = os.path.join(td, "reads.fastq.gz")
    e2e_timing.write_fastq(fq, buf, off)
    with GpuAligner(0) as al:
        args = AlignArgs(amplicon_seq=amp, expected_hdr_amplicon_seq=hdr if hdr_pass else "")
        align_reads(args, fq, al)   # warm
        pr = cProfile.Profile()
        pr.enable()
        align_reads(AlignArgs(amplicon_seq=amp, expected_hdr_amplicon_seq=hdr if hdr_pass else ""), fq, al)
        pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(22)
st.sort_stats("cumulative").print_stats(18)
