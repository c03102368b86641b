#!/usr/bin/env python3
"""Host-inclusive timings of the aligner path: what a CRISPResso
run sees, as opposed to bench.py's device-resident `value`.

Stages for N synthetic C3 reads (85 % from the amplicon, 15 % from the HDR amplicon), one MI355X:
  fastq_gz / fastq_gz_py  FASTQ.gz -> names + packed reads: native (nw_fastq_read) / Python restatement
  align_ops     nw_align_ops: reads in, records + runs out (the call-level path)
  dataframe_ops ops_to_dataframe (the DataFrame parse_needle_output would give)
  align_reads   CRISPRessoCORE.py:1788-2000 end to end (FASTQ.gz .. filtered DataFrame), C2 and C3
Usage: e2e_timing.py [n_reads] [out.json]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from crispresso_amd import fastq, synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner  # noqa: E402
from crispresso_amd.needle import AlignArgs, align_reads, ops_to_dataframe  # noqa: E402


def write_fastq(path, buf, offsets):
    import gzip

    n = len(offsets) - 1
    with gzip.open(path, "wb", compresslevel=1) as f:
        for lo in range(0, n, 100_000):
            hi = min(n, lo + 100_000)
            parts = []
            for i in range(lo, hi):
                s = bytes(buf[offsets[i]:offsets[i + 1]])
                parts.append(b"@SYN:1:FC:1:%d:%d 1:N:0:1\n%s\n+\n%s\n" % (i // 1000, i % 1000, s, b"I" * len(s)))
            f.write(b"".join(parts))


def timed(fn, *a, **k):
    t = time.perf_counter()
    r = fn(*a, **k)
    return r, time.perf_counter() - t


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "e2e.json")
    amp, hdr, buf, off = synth.c3_workload(n)
    res = {"n_reads": n, "amplicon_len": len(amp)}
    with tempfile.TemporaryDirectory() as td:
        fq = os.path.join(td, "reads.fastq.gz")
        _, res["write_fastq_s"] = timed(write_fastq, fq, buf, off)
        (names, b2, o2), res["fastq_gz_s"] = timed(fastq.read_fastq_as_fasta, fq)
        _, res["fastq_gz_py_s"] = timed(fastq.read_fastq_as_fasta_py, fq)
        with GpuAligner(0) as al:
            al.set_reference(amp)
            al.align_ops(b2[: o2[min(n, 1000)]], o2[: min(n, 1000) + 1])   # warm-up
            ob, res["align_ops_s"] = timed(al.align_ops, b2, o2)
            res["align_ops_pcie"] = al.ops_times()
            _, res["dataframe_ops_s"] = timed(ops_to_dataframe, ob, amp, b2, o2, names, "ref")
            # first call (one-time costs: host pools, pinned staging) and the best of two more
            c2 = [timed(align_reads, AlignArgs(amplicon_seq=amp), fq, al) for _ in range(3)]
            res["align_reads_c2_first_s"] = c2[0][1]
            res["align_reads_c2_s"] = min(t for _, t in c2[1:])
            res["align_reads_c2_rows"] = int(len(c2[0][0]))
            c3 = [timed(align_reads, AlignArgs(amplicon_seq=amp, expected_hdr_amplicon_seq=hdr), fq, al)
                  for _ in range(3)]
            res["align_reads_c3_first_s"] = c3[0][1]
            res["align_reads_c3_s"] = min(t for _, t in c3[1:])
            res["align_reads_c3_rows"] = int(len(c3[0][0]))
    res["align_reads_c2_reads_per_s"] = n / res["align_reads_c2_s"]
    res["align_reads_c3_reads_per_s"] = n / res["align_reads_c3_s"]
    res["align_reads_c2_without_fastq_reads_per_s"] = n / (res["align_reads_c2_s"] - res["fastq_gz_s"])
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
