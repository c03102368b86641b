"""FASTQ(.gz) ingest timing: nw_fastq_read_filtered on a synthetic 1M-read C2 file, the
libdeflate whole-member path against zlib gzread (CRISPR_NW_FASTQ_ZLIB=1), gz and plain;
outputs compared.  Usage: fastq_ingest.py [n_reads] [dir]"""
import ctypes
import gzip
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402

import e2e_timing  # noqa: E402
from crispresso_amd import _lib, fastq, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
d = sys.argv[2] if len(sys.argv) > 2 else "/tmp"
gz = os.path.join(d, "ingest_c2.fastq.gz")
plain = os.path.join(d, "ingest_c2.fastq")
amp = synth.random_amplicon(250, 1)
buf, off = synth.reads_from(amp, n, 2)
e2e_timing.write_fastq(gz, buf, off)
with gzip.open(gz) as f, open(plain, "wb") as g:
    g.write(f.read())
lib = _lib.load()
res = {}
for path in (gz, plain):
    for env in ("0", "1"):
        os.environ["CRISPR_NW_FASTQ_ZLIB"] = env
        ts = []
        for _ in range(3):
            h = ctypes.c_void_p()
            t = time.perf_counter()
            assert lib.nw_fastq_read_filtered(os.fsencode(path), 0, 0, ctypes.byref(h)) == _lib.NW_OK
            ts.append(time.perf_counter() - t)
            lib.nw_fastq_free(h)
        t = time.perf_counter()
        out = fastq.read_fastq_as_fasta(path)
        full = time.perf_counter() - t
        res[(path, env)] = out
        print(f"{os.path.basename(path):20s} {'zlib' if env == '1' else 'fast'}: native {min(ts):.3f} s "
              f"(runs {', '.join(f'{x:.3f}' for x in ts)}), read_fastq_as_fasta {full:.3f} s", flush=True)
a, b = res[(gz, "0")], res[(gz, "1")]
print("same output:", a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]))
