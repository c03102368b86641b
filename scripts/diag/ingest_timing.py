"""Host ingest timing on this machine: the 1M-read C2 FASTQ.gz (written here, gzip level 1)
through nw_gunzip_parallel (threads 8 / 16), libdeflate on one thread, nw_fastq_read +
nw_fastq_pack, and the DataFrame hand-off pieces.  Usage: ingest_timing.py [reads]"""
import ctypes
import gzip
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402

from crispresso_amd import _lib, fastq, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
amp = synth.random_amplicon(250, 1)
buf, off = synth.reads_from(amp, n, 2)
path = "/tmp/ingest_c2.fastq.gz"
seqs = bytes(buf).decode()
o = off.tolist()
with gzip.open(path, "wb", compresslevel=1) as f:
    for lo in range(0, n, 100_000):
        f.write("".join(f"@SYN:1:FC{r // 65536}:1:{r % 65536}:{r} 1:N:0\n{seqs[o[r]:o[r + 1]]}\n+\n{'I' * (o[r + 1] - o[r])}\n"
                        for r in range(lo, min(n, lo + 100_000))).encode())
gz = np.fromfile(path, np.uint8)
print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), "gz MB", len(gz) / 1e6, flush=True)
lib = _lib.load()
PINNED = int(os.environ.get("PINNED", "1"))
need = ctypes.c_int64()
out = np.empty(int(off[-1]) * 3 + 100 * n, np.uint8)   # > the decompressed size
for th in (8, 16):
    ts = []
    for _ in range(4):
        t = time.perf_counter()
        rc = lib.nw_gunzip_parallel(_lib.ptr(gz), len(gz), th, _lib.ptr(out), len(out), ctypes.byref(need))
        ts.append(time.perf_counter() - t)
    print("gunzip_parallel threads", th, "rc", rc, "s", [round(x, 4) for x in ts], flush=True)
try:
    L = ctypes.CDLL("libdeflate.so.0")
    L.libdeflate_alloc_decompressor.restype = ctypes.c_void_p
    L.libdeflate_gzip_decompress_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    d = L.libdeflate_alloc_decompressor()
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        L.libdeflate_gzip_decompress_ex(d, _lib.ptr(gz), len(gz), _lib.ptr(out), len(out), None, None)
        ts.append(time.perf_counter() - t)
    print("libdeflate 1 thread s", [round(x, 4) for x in ts], "crc32 sym", hasattr(L, "libdeflate_crc32"), flush=True)
except OSError as e:
    print("libdeflate absent", e)
h = ctypes.c_void_p()
for _ in range(3):
    t = time.perf_counter()
    lib.nw_fastq_read(path.encode(), ctypes.byref(h))
    t1 = time.perf_counter()
    pk, po, ep, eb = (ctypes.c_void_p() for _ in range(4))
    ne = ctypes.c_int64()
    lib.nw_fastq_pack(h, PINNED, ctypes.byref(pk), ctypes.byref(po), ctypes.byref(ep), ctypes.byref(eb), ctypes.byref(ne))
    t2 = time.perf_counter()
    lib.nw_fastq_free(h)
    print("nw_fastq_read", round(t1 - t, 4), "pack(pinned)", round(t2 - t1, 4), flush=True)
for _ in range(2):
    t = time.perf_counter()
    r = fastq.read_fastq_packed(path, pinned=bool(PINNED))
    print("read_fastq_packed", round(time.perf_counter() - t, 4), flush=True)
    del r
