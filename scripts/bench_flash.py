#!/usr/bin/env python3
"""Throughput of the GPU paired-end merge (crispresso_amd/flash.py) on synthetic
CRISPResso-like pairs: a 250 bp amplicon, 2 x 150 bp reads (100 bp overlap), 1 %
substitution noise per read, PCG64 seed 7.  Prints one JSON line: pairs/s of the
kernel (inputs resident) and of the whole call (with PCIe), and the CPU
restatement (oracle/flash_oracle.py, 1 thread) on a sample, for scale."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from crispresso_amd.flash import FlashOptions, merge_packed  # noqa: E402

N = int(os.environ.get("FLASH_BENCH_PAIRS", "1000000"))
L, AMP = 150, 250
rng = np.random.Generator(np.random.PCG64(7))
alpha = np.frombuffer(b"ACGT", np.uint8)
amp = rng.choice(alpha, AMP)
comp = np.zeros(256, np.uint8)
for a, b in zip(b"ACGT", b"TGCA"):
    comp[a] = b
r1 = np.tile(amp[:L], (N, 1))
r2 = np.tile(comp[amp[::-1]][:L], (N, 1))
for r in (r1, r2):
    m = rng.random(r.shape) < 0.01
    r[m] = rng.choice(alpha, int(m.sum()))
q1 = rng.integers(53, 74, (N, L)).astype(np.uint8)
q2 = rng.integers(53, 74, (N, L)).astype(np.uint8)
off = np.arange(N + 1, dtype=np.int64) * L
opts = FlashOptions(min_overlap=4, max_overlap=100, allow_outies=True)   # CRISPResso's FLASH options
merge_packed(r1[:1000].ravel(), q1[:1000].ravel(), off[:1001], r2[:1000].ravel(), q2[:1000].ravel(), off[:1001], opts)
t0 = time.perf_counter()
res = merge_packed(r1.ravel(), q1.ravel(), off, r2.ravel(), q2.ravel(), off, opts)
wall = time.perf_counter() - t0
out = {"metric": "merged read pairs/s", "pairs": N, "read_len": L, "kernel_ms": res.kernel_ms,
       "kernel_pairs_per_s": N / (res.kernel_ms / 1e3), "call_pairs_per_s": N / wall,
       "combined": int((res.length > 0).sum())}
if os.environ.get("FLASH_BENCH_CPU", "1") == "1":
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import flash_oracle  # noqa: E402
    mg = flash_oracle.Merger(min_overlap=4, max_overlap=100, allow_outies=True)
    k = 300
    t0 = time.perf_counter()
    for i in range(k):
        mg.merge_pair(r1[i].tobytes(), q1[i].tobytes(), r2[i].tobytes(), q2[i].tobytes())
    out["cpu_restatement_pairs_per_s_1thread"] = k / (time.perf_counter() - t0)
print(json.dumps(out))
