"""The headline call (nw_align_ops_packed, C2 1M reads) under a host placement: the process bound
to CPUs of the GPU's NUMA node ("local"), of another node ("remote"), or left free, before any
pinned buffer exists; prints the call median and its upload span.  Usage: h2d_probe.py MODE [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from crispresso_amd import placement  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "free"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
pcis = placement.gpu_pci_addresses()
node = placement.numa_node_of(pcis[0]) if pcis else None
nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit())
allowed = set(os.sched_getaffinity(0))
pick = node if mode == "local" else next((k for k in nodes if k != node), None) if mode == "remote" else None
cpus = [c for c in placement.node_cpus(pick) if c in allowed][:16] if pick is not None else []
if cpus:
    os.sched_setaffinity(0, cpus)
    os.environ["CRISPR_NW_HOST_THREADS"] = str(len(cpus))

import numpy as np  # noqa: E402

import bench  # noqa: E402
from crispresso_amd import _lib, synth  # noqa: E402
from crispresso_amd.aligner import GpuAligner, pack_2bit  # noqa: E402

nr = bench.READS_PER_GPU
amplicon = synth.random_amplicon(bench.AMPLICON_LEN, 1)
buf, off = synth.reads_from(amplicon, nr, 2)
pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
stats = _lib.PinnedBuffer(nr, _lib.STAT_DTYPE)
ops_off = _lib.PinnedBuffer(nr + 1, np.int64)
ops = _lib.PinnedBuffer(4 * nr + 4096, np.uint32)
p_packed = _lib.PinnedBuffer((int(off[-1]) + 3) // 4 + 1, np.uint8)
p_lens = _lib.PinnedBuffer(max(nr, 1), np.uint16)
pr = pack_2bit(pb.array, po.array, packed=p_packed.array, lens=p_lens.array)
al = GpuAligner(0)
al.set_reference(amplicon)
v = []
for i in range(rounds + 4):
    t0 = time.perf_counter()
    al.align_ops_packed(pr, out=(stats.array, ops.array, ops_off.array))
    dt = (time.perf_counter() - t0) * 1e3
    if i >= 4:
        v.append((dt, al.ops_times()["h2d_ms"]))
v = np.array(v)
print(f"{mode} (gpu node {node}, cpus {cpus[:3]}..{len(cpus)}): call median {np.median(v[:, 0]):.3f} ms, "
      f"upload span median {np.median(v[:, 1]):.3f} ms", flush=True)
al.close()
