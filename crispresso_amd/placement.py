"""Host placement of the ranks of one node ("each GPU has its own host thread
doing decode -> H2D -> kernel -> D2H").

With one process per GPU, every rank's host work (the call's length scan, the FASTQ ingest,
packing, the DataFrame hand-off) runs on its process's native pool (``csrc/host_pool.h``) and
its pinned buffers are page-locked wherever the process first touches them.  Left alone, 8 ranks
would each start a pool sized for the whole CPU share and allocate pinned memory on whatever
NUMA node they happen to run on.  :func:`bind_rank` fixes both before anything is allocated:

* the GPU of the rank is found in the KFD topology (``/sys/class/kfd/kfd/topology/nodes``: GPU
  nodes in HIP's enumeration order, filtered by ``ROCR_VISIBLE_DEVICES`` /
  ``HIP_VISIBLE_DEVICES``), its PCI address gives its NUMA node
  (``/sys/bus/pci/devices/<bdf>/numa_node``) and that node's CPUs
  (``/sys/devices/system/node/node<k>/cpulist``);
* the process's CPU share (``sched_getaffinity`` capped by the cgroup CPU quota) is split
  evenly over the node's local ranks, ``share // LOCAL_WORLD_SIZE`` CPUs each; the ranks whose
  GPUs sit on one NUMA node take disjoint consecutive slices of that node's allowed CPUs (a
  node with too few CPUs for its ranks, or no topology at all, falls back to slices of the
  whole allowed set);
* the process is bound to its slice (``sched_setaffinity``; threads started later inherit it)
  and ``CRISPR_NW_HOST_THREADS`` is set to the slice's size, so the native pool -- created at
  the library's first parallel call -- has exactly one thread per CPU of the rank.

Nothing here touches the GPU: it runs before the HIP runtime is initialised.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def parse_cpulist(text: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def cgroup_quota() -> Optional[float]:
    """CPUs the cgroup allows (cpu.max / cfs quota), None when unlimited or unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return q / per if q > 0 else None
    except (OSError, ValueError):
        return None


def _props(path: str) -> Dict[str, int]:
    out = {}
    try:
        with open(path) as f:
            for line in f:
                kv = line.split()
                if len(kv) == 2:
                    try:
                        out[kv[0]] = int(kv[1])
                    except ValueError:
                        pass
    except OSError:
        pass
    return out


def gpu_pci_addresses(root: str = KFD_NODES) -> List[str]:
    """PCI addresses ("dddd:bb:dd.f") of the GPUs in the KFD topology, in node order (the
    order ROCr enumerates its GPU agents), filtered by ROCR_VISIBLE_DEVICES and then
    HIP_VISIBLE_DEVICES when set.  [] without a topology."""
    try:
        nodes = sorted((int(d) for d in os.listdir(root) if d.isdigit()))
    except OSError:
        return []
    out = []
    for k in nodes:
        p = _props(os.path.join(root, str(k), "properties"))
        if p.get("simd_count", 0) <= 0:
            continue   # a CPU node
        loc, dom = p.get("location_id", 0), p.get("domain", 0)
        out.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7:x}")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        sel = os.environ.get(var)
        if sel:
            try:
                out = [out[int(x)] for x in sel.split(",") if x.strip() != ""]
            except (ValueError, IndexError):
                return []
    return out


def numa_node_of(pci: str) -> Optional[int]:
    try:
        with open(f"/sys/bus/pci/devices/{pci}/numa_node") as f:
            v = int(f.read())
        return v if v >= 0 else None
    except (OSError, ValueError):
        return None


def node_cpus(node: int) -> List[int]:
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            return parse_cpulist(f.read())
    except OSError:
        return []


def plan(local_rank: int, local_world: int, allowed: List[int], quota: Optional[float],
         gpu_nodes: List[Optional[int]], cpus_of_node) -> dict:
    """The CPU slice of `local_rank` (pure: tests call it with made-up topologies).

    `gpu_nodes[r]` is the NUMA node of local rank r's GPU (None: unknown), `cpus_of_node(k)` the
    CPUs of node k.  Every rank gets `per = max(1, share // local_world)` CPUs, share =
    min(len(allowed), quota); ranks of one node take consecutive disjoint slices of that node's
    allowed CPUs when the node has room for all of them, else every rank takes its slice of the
    whole allowed set (disjoint by construction)."""
    allowed = sorted(set(allowed))
    share = len(allowed) if quota is None else max(1, min(len(allowed), int(quota)))
    per = max(1, share // max(1, local_world))
    node = gpu_nodes[local_rank] if local_rank < len(gpu_nodes) else None
    numa_ok = node is not None and all(g is not None for g in gpu_nodes[:local_world])
    if numa_ok:
        # every node must hold per CPUs for each of its ranks, or the split falls back
        for k in set(gpu_nodes[:local_world]):
            room = [c for c in cpus_of_node(k) if c in set(allowed)]
            if len(room) < per * sum(1 for g in gpu_nodes[:local_world] if g == k):
                numa_ok = False
                break
    if numa_ok:
        room = [c for c in cpus_of_node(node) if c in set(allowed)]
        i = sum(1 for g in gpu_nodes[:local_rank] if g == node)   # this rank's index among its node's ranks
        cpus = room[i * per:(i + 1) * per]
        source = "numa"
    else:
        per = max(1, min(per, len(allowed) // max(1, local_world))) if len(allowed) >= local_world else 1
        lo = (local_rank * per) % max(1, len(allowed))
        cpus = allowed[lo:lo + per] or allowed[:1]
        node = None
        source = "split"
    return {"cpus": cpus, "threads": len(cpus), "numa_node": node, "source": source, "share": share,
            "per_rank": per}


def bind_rank(local_rank: int, local_world: int, apply: bool = True, device_of=None) -> dict:
    """Bind this process (local rank `local_rank` of `local_world` on this node) to its CPU
    slice and size the native pool to it (CRISPR_NW_HOST_THREADS) -- before the library's pool
    exists and before any pinned buffer is allocated.  `device_of(r)`: the GPU of local rank r
    (default r).  Returns what was chosen (reported in the bench line).  An explicit
    CRISPR_NW_HOST_THREADS is left as the user set it."""
    device_of = device_of or (lambda r: r)
    allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    quota = cgroup_quota()
    pcis = gpu_pci_addresses()
    devs = [device_of(r) for r in range(local_world)]
    nodes = [numa_node_of(pcis[d]) for d in devs] if pcis and max(devs) < len(pcis) else []
    res = plan(local_rank, local_world, allowed, quota, nodes, node_cpus)
    res["gpu_pci"] = pcis[devs[local_rank]] if devs[local_rank] < len(pcis) else None
    res["local_rank"], res["local_world"] = local_rank, local_world
    if apply:
        if hasattr(os, "sched_setaffinity") and res["cpus"]:
            try:
                os.sched_setaffinity(0, res["cpus"])
                res["bound"] = True
            except OSError as exc:
                res["bound"] = False
                res["bind_error"] = str(exc)
        if "CRISPR_NW_HOST_THREADS" in os.environ:
            res["threads"] = int(os.environ["CRISPR_NW_HOST_THREADS"])
            res["threads_from_env"] = True
        else:
            os.environ["CRISPR_NW_HOST_THREADS"] = str(res["threads"])
    return res


def device_pci(device: int) -> Optional[str]:
    """The PCI address HIP reports for `device` (hipDeviceGetPCIBusId; initialises the HIP
    runtime, so call it only once the process uses the GPU anyway): checks the KFD-order
    mapping bind_rank assumed."""
    import ctypes

    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, int(device)) != 0:
            return None
        return buf.value.decode().lower()
    except OSError:
        return None
