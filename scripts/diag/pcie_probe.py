"""PCIe copy rates of the box under host placements: the pinned buffers' NUMA node against the
GPU's (the process bound to CPUs of the GPU's node, of another node, or left free), one copy vs
chunked copies on one or two streams, D2H alone and concurrent with H2D, SDMA vs blit copies.
Each placement runs in a child process (binding happens before the child allocates anything).
Usage: pcie_probe.py            (parent: runs the children)
       pcie_probe.py child MODE (one placement: free | local | remote)"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def child(mode):
    from crispresso_amd import placement
    pcis = placement.gpu_pci_addresses()
    node = placement.numa_node_of(pcis[0]) if pcis else None
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit())
    allowed = set(os.sched_getaffinity(0))
    cpus = None
    if mode == "local" and node is not None:
        cpus = [c for c in placement.node_cpus(node) if c in allowed][:16]
    elif mode == "remote" and node is not None:
        other = [k for k in nodes if k != node]
        if other:
            cpus = [c for c in placement.node_cpus(other[0]) if c in allowed][:16]
    if cpus:
        os.sched_setaffinity(0, cpus)
    import torch
    H, D = 64 << 20, 45 << 20
    hb = torch.empty(H, dtype=torch.uint8, pin_memory=True)
    hb.fill_(1)
    db = torch.empty(H, dtype=torch.uint8, device="cuda")
    ho = torch.empty(D, dtype=torch.uint8, pin_memory=True)
    ho.fill_(2)
    do = torch.empty(D, dtype=torch.uint8, device="cuda")
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn, reps=15):
        out = []
        for i in range(reps + 3):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch.cuda.current_stream())
            for s in (s1, s2, s3):
                s.wait_event(e0)
            fn()
            for s in (s1, s2, s3):
                torch.cuda.current_stream().wait_stream(s)
            e1.record(torch.cuda.current_stream())
            torch.cuda.synchronize()
            if i >= 3:
                out.append(e0.elapsed_time(e1))
        out.sort()
        return out[len(out) // 2]

    def h2d(parts, streams):
        step = H // parts
        for k in range(parts):
            with torch.cuda.stream(streams[k % len(streams)]):
                db[k * step:(k + 1) * step].copy_(hb[k * step:(k + 1) * step], non_blocking=True)

    def d2h():
        with torch.cuda.stream(s3):
            ho.copy_(do, non_blocking=True)

    res = {"mode": mode, "gpu_node": node, "nodes": nodes, "cpus": cpus[:4] + ["..."] if cpus else "free",
           "sdma": os.environ.get("HSA_ENABLE_SDMA", "default")}
    for name, fn in (("h2d_1", lambda: h2d(1, [s1])), ("h2d_8", lambda: h2d(8, [s1])),
                     ("h2d_8x2", lambda: h2d(8, [s1, s2])), ("h2d_32x2", lambda: h2d(32, [s1, s2])),
                     ("d2h_1", d2h), ("h2d_8+d2h", lambda: (h2d(8, [s1]), d2h()))):
        ms = timed(fn)
        nb = (H if name.startswith("h2d") else 0) + (D if "d2h" in name else 0)
        res[name] = {"ms": round(ms, 4), "GBps": round(nb / ms / 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(sys.argv[2])
        sys.exit(0)
    rc = 0
    for mode, env in (("free", {}), ("local", {}), ("remote", {}), ("local", {"HSA_ENABLE_SDMA": "0"})):
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, __file__, "child", mode], env=e, timeout=180)
        rc = rc or r.returncode
        if r.returncode:
            break
    sys.exit(rc)
