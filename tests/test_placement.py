"""Host placement of the ranks of one node (crispresso_amd/placement.py): disjoint CPU
slices on each GPU's NUMA node, native pools sized to them."""
import json
import os

from crispresso_amd import placement

from .test_bench_host import _run_bench


def _topo(nodes_cpus):
    return lambda k: nodes_cpus[k]


def test_parse_cpulist():
    assert placement.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert placement.parse_cpulist("") == []


def test_plan_numa_slices_are_disjoint_and_local():
    # 8 GPUs, 4 on each of 2 NUMA nodes of 64 CPUs; the cgroup allows 128 CPUs
    nodes = {0: list(range(0, 64)), 1: list(range(64, 128))}
    gpu_nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    plans = [placement.plan(r, 8, list(range(128)), 128.0, gpu_nodes, _topo(nodes)) for r in range(8)]
    sets = [set(p["cpus"]) for p in plans]
    assert all(p["source"] == "numa" and p["threads"] == 16 for p in plans)
    assert all(not (sets[a] & sets[b]) for a in range(8) for b in range(a + 1, 8))
    for r, p in enumerate(plans):
        assert set(p["cpus"]) <= set(nodes[gpu_nodes[r]])
    # a 16-CPU quota over 8 ranks: 2 CPUs each, still on the GPU's node
    plans = [placement.plan(r, 8, list(range(128)), 16.0, gpu_nodes, _topo(nodes)) for r in range(8)]
    assert sum(p["threads"] for p in plans) == 16
    assert all(set(p["cpus"]) <= set(nodes[gpu_nodes[r]]) for r, p in enumerate(plans))
    sets = [set(p["cpus"]) for p in plans]
    assert all(not (sets[a] & sets[b]) for a in range(8) for b in range(a + 1, 8))


def test_plan_falls_back_when_a_node_is_too_small_or_unknown():
    nodes = {0: [0, 1], 1: list(range(2, 32))}
    gpu_nodes = [0, 0, 0, 0, 1, 1, 1, 1]   # node 0 cannot give 4 ranks 4 CPUs each
    plans = [placement.plan(r, 8, list(range(32)), None, gpu_nodes, _topo(nodes)) for r in range(8)]
    assert all(p["source"] == "split" for p in plans)
    sets = [set(p["cpus"]) for p in plans]
    assert all(not (sets[a] & sets[b]) for a in range(8) for b in range(a + 1, 8))
    assert sum(p["threads"] for p in plans) <= 32
    plans = [placement.plan(r, 2, list(range(8)), None, [], _topo(nodes)) for r in range(2)]
    assert [p["cpus"] for p in plans] == [[0, 1, 2, 3], [4, 5, 6, 7]]


def test_plan_single_rank_takes_the_share():
    p = placement.plan(0, 1, list(range(256)), 16.0, [3], _topo({3: list(range(192, 256))}))
    assert p["threads"] == 16 and set(p["cpus"]) <= set(range(192, 256))


def test_bench_gpus_8_dry_run_binds_disjoint_cpu_sets():
    """`bench.py --gpus 8 --dry-run` (8 ranks, no GPU): every rank bound to its own CPUs, its native
    pool sized to them, the pools summing to at most the share."""
    p = _run_bench("--gpus", "8", "--dry-run", "--pooled-reads", "100", env_extra={"CRISPR_BENCH_DEVICES": "1"},
                   timeout=400)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    d = json.loads(lines[0])
    pl = d["host_placement"]
    assert len(pl) == 8 and sorted(x["local_rank"] for x in pl) == list(range(8))
    sets = [set(x["cpus"]) for x in pl]
    share = pl[0]["share"]
    if share >= 8:
        assert all(not (sets[a] & sets[b]) for a in range(8) for b in range(a + 1, 8))
    assert all(x["bound"] and x["pool_threads"] == len(x["cpus"]) for x in pl)
    assert sum(x["pool_threads"] for x in pl) <= max(share, 8)
    assert set().union(*sets) <= set(os.sched_getaffinity(0))
