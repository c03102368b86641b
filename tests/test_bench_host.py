"""bench.py's host-side pieces (no GPU): the PMC traffic it reports comes from the committed
rocprofv3 summaries of the TIMED resident pass's kernels (per pass), of call_pcie's calls and of
the quantification leg (per call), and records which library build they profiled."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)   # module level: imports and constants only
    return mod


import pytest  # noqa: E402


@pytest.mark.parametrize("which", ["RESIDENT_PMC", "CALL_PMC"])
def test_pmc_summary_covers_the_timed_kernels(which):
    b = load_bench()
    path = getattr(b, which)
    with open(path) as f:
        summ = json.load(f)
    assert summ["_meta"]["calls"] and summ["_meta"]["lib_sha1"]
    for k in ("nw_band_classify", "nw_band_segsort", "nw_band_fill<16, true>", "nw_band_walk<16, true>",
              "nw_ops_compact"):
        assert any(k in name for name in summ), k
    cp = b.pmc_per_call(path, lambda k: ("nw::" in k and "nwq::" not in k) or "nw_align_kernel" in k)
    assert cp["traffic"] > 5e7 and cp["valu_fill16"] > 0   # ~0.1-1.5 GB per 1M C2 reads


def test_quant_pmc_summary():
    b = load_bench()
    qp = b.pmc_per_call(b.QUANT_PMC, lambda k: "nwq::" in k)
    assert qp is not None and qp["traffic"] > 0
    assert any("quant_lanes" in k for k in qp["kernels"])


def test_pmc_per_call_sums_kernels(tmp_path):
    b = load_bench()
    p = tmp_path / "s.json"
    p.write_text(json.dumps({"_meta": {"calls": 4, "lib_sha1": "x"},
                             "void nw::nw_band_fill<16, 1, false>(nw::KernelArgs)": {"hbm_bytes_per_call": 10.0,
                                                                                    "valu_per_call": 7.0},
                             "nw::nw_band_segsort(nw::KernelArgs, unsigned int)": {"hbm_bytes_per_call": 5.0},
                             "nwq::quant_lanes(nwq::LArgs)": {"hbm_bytes_per_call": 100.0}}))
    cp = b.pmc_per_call(str(p), lambda k: "nwq::" not in k)
    assert cp["traffic"] == 15.0 and cp["valu_fill16"] == 7.0 and cp["calls_profiled"] == 4
    assert cp["lib_matches_loaded"] in (False, None)


def _bench_rank(rank, world, port, out_dir):
    """bench.py's multi-process plumbing (gloo barrier, max over ranks) never
    initialises torch's HIP runtime: libcrispr_nw.so owns the GPU in that process."""
    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    b = load_bench()
    r, local, w, dist = b.dist_setup()
    assert (r, local, w) == (rank, rank, world)
    b.barrier(dist)
    m = b.max_over_ranks(dist, float(rank + 1))
    assert m == float(world)
    assert not torch.cuda.is_initialized()
    with open(os.path.join(out_dir, f"ok{rank}"), "w") as f:
        f.write(str(m))
    dist.destroy_process_group()


def test_bench_multi_rank_path_is_torch_cuda_free(tmp_path):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_bench_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="fork")
    assert (tmp_path / "ok0").read_text() == "2.0" and (tmp_path / "ok1").read_text() == "2.0"


def _run_bench(*args, env_extra=None, timeout=240):
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_gpus_n_launches_n_ranks_itself():
    """`python bench.py --gpus 2` with no launcher forms a 2-rank world (one process per GPU),
    every rank takes its share of the C4 / pooled work, and one line comes back."""
    p = _run_bench("--gpus", "2", "--dry-run", "--pooled-reads", "1000", env_extra={"CRISPR_BENCH_DEVICES": "1"})
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2
    assert [r["rank"] for r in d["ranks"]] == [0, 1] and all(r["device"] == 0 for r in d["ranks"])
    assert d["c4_reads_total"] == 100_000_000 and all(r["c4_reads"] == 50_000_000 for r in d["ranks"])
    rng = [r["pooled_range"] for r in d["ranks"]]
    assert rng[0][0] == 0 and rng[0][1] == rng[1][0] and rng[1][1] == d["pooled_reads_total"] == 96_000


def test_bench_refuses_a_world_that_is_not_gpus():
    p = _run_bench("--gpus", "1", "--dry-run", "--pooled-reads", "100",
                   env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                              "MASTER_PORT": "1"}, timeout=60)
    assert p.returncode == 2 and "formed a world of 2" in p.stderr
