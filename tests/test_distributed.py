"""Sharding across devices / ranks (CPU: gloo world_size 2, oracle-backed aligner)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from crispresso_amd import synth
from crispresso_amd.distributed import MultiGpuAligner, align_sharded, shard_range


def test_shard_ranges_cover_everything():
    for n in (0, 1, 7, 8, 1001):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def _same(a, b):
    assert len(a) == len(b)
    for f in ("aln_len", "n_ident", "n_sim", "n_gaps", "score", "end_i", "end_j", "flags"):
        assert np.array_equal(a.stats[f], b.stats[f]), f
    for i in range(len(a)):
        L = int(a.stats["aln_len"][i])
        assert np.array_equal(a.aln[i, :, :L], b.aln[i, :, :L])


def test_multi_device_threads_equal_single():
    from tests.helpers import OracleAligner

    amp = synth.random_amplicon(150, 3)
    buf, off = synth.reads_from(amp, 301, 4, synth.PARITY_MIX)
    single = OracleAligner()
    single.set_reference(amp)
    ref = single.align_packed(buf, off)
    multi = MultiGpuAligner([0, 1, 2], factory=lambda d, o: OracleAligner(d, o))
    multi.set_reference(amp)
    _same(multi.align_packed(buf, off), ref)
    multi.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    from tests.helpers import OracleAligner

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    amp = synth.random_amplicon(120, 5)
    buf, off = synth.reads_from(amp, 97, 6, synth.PARITY_MIX)
    res = align_sharded(amp, buf, off, OracleAligner(), dist)
    if rank == 0:
        np.save(os.path.join(out_dir, "stats.npy"), res.stats)
        np.save(os.path.join(out_dir, "aln.npy"), res.aln)
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gathers_in_read_order(tmp_path):
    from tests.helpers import OracleAligner

    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="fork")
    amp = synth.random_amplicon(120, 5)
    buf, off = synth.reads_from(amp, 97, 6, synth.PARITY_MIX)
    al = OracleAligner()
    al.set_reference(amp)
    ref = al.align_packed(buf, off)
    stats = np.load(tmp_path / "stats.npy")
    aln = np.load(tmp_path / "aln.npy")
    assert np.array_equal(stats, ref.stats)
    for i in range(len(stats)):
        L = int(stats["aln_len"][i])
        assert np.array_equal(aln[i, :, :L], ref.aln[i, :, :L])
