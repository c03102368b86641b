#!/usr/bin/env python3
"""Benchmark: aligned reads/sec, 250 bp amplicon x 1M synthetic reads per GPU.

BASELINE.json metric: "aligned reads/sec (250 bp amplicon x 1M reads) at
1/2/4/8 MI355X".  value (round 5 on): whole-job throughput with the rank's batch
already resident in HBM when the timed region starts, as the build contract asks
("the PCIe-inclusive rate is never value").  One step = one pass of the hot path
over the rank's 1M C2 reads held in HBM as 2 bits per base (+ exceptions +
uint16 lengths, nw_batch_upload_packed, include/crispr_nw.h): classify (exact
copies, certificates, the DP reads' bytes), length sort, the certified band
levels with traceback, the wide and exact levels, and the ops compaction --
every read's record (nw_stat) and traceback runs written to HBM
(nw_batch_run_async + nw_batch_sync, one launch of each kernel over the batch,
the kernels the pipelined call runs on its chunks of >= 65536 reads).  K steps
between barriers, wall clock, max over ranks.

The boundary of SURVEY.md 8d (CRISPRessoCORE.py:1791-1806: host batch in ->
per-read records in host memory) is reported beside it as "call_pcie": one
nw_align_ops_packed call on the same batch in pinned host memory, chunks
pipelined over PCIe (2 bits per base in; records, run offsets and runs back to
pinned host memory) -- the rate a caller with host buffers sees; it was value
up to round 4.  The same call on the text (one byte per base, nw_align_ops) is
"text_input"; nw_pack_reads making the 2-bit batch is "ingest_pack"; the host
rebuilding the rows from the runs is "expand".

N GPUs: one process per GPU (torch.distributed.run), each aligning its own 1M
read shard (reads are independent, no collective on the data
path).  The timing barrier and the max-over-ranks run over a gloo process group
on the host: this process never initialises torch's HIP runtime (libcrispr_nw.so
owns the GPU).  value = N * 1M * K / max-over-ranks time of K steps ("weak").
At every N the line also carries the two multi-GPU configs of BASELINE.json at
their own shapes, timed the same way (barrier, max over ranks): "c4" (configs[3]:
100M reads over the N GPUs, each rank aligning 100M / N reads of the C4 generator,
seed 10 + rank, in calls of at most 12.5M reads; at N = 1 one 12.5M-read call,
"c4_shard") and "pooled" (configs[4]: 96 amplicons x 100k reads split over the
ranks by DP cells, crispresso_amd.distributed.cell_partition, one
nw_align_multi_ops_packed call per rank).

Extra keys: "kernel_rate" (the same resident pass timed by HIP events on the
aligner's stream, per phase and per path), "resident_check" (the timed pass's
records and runs against the pipelined call's, every read), "sample_check"
(every 100th read of the call's output re-aligned by the CPU oracle, outside the
timed region), "roofline" (HBM: algorithmic bytes per pass over the resident
pass's HIP-event time; VALU: issue fraction of nw_band_fill<16>),
"cpu_baseline" (the CPU oracle -- a port, EMBOSS is absent -- on bounded samples,
1 thread and the process's CPU share, rank 0 at N = 1 only); legs either side of the
path at N = 1: "e2e" (a 1M-read C2 FASTQ.gz through needle.align_reads to the
DataFrame, CORE:1788-2000), "dual_alignment" (C3, CORE:1808-1828),
"downstream_quantification", "upstream_merge".
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
# VALU issue peak: 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction (MI355X_MICROARCH.md "Wave scheduling")
VALU_ISSUE_PEAK = 1024 * 2.4e9 / 2
# a micro-benchmark's rate, not a validated hardware ceiling: packed 16-bit / VOP3 / DPP VALU ops issued at 0.228
# wave-instructions per SIMD-cycle (8 independent chains, 8 waves per SIMD; v_add_u32 reached only 0.39-0.41 of the
# nominal 0.5 in the same benchmark), profiles/r04_ubench/ubench_issue_rate.txt
UBENCH_VOP3P_RATE = 1024 * 2.4e9 * 0.228
READS_PER_GPU = 1_000_000
# rocprofv3 --pmc summaries (scripts/gpu_pmc_call.sh + pmc_summary.py: 2 x FETCH_SIZE + WRITE_SIZE, the guide's
# gfx950 correction) of the TIMED CALL's kernels (every launch of warmup + steps calls, per call) and of the
# quantification leg's kernels; each records the sha1 of the library it profiled (checked against the one loaded)
PMC_DIR = os.path.join(ROOT, "profiles", "r06_pmc")
RESIDENT_PMC = os.path.join(PMC_DIR, "summary_resident.json")   # bench.py --kernel-only: the value's pass
CALL_PMC = os.path.join(PMC_DIR, "summary_call.json")           # bench.py --skip-kernel-pass: call_pcie's calls
QUANT_PMC = os.path.join(PMC_DIR, "summary_quant.json")
LIB_SO = os.path.join(ROOT, "crispresso_amd", "lib", "libcrispr_nw.so")
AMPLICON_LEN = 250


C4_TOTAL_READS = 100_000_000   # BASELINE.json configs[3]
C4_CALL_READS = 12_500_000     # reads per call (100M / 8 GPUs: one call per rank at N = 8)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_share():
    """(threads, detail): the CPUs this process may run on (sched_getaffinity), capped by the
    cgroup's CPU quota when there is one (the GPU box shows the whole machine's CPUs to
    os.cpu_count() and affinity, but gives a job a share of them)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, {"sched_getaffinity": aff, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(),
                 "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def dist_setup():
    """(rank, local, world, dist) -- gloo on the host; torch.cuda is never touched."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 0, 1, None
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # rehearsal of the N > 1 path on a box with fewer GPUs than ranks (several ranks share a device)
    if os.environ.get("CRISPR_BENCH_DEVICES"):
        local %= max(1, int(os.environ["CRISPR_BENCH_DEVICES"]))
    # gloo prints its connection report on the C stdout: keep stdout for the one JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo")
        dist.barrier()
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    return rank, local, world, dist


def launch_ranks(n):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE): start the N ranks as a
    torch.distributed.run child (one process per GPU, rank r on device r) and relay its exit
    status.  This process never touches the GPU (nothing GPU-related is imported before this
    point), so the ranks start from a clean runtime; rank 0 writes the JSON line straight to
    the inherited stdout."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n} without a launcher: starting {n} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.run(cmd, env=dict(os.environ, CRISPR_BENCH_LAUNCHED="1")).returncode


def ranks_seen(dist):
    """Ranks that reached this point (a sum over the process group), 1 without one."""
    if dist is None:
        return 1
    import torch

    t = torch.ones(1, dtype=torch.float64)
    dist.all_reduce(t)
    return int(t.item())


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, value):
    if dist is None:
        return value
    import torch

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def lib_sha1():
    import hashlib

    try:
        with open(LIB_SO, "rb") as f:
            return hashlib.sha1(f.read()).hexdigest()
    except OSError:
        return None


def pmc_per_call(path, select):
    """(HBM bytes per call, VALU per call of the fill<16> kernels, kernels, source note) summed over the
    kernels of a per-call PMC summary whose names satisfy `select`; None when the summary is absent."""
    try:
        with open(path) as f:
            summ = json.load(f)
    except (OSError, ValueError):
        return None
    meta = summ.pop("_meta", {})
    names = sorted(k for k in summ if select(k) and "hbm_bytes_per_call" in summ[k])
    if not names:
        return None
    traffic = float(sum(summ[k]["hbm_bytes_per_call"] for k in names))
    valu16 = sum(summ[k].get("valu_per_call", 0.0) for k in names if "nw_band_fill<16" in k) or None
    here = lib_sha1()
    return {"traffic": traffic, "valu_fill16": valu16, "kernels": names,
            "source": os.path.relpath(path, ROOT), "calls_profiled": meta.get("calls"),
            "lib_sha1": meta.get("lib_sha1"), "lib_matches_loaded": (meta.get("lib_sha1") == here) if here else None}


def sample_check(amplicon, buf, offsets, ob, every, threads):
    """Every `every`-th read of the timed batch: its record and the rows expanded from its
    runs against the CPU oracle (outside the timed region)."""
    from tests.every_read import check_subset

    offsets = np.asarray(offsets, dtype=np.int64)
    idx = np.arange(0, len(offsets) - 1, every, dtype=np.int64)
    bad = check_subset(amplicon, buf, offsets, ob, idx, threads)
    return {"reads_checked": int(len(idx)), "every": every, "sample_mismatches": int(bad.sum()),
            "what": "record (length, identity, similarity, gaps, score, start cell) and the three rows expanded "
                    "from the runs, vs oracle/nw_oracle.c on the same reads"}


def sample_check_multi(amplicons, buf, offsets, which, ob, every, threads):
    """sample_check of a pooled batch (reads grouped by amplicon): every `every`-th read, each
    against its own amplicon."""
    from crispresso_amd.aligner import OpsBatch
    from tests.every_read import check_subset

    offsets = np.asarray(offsets, dtype=np.int64)
    idx = np.arange(0, len(offsets) - 1, every, dtype=np.int64)
    bounds = np.searchsorted(which, np.arange(len(amplicons) + 1))
    bad = 0
    for g, amp in enumerate(amplicons):
        lo, hi = int(bounds[g]), int(bounds[g + 1])
        sel = idx[(idx >= lo) & (idx < hi)]
        if not len(sel):
            continue
        sub_off = offsets[lo:hi + 1] - offsets[lo]
        r0, r1 = int(ob.ops_off[lo]), int(ob.ops_off[hi])
        sub = OpsBatch(ob.stats[lo:hi], ob.ops[r0:r1], ob.ops_off[lo:hi + 1] - r0, np.diff(sub_off), ob.scale)
        bad += int(check_subset(amp, buf[offsets[lo]:offsets[hi]], sub_off, sub, sel - lo, threads).sum())
    return {"reads_checked": int(len(idx)), "every": every, "sample_mismatches": bad,
            "what": "record and the three rows expanded from the runs, each read against its own amplicon, vs "
                    "oracle/nw_oracle.c"}


def sample_check_records(amplicon, buf, offsets, stats, every, threads):
    """Records of every `every`-th read of a records-only pass (the HDR pass) vs the oracle."""
    from oracle import oracle_py
    from tests.every_read import FIELDS

    offsets = np.asarray(offsets, dtype=np.int64)
    idx = np.arange(0, len(offsets) - 1, every, dtype=np.int64)
    lens = offsets[idx + 1] - offsets[idx]
    soff = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(lens, out=soff[1:])
    sbuf = np.concatenate([buf[offsets[r]:offsets[r + 1]] for r in idx.tolist()]) if len(idx) else np.zeros(1, np.uint8)
    res, _ = oracle_py.align_batch(amplicon, sbuf, soff, nthreads=threads)
    bad = np.zeros(len(idx), bool)
    for f in FIELDS:
        bad |= stats[f][idx] != res[f]
    return {"reads_checked": int(len(idx)), "every": every, "sample_mismatches": int(bad.sum()),
            "what": "records (length, identity, similarity, gaps, score, start cell) of the records-only pass vs "
                    "oracle/nw_oracle.c"}


def cpu_baseline(amplicon, buf, offsets, n_sample, threads, n_sample_1t, share_detail):
    from oracle import oracle_py

    t0 = time.perf_counter()
    oracle_py.align_batch(amplicon, buf, offsets[: n_sample + 1], nthreads=threads)
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    oracle_py.align_batch(amplicon, buf, offsets[: n_sample_1t + 1], nthreads=1)
    dt1 = time.perf_counter() - t1
    return {
        "value": n_sample / dt,
        "unit": "aligned reads/s",
        "cores": threads,
        "kind": "port",
        "one_thread": {"value": n_sample_1t / dt1, "cores": 1, "reads": n_sample_1t, "seconds": dt1},
        "cpu_share": share_detail,
        "sample": f"first {n_sample} reads of the same synthetic C2 batch, CPU oracle (oracle/nw_oracle.c, scalar "
                  f"Gotoh + traceback per read) on {threads} host threads (len(os.sched_getaffinity(0)) = "
                  f"{share_detail['sched_getaffinity']}, capped by the cgroup CPU quota "
                  f"{share_detail['cgroup_quota_cpus']}), {dt:.2f} s wall; one_thread: first {n_sample_1t} reads, "
                  "1 thread; EMBOSS needle itself is not installed on the box",
    }


def kernel_pass(al, pr, steps, warmup, lane_walk=False):
    """The packed call's kernels + ops compaction on the batch resident in HBM (upload once, in
    nw_align_ops_packed_lens' layout: classify decodes the 2-bit reads as in the call), one
    launch of each over the whole batch.  lane_walk: the first level's lane walk + stop summary
    instead of the call's wave-per-read walk (no pipelined call runs it)."""
    al.upload_packed(pr)
    al.set_lane_walk(lane_walk)
    for _ in range(warmup):
        al.run_async()
        al.sync()
    kms, phases = [], []
    for _ in range(max(steps, 1)):
        al.run_async()
        kms.append(al.sync())
        phases.append(al.phase_times())
    ph = {k: float(np.mean([d[k] for d in phases])) for k in phases[0]}
    al.set_lane_walk(False)
    return float(np.mean(kms)), ph, al.path_counts(), al.algo_bytes(), al.geometry()


def quant_leg(al, amplicon, buf, offsets, n_reads, steps, warmup, rank, world, cpu_sample, no_cpu):
    """Downstream quantification (process_df_chunk, CORE:428-753) of this rank's aligned
    reads, chained on the device: the aligner's resident OPS output (records + runs, the
    default output; nw_batch_device_ops) goes straight into nwq_run_device_ops, which
    rebuilds the rows it needs from the runs on the device and quantifies them.
    Settings: one guide cutting mid-amplicon, CRISPResso defaults otherwise
    (window_around_sgrna 1, exclude 15 bp each side)."""
    from crispresso_amd import quantify
    from crispresso_amd.aligner import OpsBatch
    from crispresso_amd.devmem import DeviceBuffer

    al.set_output("ops")
    al.upload(buf, offsets)
    al.run_async()
    al.sync()
    dev = al.device_ops()
    stride = dev["max_cols"]
    ob = al.download_ops(n_reads)
    lens = ob.stats["aln_len"].astype(np.int64)
    ident = ob.stats["n_ident"].astype(np.int64)
    um = ident == lens
    args = argparse.Namespace(amplicon_seq=amplicon, guide_seq=amplicon[105:125], cleavage_offset=-3,
                              window_around_sgrna=1, exclude_bp_from_left=15, exclude_bp_from_right=15,
                              coding_seq=None, expected_hdr_amplicon_seq=None)
    g = quantify.globals_from_args(args)
    q = quantify.GpuQuantifier(al.device)
    q.set_params(g, args)
    pre = quantify.pre_flags(um)
    d_pre = DeviceBuffer.from_array(pre, al.device)
    d_out = DeviceBuffer(16 * n_reads, al.device)
    for _ in range(warmup):
        q.run_device_ops(amplicon, dev, d_pre.ptr, n_reads, d_out.ptr)
    kms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        q.run_device_ops(amplicon, dev, d_pre.ptr, n_reads, d_out.ptr)
        kms.append(q.last_kernel_ms)
    elapsed = time.perf_counter() - t0
    nruns = np.diff(np.asarray(ob.ops_off, dtype=np.int64))
    rlen = np.diff(np.asarray(offsets[: n_reads + 1], dtype=np.int64))
    algo = int(n_reads * (1 + 4 + 8 + 16) + (4 * nruns[~um] + rlen[~um]).sum())
    kavg = float(np.mean(kms))
    qp = pmc_per_call(QUANT_PMC, lambda k: "nwq::" in k)
    out = {
        "metric": "quantified reads/s (process_df_chunk on the aligned C2 batch, device-resident)",
        "value": n_reads * steps / elapsed,
        "unit": "reads/s",
        "ms_per_step": elapsed / steps * 1e3,
        "input": "the aligner's resident ops output (records + runs + reads in HBM; no rows-mode re-run)",
        "kernel": "nwq::quant_lanes (process_df_chunk's substitution / insertion / deletion positions straight "
                  "from each read's runs and bytes, one lane per read; the few reads it does not take -- non-ACGT "
                  "bytes, more runs than a lane holds -- through nwq::expand_rows + nwq::quant_kernel) + "
                  "nwq::quant_reduce",
        "kernel_ms_avg": kavg,
        "lane_fallbacks": q.last_lane_fallbacks,
        "roofline": {"bound": "hbm", "achieved": algo / (kavg * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": algo / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": qp["traffic"] if qp else None,
                     "traffic_source": (f"{qp['source']} (rocprofv3 --pmc of bench.py --quant-only, per run, "
                                        f"library sha1 {qp['lib_sha1']}, matches the loaded one: "
                                        f"{qp['lib_matches_loaded']})") if qp else None,
                     "traffic_kernels": qp["kernels"] if qp else None,
                     "algo_bytes_per_launch": algo,
                     "algo_bytes_def": "per read 1 (flags) + 4 (aln_len) + 8 (run offset) + 16 (result); + 4 per "
                                       "run + the read's bytes for reads not UNMODIFIED on input"},
        "settings": "guide mid-amplicon, window_around_sgrna 1, exclude 15/15",
    }
    if rank == 0 and world == 1 and not no_cpu:
        from oracle import quant_oracle as qo

        k = min(cpu_sample, n_reads)
        sub = OpsBatch(ob.stats[:k], ob.ops[: int(ob.ops_off[k])], ob.ops_off[: k + 1], None, ob.scale,
                       offsets=offsets[: k + 1])
        batch = sub.expand(amplicon, buf, offsets[: k + 1])
        rows = [(batch.ref_seq(i), batch.align_str(i), batch.align_seq(i)) for i in range(k)]
        prm = qo.QuantParams(len_amplicon=g.LEN_AMPLICON, include_idxs=frozenset(g.INCLUDE_IDXS),
                             window_around_sgrna=1)
        t1 = time.perf_counter()
        qo.process_rows([r[0] for r in rows], [r[1] for r in rows], [r[2] for r in rows], um[:k], None, None, prm)
        dt = time.perf_counter() - t1
        out["cpu_baseline"] = {"value": k / dt, "unit": "reads/s", "cores": 1, "kind": "port",
                               "sample": f"first {k} aligned reads, oracle/quant_oracle.py (pure-Python restatement "
                                         f"of process_df_chunk), 1 thread, {dt:.2f} s"}
    d_pre.free()
    d_out.free()
    q.close()
    return out


def dual_leg(al, n_reads, steps, warmup, threads, sample_every):
    """C3: every read against the amplicon (records + runs) and against the HDR
    amplicon (records only: the repair pass reads scores, CORE:1808-1828 with just_score).
    One call per step (nw_align_dual_ops_packed_lens): the reads cross PCIe once, 2-bit packed
    as in the headline, and each uploaded read range is aligned against both amplicons, the HDR
    pass's chunks interleaved with the amplicon pass's.  Also timed: the two-call form of round 4
    (nw_align_ops_packed, then nw_align_ops_resident on the batch still in HBM after switching the
    amplicon), reported as "two_calls".  `al`: the headline's aligner (one context per process:
    a second one's streams would share the GPU's hardware queues with the first's)."""
    from crispresso_amd import _lib, synth
    from crispresso_amd.aligner import pack_2bit

    amp, hdr, buf, off = synth.c3_workload(n_reads)
    n = len(off) - 1
    pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
    stats = _lib.PinnedBuffer(n, _lib.STAT_DTYPE)
    stats2 = _lib.PinnedBuffer(n, _lib.STAT_DTYPE)
    ops_off = _lib.PinnedBuffer(n + 1, np.int64)
    ops_off2 = _lib.PinnedBuffer(n + 1, np.int64)
    ops = _lib.PinnedBuffer(4 * n + 4096, np.uint32)
    p_packed = _lib.PinnedBuffer((int(off[-1]) + 3) // 4 + 1, np.uint8)
    p_lens = _lib.PinnedBuffer(max(n, 1), np.uint16)
    pr = pack_2bit(pb.array, po.array, packed=p_packed.array, lens=p_lens.array)

    state = {}

    def two_calls():
        al.set_reference(amp)
        al.set_known(hdr)   # the HDR amplicon's copies: one alignment (needle.align_reads does the same)
        state["ob"] = al.align_ops_packed(pr, out=(stats.array, ops.array, ops_off.array))
        al.set_known(None)
        al.set_reference(hdr)   # the resident pass: the reference amplicon's copies from one alignment
        al.align_ops(None, po.array, out=(stats2.array, None, ops_off2.array), resident=True, records_only=True)

    dt2 = timed_calls(None, two_calls, max(2, steps // 2), 1, 0.0) / max(2, steps // 2)
    al.set_reference(amp)

    def step():
        state["ob"], _ = al.align_dual_packed(pr, hdr, out=(stats.array, ops.array, ops_off.array),
                                              out2=(stats2.array, None, ops_off2.array), records_only2=True)

    dt = timed_calls(None, step, steps, warmup, LEG_WARM_S) / steps
    checks = None
    if sample_every:   # the last timed step's outputs, both passes
        checks = {"amplicon_pass": sample_check(amp, buf, off, state["ob"], sample_every, threads),
                  "hdr_pass": sample_check_records(hdr, buf, off, stats2.array, sample_every, threads)}
    hdr_better = int((stats2.array["n_ident"] * stats.array["aln_len"] >
                      stats.array["n_ident"] * stats2.array["aln_len"]).sum())
    out = {"metric": "dual-aligned reads/s (C3: 1M reads x amplicon + HDR amplicon, 1 GPU)",
           "value": n / dt, "unit": "reads/s", "ms_per_step": dt * 1e3, "reads": n,
           "reads_closer_to_hdr": hdr_better, "sample_check": checks,
           "pcie": al.ops_times(), "path_counts_amplicon_pass": al.path_counts(),
           "two_calls": {"ms_per_step": dt2 * 1e3,
                         "note": "set the amplicon, nw_align_ops_packed, set the HDR amplicon, "
                                 "nw_align_ops_resident (round 4's step)"},
           "note": "per step: one nw_align_dual_ops_packed_lens call (pinned 2-bit reads in; amplicon pass: records "
                   "+ runs out, HDR pass: records out), synchronous; packing outside the timed region, as in the "
                   "headline"}
    for b in (pb, po, stats, stats2, ops_off, ops_off2, ops, p_packed):
        b.close()
    return out


def c1_shape_leg(al, n_reads, steps, warmup, threads, sample_every):
    """The reference's own read shape at volume (tests/crispresso_tests.py:145-155: 151 bp reads
    against the 280 bp amplicon; CORE:1791-1806): 1M 151 bp windows of a 280 bp amplicon (seed 6)
    at uniform offsets with the C2 edit mix (synth.c1_shape_workload), one nw_align_ops_packed
    call per step as in the headline."""
    from crispresso_amd import _lib, synth

    t0 = time.perf_counter()
    amp, buf, off = synth.c1_shape_workload(n_reads)
    pr, bufs = pack_pinned(buf, off, threads)
    n = len(off) - 1
    out = (_lib.PinnedBuffer(n, _lib.STAT_DTYPE), _lib.PinnedBuffer(4 * n + 4096, np.uint32),
           _lib.PinnedBuffer(n + 1, np.int64))
    outs = tuple(b.array for b in out)
    gen_s = time.perf_counter() - t0
    al.set_reference(amp)
    state = {}

    def call():
        state["ob"] = al.align_ops_packed(pr, out=outs)

    dt = timed_calls(None, call, steps, warmup, LEG_WARM_S) / steps
    res = {"metric": "aligned reads/s (C1 shape: 151 bp reads x 280 bp amplicon, 1 GPU)", "value": n / dt,
           "unit": "aligned reads/s", "ms_per_step": dt * 1e3, "reads": n, "amplicon_len": len(amp),
           "path_counts": al.path_counts(), "pcie": al.ops_times(), "input_prep_s": gen_s,
           "sample_check": sample_check(amp, buf, off, state["ob"], sample_every, threads) if sample_every else None,
           "note": "reads at uniform offsets 0..129 of the amplicon (La - Lb = -129), C2 edit mix within each "
                   "window; same call and buffers as the headline (pinned 2-bit reads in, records + runs out)"}
    for b in bufs + out:
        b.close()
    return res


RESIDENT_WARM_S = 0.2   # untimed seconds of resident passes before the headline's timed steps (steady clocks)
LEG_WARM_S = 0.5   # untimed seconds of calls before a leg's timed steps (steady GPU clocks)


def timed_calls(dist, call, steps, warmup, warm_s=0.0):
    """warmup untimed calls (and, for the legs, more until warm_s seconds of calls have run:
    after the host-side input generation the GPU has clocked down, and a 25-50 ms call
    needs several calls to reach steady clocks), then `steps` timed ones between barriers;
    max over ranks (s)."""
    t_w = time.perf_counter()
    k = 0
    while k < warmup or time.perf_counter() - t_w < warm_s:
        call()
        k += 1
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(steps):
        call()
    barrier(dist)
    return max_over_ranks(dist, time.perf_counter() - t0)


def pack_pinned(buf, offsets, threads):
    """(PackedReads in pinned memory, its buffers): text batch -> 2 bits per base."""
    from crispresso_amd import _lib
    from crispresso_amd.aligner import PackedReads, pack_2bit

    po = _lib.pinned_copy(offsets)
    pp = _lib.PinnedBuffer((int(offsets[-1]) + 3) // 4 + 16, np.uint8)
    pl = _lib.PinnedBuffer(max(len(offsets) - 1, 1), np.uint16)
    pr = pack_2bit(buf, po.array, nthreads=threads, packed=pp.array, lens=pl.array)
    return PackedReads(pr.packed, po.array, pr.exc_pos, pr.exc_byte, pr.lens), (po, pp, pl)


def c4_leg(al, amplicon, rank, world, dist, threads, steps, warmup, sample_every):
    """BASELINE configs[3] (C4: 100M synthetic 250 bp reads over N GPUs, SURVEY 8d seeds 10 + g):
    this rank aligns reads of the C4 generator, seed 10 + rank -- 100M / N of them in calls
    of at most 12.5M reads (N > 1), or one 12.5M-read call, the N = 8 shard (N = 1, "c4_shard").
    Inputs 2-bit packed in pinned memory before the timed region; outputs to pinned memory;
    value = reads of all ranks / max-over-ranks time.  The native generator
    (include/crispr_synth.h: the C2 mix, counter-based RNG) draws 12.5M reads in ~1 s."""
    from crispresso_amd import _lib, synth

    per_rank = C4_CALL_READS if world == 1 else C4_TOTAL_READS // world
    ncalls = (per_rank + C4_CALL_READS - 1) // C4_CALL_READS
    t0 = time.perf_counter()
    batches, keep = [], []
    scratch = np.empty(min(C4_CALL_READS, per_rank) * (len(amplicon) + 10), np.uint8)   # reads are <= La + 10
    text = off = None
    for k in range(ncalls):
        m = min(C4_CALL_READS, per_rank - k * C4_CALL_READS)
        text, off = synth.native_reads(amplicon, m, 10 + rank, first=k * C4_CALL_READS, buf=scratch)
        pr, bufs = pack_pinned(text, off, threads)
        batches.append(pr)
        keep.append(bufs)
    gen_s = time.perf_counter() - t0
    m_out = min(C4_CALL_READS, per_rank)
    out = (_lib.PinnedBuffer(m_out, _lib.STAT_DTYPE), _lib.PinnedBuffer(2 * m_out + 4096, np.uint32),
           _lib.PinnedBuffer(m_out + 1, np.int64))
    outs = tuple(b.array for b in out)
    state = {}

    def one_pass():
        for pr in batches:
            n = len(pr.offsets) - 1
            state["ob"] = al.align_ops_packed(pr, out=(outs[0][:n], outs[1], outs[2][:n + 1]))

    elapsed = timed_calls(dist, one_pass, steps, warmup, LEG_WARM_S)
    pcie = al.ops_times()
    ob = state["ob"]
    check = None
    if sample_every:
        check = sample_check(amplicon, text, off, ob, sample_every, threads)
    total = per_rank * world
    res = {"metric": "aligned reads/s (C4: 100M synthetic 250 bp reads sharded across the GPUs)" if world > 1
           else "aligned reads/s (C4 shard: 12.5M reads = 100M / 8 GPUs, one call, 1 GPU)",
           "value": total * steps / elapsed, "unit": "aligned reads/s", "n_gpus": world,
           "reads_per_rank": per_rank, "reads_total": total, "calls_per_rank": ncalls,
           "ms_per_pass": elapsed / steps * 1e3, "steps": steps, "warmup": warmup,
           "path_counts_last_call": al.path_counts(), "pcie_last_call": pcie, "sample_check_last_call": check,
           "input_prep_s": gen_s,
           "note": "pass = every call of this rank's share (inputs 2-bit packed in pinned host memory before the "
                   "timed region; records + runs to pinned host memory); reads of the C4 generator (native, seed "
                   "10 + rank, reads k*12.5M.. of its set for call k); barrier + max over ranks"}
    for bufs in keep:
        for b in bufs:
            b.close()
    for b in out:
        b.close()
    return res


def pooled_workload(n_amplicons, reads_per_amplicon, lo=None, hi=None):
    """C5: 96 amplicons of U[150, 300] bp (seed 5), reads from each with the C2 mix
    (native generator, seed 100 + g), grouped by amplicon as CRISPRessoPooled's
    demultiplexing leaves them.  -> (amplicons, offsets of all reads, amplicon of each read,
    bytes of reads [lo, hi) only (all by default))."""
    from crispresso_amd import synth

    amps = synth.pooled_amplicons(n_amplicons, 5)
    lens = np.concatenate([np.diff(synth.native_offsets(a, reads_per_amplicon, 100 + g)) for g, a in enumerate(amps)])
    off = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    which = np.repeat(np.arange(n_amplicons, dtype=np.int32), reads_per_amplicon)
    lo = 0 if lo is None else lo
    hi = len(lens) if hi is None else hi
    buf = np.empty(max(int(off[hi] - off[lo]), 1), np.uint8)
    for g, amp in enumerate(amps):
        a, b = max(lo, g * reads_per_amplicon), min(hi, (g + 1) * reads_per_amplicon)
        if a < b:
            seg = buf[off[a] - off[lo]:off[b] - off[lo]]
            synth.native_reads(amp, b - a, 100 + g, first=a - g * reads_per_amplicon, buf=seg)
    return amps, buf, off, which


def pooled_leg(al, rank, world, dist, n_amplicons, reads_per_amplicon, steps, warmup, threads, text_too,
               sample_every):
    """BASELINE configs[4] (C5: CRISPRessoPooled, 96 amplicons x 100k reads, 150-300 bp, over the
    N GPUs): the reads are split by DP cells (distributed.cell_partition, the same split
    align_pooled_sharded makes; CRISPRessoPooled.py:882-908 ran one CRISPResso per amplicon,
    serially), each rank aligns its range with one nw_align_multi_ops_packed call (pinned
    2-bit input).  value = all reads / max-over-ranks time.  `al` is the headline's context
    (a second context's streams would share the hardware queues); the call leaves it
    without an amplicon."""
    from crispresso_amd import _lib
    from crispresso_amd.distributed import cell_partition, pooled_costs

    from crispresso_amd import synth

    amps = synth.pooled_amplicons(n_amplicons, 5)
    t0 = time.perf_counter()
    lens = np.concatenate([np.diff(synth.native_offsets(a, reads_per_amplicon, 100 + g)) for g, a in enumerate(amps)])
    off_all = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=off_all[1:])
    which_all = np.repeat(np.arange(n_amplicons, dtype=np.int32), reads_per_amplicon)
    parts = cell_partition(pooled_costs(amps, off_all, which_all), world)
    lo, hi = parts[rank]
    _, buf, _, _ = pooled_workload(n_amplicons, reads_per_amplicon, lo, hi)
    off = off_all[lo:hi + 1] - off_all[lo]
    which = which_all[lo:hi]
    n = hi - lo
    pr, bufs = pack_pinned(buf, off, threads)
    pw = _lib.pinned_copy(which)
    gen_s = time.perf_counter() - t0
    out = (_lib.PinnedBuffer(n, _lib.STAT_DTYPE), _lib.PinnedBuffer(4 * n + 4096, np.uint32),
           _lib.PinnedBuffer(n + 1, np.int64))
    outs = tuple(b.array for b in out)
    state = {}

    def call():
        state["ob"] = al.align_multi_ops(amps, pr, None, pw.array, out=outs)

    elapsed = timed_calls(dist, call, steps, warmup, LEG_WARM_S)
    ob = state["ob"]
    res = {"metric": "pooled aligned reads/s (C5: 96 amplicons x 100k reads, 150-300 bp, over the GPUs)",
           "value": len(lens) * steps / elapsed, "unit": "aligned reads/s", "n_gpus": world,
           "ms_per_step": elapsed / steps * 1e3, "reads_total": int(len(lens)), "reads_this_rank": int(n),
           "amplicons": n_amplicons, "reads_per_amplicon": reads_per_amplicon,
           "partition": [[int(a), int(b)] for a, b in parts],
           "cells_this_rank": int(pooled_costs(amps, off_all, which_all)[lo:hi].sum()),
           "mean_read_len": float(lens.mean()), "path_counts": al.path_counts(), "pcie": al.ops_times(),
           "runs_per_read": int(ob.ops_off[n]) / max(n, 1), "input_prep_s": gen_s,
           "algo_bytes_this_rank": int((off[-1] - off[0]) + 3 * outs[0]["aln_len"].astype(np.int64).sum() + 16 * n),
           "sample_check": (sample_check_multi(amps, buf, off, which, ob, sample_every, threads)
                            if sample_every else None),
           "note": "step = one nw_align_multi_ops_packed call per rank on its cell_partition range (2-bit reads + "
                   "exceptions in, pinned; every amplicon's tables uploaded once; chunks of one amplicon each); "
                   "barrier + max over ranks"}
    if text_too:   # the same call on the text: same records and runs
        pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(off)
        packed_ops = (ob.ops_off.copy(), ob.ops[: int(ob.ops_off[n])].copy(), outs[0].copy())
        t1 = time.perf_counter()
        tob = al.align_multi_ops(amps, pb.array, po.array, pw.array)
        dt = time.perf_counter() - t1
        res["text_input"] = {"value": n / dt, "ms_per_step": dt * 1e3, "pcie": al.ops_times(),
                             "same_output_as_packed": bool(np.array_equal(tob.ops_off, packed_ops[0])
                                                           and np.array_equal(tob.ops, packed_ops[1])
                                                           and np.array_equal(tob.stats, packed_ops[2]))}
        pb.close()
        po.close()
    for b in bufs + (pw,) + out:
        b.close()
    return res


def e2e_leg(al, amplicon, buf, offsets, threads, repeats=2):
    """The product path end to end (CORE:1788-2000): a FASTQ.gz of the rank's 1M C2 reads through
    needle.align_reads to the DataFrame parse_needle_output would build -- native ingest
    (libdeflate + parallel parse + 2-bit packing into pinned memory), one nw_align_ops_packed
    call, the DataFrame hand-off.  Reports the wall time and each stage's share."""
    import gzip
    import tempfile

    from crispresso_amd.needle import AlignArgs, align_reads

    n = len(offsets) - 1
    tmp = tempfile.mkdtemp(prefix="crispr_e2e_")
    path = os.path.join(tmp, "c2_reads.fastq.gz")
    t0 = time.perf_counter()
    seqs = bytes(buf).decode("ascii")
    off = offsets.tolist()
    qual = "I" * 400
    with gzip.open(path, "wb", compresslevel=1) as f:
        step = 100_000
        for lo in range(0, n, step):
            hi = min(n, lo + step)
            f.write("".join(f"@SYN:1:FC{r // 65536}:1:{r % 65536}:{r} 1:N:0\n{seqs[off[r]:off[r + 1]]}\n+\n"
                            f"{qual[: off[r + 1] - off[r]]}\n" for r in range(lo, hi)).encode("ascii"))
    write_s = time.perf_counter() - t0
    gz_bytes = os.path.getsize(path)
    runs = []
    rows = None
    for _ in range(repeats):
        tm = {}
        t1 = time.perf_counter()
        df = align_reads(AlignArgs(amplicon_seq=amplicon), path, aligner=al, timings=tm)
        tm["wall_s"] = time.perf_counter() - t1
        runs.append(tm)
        rows = len(df)
        del df
    try:
        os.remove(path)
        os.rmdir(tmp)
    except OSError:
        pass
    best = min(runs, key=lambda t: t["wall_s"])
    return {"metric": "reads/s end to end (C2 FASTQ.gz -> DataFrame, needle.align_reads)",
            "value": n / best["wall_s"], "unit": "reads/s", "reads": n, "rows": rows,
            "seconds": best, "first_call_seconds": runs[0],
            "aligner_call_ms": best["align_s"] * 1e3, "aligner_call_share": best["align_s"] / best["wall_s"],
            "fastq_gz_bytes": gz_bytes, "write_s": write_s,
            "note": "best of the runs; align_s = the nw_align_ops_packed call inside align_reads (pinned 2-bit batch "
                    "from the ingest in, records + runs to pinned pool memory out); ingest_s = nw_fastq_read + "
                    "nw_fastq_pack; dataframe_s = ops_to_dataframe; FASTQ.gz written with gzip level 1 outside the "
                    "timing"}


def merge_leg(device, n_pairs):
    """The paired-end merge (crispresso_amd/flash.py, FLASH semantics) on synthetic pairs of the
    same shape as scripts/bench_flash.py: 2 x 150 bp over a 250 bp amplicon, 1 % noise, seed 7,
    CRISPResso's FLASH options.  Informational (upstream of the metric's path)."""
    from crispresso_amd.flash import FlashOptions, merge_packed

    L, amp_len = 150, 250
    rng = np.random.Generator(np.random.PCG64(7))
    alpha = np.frombuffer(b"ACGT", np.uint8)
    amp = rng.choice(alpha, amp_len)
    comp = np.zeros(256, np.uint8)
    for x, y in zip(b"ACGT", b"TGCA"):
        comp[x] = y
    r1 = np.tile(amp[:L], (n_pairs, 1))
    r2 = np.tile(comp[amp[::-1]][:L], (n_pairs, 1))
    for r in (r1, r2):
        m = rng.random(r.shape) < 0.01
        r[m] = rng.choice(alpha, int(m.sum()))
    q = rng.integers(53, 74, (n_pairs, L)).astype(np.uint8)
    off = np.arange(n_pairs + 1, dtype=np.int64) * L
    opts = FlashOptions(min_overlap=4, max_overlap=100, allow_outies=True)
    merge_packed(r1[:1000].ravel(), q[:1000].ravel(), off[:1001], r2[:1000].ravel(), q[:1000].ravel(), off[:1001],
                 opts, device)
    t0 = time.perf_counter()
    res = merge_packed(r1.ravel(), q.ravel(), off, r2.ravel(), q.ravel(), off, opts, device)
    wall = time.perf_counter() - t0
    return {"metric": "merged read pairs/s", "pairs": n_pairs, "read_len": L, "kernel_ms": res.kernel_ms,
            "value": n_pairs / (res.kernel_ms / 1e3), "call_pairs_per_s": n_pairs / wall,
            "combined": int((res.length > 0).sum()),
            "note": "nwf_merge_batch kernel time (inputs resident); call_pairs_per_s includes PCIe and allocation"}


def band_cells(counts, La, mean_len):
    """DP cells the band path computes per pass: W diagonals x (La + Lb) / 2 anti-diagonal steps per read
    and level (16, 32 and the 128-diagonal wide level), the full La x Lb matrix for the exact kernel, none
    for exact copies."""
    steps = (La + mean_len) / 2.0
    return (counts["band16"] * 16 * steps + counts["band32"] * 32 * steps + counts["band_fallback"] * 128 * steps +
            counts["exact_kernel"] * La * mean_len)


def dry_run(args, rank, local, world, dist, seen, place):
    """--dry-run: the N-rank plumbing without a GPU (CPU tests).  Each rank derives its share of
    the C2 / C4 / pooled work exactly as a measured run would and reports it, with its host
    placement (CPU slice, native pool threads); rank 0 prints them all in one line."""
    from crispresso_amd import _lib, synth
    from crispresso_amd.distributed import cell_partition, pooled_costs

    per_rank_c4 = C4_CALL_READS if world == 1 else C4_TOTAL_READS // world
    amps = synth.pooled_amplicons(args.pooled_amplicons, 5)
    lens = np.concatenate([np.diff(synth.native_offsets(a, args.pooled_reads, 100 + g)) for g, a in enumerate(amps)])
    off_all = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=off_all[1:])
    which_all = np.repeat(np.arange(len(amps), dtype=np.int32), args.pooled_reads)
    parts = cell_partition(pooled_costs(amps, off_all, which_all), world)
    mine = {"rank": rank, "device": local, "c2_reads": args.reads, "c2_seed": 2 if world == 1 else 10 + rank,
            "c4_reads": per_rank_c4, "pooled_range": list(map(int, parts[rank]))}
    import torch

    t = torch.tensor([rank, local, mine["c4_reads"], *mine["pooled_range"]], dtype=torch.int64)
    gathered = [torch.zeros_like(t) for _ in range(world)] if dist is not None else [t]
    if dist is not None:
        dist.all_gather(gathered, t)
    place = dict(place, pool_threads=int(_lib.load().nw_host_threads()))
    places = [None] * world
    if dist is not None:
        dist.all_gather_object(places, place)
    else:
        places = [place]
    barrier(dist)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": seen,
                          "ranks": [{"rank": int(g[0]), "device": int(g[1]), "c4_reads": int(g[2]),
                                     "pooled_range": [int(g[3]), int(g[4])]} for g in gathered],
                          "host_placement": places,
                          "c4_reads_total": int(sum(int(g[2]) for g in gathered)),
                          "pooled_reads_total": int(len(lens))}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=READS_PER_GPU)
    ap.add_argument("--cpu-sample", type=int, default=300_000)
    ap.add_argument("--cpu-sample-1t", type=int, default=20_000)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline and host packing (default: the process's CPU share: "
                         "sched_getaffinity capped by the cgroup quota)")
    ap.add_argument("--sample-every", type=int, default=100)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the oracle sample checks of the timed batches")
    ap.add_argument("--no-quant", action="store_true", help="skip the downstream quantification leg")
    ap.add_argument("--quant-cpu-sample", type=int, default=20_000)
    ap.add_argument("--no-legs", action="store_true", help="skip the e2e / C3 / merge legs (N = 1 only)")
    ap.add_argument("--no-multi", action="store_true", help="skip the C4 and pooled (C5) legs")
    ap.add_argument("--multi-steps", type=int, default=3, help="timed passes of the C4 / pooled legs")
    ap.add_argument("--merge-pairs", type=int, default=1_000_000)
    ap.add_argument("--kernel-only", action="store_true",
                    help="profiling: only the kernel-resident pass (one launch of each kernel per step over the whole "
                         "batch, so rocprofv3 per-dispatch figures are per-pass figures); value = the kernel rate")
    ap.add_argument("--quant-only", action="store_true",
                    help="profiling: only the downstream quantification leg (its kernels on the resident batch)")
    ap.add_argument("--skip-kernel-pass", action="store_true",
                    help="tracing: stop after the timed packed calls (no text call, kernel-resident pass or legs)")
    ap.add_argument("--phase-events", action="store_true",
                    help="A/B: keep the resident pass's per-phase timing events in the timed steps")
    ap.add_argument("--pooled-amplicons", type=int, default=96)
    ap.add_argument("--pooled-reads", type=int, default=100_000, help="C5 reads per amplicon")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch check without a GPU: form the world, partition the C4 / pooled work over the ranks, "
                         "print rank 0's line with \"dry_run\": true; no alignment, no value")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:   # checked before joining the process group
        log(f"[bench] --gpus {args.gpus} but the launcher formed a world of {world_env} ranks")
        sys.exit(2)
    rank, local, world, dist = dist_setup()
    seen = ranks_seen(dist)
    if seen != world:
        log(f"[rank {rank}] {seen} of {world} ranks reached the start")
        sys.exit(2)
    # host placement before anything is allocated or the library's pool exists (one
    # host thread set per GPU): at N > 1 every rank is bound to its slice of the CPU share on its
    # GPU's NUMA node and its native pool sized to that slice; at N = 1 nothing changes
    from crispresso_amd import placement

    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    local_rank = int(os.environ.get("LOCAL_RANK", local))
    ndev = int(os.environ.get("CRISPR_BENCH_DEVICES", "0"))   # the rehearsal's shared devices
    place = placement.bind_rank(local_rank, local_world, apply=local_world > 1,
                                device_of=(lambda r: r % ndev) if ndev > 0 else None)
    if args.dry_run:
        dry_run(args, rank, local, world, dist, seen, place)
        return
    from crispresso_amd import _lib, synth
    from crispresso_amd.aligner import GpuAligner

    share, share_detail = cpu_share()
    place["pool_threads"] = int(_lib.load().nw_host_threads())
    # the ranks of a node share its CPUs: a bound rank uses its slice
    threads = args.cpu_threads or (place["threads"] if local_world > 1 else max(1, share // max(1, local_world)))
    amplicon = synth.random_amplicon(AMPLICON_LEN, 1)
    seed = 2 if world == 1 else 10 + rank
    t0 = time.perf_counter()
    buf, offsets = synth.reads_from(amplicon, args.reads, seed)
    n = len(offsets) - 1
    log(f"[rank {rank}] generated {n} reads in {time.perf_counter() - t0:.1f}s; host threads {threads} {share_detail}")

    al = GpuAligner(local)
    al.set_reference(amplicon)
    place["device_pci"] = placement.device_pci(local)   # the device HIP opened: does it match the KFD order?
    place["pci_match"] = place["device_pci"] == place["gpu_pci"] if place["gpu_pci"] else None
    # the host batch and the outputs in pinned memory (the native FASTQ ingest, nw_fastq_pack, hands the
    # aligner exactly such a batch: the e2e leg)
    pb, po = _lib.pinned_copy(buf), _lib.pinned_copy(offsets)
    p_packed = _lib.PinnedBuffer((int(offsets[-1]) + 3) // 4 + 16, np.uint8)
    p_lens = _lib.PinnedBuffer(max(n, 1), np.uint16)
    p_stats = _lib.PinnedBuffer(n, _lib.STAT_DTYPE)
    p_off = _lib.PinnedBuffer(n + 1, np.int64)
    p_ops = _lib.PinnedBuffer(4 * n + 4096, np.uint32)
    out = (p_stats.array, p_ops.array, p_off.array)
    if args.quant_only:
        q = quant_leg(al, amplicon, buf, offsets, n, args.steps, args.warmup, rank, world, args.quant_cpu_sample, True)
        if rank == 0:
            print(json.dumps(q), flush=True)
        al.close()
        return
    if args.kernel_only:
        from crispresso_amd.aligner import pack_2bit

        pr = pack_2bit(pb.array, po.array, nthreads=threads, packed=p_packed.array, lens=p_lens.array)
        kms, phases, counts, algo_bytes, geo = kernel_pass(al, pr, args.steps, args.warmup, lane_walk=True)
        if rank == 0:
            print(json.dumps({"metric": "kernel-resident aligned reads/s (profiling run, not the bench metric)",
                              "value": n / (kms * 1e-3), "kernel_ms": kms, "phases_ms": phases,
                              "path_counts": counts, "algo_bytes_per_launch": algo_bytes}), flush=True)
        al.close()
        return
    from crispresso_amd.aligner import pack_2bit

    t1 = time.perf_counter()
    pr = pack_2bit(pb.array, po.array, nthreads=threads, packed=p_packed.array, lens=p_lens.array)
    pack_s = time.perf_counter() - t1
    state = {}

    def headline_call():
        state["ob"] = al.align_ops_packed(pr, out=out)   # synchronous: records + runs are in host memory

    elapsed_call = timed_calls(dist, headline_call, args.steps, args.warmup)
    ob = state["ob"]
    pcie = al.ops_times()
    n_runs = int(ob.ops_off[n])
    call_counts = al.path_counts()

    if args.skip_kernel_pass:   # tracing / call A/B: the timed calls only
        if rank == 0:
            print(json.dumps({"metric": "aligned reads/s (timed calls only, --skip-kernel-pass)",
                              "value": n * world * args.steps / elapsed_call,
                              "ms_per_step": elapsed_call / args.steps * 1e3,
                              "n_gpus": world, "pcie": pcie, "path_counts": call_counts}), flush=True)
        al.close()
        return
    # the timed call's own outputs against the oracle (before anything reuses the buffers)
    check = None if args.no_check else sample_check(amplicon, buf, offsets, ob, args.sample_every, threads)

    # the same call on the text (one byte per base over PCIe), into its own (pool) buffers
    al.align_ops(pb.array, po.array)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        ob_text = al.align_ops(pb.array, po.array)
    text_s = (time.perf_counter() - t1) / args.steps
    text_pcie = al.ops_times()
    text_same = bool(np.array_equal(ob_text.stats, ob.stats) and np.array_equal(ob_text.ops_off, ob.ops_off)
                     and np.array_equal(ob_text.ops, ob.ops[:n_runs]))
    del ob_text

    t1 = time.perf_counter()
    ob.expand(amplicon, pb.array, po.array, nthreads=threads)
    expand_s = time.perf_counter() - t1

    # value: the hot path over the batch resident in HBM (wall clock, barriers, max over ranks); the
    # 1M-read call runs the first level's lane walk + stop summary on every chunk (>= 65536 reads,
    # DESIGN.md 4a), so the resident pass does too
    al.upload_packed(pr)
    al.set_lane_walk(True)
    al.set_phase_events(args.phase_events)   # off: kernel_rate below times the phases, with their events

    step_kms = []

    def resident_step():
        al.run_async()
        step_kms.append(al.sync())   # records + runs of every read in HBM; the pass's HIP-event time

    elapsed = timed_calls(dist, resident_step, args.steps, args.warmup, warm_s=RESIDENT_WARM_S)
    kms_timed = float(np.mean(step_kms[-args.steps:]))   # the timed steps' own device time (roofline)
    res = al.download_ops(n)
    n_res = int(res.ops_off[n])
    resident_check = {
        "reads": n, "runs": n_res,
        "same_as_call": bool(n_res == n_runs and np.array_equal(res.ops_off, ob.ops_off[:n + 1])
                             and np.array_equal(res.stats, ob.stats) and np.array_equal(res.ops[:n_res], ob.ops[:n_runs])),
        "what": "every record, run offset and run of the timed resident pass (downloaded after it) against the "
                "pipelined call's output on the same reads (which sample_check holds against the oracle)",
    }
    del res
    al.set_lane_walk(False)
    al.set_phase_events(True)
    # the same pass by HIP events (per phase), and with the wave-per-read walk for reference
    kms, phases, counts, algo_bytes, geo = kernel_pass(al, pr, args.steps, args.warmup, lane_walk=True)
    kms_ww, phases_ww, _, _, _ = kernel_pass(al, pr, args.steps, args.warmup)
    geo["fallback_reads"] = counts["band_fallback"]
    geo["exact_kernel_reads"] = counts["exact_kernel"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(amplicon, buf, offsets, min(args.cpu_sample, n), threads, min(args.cpu_sample_1t, n),
                           share_detail)

    quant = None
    if not args.no_quant:
        quant = quant_leg(al, amplicon, buf, offsets, n, args.steps, args.warmup, rank, world, args.quant_cpu_sample,
                          args.no_cpu)

    # the multi-GPU configs at their own shapes (every rank takes part: barriers inside)
    multi = {"c4": None, "pooled": None}
    if not args.no_multi:
        for name in multi:
            try:   # never cost the bench line (the error is reported instead)
                if name == "c4":
                    al.set_reference(amplicon)
                    multi[name] = c4_leg(al, amplicon, rank, world, dist, threads, args.multi_steps, 1,
                                         0 if args.no_check else 1250)
                else:
                    multi[name] = pooled_leg(al, rank, world, dist, args.pooled_amplicons, args.pooled_reads,
                                             args.multi_steps, 1, threads, text_too=world == 1,
                                             sample_every=0 if args.no_check else 1000)
            except Exception as exc:
                multi[name] = {"error": f"{type(exc).__name__}: {exc}"}

    legs = {"e2e": None, "dual": None, "c1": None, "merge": None}
    if rank == 0 and world == 1 and not args.no_legs:
        for name in legs:
            try:   # informational legs: never cost the bench line
                if name == "e2e":
                    al.set_reference(amplicon)
                    legs[name] = e2e_leg(al, amplicon, buf, offsets, threads)
                elif name == "c1":
                    legs[name] = c1_shape_leg(al, args.reads, args.steps, args.warmup, threads,
                                              0 if args.no_check else args.sample_every)
                elif name == "dual":
                    legs[name] = dual_leg(al, args.reads, args.steps, args.warmup, threads,
                                          0 if args.no_check else args.sample_every)
                else:
                    legs[name] = merge_leg(local, args.merge_pairs)
            except Exception as exc:
                legs[name] = {"error": f"{type(exc).__name__}: {exc}"}

    # HBM traffic and the fill<16> VALU count per pass of the timed resident pass (PMC of bench.py
    # --kernel-only: the same kernels, one launch each per pass); the call's per-call traffic beside it
    aligner_kernel = lambda k: ("nw::" in k and "nwq::" not in k) or "nw_align_kernel" in k  # noqa: E731
    cp = pmc_per_call(RESIDENT_PMC, aligner_kernel)
    ccp = pmc_per_call(CALL_PMC, aligner_kernel)
    traffic = cp["traffic"] if cp else None
    fill_valu = cp["valu_fill16"] if cp else None
    lens = np.diff(offsets)
    cells = band_cells(counts, AMPLICON_LEN, float(lens.mean()) if n else 0.0)
    pass_gbs = algo_bytes / (kms_timed * 1e-3) / 1e9
    ms_step = elapsed / args.steps * 1e3
    ms_call = elapsed_call / args.steps * 1e3
    call_gbs = algo_bytes / (ms_call * 1e-3) / 1e9
    fill_ms = phases["fill16_ms"]
    value = n * world * args.steps / elapsed
    if rank == 0:
        line = {
            "metric": "aligned reads/sec (250 bp amplicon x 1M reads) at 1/2/4/8 MI355X",
            "value": value,
            "unit": "aligned reads/s",
            "n_gpus": world,
            "ranks_seen": seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16x2",
            "data": "synthetic (SURVEY 8d C2 mix: 60% exact, 20% 1-3 subs, 10% del, 5% ins, 5% 1% noise)",
            "config": {
                "workload": f"C2: {n} synthetic ~250 bp reads x 250 bp amplicon per GPU, EMBOSS needle semantics "
                            "(EDNAFULL, gapopen 10, gapextend 0.5, free end gaps); step = one pass of the hot path over "
                            "the batch resident in HBM (2 bits per base + lengths): every read's record + traceback "
                            "runs written to HBM (nw_batch_run_async + nw_batch_sync); the PCIe-inclusive call "
                            "(pinned host batch in -> pinned host records out) is call_pcie",
                "reads_per_gpu": n,
                "amplicon_len": AMPLICON_LEN,
                "parallelism": f"read shards x{world} (no collective on the data path; gloo host barrier)",
                "kernel_geometry": geo,
            },
            "resident_check": resident_check,
            "call_pcie": {
                "value": n * world * args.steps / elapsed_call, "unit": "aligned reads/s", "ms_per_step": ms_call,
                "path_counts": call_counts,
                "note": "SURVEY 8d's boundary: one nw_align_ops_packed call per step, the pinned host batch (2 bits "
                        "per base) in -> records + runs in pinned host memory, chunks pipelined over PCIe (value up "
                        "to round 4); same barriers and max over ranks",
            },
            "host_placement": place,
            "ingest_pack": {"ms": pack_s * 1e3, "bases_per_s": (int(offsets[-1]) - int(offsets[0])) / pack_s,
                            "threads": threads, "exceptions": int(len(pr.exc_pos)),
                            "note": "nw_pack_reads: the text batch -> 2 bits per base + exception list (host; the "
                                    "native FASTQ ingest does the same inside nw_fastq_pack, timed in e2e)"},
            "text_input": {"value": n / text_s, "ms_per_step": text_s * 1e3, "h2d_ms": text_pcie["h2d_ms"],
                           "h2d_bytes": text_pcie["h2d_bytes"], "same_output_as_packed": text_same,
                           "note": "nw_align_ops on the text batch (one byte per base over PCIe), own output buffers"},
            "pcie": {
                "h2d_ms": pcie["h2d_ms"], "h2d_bytes": pcie["h2d_bytes"],
                "h2d_gbs": pcie["h2d_bytes"] / max(pcie["h2d_ms"], 1e-9) / 1e6,
                "d2h_bytes": pcie["d2h_bytes"], "compute_ms_in_call": pcie["compute_ms"],
                "runs_per_read": n_runs / max(n, 1),
                "note": "last timed call_pcie call: upload span on the copy stream; d2h = records (32 B) + run offsets (8 B) "
                        "per read + 4 B per run; compute = the call's device span, first upload to the last chunk's end",
            },
            "kernel_rate": {
                "value": n / (kms * 1e-3), "unit": "aligned reads/s", "kernel_ms": kms, "phases_ms": phases,
                "path_counts": counts,
                "note": "the call's own kernels (the first level's lane walk + stop summary, as the call's chunks of "
                        ">= 65536 reads run them) + ops compaction on the batch resident in HBM, one launch of each "
                        "over the batch, outputs left in HBM (HIP events on the aligner's stream)",
            },
            "kernel_rate_wave_walk": {
                "value": n / (kms_ww * 1e-3), "unit": "aligned reads/s", "kernel_ms": kms_ww, "phases_ms": phases_ww,
                "note": "the same resident pass with the wave-per-read walk (what the pooled call's small chunks run)",
            },
            "expand": {"ms": expand_s * 1e3, "reads_per_s": n / expand_s, "threads": threads,
                       "note": "nw_expand_ops: the three rows of every read rebuilt from its runs on the host "
                               "(not in value)"},
            "sample_check": check,
            "roofline": {
                "bound": "hbm",
                "achieved": pass_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": pass_gbs / HBM_PEAK_GBS,
                "call_achieved": call_gbs,   # the same bytes over call_pcie's ms_per_step
                "call_frac": call_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": (f"{cp['source']} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py "
                                   f"--kernel-only: every launch of {cp['calls_profiled']} resident passes, summed "
                                   f"per pass; library sha1 {cp['lib_sha1']}, matches the loaded one: "
                                   f"{cp['lib_matches_loaded']})") if cp else None,
                "traffic_kernels": cp["kernels"] if cp else None,
                "call_traffic": ccp["traffic"] if ccp else None,
                "call_traffic_source": (f"{ccp['source']} (bench.py --skip-kernel-pass: every launch of "
                                        f"{ccp['calls_profiled']} call_pcie calls, summed per call; library sha1 "
                                        f"{ccp['lib_sha1']}, matches the loaded one: {ccp['lib_matches_loaded']})")
                                       if ccp else None,
                "kernel": "the timed pass's kernels over the 1M resident reads: nw_band_classify<true> + "
                          "nw_band_cert (the three-substitution and one-indel checks on classify's queues) + "
                          "nw_band_segsort + nw_band_fill<16, true> + "
                          "nw_band_walk<16, true> (lane walk + stop summary) + redo compaction + nw_band_fill/walk<32> "
                          "+ nw_band_fill/walk<128> (wide level) + nw_align_kernel + nw_ops_compact, one launch each "
                          "(the kernels call_pcie runs per chunk of >= 65536 reads); call_achieved: the same bytes over "
                          "call_pcie's time",
                "kernel_ms_avg": kms_timed,
                "kernel_ms_with_phase_events": kms,
                "achieved_def": "algorithmic bytes of the pass / its device time in the timed steps (HIP events "
                                "on the aligner's stream around each pass, mean over the K steps; batch resident in "
                                "HBM); call_achieved: the same bytes / call_pcie.ms_per_step (the whole call: PCIe "
                                "both ways, host scan, every kernel)",
                "algo_bytes_per_launch": algo_bytes,
                "algo_bytes_def": "sum over reads of read_len + 3*aln_len + 16 (SURVEY 8d)",
                "valu": {
                    "kernel": "nw_band_fill<16, true> (the first level's traceback fill)",
                    "fill16_ms": fill_ms,
                    "valu_instructions_per_launch": fill_valu,
                    "valu_source": cp["source"] if cp else None,
                    "issue_frac": (fill_valu / (fill_ms * 1e-3) / VALU_ISSUE_PEAK) if fill_valu and fill_ms else None,
                    "issue_peak_per_s": VALU_ISSUE_PEAK,
                    # the rate the fills' packed (VOP3P) instructions reached in a micro-benchmark: a
                    # measured rate, NOT a validated hardware ceiling
                    "ubench_vop3p_rate_per_s": UBENCH_VOP3P_RATE,
                    "ubench_rate_frac": (fill_valu / (fill_ms * 1e-3) / UBENCH_VOP3P_RATE) if fill_valu and fill_ms else None,
                    "ubench_source": "profiles/r04_ubench/ubench_issue_rate.txt: v_pk_* / v_perm / v_and_or / DPP moves at "
                                     "0.228 wave-instructions per SIMD-cycle with 8 independent chains and 8 waves per "
                                     "SIMD; unvalidated as a ceiling (v_add_u32 reached 0.39, not the nominal 0.5)",
                    "band_cells_per_pass": cells,
                    "band_gcups": cells / (kms * 1e-3) / 1e9,
                    "note": "issue_frac = SQ_INSTS_VALU of one fill<16> launch (PMC, chip total) / its live HIP-event "
                            "time / (1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction); band cells = "
                            "cells the bands and the exact kernel actually compute (W x (La + Lb)/2 per read and "
                            "level), not the La x Lb matrices the certificate makes unnecessary",
                },
            },
            "cpu_baseline": cpu,
            "c4" if world > 1 else "c4_shard": multi["c4"],
            "pooled": multi["pooled"],
            "e2e": legs["e2e"],
            "dual_alignment": legs["dual"],
            "c1_shape": legs["c1"],
            "downstream_quantification": quant,
            "upstream_merge": legs["merge"],
        }

        def pick(d, *ks):
            return {k: d.get(k) for k in ks} if isinstance(d, dict) else None
        # the line's last key (a driver record keeps the line's tail): the figures the long keys above hold
        line["summary"] = {
            "value_resident": value, "ms_per_step": ms_step,
            "call_pcie": pick(line["call_pcie"], "value", "ms_per_step"),
            "roofline": pick(line["roofline"], "frac", "achieved", "traffic", "call_frac"),
            "cpu_baseline": pick(cpu, "value", "cores", "kind"),
            "sample_mismatches": (check or {}).get("sample_mismatches") if isinstance(check, dict) else None,
            "resident_same_as_call": (resident_check or {}).get("same_as_call") if isinstance(resident_check, dict) else None,
            "legs_ms_per_step": {k: (line.get(k) or {}).get("ms_per_step") if isinstance(line.get(k), dict) else None
                                 for k in ("c4" if world > 1 else "c4_shard", "pooled", "dual_alignment", "c1_shape",
                                           "downstream_quantification", "upstream_merge")},
        }
        print(json.dumps(line), flush=True)
    for b in (pb, po, p_packed, p_stats, p_off, p_ops):
        b.close()
    al.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
