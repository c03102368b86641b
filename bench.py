#!/usr/bin/env python3
"""Benchmark: aligned reads/sec, 250 bp amplicon x 1M synthetic reads per GPU.

BASELINE.json metric: "aligned reads/sec (250 bp amplicon x 1M reads) at
1/2/4/8 MI355X".  One step = one pass of the GPU aligner (the kernel that
replaces EMBOSS needle, CRISPRessoCORE.py:1791-1806) over the rank's batch of
1M reads that is already resident in HBM; outputs (three alignment strings
and per-read statistics) are written to HBM.

N GPUs: one process per GPU (torch.distributed.run), each aligning its own 1M
read shard (reads are independent, no collective on the data
path; the only collectives are the timing barrier and the max-over-ranks).
value = N * 1M * K / max-over-ranks time of K steps  ("scaling": "weak").

Extra keys: "roofline" (HBM, algorithmic bytes per launch / kernel time from
HIP events on the aligner's stream) with a VALU-side GCUPS figure, and
"cpu_baseline" (the CPU oracle -- a port, not EMBOSS, which is absent -- on a
bounded sample, rank 0 at N=1 only); informational legs either side of the
path: "downstream_quantification" (process_df_chunk on the aligned batch) and,
at N=1, "upstream_merge" (the paired-end merge, FLASH semantics, 1M 2 x 150 bp
pairs; --no-merge skips it).
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
VALU_PEAK_TOPS = 78.6          # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz int32 lane-ops/s (x1e12)
READS_PER_GPU = 1_000_000
# rocprofv3 --pmc summary of this build's kernels on this workload (scripts/gpu_pmc.sh + pmc_summary.py:
# 2 x FETCH_SIZE + WRITE_SIZE per launch, the guide's gfx950 correction); source of roofline.traffic
# (newest first: the aligner kernels' latest summary, then the one that also holds the quantification kernels)
PMC_SUMMARIES = [os.path.join(ROOT, "profiles", "r01_v24", "pmc_summary.json"),
                 os.path.join(ROOT, "profiles", "r01_v23", "pmc_summary.json"),
                 os.path.join(ROOT, "profiles", "r01_v22", "pmc_summary.json"),
                 os.path.join(ROOT, "profiles", "r01_v21", "pmc_summary.json"),
                 os.path.join(ROOT, "profiles", "r01_v19", "pmc_summary.json"),
                 os.path.join(ROOT, "profiles", "r01_diag_pmc", "pmc_summary.json"),
                 os.path.join(ROOT, "profiles", "r01_bias_pmc", "pmc_summary.json"),
                 os.path.join(ROOT, "profiles", "r01_quant", "pmc_summary.json")]
AMPLICON_LEN = 250


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 0, 1, None
    import torch
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl")
    return rank, local, world, dist


def barrier(dist, local):
    if dist is None:
        return
    import torch

    dist.barrier(device_ids=[local])
    torch.cuda.synchronize()


def max_over_ranks(dist, local, value):
    if dist is None:
        return value
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_traffic(*prefixes, required=None):
    """(HBM bytes per launch of the kernels whose names start with `prefixes`, source file), from the
    first summary in PMC_SUMMARIES that holds them (and a kernel starting with `required`)."""
    for path in PMC_SUMMARIES:
        try:
            with open(path) as f:
                summ = json.load(f)
        except (OSError, ValueError):
            continue
        if required and not any(required in k for k in summ):
            continue
        vals = [v["hbm_bytes_per_launch"] for k, v in summ.items()
                if any(k.startswith(p) for p in prefixes) and "hbm_bytes_per_launch" in v]
        if vals:
            return float(sum(vals)), os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(amplicon, buf, offsets, n_sample, threads):
    from oracle import oracle_py

    sub = offsets[: n_sample + 1]
    t0 = time.perf_counter()
    oracle_py.align_batch(amplicon, buf, sub, nthreads=threads)
    dt = time.perf_counter() - t0
    return {
        "value": n_sample / dt,
        "unit": "aligned reads/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {n_sample} reads of the same synthetic C2 batch, CPU oracle (oracle/nw_oracle.c, "
                  f"scalar Gotoh + traceback per read) on {threads} host threads, {dt:.2f} s wall; "
                  "EMBOSS needle itself is not installed on the box",
    }


def quant_leg(al, amplicon, n_reads, steps, warmup, dist, local, rank, world, cpu_sample, no_cpu):
    """Downstream quantification (process_df_chunk, CORE:428-753) of this rank's
    aligned reads, straight from the aligner's HBM output (nwq_run_device).
    Settings: one guide cutting mid-amplicon, CRISPResso defaults otherwise
    (window_around_sgrna 1, exclude 15 bp each side)."""
    from crispresso_amd import quantify
    from crispresso_amd.devmem import DeviceBuffer

    d_aln, stride, d_stats = al.device_output()
    batch = al.download(n_reads, AMPLICON_LEN + 64)
    lens = batch.stats["aln_len"].astype(np.int64)
    ident = batch.stats["n_ident"].astype(np.int64)
    um = ident == lens
    args = argparse.Namespace(amplicon_seq=amplicon, guide_seq=amplicon[105:125], cleavage_offset=-3,
                              window_around_sgrna=1, exclude_bp_from_left=15, exclude_bp_from_right=15,
                              coding_seq=None, expected_hdr_amplicon_seq=None)
    g = quantify.globals_from_args(args)
    q = quantify.GpuQuantifier(local)
    q.set_params(g, args)
    pre = quantify.pre_flags(um)
    d_pre = DeviceBuffer.from_array(pre, local)
    d_out = DeviceBuffer(16 * n_reads, local)
    for _ in range(warmup):
        q.run_device(d_aln, stride, d_stats, 8, d_pre.ptr, n_reads, d_out.ptr)
    barrier(dist, local)
    kms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        q.run_device(d_aln, stride, d_stats, 8, d_pre.ptr, n_reads, d_out.ptr)
        kms.append(q.last_kernel_ms)
    barrier(dist, local)
    elapsed = max_over_ranks(dist, local, time.perf_counter() - t0)
    algo = int(n_reads * (1 + 4 + 16) + 3 * lens[~um].sum())
    kavg = float(np.mean(kms))
    q_traffic, q_src = pmc_traffic("nwq::quant_kernel", "nwq::quant_reduce")
    out = {
        "metric": "quantified reads/s (process_df_chunk on the aligned C2 batch, device-resident)",
        "value": n_reads * world * steps / elapsed,
        "unit": "reads/s",
        "ms_per_step": elapsed / steps * 1e3,
        "kernel": "nwq::quant_kernel + nwq::quant_reduce",
        "kernel_ms_avg": kavg,
        "roofline": {"bound": "hbm", "achieved": algo / (kavg * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": algo / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": q_traffic,
                     "traffic_source": q_src,
                     "algo_bytes_per_launch": algo,
                     "algo_bytes_def": "per read 1 (flags) + 4 (aln_len) + 16 (result); + 3*aln_len for rows not "
                                       "UNMODIFIED on input (the three alignment rows)"},
        "settings": "guide mid-amplicon, window_around_sgrna 1, exclude 15/15",
    }
    if rank == 0 and world == 1 and not no_cpu:
        from oracle import quant_oracle as qo

        k = min(cpu_sample, n_reads)
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=READS_PER_GPU)
    ap.add_argument("--cpu-sample", type=int, default=300_000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-quant", action="store_true", help="skip the downstream quantification leg")
    ap.add_argument("--quant-cpu-sample", type=int, default=20_000)
    ap.add_argument("--no-merge", action="store_true", help="skip the paired-end merge leg (N = 1 only)")
    ap.add_argument("--merge-pairs", type=int, default=1_000_000)
    args = ap.parse_args()

    rank, local, world, dist = dist_setup(args.gpus)
    from crispresso_amd import synth
    from crispresso_amd.aligner import GpuAligner

    amplicon = synth.random_amplicon(AMPLICON_LEN, 1)
    seed = 2 if world == 1 else 10 + rank
    t0 = time.perf_counter()
    buf, offsets = synth.reads_from(amplicon, args.reads, seed)
    log(f"[rank {rank}] generated {args.reads} reads in {time.perf_counter() - t0:.1f}s")

    al = GpuAligner(local)
    al.set_reference(amplicon)
    al.upload(buf, offsets)
    for _ in range(args.warmup):
        al.run_async()
        al.sync()

    barrier(dist, local)
    kernel_ms = []
    split = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        al.run_async()
        kernel_ms.append(al.sync())
        split.append(al.kernel_times())
    barrier(dist, local)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(dist, local, elapsed)

    algo_bytes = al.algo_bytes()       # per launch, from this batch's own results
    cells = al.cells()
    geo = al.geometry()
    geo["fallback_reads"] = al.fallbacks()
    avg_ms = float(np.mean(kernel_ms))
    split_ms = {k: float(np.mean([d[k] for d in split])) for k in split[0]} if split else {}
    achieved_gbs = algo_bytes / (avg_ms * 1e-3) / 1e9
    gcups = cells / (avg_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(amplicon, buf, offsets, min(args.cpu_sample, args.reads), args.cpu_threads)

    quant = None
    if not args.no_quant:
        quant = quant_leg(al, amplicon, args.reads, args.steps, args.warmup, dist, local, rank, world,
                          args.quant_cpu_sample, args.no_cpu)

    merge = None
    if rank == 0 and world == 1 and not args.no_merge:
        try:
            merge = merge_leg(local, args.merge_pairs)
        except Exception as exc:   # informational leg: never costs the bench line
            merge = {"error": f"{type(exc).__name__}: {exc}"}

    diag = geo["tb_mode"].startswith("diag")
    if diag:
        traffic, traffic_src = pmc_traffic("void nw::nw_band_", "nw::nw_band_", "void nw::nw_align_kernel",
                                           required="nw::nw_band_fill<16>")
    elif geo["tb_mode"].startswith("stream"):
        traffic, traffic_src = pmc_traffic("void nw::nw_stream_fill", "void nw::nw_stream_walk", "void nw::nw_align_kernel",
                                           required="void nw::nw_stream_fill")
    else:
        traffic, traffic_src = None, None
    total_reads = args.reads * world * args.steps
    value = total_reads / elapsed
    if rank == 0:
        line = {
            "metric": "aligned reads/sec (250 bp amplicon x 1M reads) at 1/2/4/8 MI355X",
            "value": value,
            "unit": "aligned reads/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16x2" if geo["tb_mode"].startswith(("pair", "stream", "diag")) else "int32",
            "data": "synthetic (SURVEY 8d C2 mix: 60% exact, 20% 1-3 subs, 10% del, 5% ins, 5% 1% noise)",
            "config": {
                "workload": f"C2: {args.reads} synthetic ~250 bp reads x 250 bp amplicon per GPU, "
                            "EMBOSS needle semantics (EDNAFULL, gapopen 10, gapextend 0.5, free end gaps)",
                "reads_per_gpu": args.reads,
                "amplicon_len": AMPLICON_LEN,
                "parallelism": f"read shards x{world} (no collective on the data path)",
                "kernel_geometry": geo,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": f"{traffic_src} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the same bench "
                                  "command, per launch of fill + walk + fallback)",
                "kernel": ("nw_band_classify (exact copies, no DP) + length sort + nw_band_fill<16> + "
                           "nw_band_walk<16> (certified 16-diagonal band) + nw_band_fill/walk<32> on its redo list "
                           "+ nw_align_kernel on what neither band certifies" if diag
                           else f"nw_stream_fill<{geo['rows_per_lane']}> + nw_stream_walk<{geo['rows_per_lane']}>"
                           if geo["tb_mode"].startswith("stream")
                           else f"nw_align_kernel<{geo['rows_per_lane']},{geo['tb_mode']}>"),
                "kernel_ms_avg": avg_ms,
                "kernel_ms_split": split_ms,
                "achieved_def": "algorithmic bytes / device time of the whole batch (fill + walk + fallback "
                                "kernels, HIP events on the aligner's stream)",
                "algo_bytes_per_launch": algo_bytes,
                "algo_bytes_def": "sum over reads of read_len + 3*aln_len + 16 (SURVEY 8d)",
                "valu": {
                    "gcups": gcups,
                    "cells_per_launch": cells,
                    "note": ("gcups counts the full La x Lb matrix of every read (the work the reference's needle "
                             "does); the certified bands compute 16 (or 32) diagonals per read, exact copies none, and "
                             "prove the rest cannot "
                             "change the result (DESIGN.md §4)" if diag else
                             "the DP is a dependent integer recurrence: VALU-bound, HBM frac is small by construction"),
                },
            },
            "cpu_baseline": cpu,
            "downstream_quantification": quant,
            "upstream_merge": merge,
        }
        print(json.dumps(line), flush=True)
    al.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
