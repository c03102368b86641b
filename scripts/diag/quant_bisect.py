"""Find reads on which the device quantification (lane path, or the forced row path) differs from
the oracle (tests/test_gpu_quant.py::test_device_ops_lane_path_vs_oracle setup): bisects the
read set down to single reads and prints their rows and runs.  Usage: quant_bisect.py La n pad pname"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import math  # noqa: E402

import numpy as np  # noqa: E402

from crispresso_amd import quantify  # noqa: E402
from crispresso_amd.aligner import GpuAligner  # noqa: E402
from crispresso_amd.devmem import DeviceBuffer  # noqa: E402
from oracle import quant_oracle as qo  # noqa: E402
from tests.test_gpu_quant import PARAMS, args_for, globals_for, make_params, odd_reads  # noqa: E402

La, n, pad, pname = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
amp, buf, off = odd_reads(La, n, 90 + La, pad)
prm = make_params(amp, PARAMS[pname])
al = GpuAligner(0)
al.set_reference(amp)
al.set_output("ops")


def run_subset(sel, q):
    b = np.concatenate([buf[off[i]:off[i + 1]] for i in sel]) if len(sel) else np.zeros(1, np.uint8)
    o = np.r_[0, np.cumsum([off[i + 1] - off[i] for i in sel])].astype(np.int64)
    m = len(sel)
    al.upload(b, o)
    al.run_async()
    al.sync()
    dev = al.device_ops()
    ob = al.download_ops(m)
    rows = ob.expand(amp, b, o)
    lens = rows.stats["aln_len"]
    score = np.array([float("%.1f" % (100.0 * x / y)) if y else 0.0 for x, y in zip(rows.stats["n_ident"], lens)])
    um = score == 100
    rng = np.random.Generator(np.random.PCG64(La + 5))
    sr = rng.choice([100.0, 99.0, 97.0, 50.0, math.nan], size=n)[sel]
    sd = score - sr
    pre = quantify.pre_flags(um, sd if prm.expected_hdr else None, sr if prm.expected_hdr else None,
                             prm.hdr_perfect_alignment_threshold)
    R = [rows.aln[i, 0, :lens[i]].tobytes().decode("latin-1") for i in range(m)]
    M = [rows.aln[i, 1, :lens[i]].tobytes().decode("latin-1") for i in range(m)]
    S = [rows.aln[i, 2, :lens[i]].tobytes().decode("latin-1") for i in range(m)]
    ref = qo.process_rows(R, M, S, um, sd if prm.expected_hdr else None, sr if prm.expected_hdr else None, prm)
    q.set_params(globals_for(prm), args_for(prm, prm.exon_positions is not None))
    with DeviceBuffer.from_array(pre) as d_pre, DeviceBuffer(16 * max(m, 1)) as d_out:
        tot = q.unpack_totals(q.run_device_ops(amp, dev, d_pre.ptr, m, d_out.ptr), dev["max_cols"])
        rd = d_out.download(np.zeros((max(m, 1), 4), np.int32))[:m]
    bad = [k for k in qo.VECTORS if not np.array_equal(tot["vectors"][k], ref["vectors"][k])]
    if not np.array_equal(rd[:, 0].astype(np.int8), ref["cls"]):
        bad.append("cls")
    for c, k in ((1, "n_mutated"), (2, "n_inserted"), (3, "n_deleted")):
        if not np.array_equal(rd[:, c], ref[k]):
            bad.append(k)
    if tot["counters"] != ref["counters"]:
        bad.append("counters")
    return bad, (R, M, S, ob, tot, ref, rd)


os.environ["CRISPR_NWQ_ROWS"] = "1"
q_rows = quantify.GpuQuantifier(0)
os.environ.pop("CRISPR_NWQ_ROWS")
q_lanes = quantify.GpuQuantifier(0)
for name, q in (("lanes", q_lanes), ("rows", q_rows)):
    sel = list(range(n))
    bad, _ = run_subset(sel, q)
    print(name, "all reads:", bad or "ok", flush=True)
    if not bad:
        continue
    while len(sel) > 1:
        h = len(sel) // 2
        b1, _ = run_subset(sel[:h], q)
        if b1:
            sel = sel[:h]
            continue
        b2, _ = run_subset(sel[h:], q)
        if b2:
            sel = sel[h:]
            continue
        print(name, "no single half fails (interaction); stopping at", len(sel), "reads")
        break
    bad, (R, M, S, ob, tot, ref, rd) = run_subset(sel, q)
    print(name, "minimal set", sel, "bad", bad)
    for j, i in enumerate(sel[:4]):
        print(" read", i, bytes(buf[off[i]:off[i + 1]]).decode("latin-1"))
        print("  R", R[j]); print("  M", M[j]); print("  S", S[j])
        print("  runs", [(int(x) >> 28, int(x) & 0xfffffff) for x in ob.ops[ob.ops_off[j]:ob.ops_off[j + 1]]],
              "stats", ob.stats[j])
        print("  gpu", rd[j], "oracle cls", ref["cls"][j], ref["n_mutated"][j], ref["n_inserted"][j], ref["n_deleted"][j])
    for k in qo.VECTORS:
        g, r = tot["vectors"][k], ref["vectors"][k]
        if not np.array_equal(g, r):
            d = np.flatnonzero(g != r)
            print("  ", k, "positions", d[:10].tolist(), "gpu", g[d[:10]].tolist(), "oracle", r[d[:10]].tolist())
al.close()
