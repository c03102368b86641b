#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh) per kernel.

Per kernel: mean counter value per dispatch.  HBM traffic per launch follows
MI355X_MICROARCH.md's rocprofv3 notes: FETCH_SIZE / WRITE_SIZE are kilobytes
from the L2's fabric-side request counters; on gfx950 FETCH_SIZE reports half
the bytes of wide streaming reads, so it is doubled here (an upper estimate for
narrower reads).  Usage: pmc_summary.py <pmc dir> <out.json> [calls: the timed program made this many pipelined calls]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def lib_hash(root_dir):
    """sha1 of the library the passes ran (crispresso_amd/lib/libcrispr_nw.so): bench.py compares it
    with the library it loads and flags a summary of another build."""
    import hashlib

    p = os.path.join(root_dir, "crispresso_amd", "lib", "libcrispr_nw.so")
    try:
        with open(p, "rb") as f:
            return hashlib.sha1(f.read()).hexdigest()
    except OSError:
        return None


def main(root, out, calls=None):
    vals = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if "rocclr" in name:
                    continue
                vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    summary = {}
    for k, cs in vals.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = float(max(len(v) for v in cs.values()))
        if "FETCH_SIZE" in d or "WRITE_SIZE" in d:
            fetch = 2.0 * d.get("FETCH_SIZE", 0.0) * 1024
            write = d.get("WRITE_SIZE", 0.0) * 1024
            d["hbm_bytes_per_launch"] = fetch + write
            d["hbm_note"] = "2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes; gfx950 FETCH_SIZE halving corrected)"
            if calls:   # a pipelined call launches each kernel once per chunk: bytes per call
                tot = 2.0 * sum(cs.get("FETCH_SIZE", [0.0])) * 1024 + sum(cs.get("WRITE_SIZE", [0.0])) * 1024
                d["hbm_bytes_per_call"] = tot / calls
        if calls and "SQ_INSTS_VALU" in cs:
            d["valu_per_call"] = sum(cs["SQ_INSTS_VALU"]) / calls
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
            d["valu_per_wave"] = d["SQ_INSTS_VALU"] / max(d["SQ_WAVES"], 1)
        summary[k] = d
    summary["_meta"] = {"lib_sha1": lib_hash(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                        "calls": calls}
    with open(out, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    for k, d in summary.items():
        print(k[:60], {c: round(v, 1) for c, v in d.items() if isinstance(v, float)})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
