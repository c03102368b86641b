#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh) per kernel.

Per kernel: mean counter value per dispatch.  HBM traffic per launch follows
MI355X_MICROARCH.md's rocprofv3 notes: FETCH_SIZE / WRITE_SIZE are kilobytes
from the L2's fabric-side request counters; on gfx950 FETCH_SIZE reports half
the bytes of wide streaming reads, so it is doubled here (an upper estimate for
narrower reads).  Usage: pmc_summary.py <pmc dir> <out.json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root, out):
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
        if "FETCH_SIZE" in d or "WRITE_SIZE" in d:
            fetch = 2.0 * d.get("FETCH_SIZE", 0.0) * 1024
            write = d.get("WRITE_SIZE", 0.0) * 1024
            d["hbm_bytes_per_launch"] = fetch + write
            d["hbm_note"] = "2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes; gfx950 FETCH_SIZE halving corrected)"
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
            d["valu_per_wave"] = d["SQ_INSTS_VALU"] / max(d["SQ_WAVES"], 1)
        summary[k] = d
    with open(out, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    for k, d in summary.items():
        print(k[:60], {c: round(v, 1) for c, v in d.items() if isinstance(v, float)})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
