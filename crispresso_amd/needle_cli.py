"""`needle`-compatible command line over the GPU aligner (drop-in at the process boundary).

CRISPResso runs (CRISPRessoCORE.py:1797-1801)::

    ... | needle -asequence=AMPL.fa -bsequence=/dev/stdin -outfile=/dev/stdout \\
            -gapopen=10 -gapextend=0.5 -awidth3=5000 2>> LOG | gzip > needle_output.txt.gz

Putting ``crispresso_amd/bin`` first on PATH makes that pipeline use this
program: same qualifiers, FASTA in, srspair out.  Options are parsed by
:mod:`crispresso_amd.needle_options`; unsupported ones exit non-zero with a
message on stderr (as EMBOSS does for bad qualifiers).
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional, Tuple

import numpy as np

from . import fastq
from .needle_options import NeedleOptions, UnsupportedNeedleOption

BATCH = 1 << 20


def split_args(argv: List[str]) -> Tuple[Optional[str], Optional[str], str, str]:
    """-> (asequence, bsequence, outfile, the remaining options as one string)."""
    a = b = None
    out = "stdout"
    rest: List[str] = []
    i = 0
    while i < len(argv):
        t = argv[i]
        i += 1
        key, eq, val = t.lstrip("-").partition("=")
        if t.startswith("-") and key.lower() in ("asequence", "bsequence", "outfile"):
            if not eq:
                if i >= len(argv):
                    raise UnsupportedNeedleOption(f"-{key} needs a value")
                val = argv[i]
                i += 1
            if key.lower() == "asequence":
                a = val
            elif key.lower() == "bsequence":
                b = val
            else:
                out = val
        else:
            rest.append(t)
    return a, b, out, " ".join(rest)


def read_fasta(path: str):
    if path in ("/dev/stdin", "stdin", "-"):
        text = sys.stdin.buffer.read().decode("ascii", "replace")
    else:
        with open(path, "rb") as f:
            data = f.read()
        if data[:2] == b"\x1f\x8b":
            import gzip

            data = gzip.decompress(data)
        text = data.decode("ascii", "replace")
    return fastq.parse_fasta_text(text)


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    try:
        a_path, b_path, out_path, rest = split_args(argv)
        opts = NeedleOptions.parse(rest)
        if not a_path or not b_path:
            raise UnsupportedNeedleOption("-asequence and -bsequence are required")
    except (UnsupportedNeedleOption, ValueError) as exc:
        print(f"Error: {exc}", file=sys.stderr)
        return 1
    from .aligner import GpuAligner, format_srspair
    from .needle import SRSPAIR_HEADER, SRSPAIR_TRAILER

    anames, abuf, aoff = read_fasta(a_path)
    if not anames or aoff[1] == 0:
        print("Error: empty -asequence", file=sys.stderr)
        return 1
    amplicon = abuf[aoff[0]:aoff[1]].tobytes().decode()
    names, buf, off = read_fasta(b_path)
    device = int(os.environ.get("CRISPR_NW_DEVICE", "0"))
    out = sys.stdout if out_path in ("stdout", "/dev/stdout") else open(out_path, "w")
    try:
        with GpuAligner(device, opts) as al:
            al.set_reference(amplicon)
            out.write(SRSPAIR_HEADER.format(a=a_path))
            for lo in range(0, len(names), BATCH):
                hi = min(len(names), lo + BATCH)
                sub = off[lo:hi + 1]
                batch = al.align_packed(buf[sub[0]:sub[-1]], sub - sub[0])
                out.write(format_srspair(batch, anames[0], names[lo:hi], opts))
            out.write(SRSPAIR_TRAILER)
    finally:
        if out is not sys.stdout:
            out.close()
        else:
            out.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
