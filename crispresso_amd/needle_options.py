"""Parse CRISPResso's ``--needle_options_string`` into aligner parameters.

The reference splices the string verbatim into the ``needle`` command line
(``CRISPRessoCORE.py:1800``; default ``"-gapopen=10 -gapextend=0.5  -awidth3=5000"``,
``CRISPRessoCORE.py:4226-4231``; forwarded by CRISPRessoPooled,
``CRISPRessoPooledCORE.py:514``).  EMBOSS accepts ``-qualifier=value`` and
``-qualifier value``; booleans as ``-endweight``, ``-endweight=Y``, ``-noendweight``.
Options that change the alignment and that the GPU path does not implement
raise :class:`UnsupportedNeedleOption` (the reference would run needle with
them; we refuse loudly rather than silently ignore).  ``-endweight`` with
``-endopen`` / ``-endextend`` is implemented by the exact kernels (DESIGN.md 2.9;
parity vs EMBOSS unpinned: CRISPResso never sets it).
"""
from __future__ import annotations

import shlex
from dataclasses import dataclass

DEFAULT_NEEDLE_OPTIONS = "-gapopen=10 -gapextend=0.5  -awidth3=5000"

# Qualifiers that only affect the report text or I/O (accepted and ignored).
_IGNORED = {"auto", "stdout", "filter", "warning", "error", "fatal", "die", "debug", "verbose",
            "help", "aformat", "aformat3", "brief", "nobrief", "aglobal3", "aaccshow3", "aname3",
            "aextension3", "adirectory3", "sprotein", "snucleotide", "sformat", "sformat1", "sformat2",
            "sask", "supper", "slower", "outfile", "asequence", "bsequence", "datafile2"}


class UnsupportedNeedleOption(ValueError):
    pass


def _bool(v: str) -> bool:
    return v.strip().upper() in ("Y", "YES", "T", "TRUE", "1")


@dataclass
class NeedleOptions:
    gap_open: float = 10.0
    gap_extend: float = 0.5
    end_weight: bool = False
    end_open: float = 10.0
    end_extend: float = 0.5
    matrix: str = "EDNAFULL"
    awidth: int = 5000

    @classmethod
    def parse(cls, text: str) -> "NeedleOptions":
        o = cls()
        toks = shlex.split(text or "")
        i = 0
        while i < len(toks):
            t = toks[i]
            i += 1
            if not t.startswith("-"):
                raise UnsupportedNeedleOption(f"unexpected needle argument {t!r}")
            key, eq, val = t[1:].partition("=")
            key = key.lower()
            negated = False
            if not eq:
                # "-q value" unless the next token is another qualifier (boolean flag)
                if key in ("endweight", "noendweight"):
                    val = "Y"
                elif i < len(toks) and not toks[i].startswith("-"):
                    val = toks[i]
                    i += 1
                else:
                    val = "Y"
            if key.startswith("no") and key[2:] in ("endweight",):
                key, negated = key[2:], True
            if key == "gapopen":
                o.gap_open = float(val)
            elif key == "gapextend":
                o.gap_extend = float(val)
            elif key == "endweight":
                o.end_weight = (not _bool(val)) if negated else _bool(val)
            elif key == "endopen":
                o.end_open = float(val)
            elif key == "endextend":
                o.end_extend = float(val)
            elif key in ("datafile",):
                o.matrix = val
            elif key == "awidth3" or key == "awidth":
                o.awidth = int(val)
            elif key in _IGNORED:
                continue
            else:
                raise UnsupportedNeedleOption(f"needle option -{key} is not supported by the GPU aligner")
        if o.matrix.upper() != "EDNAFULL":
            raise UnsupportedNeedleOption(f"-datafile {o.matrix}: only EDNAFULL is supported")
        if o.end_weight and (o.end_open < 0 or o.end_extend < 0):
            raise UnsupportedNeedleOption("-endopen / -endextend must be non-negative")
        if o.awidth <= 0:
            raise UnsupportedNeedleOption("-awidth3 must be positive")
        return o
