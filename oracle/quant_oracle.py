"""CPU restatement of CRISPResso's indel/substitution quantification.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / baseline -- never by the product
path (crispresso_amd.quantify runs the HIP kernel and fails without it).

Follows, row by row, ``process_df_chunk`` (``CRISPResso/CRISPRessoCORE.py:428-753``)
together with the state it reads from ``run_crispresso``:

* ``compute_ref_positions``                      CORE:2055-2067
* ``UNMODIFIED`` initialisation (score_ref==100) CORE:2014
* ``ignore_n_in_alignment`` (amplicon with N)    CORE:2031-2046
* ``INCLUDE_IDXS`` / exclude_bp_from_left/right  CORE:2740-2762
* cut points from guides                         CORE:1290-1341
* ``EXON_POSITIONS`` / ``SPLICING_POSITIONS``    CORE:1414-1455

The reference works on numpy index arrays; the restatement works on runs and
reproduces the numpy behaviours the results depend on:

* ``vec[idx] += 1`` with repeated indices adds ONCE per distinct element
  (buffered fancy indexing), and negative indices wrap (``-1`` -> ``LEN-1``).
  Only insertion flanks can be negative: an insertion starting at column 0
  contributes ``ref_positions[0] == -1`` and one ending at the last column
  contributes ``ref_positions[L-1] == -LEN`` (CORE:520-526, 2055-2067).
* ``INCLUDE_IDXS.intersection(...)`` sees the raw (unwrapped) values.
* With ``window_around_sgrna`` set, NHEJ rows filter substitutions and the
  insertion/deletion RUN lists by the window (CORE:611-641), but
  ``insertion_positions_flat`` is never rebuilt and ``deletion_positions_flat``
  only when at least one deletion run survives (CORE:640-641).
* effect_vector_any is taken BEFORE the window filter (CORE:598-607).

Parity: pinned against the reference's own ``process_df_chunk`` run in this
container on recorded DataFrames (tests/golden/quant_*.json.gz,
tests/golden/make_quant_golden.py; and the end-to-end captures of
tests/golden/make_golden.py).
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

BASES = frozenset("ATCGN")

# output vector order (the positions 1..13 and 16..17 of process_df_chunk's tuple)
VECTORS = (
    "effect_vector_insertion", "effect_vector_deletion", "effect_vector_mutation", "effect_vector_any",
    "effect_vector_insertion_mixed", "effect_vector_deletion_mixed", "effect_vector_mutation_mixed",
    "effect_vector_insertion_hdr", "effect_vector_deletion_hdr", "effect_vector_mutation_hdr",
    "effect_vector_insertion_noncoding", "effect_vector_deletion_noncoding", "effect_vector_mutation_noncoding",
    "avg_vector_del_all", "avg_vector_ins_all",
)
COUNTERS = ("modified_frameshift", "modified_non_frameshift", "non_modified_non_frameshift",
            "splicing_sites_modified")


@dataclass
class QuantParams:
    """The run_crispresso globals and args fields process_df_chunk reads."""
    len_amplicon: int
    include_idxs: frozenset                       # INCLUDE_IDXS
    exon_positions: Optional[frozenset] = None    # EXON_POSITIONS (None: no coding_seq)
    splicing_positions: Optional[frozenset] = None
    ignore_substitutions: bool = False
    ignore_insertions: bool = False
    ignore_deletions: bool = False
    window_around_sgrna: int = 1
    hide_mutations_outside_window_NHEJ: bool = False
    expected_hdr: bool = False                    # args.expected_hdr_amplicon_seq truthy
    hdr_perfect_alignment_threshold: float = 98.0


# ------------------------------------------------------------ run_crispresso state

def compute_ref_positions(ref_seq: str) -> List[int]:
    """CORE:2055-2067: base columns get their 0-based amplicon index, gap
    columns get -(bases so far), or -1 before the first base."""
    out, idx = [], 0
    for c in ref_seq:
        if c in BASES:
            out.append(idx)
            idx += 1
        else:
            out.append(-idx if idx else -1)
    return out


def _rc(s: str) -> str:
    return s.upper()[::-1].translate(str.maketrans("ATCGN", "TAGCN"))


def cut_points(amplicon: str, guide_seq: Optional[str], cleavage_offset: int = -3) -> List[int]:
    """CORE:1290-1341 (guides are matched with re.finditer: non-overlapping)."""
    if not guide_seq:
        return []
    pts: List[int] = []
    for g in guide_seq.strip().upper().split(","):
        fw = cleavage_offset + len(g) - 1
        rc = -cleavage_offset - 1
        pts += [m.start() + fw for m in re.finditer(g, amplicon)]
        pts += [m.start() + rc for m in re.finditer(_rc(g), amplicon)]
    return pts


def include_idxs(len_amplicon: int, cuts: Sequence[int], window_around_sgrna: int,
                 exclude_bp_from_left: int, exclude_bp_from_right: int) -> frozenset:
    """CORE:2740-2762."""
    if cuts and window_around_sgrna > 0:
        half = max(1, window_around_sgrna // 2)
        inc = set()
        for c in cuts:
            inc.update(range(max(0, c - half + 1), min(len_amplicon - 1, c + half + 1)))
    else:
        inc = set(range(len_amplicon))
    exc = set()
    if exclude_bp_from_left:
        exc.update(range(exclude_bp_from_left))
    if exclude_bp_from_right:
        exc.update(range(len_amplicon)[-exclude_bp_from_right:])
    return frozenset(inc - exc)


def exon_splicing_positions(amplicon: str, coding_seq: Optional[str]):
    """CORE:1414-1455 -> (EXON_POSITIONS, SPLICING_POSITIONS) or (None, None)."""
    if not coding_seq:
        return None, None
    L = len(amplicon)
    exon, splice = set(), []
    for e in coding_seq.strip().upper().split(","):
        st = amplicon.find(e)
        if st < 0:
            raise ValueError(f"coding subsequence {e} not in the amplicon")
        en = st + len(e)
        exon.update(range(st, en))
        splice += [max(0, st - 2), max(0, st - 1), min(L - 1, en), min(L - 1, en + 1)]
    return frozenset(exon), frozenset(set(splice) - exon)


def ignore_n_in_alignment(ref_seq: str, align_str: str, unmodified: bool):
    """CORE:2038-2046: markup under an amplicon N becomes '|'; a row whose markup
    is then a single repeated character is UNMODIFIED."""
    s = "".join("|" if ref_seq[i] == "N" else c for i, c in enumerate(align_str))
    if len(set(s)) == 1:
        unmodified = True
    return s, unmodified


# ------------------------------------------------------------------- rows

def _runs(s: str, ch: str):
    """Maximal runs of ch in s as (start, end) column spans (re '(-*-)', '(\\.*\\.)')."""
    out, i, n = [], 0, len(s)
    while i < n:
        if s[i] == ch:
            j = i
            while j < n and s[j] == ch:
                j += 1
            out.append((i, j))
            i = j
        else:
            i += 1
    return out


def _wrap(p: int, L: int) -> int:
    return p + L if p < 0 else p


def process_rows(ref_seqs, align_strs, align_seqs, unmodified, score_diff, score_repaired,
                 prm: QuantParams) -> Dict:
    """process_df_chunk over rows; returns per-row outputs and the aggregates.

    unmodified: the incoming UNMODIFIED flags (score_ref == 100, after the N rule).
    score_diff / score_repaired: floats (NaN allowed) or None when no HDR amplicon.
    """
    L = prm.len_amplicon
    n = len(ref_seqs)
    vec = {k: np.zeros(L, dtype=np.int64) for k in VECTORS}
    cnt = {k: 0 for k in COUNTERS}
    hist_inframe: Dict[int, int] = {}
    hist_frameshift: Dict[int, int] = {}
    out_cls = np.zeros(n, dtype=np.int8)      # 0 UNMODIFIED, 1 NHEJ, 2 HDR, 3 MIXED
    out_mut = np.zeros(n, dtype=np.int64)
    out_ins = np.zeros(n, dtype=np.int64)
    out_del = np.zeros(n, dtype=np.int64)
    INC = prm.include_idxs
    frameshift = prm.exon_positions is not None
    EXON = prm.exon_positions or frozenset()
    SPL = prm.splicing_positions or frozenset()

    def bump(name, positions):
        for p in {_wrap(int(q), L) for q in positions}:
            vec[name][p] += 1

    for r in range(n):
        if unmodified[r]:
            continue
        R, M, S = ref_seqs[r], align_strs[r], align_seqs[r]
        rp = compute_ref_positions(R)
        sub = [] if prm.ignore_substitutions else [rp[c] for st, en in _runs(M, ".") for c in range(st, en)]
        dels = [] if prm.ignore_deletions else [([rp[c] for c in range(st, en)], en - st) for st, en in _runs(S, "-")]
        inss = [] if prm.ignore_insertions else \
            [([rp[max(0, st - 1)], rp[min(len(rp) - 1, en)]], en - st) for st, en in _runs(R, "-")]
        del_flat = [p for ps, _ in dels for p in ps]
        ins_flat = [p for ps, _ in inss for p in ps]

        def hits_window(ps):
            return any(p in INC for p in ps)

        cls = 0
        if prm.expected_hdr and score_diff[r] < 0 and score_repaired[r] >= prm.hdr_perfect_alignment_threshold:
            cls = 2
        elif prm.expected_hdr and score_diff[r] < 0 and score_repaired[r] < prm.hdr_perfect_alignment_threshold:
            cls = 3
        elif hits_window(sub) or hits_window(ins_flat) or hits_window(del_flat):
            cls = 1
        out_cls[r] = cls

        tag = {3: "_mixed", 2: "_hdr"}.get(cls)
        if tag is not None:
            bump("effect_vector_mutation" + tag, sub)
            bump("effect_vector_deletion" + tag, del_flat)
            bump("effect_vector_insertion" + tag, ins_flat)
        elif cls == 1 and not prm.hide_mutations_outside_window_NHEJ:
            bump("effect_vector_mutation", sub)
            bump("effect_vector_deletion", del_flat)
            bump("effect_vector_insertion", ins_flat)
        bump("effect_vector_any", del_flat + ins_flat + sub)

        if cls == 1 and prm.window_around_sgrna:
            sub = [p for p in set(sub) if p in INC]
            inss = [x for x in inss if hits_window(x[0])]
            dels = [x for x in dels if hits_window(x[0])]
            if dels:
                del_flat = [p for ps, _ in dels for p in ps]
        if cls == 1 and prm.hide_mutations_outside_window_NHEJ:
            bump("effect_vector_mutation", sub)
            bump("effect_vector_deletion", del_flat)
            bump("effect_vector_insertion", ins_flat)

        if cls == 0:
            continue
        out_mut[r] = len(sub)
        out_ins[r] = sum(s for _, s in inss)
        out_del[r] = sum(s for _, s in dels)
        exon_lens, exon_mod = [], False
        for ps, size in inss:
            for p in {_wrap(q, L) for q in ps}:
                vec["avg_vector_ins_all"][p] += size
            if frameshift and EXON.intersection(ps):
                exon_lens.append(size)
                exon_mod = True
        for ps, size in dels:
            for p in ps:
                vec["avg_vector_del_all"][p] += size
        if not frameshift:
            continue
        d_exon = EXON.intersection(del_flat)
        if d_exon:
            exon_mod = True
            exon_lens.append(-len(d_exon))
        if EXON.intersection(sub):
            exon_mod = True
        if SPL.intersection(sub) or SPL.intersection(del_flat) or SPL.intersection(ins_flat):
            cnt["splicing_sites_modified"] += 1
        if exon_mod:
            if not exon_lens:
                cnt["modified_non_frameshift"] += 1
                hist_inframe[0] = hist_inframe.get(0, 0) + 1
            else:
                eff = sum(exon_lens)
                if eff % 3 == 0:
                    cnt["modified_non_frameshift"] += 1
                    hist_inframe[eff] = hist_inframe.get(eff, 0) + 1
                else:
                    cnt["modified_frameshift"] += 1
                    hist_frameshift[eff] = hist_frameshift.get(eff, 0) + 1
        else:
            cnt["non_modified_non_frameshift"] += 1
            bump("effect_vector_insertion_noncoding", ins_flat)
            bump("effect_vector_deletion_noncoding", del_flat)
            bump("effect_vector_mutation_noncoding", sub)

    return {"cls": out_cls, "n_mutated": out_mut, "n_inserted": out_ins, "n_deleted": out_del,
            "vectors": vec, "counters": cnt, "hist_inframe": hist_inframe, "hist_frameshift": hist_frameshift}


def class_flags(cls: np.ndarray, unmodified_in) -> Dict[str, np.ndarray]:
    """Per-row UNMODIFIED/NHEJ/HDR/MIXED columns as the DataFrame holds them after the chunk."""
    um = np.asarray(unmodified_in, dtype=bool)
    return {"UNMODIFIED": um | (cls == 0), "NHEJ": (cls == 1) & ~um, "HDR": (cls == 2) & ~um,
            "MIXED": (cls == 3) & ~um}


def is_nan(x) -> bool:
    return x is None or (isinstance(x, float) and math.isnan(x))
