/*
 * nw_oracle.h -- CPU restatement of EMBOSS `needle` 6.6.0 as CRISPResso calls it.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this.  The product path (crispresso_amd/) never links
 * or calls it; there is no CPU fallback in the product.
 *
 * PARITY STATUS: "parity unpinned" against EMBOSS itself.  EMBOSS (the module
 * that owns the arithmetic, pinned at emboss=6.6.0 in reference
 * environment.yml:19) is not vendored in /root/reference and is not installed in
 * this image, and the reference's tests hold no alignment-level fixtures
 * (SURVEY.md 8c).  What this file restates is the published EMBOSS needle
 * algorithm (embAlignPathCalcWithEndGapPenalties + embAlignWalkNWMatrixUsingCompass
 * + embAlignReportGlobal, endweight off) with every unverifiable choice made
 * explicit in DESIGN.md "EMBOSS semantics".  The DP optimum itself is pinned
 * independently (brute-force enumeration, tests/test_oracle.py).
 *
 * Reference call sites this replaces (CRISPResso/CRISPRessoCORE.py):
 *   forward pass   1791-1806, HDR pass 1812-1828, RC passes 1910-1936
 *   output format consumed by parse_needle_output 1707-1786
 *   needle options default  "-gapopen=10 -gapextend=0.5 -awidth3=5000" 4226-4231
 */
#ifndef CRISPR_NW_ORACLE_H
#define CRISPR_NW_ORACLE_H

#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Scores are integers: every EMBOSS float is multiplied by `scale` (a power of
 * two chosen so the penalties are exact).  gapopen=10, gapextend=0.5 -> scale 2,
 * open 20, extend 1, EDNAFULL match 10 / mismatch -8. */
typedef struct {
    int32_t scale;
    int32_t gap_open;    /* scaled */
    int32_t gap_extend;  /* scaled */
    float gap_open_f;    /* as given, for the report header */
    float gap_extend_f;
    /* needle -endweight / -endopen / -endextend (EMBOSS defaults N / 10.0 / 0.5):
     * with end_weight, an end gap of k residues costs end_open + (k-1) * end_extend
     * (scaled) instead of nothing.  PARITY UNPINNED: CRISPResso never sets these, the
     * reference holds no output made with them, and EMBOSS is absent. */
    int32_t end_weight;
    int32_t end_open;    /* scaled */
    int32_t end_extend;  /* scaled */
} oracle_params;

typedef struct {
    int32_t aln_len;
    int32_t n_ident;
    int32_t n_sim;
    int32_t n_gaps;
    int32_t score;       /* scaled */
    int32_t end_i;       /* 1-based row (amplicon) of the last aligned pair */
    int32_t end_j;       /* 1-based column (read) of the last aligned pair */
    int32_t read_end;    /* last read coordinate printed on the srspair line */
    int32_t ref_end;     /* last amplicon coordinate printed */
} oracle_result;

/* EDNAFULL code of an ASCII residue (case-insensitive); 16 = not in the matrix. */
int oracle_code(unsigned char c);
/* Unscaled EDNAFULL score of two codes (0 when either is 16). */
int oracle_sub(int ca, int cb);

/* Derive scale/open/extend from EMBOSS float penalties. 0 ok, -1 inexact. */
int oracle_params_init(oracle_params* p, float gap_open, float gap_extend);
/* The same with -endweight / -endopen / -endextend (one scale for all four). */
int oracle_params_init_end(oracle_params* p, float gap_open, float gap_extend, int end_weight, float end_open,
                           float end_extend);

/* Align read b (columns) against amplicon a (rows).  The three output buffers
 * must hold la+lb+1 bytes; they are NUL-terminated.  Returns 0, or -1 when
 * la==0 or lb==0 or on allocation failure. */
int oracle_align(const char* a, int32_t la, const char* b, int32_t lb,
                 const oracle_params* p, oracle_result* out,
                 char* ref_aln, char* markup, char* read_aln);

/* Score-only DP (same recurrence, no traceback); used by the brute-force test. */
int32_t oracle_score(const char* a, int32_t la, const char* b, int32_t lb,
                     const oracle_params* p);

/* Batch over n reads with `nthreads` POSIX threads (CPU baseline).  Outputs are
 * written at fixed stride `stride` per read (>= la + max lb + 1). */
int oracle_align_batch(const char* a, int32_t la, const char* reads,
                       const int64_t* offsets, int32_t n, const oracle_params* p,
                       int nthreads, oracle_result* res, char* ref_aln,
                       char* markup, char* read_aln, int64_t stride);

/* srspair text of one pair (the block parse_needle_output reads,
 * CRISPRessoCORE.py:1715-1765).  Returns bytes written (excluding NUL) or the
 * size needed when buf is too small (nothing written then). */
int64_t oracle_format_srspair(char* buf, int64_t cap, const char* aname,
                              const char* bname, const oracle_params* p,
                              const oracle_result* r, const char* ref_aln,
                              const char* markup, const char* read_aln);

#ifdef __cplusplus
}
#endif
#endif
