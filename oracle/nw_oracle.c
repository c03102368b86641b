/*
 * nw_oracle.c -- scalar CPU restatement of EMBOSS needle 6.6.0 (endweight off).
 *
 * TEST INFRASTRUCTURE ONLY (see nw_oracle.h).  Parity vs EMBOSS: pinned end to end
 * by the reference's own e2e test values (see the tie rules below); no EMBOSS binary
 * or source exists offline, so per-alignment golden files are not available.
 *
 * Model (DESIGN.md "EMBOSS semantics"):
 *  - a = amplicon = rows (needle -asequence, CRISPRessoCORE.py:1798),
 *    b = read = columns (-bsequence=/dev/stdin, CRISPRessoCORE.py:1799).
 *  - Gotoh affine DP with three states, as EMBOSS embAlignPathCalcWithEndGapPenalties:
 *      M[i][j] = best(M,X,Y)[i-1][j-1] + s(a_i, b_j)
 *      X[i][j] = max(M[i][j-1] - open, X[i][j-1] - extend)   (gap in a, consumes b_j)
 *      Y[i][j] = max(M[i-1][j] - open, Y[i-1][j] - extend)   (gap in b, consumes a_i)
 *    The values need no tie rule; the traceback's choices do:
 *    predecessor of an M cell: M if M >= X and M >= Y (ties stay on the diagonal),
 *    else X if X >= Y (X wins an X == Y tie), else Y; a gap run ends (was opened)
 *    only when open > extend (ties extend the gap).  These rules are PINNED against
 *    real EMBOSS through the reference's own end-to-end assertions
 *    (tests/golden/make_e2e_golden.py): on tests/crispresso_tests.py:181-195 the
 *    previous choice (strict M, open on ties) misses 10 of the 14 asserted values,
 *    this one reproduces all 14; on the indel-rich second run
 *    (tests/crispresso_tests.py:198-272, --case test1) "Y wins an X == Y tie" misses
 *    the insertion and indel-size histograms, "X wins" matches them (DESIGN.md
 *    2.5).  The start-cell scan order is not exercised by either data set.
 *  - Free end gaps (needle -endweight defaults to false; CRISPResso never sets it):
 *    row 0 / column 0 hold M = 0, X = Y = -inf.  This reproduces EMBOSS's first
 *    row/column initialisation (m = match, ix/iy = -gapopen).
 *  - -endweight (PARITY UNPINNED): an end gap of k residues costs
 *    endopen + (k-1) * endextend.  Leading: row 0 / column 0 hold M = -(endopen +
 *    (k-1) * endextend) for the k residues before the cell (M[0][0] = 0); trailing:
 *    the start-cell scan compares M of a last-column cell minus the penalty of the
 *    la - i amplicon residues after it (last row: lb - j read residues), and that
 *    penalised value is the reported score.
 *  - The walk starts at the best M cell of the last row or last column
 *    (scan: corner, then last column bottom->top, then last row right->left,
 *    strict >); the unmatched tail is emitted as end gaps first, the unmatched
 *    head after the walk, as embAlignWalkNWMatrixUsingCompass does.
 *  - Report (embAlignReportGlobal -> srspair): Length counts every column
 *    including end gaps; Identity = identical pairs (case-insensitive);
 *    Similarity = identical or positive-scoring pairs; Gaps = gap columns;
 *    Score = DP value of the start cell.  Markup '|' identical, ':' similar,
 *    '.' other pair, ' ' gap.
 */
#include "nw_oracle.h"

#include <ctype.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* EDNAFULL (NCBI NUC.4.4), order A T G C S W R Y K M B V H D N U. */
static const signed char kEdnaFull[16][16] = {
    /*        A   T   G   C   S   W   R   Y   K   M   B   V   H   D   N   U */
    /* A */ { 5, -4, -4, -4, -4,  1,  1, -4, -4,  1, -4, -1, -1, -1, -2, -4},
    /* T */ {-4,  5, -4, -4, -4,  1, -4,  1,  1, -4, -1, -4, -1, -1, -2,  5},
    /* G */ {-4, -4,  5, -4,  1, -4,  1, -4,  1, -4, -1, -1, -4, -1, -2, -4},
    /* C */ {-4, -4, -4,  5,  1, -4, -4,  1, -4,  1, -1, -1, -1, -4, -2, -4},
    /* S */ {-4, -4,  1,  1, -1, -4, -2, -2, -2, -2, -1, -1, -3, -3, -1, -4},
    /* W */ { 1,  1, -4, -4, -4, -1, -2, -2, -2, -2, -3, -3, -1, -1, -1,  1},
    /* R */ { 1, -4,  1, -4, -2, -2, -1, -4, -2, -2, -3, -1, -3, -1, -1, -4},
    /* Y */ {-4,  1, -4,  1, -2, -2, -4, -1, -2, -2, -1, -3, -1, -3, -1,  1},
    /* K */ {-4,  1,  1, -4, -2, -2, -2, -2, -1, -4, -1, -3, -3, -1, -1,  1},
    /* M */ { 1, -4, -4,  1, -2, -2, -2, -2, -4, -1, -3, -1, -1, -3, -1, -4},
    /* B */ {-4, -1, -1, -1, -1, -3, -3, -1, -1, -3, -1, -2, -2, -2, -1, -1},
    /* V */ {-1, -4, -1, -1, -1, -3, -1, -3, -3, -1, -2, -1, -2, -2, -1, -4},
    /* H */ {-1, -1, -4, -1, -3, -1, -3, -1, -3, -1, -2, -2, -1, -2, -1, -1},
    /* D */ {-1, -1, -1, -4, -3, -1, -1, -3, -1, -3, -2, -2, -2, -1, -1, -1},
    /* N */ {-2, -2, -2, -2, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -2},
    /* U */ {-4,  5, -4, -4, -4,  1, -4,  1,  1, -4, -1, -4, -1, -1, -2,  5},
};

int oracle_code(unsigned char c) {
    switch (toupper(c)) {
        case 'A': return 0;  case 'T': return 1;  case 'G': return 2;
        case 'C': return 3;  case 'S': return 4;  case 'W': return 5;
        case 'R': return 6;  case 'Y': return 7;  case 'K': return 8;
        case 'M': return 9;  case 'B': return 10; case 'V': return 11;
        case 'H': return 12; case 'D': return 13; case 'N': return 14;
        case 'U': return 15;
        default: return 16;
    }
}

int oracle_sub(int ca, int cb) {
    if (ca > 15 || cb > 15) return 0;
    return kEdnaFull[ca][cb];
}

int oracle_params_init_end(oracle_params* p, float gap_open, float gap_extend, int end_weight, float end_open,
                           float end_extend) {
    for (int scale = 1; scale <= 64; scale *= 2) {
        double o = (double)gap_open * scale, e = (double)gap_extend * scale;
        double eo = end_weight ? (double)end_open * scale : 0.0, ee = end_weight ? (double)end_extend * scale : 0.0;
        if (o == floor(o) && e == floor(e) && eo == floor(eo) && ee == floor(ee)) {
            p->scale = scale;
            p->gap_open = (int32_t)o;
            p->gap_extend = (int32_t)e;
            p->gap_open_f = gap_open;
            p->gap_extend_f = gap_extend;
            p->end_weight = end_weight != 0;
            p->end_open = (int32_t)eo;
            p->end_extend = (int32_t)ee;
            return 0;
        }
    }
    return -1;
}

int oracle_params_init(oracle_params* p, float gap_open, float gap_extend) {
    return oracle_params_init_end(p, gap_open, gap_extend, 0, 10.0f, 0.5f);
}

/* Penalty of an end gap of k residues (0 without -endweight). */
static inline int32_t end_gap(const oracle_params* p, int32_t k) {
    return (p->end_weight && k > 0) ? p->end_open + (k - 1) * p->end_extend : 0;
}

#define NEG_INF (-(1 << 28))

enum { ST_M = 0, ST_X = 1, ST_Y = 2 };

/* Tie-rule probes (test infrastructure only: tests/golden/make_e2e_golden.py bisects the unpinned rules
 * against the reference's e2e assertions with ORACLE_TIE_VARIANT; unset = the pinned rules above):
 * "xy_y" Y wins an X == Y tie (the rule before test1 pinned it), "m_strict" M must beat X and Y, "gap_open" a gap opens on an open ==
 * extend tie, "start_row" the start-cell scan takes the last row before the last column, "start_ge"
 * a later equal start-cell candidate replaces an earlier one. */
static int g_variant = -1;
enum { V_XY_Y = 1, V_M_STRICT = 2, V_GAP_OPEN = 4, V_START_ROW = 8, V_START_GE = 16 };
static int variant(void) {
    if (g_variant < 0) {
        const char* v = getenv("ORACLE_TIE_VARIANT");
        int f = 0;
        if (v) {
            if (strstr(v, "xy_y")) f |= V_XY_Y;
            if (strstr(v, "m_strict")) f |= V_M_STRICT;
            if (strstr(v, "gap_open")) f |= V_GAP_OPEN;
            if (strstr(v, "start_row")) f |= V_START_ROW;
            if (strstr(v, "start_ge")) f |= V_START_GE;
        }
        g_variant = f;
    }
    return g_variant;
}

static inline int best_state(int m, int x, int y) {
    const int v = variant();
    if (v & V_M_STRICT) { if (m > x && m > y) return ST_M; }
    else if (m >= x && m >= y) return ST_M;
    if (v & V_XY_Y) return x > y ? ST_X : ST_Y;
    return x >= y ? ST_X : ST_Y;
}

typedef struct {
    int32_t *M, *X, *Y;
    int32_t cap;
} dp_mats;

static int mats_reserve(dp_mats* d, int64_t cells) {
    if (cells <= d->cap) return 0;
    free(d->M); free(d->X); free(d->Y);
    d->M = (int32_t*)malloc(sizeof(int32_t) * cells);
    d->X = (int32_t*)malloc(sizeof(int32_t) * cells);
    d->Y = (int32_t*)malloc(sizeof(int32_t) * cells);
    if (!d->M || !d->X || !d->Y) { d->cap = 0; return -1; }
    d->cap = (int32_t)cells;
    return 0;
}

static void mats_free(dp_mats* d) {
    free(d->M); free(d->X); free(d->Y);
    d->M = d->X = d->Y = NULL; d->cap = 0;
}

/* Fill the (la+1) x (lb+1) matrices; row-major with stride lb+1. */
static void fill(const int* ca, int32_t la, const int* cb, int32_t lb,
                 const oracle_params* p, dp_mats* d) {
    const int64_t W = lb + 1;
    const int32_t O = p->gap_open, E = p->gap_extend, S = p->scale;
    int32_t *M = d->M, *X = d->X, *Y = d->Y;
    for (int32_t j = 0; j <= lb; j++) { M[j] = -end_gap(p, j); X[j] = NEG_INF; Y[j] = NEG_INF; }
    for (int32_t i = 1; i <= la; i++) {
        int64_t r = i * W, u = r - W;
        M[r] = -end_gap(p, i); X[r] = NEG_INF; Y[r] = NEG_INF;
        const signed char* srow = kEdnaFull[ca[i - 1] < 16 ? ca[i - 1] : 0];
        const int unk_a = ca[i - 1] > 15;
        for (int32_t j = 1; j <= lb; j++) {
            int cbj = cb[j - 1];
            int s = (unk_a || cbj > 15) ? 0 : srow[cbj] * S;
            int32_t m = M[u + j - 1], x = X[u + j - 1], y = Y[u + j - 1];
            int32_t b = (m > x && m > y) ? m : (x > y ? x : y);
            M[r + j] = b + s;
            int32_t og = M[r + j - 1] - O, eg = X[r + j - 1] - E;
            X[r + j] = og >= eg ? og : eg;
            og = M[u + j] - O; eg = Y[u + j] - E;
            Y[r + j] = og >= eg ? og : eg;
        }
    }
}

/* Start cell: corner, then last column bottom->top, then last row right->left,
 * first strict maximum wins. */
static int32_t pick_end(const dp_mats* d, int32_t la, int32_t lb, const oracle_params* p, int32_t* ei,
                        int32_t* ej) {
    const int64_t W = lb + 1;
    int32_t bi = la, bj = lb, best = d->M[la * W + lb];
    const int ge = (variant() & V_START_GE) != 0;
    for (int pass = 0; pass < 2; pass++) {
        const int col = ((variant() & V_START_ROW) != 0) ? pass == 1 : pass == 0;
        if (col) {
            for (int32_t i = la - 1; i >= 1; i--) {
                int32_t v = d->M[i * W + lb] - end_gap(p, la - i);
                if (v > best || (ge && v == best)) { best = v; bi = i; bj = lb; }
            }
        } else {
            for (int32_t j = lb - 1; j >= 1; j--) {
                int32_t v = d->M[la * W + j] - end_gap(p, lb - j);
                if (v > best || (ge && v == best)) { best = v; bi = la; bj = j; }
            }
        }
    }
    *ei = bi; *ej = bj;
    return best;
}

int32_t oracle_score(const char* a, int32_t la, const char* b, int32_t lb,
                     const oracle_params* p) {
    if (la <= 0 || lb <= 0) return NEG_INF;
    int* ca = (int*)malloc(sizeof(int) * la);
    int* cb = (int*)malloc(sizeof(int) * lb);
    for (int32_t i = 0; i < la; i++) ca[i] = oracle_code((unsigned char)a[i]);
    for (int32_t j = 0; j < lb; j++) cb[j] = oracle_code((unsigned char)b[j]);
    dp_mats d = {0};
    if (mats_reserve(&d, (int64_t)(la + 1) * (lb + 1))) { free(ca); free(cb); return NEG_INF; }
    fill(ca, la, cb, lb, p, &d);
    int32_t ei, ej;
    const int32_t s = pick_end(&d, la, lb, p, &ei, &ej);
    mats_free(&d); free(ca); free(cb);
    return s;
}

static int align_with(const char* a, int32_t la, const int* ca, const char* b,
                      int32_t lb, const int* cb, const oracle_params* p, dp_mats* d,
                      oracle_result* out, char* ref_aln, char* markup, char* read_aln) {
    if (la <= 0 || lb <= 0) return -1;
    if (mats_reserve(d, (int64_t)(la + 1) * (lb + 1))) return -1;
    fill(ca, la, cb, lb, p, d);
    const int64_t W = lb + 1;
    const int32_t O = p->gap_open, E = p->gap_extend;
    int32_t ei, ej;
    const int32_t best = pick_end(d, la, lb, p, &ei, &ej);

    /* Columns are produced end -> start into the tail of the buffers. */
    const int32_t cap = la + lb;
    int32_t k = cap;  /* next free slot is k-1 */
    char* ra = ref_aln; char* rb = read_aln;
    /* unmatched tail */
    for (int32_t j = lb; j > ej; j--) { --k; ra[k] = '-'; rb[k] = b[j - 1]; }
    for (int32_t i = la; i > ei; i--) { --k; ra[k] = a[i - 1]; rb[k] = '-'; }
    int32_t i = ei, j = ej, st = ST_M;
    while (i > 0 && j > 0) {
        int64_t c = (int64_t)i * W + j;
        if (st == ST_M) {
            --k; ra[k] = a[i - 1]; rb[k] = b[j - 1];
            int64_t dg = c - W - 1;
            st = best_state(d->M[dg], d->X[dg], d->Y[dg]);
            i--; j--;
        } else if (st == ST_X) {
            --k; ra[k] = '-'; rb[k] = b[j - 1];
            st = (d->M[c - 1] - O > d->X[c - 1] - E || ((variant() & V_GAP_OPEN) && d->M[c - 1] - O == d->X[c - 1] - E)) ? ST_M : ST_X;
            j--;
        } else {
            --k; ra[k] = a[i - 1]; rb[k] = '-';
            st = (d->M[c - W] - O > d->Y[c - W] - E || ((variant() & V_GAP_OPEN) && d->M[c - W] - O == d->Y[c - W] - E)) ? ST_M : ST_Y;
            i--;
        }
    }
    /* unmatched head */
    for (; j > 0; j--) { --k; ra[k] = '-'; rb[k] = b[j - 1]; }
    for (; i > 0; i--) { --k; ra[k] = a[i - 1]; rb[k] = '-'; }

    const int32_t L = cap - k;
    memmove(ra, ra + k, L); ra[L] = 0;
    memmove(rb, rb + k, L); rb[L] = 0;
    int32_t ident = 0, sim = 0, gaps = 0, nb = 0;
    for (int32_t q = 0; q < L; q++) {
        char x = ra[q], y = rb[q];
        if (x == '-' || y == '-') {
            gaps++; markup[q] = ' ';
            if (y != '-') nb++;
            continue;
        }
        nb++;
        if (toupper((unsigned char)x) == toupper((unsigned char)y)) {
            ident++; sim++; markup[q] = '|';
        } else if (oracle_sub(oracle_code((unsigned char)x), oracle_code((unsigned char)y)) > 0) {
            sim++; markup[q] = ':';
        } else {
            markup[q] = '.';
        }
    }
    markup[L] = 0;
    out->aln_len = L;
    out->n_ident = ident;
    out->n_sim = sim;
    out->n_gaps = gaps;
    out->score = best;
    out->end_i = ei;
    out->end_j = ej;
    out->read_end = nb;
    out->ref_end = la;
    return 0;
}

int oracle_align(const char* a, int32_t la, const char* b, int32_t lb,
                 const oracle_params* p, oracle_result* out,
                 char* ref_aln, char* markup, char* read_aln) {
    if (la <= 0 || lb <= 0) return -1;
    int* ca = (int*)malloc(sizeof(int) * la);
    int* cb = (int*)malloc(sizeof(int) * lb);
    if (!ca || !cb) { free(ca); free(cb); return -1; }
    for (int32_t i = 0; i < la; i++) ca[i] = oracle_code((unsigned char)a[i]);
    for (int32_t j = 0; j < lb; j++) cb[j] = oracle_code((unsigned char)b[j]);
    dp_mats d = {0};
    int rc = align_with(a, la, ca, b, lb, cb, p, &d, out, ref_aln, markup, read_aln);
    mats_free(&d);
    free(ca); free(cb);
    return rc;
}

typedef struct {
    const char* a; int32_t la; const int* ca;
    const char* reads; const int64_t* offsets;
    int32_t n; const oracle_params* p;
    oracle_result* res; char *ref_aln, *markup, *read_aln; int64_t stride;
    int tid, nthreads; int rc;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* jb = (batch_job*)arg;
    dp_mats d = {0};
    int* cb = NULL; int32_t cbcap = 0;
    jb->rc = 0;
    for (int32_t r = jb->tid; r < jb->n; r += jb->nthreads) {
        const char* b = jb->reads + jb->offsets[r];
        int32_t lb = (int32_t)(jb->offsets[r + 1] - jb->offsets[r]);
        oracle_result* o = jb->res + r;
        int64_t off = (int64_t)r * jb->stride;
        if (lb <= 0) { memset(o, 0, sizeof(*o)); continue; }
        if (lb > cbcap) { free(cb); cb = (int*)malloc(sizeof(int) * lb); cbcap = lb; }
        for (int32_t j = 0; j < lb; j++) cb[j] = oracle_code((unsigned char)b[j]);
        if (align_with(jb->a, jb->la, jb->ca, b, lb, cb, jb->p, &d, o,
                       jb->ref_aln + off, jb->markup + off, jb->read_aln + off)) {
            jb->rc = -1;
            break;
        }
    }
    free(cb);
    mats_free(&d);
    return NULL;
}

int oracle_align_batch(const char* a, int32_t la, const char* reads,
                       const int64_t* offsets, int32_t n, const oracle_params* p,
                       int nthreads, oracle_result* res, char* ref_aln,
                       char* markup, char* read_aln, int64_t stride) {
    if (la <= 0) return -1;
    if (nthreads < 1) nthreads = 1;
    int* ca = (int*)malloc(sizeof(int) * la);
    for (int32_t i = 0; i < la; i++) ca[i] = oracle_code((unsigned char)a[i]);
    batch_job* jobs = (batch_job*)calloc(nthreads, sizeof(batch_job));
    pthread_t* th = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (batch_job){a, la, ca, reads, offsets, n, p, res, ref_aln, markup,
                              read_aln, stride, t, nthreads, 0};
        if (nthreads == 1) batch_worker(&jobs[t]);
        else pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    int rc = 0;
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    free(th); free(jobs); free(ca);
    return rc;
}

/* ---------------------------------------------------------------- srspair */

typedef struct { char* buf; int64_t cap, len; } sbuf;

static void sb_printf(sbuf* s, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void sb_printf(sbuf* s, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    int64_t room = s->cap - s->len;
    int n = vsnprintf(room > 0 ? s->buf + s->len : NULL, room > 0 ? (size_t)room : 0, fmt, ap);
    va_end(ap);
    s->len += n;
}

static void sb_put(sbuf* s, const char* src, int64_t n) {
    if (s->len + n < s->cap) memcpy(s->buf + s->len, src, n);
    s->len += n;
}

int64_t oracle_format_srspair(char* buf, int64_t cap, const char* aname,
                              const char* bname, const oracle_params* p,
                              const oracle_result* r, const char* ref_aln,
                              const char* markup, const char* read_aln) {
    sbuf s = {buf, cap, 0};
    const int32_t L = r->aln_len;
    double pi = L ? 100.0 * r->n_ident / L : 0.0;
    double ps = L ? 100.0 * r->n_sim / L : 0.0;
    double pg = L ? 100.0 * r->n_gaps / L : 0.0;
    sb_printf(&s, "#=======================================\n#\n");
    sb_printf(&s, "# Aligned_sequences: 2\n# 1: %s\n# 2: %s\n", aname, bname);
    sb_printf(&s, "# Matrix: EDNAFULL\n# Gap_penalty: %.1f\n# Extend_penalty: %.1f\n#\n",
              p->gap_open_f, p->gap_extend_f);
    sb_printf(&s, "# Length: %d\n", L);
    sb_printf(&s, "# Identity:    %7d/%d (%4.1f%%)\n", r->n_ident, L, pi);
    sb_printf(&s, "# Similarity:  %7d/%d (%4.1f%%)\n", r->n_sim, L, ps);
    sb_printf(&s, "# Gaps:        %7d/%d (%4.1f%%)\n", r->n_gaps, L, pg);
    sb_printf(&s, "# Score: %.1f\n# \n#\n#=======================================\n\n",
              (double)r->score / p->scale);
    /* one chunk (awidth3=5000 keeps CRISPResso amplicons on one line) */
    int32_t na = 0, nb = 0;
    for (int32_t q = 0; q < L; q++) { if (ref_aln[q] != '-') na++; if (read_aln[q] != '-') nb++; }
    sb_printf(&s, "%-13.13s %6d ", aname, na ? 1 : 0);
    sb_put(&s, ref_aln, L);
    sb_printf(&s, " %6d\n", na);
    sb_printf(&s, "%21s", "");
    sb_put(&s, markup, L);
    sb_printf(&s, "\n");
    sb_printf(&s, "%-13.13s %6d ", bname, nb ? 1 : 0);
    sb_put(&s, read_aln, L);
    sb_printf(&s, " %6d\n\n\n", nb);
    if (s.len >= cap) return s.len;  /* too small: report need */
    buf[s.len] = 0;
    return s.len;
}
