/* crispr_quant.h -- C ABI of the MI355X indel/substitution quantification.
 *
 * Replaces CRISPResso's per-read quantification loop, process_df_chunk
 * (CRISPResso/CRISPRessoCORE.py:428-753), and the per-row preparation before it
 * (UNMODIFIED = score_ref == 100, CORE:2014; ignore_n_in_alignment, CORE:2031-2046;
 * compute_ref_positions, CORE:2055-2067).  Input is the aligner's output layout
 * (rows of aligned amplicon / markup / aligned read, include/crispr_nw.h); output
 * is the per-read classification and counts the DataFrame gets, and the effect
 * vectors, histograms and counters the chunk returns, as exact integers.
 *
 * The reference has no FFI at this point (the loop is Python over a DataFrame);
 * the binding a maintainer adds is crispresso_amd/quantify.py (ctypes), whose
 * process_df_chunk(chunk_input) keeps the reference's signature and return tuple.
 */
#ifndef CRISPR_QUANT_H
#define CRISPR_QUANT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nwq_ctx nwq_ctx;

/* The run_crispresso state process_df_chunk reads (module globals and args). */
typedef struct nwq_params {
    int32_t len_amplicon;            /* LEN_AMPLICON (CORE:1288); < 32768 */
    const uint8_t* include_mask;     /* [len_amplicon] 0/1: INCLUDE_IDXS (CORE:2740-2762) */
    const uint8_t* exon_mask;        /* [len_amplicon] EXON_POSITIONS (CORE:1414-1451); NULL = no
                                        --coding_seq: frameshift analysis off (CORE:445-448) */
    const uint8_t* splicing_mask;    /* [len_amplicon] SPLICING_POSITIONS (CORE:1444-1455), or NULL */
    int32_t ignore_substitutions;    /* args.ignore_substitutions (CORE:488) */
    int32_t ignore_insertions;       /* args.ignore_insertions (CORE:517) */
    int32_t ignore_deletions;        /* args.ignore_deletions (CORE:503) */
    int32_t window_around_sgrna;     /* args.window_around_sgrna: nonzero filters NHEJ runs (CORE:611) */
    int32_t hide_mutations_outside_window_nhej;  /* CORE:591, 645 */
    int32_t amplicon_has_n;          /* "N" in amplicon: ignore_n_in_alignment (CORE:2031-2046) */
} nwq_params;

/* Per-read input flags. */
enum {
    NWQ_PRE_UNMODIFIED = 1,   /* score_ref == 100 (CORE:2014) */
    NWQ_PRE_HDR = 2,          /* score_diff < 0 and score_repaired >= threshold (CORE:536-541) */
    NWQ_PRE_MIXED = 4         /* score_diff < 0 and score_repaired <  threshold (CORE:543-548) */
};

/* Per-read output.  cls: 0 UNMODIFIED, 1 NHEJ, 2 HDR, 3 MIXED; -1 = the aligned
 * amplicon row does not hold len_amplicon bases (not an alignment of it). */
typedef struct nwq_read {
    int32_t cls, n_mutated, n_inserted, n_deleted;
} nwq_read;

/* Totals layout (int64 words), see nwq_totals_words:
 *   [15][len_amplicon] vectors, in the order of process_df_chunk's return tuple:
 *       insertion, deletion, mutation, any, insertion_mixed, deletion_mixed,
 *       mutation_mixed, insertion_hdr, deletion_hdr, mutation_hdr,
 *       insertion_noncoding, deletion_noncoding, mutation_noncoding,
 *       avg_vector_del_all, avg_vector_ins_all (sums of run sizes, before the
 *       caller's division, CORE:2962-2973)
 *   [4] modified_frameshift, modified_non_frameshift, non_modified_non_frameshift,
 *       splicing_sites_modified
 *   [H] hist_inframe, [H] hist_frameshift: entry e + len_amplicon counts the
 *       effective length e, H = len_amplicon + stride + 1. */
enum { NWQ_NVEC = 15, NWQ_NCOUNTERS = 4 };

int nwq_create(int device, nwq_ctx** out);
void nwq_destroy(nwq_ctx* c);
const char* nwq_last_error(const nwq_ctx* c);
int nwq_set_params(nwq_ctx* c, const nwq_params* p);
int64_t nwq_totals_words(const nwq_ctx* c, int64_t stride);

/* Host buffers, synchronous.  aln: [n][3][stride] bytes (stride % 4 == 0, < 32768),
 * row k of read r at aln + (r*3 + k)*stride, aln_len[r] columns used.  When
 * amplicon_has_n, the markup rows are rewritten in place (N columns -> '|'), as the
 * reference rewrites align_str.  totals: nwq_totals_words int64, overwritten. */
int nwq_run(nwq_ctx* c, uint8_t* aln, int64_t stride, const int32_t* aln_len, const uint8_t* pre, int64_t n,
            nwq_read* out, int64_t* totals, float* kernel_ms);

/* The same on DEVICE buffers of this context's GPU (e.g. the aligner's resident
 * output, nw_batch_device_output): aln_len[r * len_stride]; out is a device array;
 * totals is a HOST array.  Synchronous. */
int nwq_run_device(nwq_ctx* c, uint8_t* d_aln, int64_t stride, const int32_t* d_aln_len, int64_t len_stride,
                   const uint8_t* d_pre, int64_t n, nwq_read* d_out, int64_t* totals, float* kernel_ms);

/* The same on the aligner's device-resident OPS output (nw_batch_device_ops of an
 * NW_OUT_OPS run: runs, run offsets [n + 1], nw_stat records, the reads as aligned):
 * the rows of every read the quantification loads are rebuilt on the device from its
 * runs, the amplicon and its bytes (the bytes nw_expand_ops writes), then quantified --
 * align -> quantify without the rows layout or a host round trip.  amplicon /
 * amplicon_len: the amplicon aligned (len_amplicon of the params); stride: a multiple of
 * 4 >= every alignment length (nw_batch_device_ops' max_cols).  Synchronous; d_out a
 * device array, totals a HOST array. */
int nwq_run_device_ops(nwq_ctx* c, const char* amplicon, int32_t amplicon_len, const uint32_t* d_ops,
                       const int64_t* d_ops_off, const void* d_stats, const uint8_t* d_reads, const int64_t* d_offsets,
                       int64_t reads_bias, int64_t stride, const uint8_t* d_pre, int64_t n, nwq_read* d_out,
                       int64_t* totals, float* kernel_ms);

/* Reads the lane path of the last nwq_run_device_ops left to the row path (nwq::quant_lanes'
 * fallback list: a '-' byte in the read, more substitutions / deletions / insertions than a lane
 * holds); -1 when that run did not take the lane path.  A diagnostic (bench.py reports it). */
int64_t nwq_lane_fallbacks(const nwq_ctx* c);

#ifdef __cplusplus
}
#endif
#endif
