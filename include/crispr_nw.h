/*
 * crispr_nw.h -- C ABI of the MI355X batched global aligner (libcrispr_nw.so).
 *
 * Drop-in for the EMBOSS `needle` process boundary of CRISPResso's single-amplicon
 * pipeline.  Today's contract is a shell pipeline
 *     cat R.fastq.gz | gunzip | awk | sed 's/:/_/g' |
 *         needle -asequence=AMPL.fa -bsequence=/dev/stdin -outfile=/dev/stdout
 *                <needle_options_string> | gzip > needle_output_*.txt.gz
 * (CRISPResso/CRISPRessoCORE.py:1788-1806 forward pass, 1808-1828 HDR pass,
 *  1910-1936 reverse-complement passes), parsed back by parse_needle_output
 * (CRISPRessoCORE.py:1707-1786).  The reference has no FFI of its own; the
 * entry points below are what a ctypes binding of that boundary needs
 * (SURVEY.md 8b).  Plain C types only; no torch types.
 *
 * Threading: one nw_ctx per GPU; a context is NOT thread-safe.  Calls are
 * synchronous unless named *_async.  Every function returns NW_OK (0) or a
 * negative NW_E_* code; nw_last_error() holds the message.  Errors map to the
 * reference's NeedleException ("Needle failed to run", CRISPRessoCORE.py:381,
 * 1805-1806) in the Python host.
 */
#ifndef CRISPR_NW_H
#define CRISPR_NW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NW_OK 0
#define NW_E_INVALID (-1)      /* bad argument (null pointer, empty amplicon, ...) */
#define NW_E_INEXACT (-2)      /* penalties not exactly representable in integer units */
#define NW_E_UNSUPPORTED (-3)  /* option the GPU path does not implement (matrix other than EDNAFULL, size) */
#define NW_E_HIP (-4)          /* HIP runtime error or no device */
#define NW_E_NOMEM (-5)        /* device or host allocation failed */
#define NW_E_STATE (-6)        /* call out of order (e.g. run before upload) */
#define NW_E_CAPACITY (-7)     /* caller's ops buffer too small: ops_off[n] holds the runs needed */

/* Traceback tie policy.  NW_TIE_EMBOSS, the rule pinned against real EMBOSS 6.6.0
 * output by the reference's end-to-end assertions (oracle/nw_oracle.c):
 * the predecessor of an M cell is M when M >= X and M >= Y (ties stay on the
 * diagonal), else X when X > Y, else Y; a gap run was opened at a cell only when
 * open > extend there (ties extend the gap).  Start cell: the best M on the last
 * row / column, scanned corner, then last column bottom->top, then last row
 * right->left; the first strict maximum wins. */
#define NW_TIE_EMBOSS 0

/* nw_stat.flags */
#define NW_FLAG_EMPTY 1        /* zero-length read: no alignment (needle skips it) */

/* Output of the upload/run API (nw_batch_set_output).  NW_OUT_ROWS: the three
 * alignment strings per read in HBM ([n][3][stride], nw_batch_download /
 * nw_batch_device_output).  NW_OUT_OPS: the traceback runs per read (below). */
#define NW_OUT_ROWS 0
#define NW_OUT_OPS 1

/* A run of the ops output: type << 28 | length.  M pairs a residue of each
 * sequence (match or mismatch), X is a gap in the amplicon (read residue), Y a
 * gap in the read (amplicon residue).  A read's runs go start -> end; end gaps are
 * runs like any other. */
#define NW_RUN_M 0u
#define NW_RUN_X 1u
#define NW_RUN_Y 2u
#define NW_RUN_TYPE(op) ((op) >> 28)
#define NW_RUN_LEN(op) ((op) & 0x0fffffffu)

typedef struct nw_ctx nw_ctx;

/* One record per read, written by the GPU. */
typedef struct {
    int32_t aln_len;   /* alignment columns incl. end gaps  == srspair "# Length:" */
    int32_t n_ident;   /* == "# Identity:" numerator   */
    int32_t n_sim;     /* == "# Similarity:" numerator */
    int32_t n_gaps;    /* == "# Gaps:" numerator       */
    int32_t score;     /* "# Score:" x nw_score_scale() */
    int32_t end_i;     /* 1-based amplicon row where the traceback started */
    int32_t end_j;     /* 1-based read column where the traceback started  */
    int32_t flags;     /* NW_FLAG_* */
} nw_stat;

/* Context lifetime.  device = HIP ordinal.  Replaces launching one `needle`
 * process per pass (CRISPRessoCORE.py:1804, 1824, 1919, 1932). */
int nw_create(int device, nw_ctx** out);
void nw_destroy(nw_ctx* ctx);
const char* nw_last_error(const nw_ctx* ctx);

/* needle qualifiers (CRISPRessoCORE.py:4226-4231 default
 * "-gapopen=10 -gapextend=0.5 -awidth3=5000").  matrix must be "EDNAFULL" (or
 * NULL / empty); tie_policy NW_TIE_EMBOSS.  end_weight != 0 is needle's -endweight
 * (-endopen end_open, -endextend end_extend; CRISPResso never sets it, but
 * --needle_options_string forwards it): an end gap of k residues costs
 * end_open + (k - 1) * end_extend, and every read goes through the
 * exact int32 kernels (the band certificate assumes free end gaps).  end_open /
 * end_extend are ignored when end_weight is 0.  Returns NW_E_INEXACT when any
 * penalty in use is not a multiple of 1/16, NW_E_INVALID when one is negative or
 * over 1000. */
int nw_set_params(nw_ctx* ctx, float gap_open, float gap_extend, int end_weight,
                  float end_open, float end_extend, const char* matrix, int tie_policy);
/* Integer multiplier applied to every score (2 for the defaults). */
int nw_score_scale(const nw_ctx* ctx);

/* The amplicon (needle -asequence; CRISPRessoCORE.py:1695-1696 / 1704-1705 /
 * 1885-1907).  Uploads the substitution profile.  1 <= ref_len <= 8192 (amplicons over
 * 1024 bp go through the exact multi-wave kernel only). */
int nw_set_reference(nw_ctx* ctx, const char* ref, int32_t ref_len);

/* Bytes per string slot a caller must provide for reads up to max_read_len. */
int64_t nw_required_stride(const nw_ctx* ctx, int32_t max_read_len);

/* Align n reads (needle -bsequence stream) against the current reference.
 * reads: concatenated bytes; offsets: n+1 byte offsets (read r is
 * reads[offsets[r] .. offsets[r+1])).  Outputs (caller-owned, host memory):
 * aln_out: n * 3 * stride bytes; for read r, at r*3*stride: the aligned
 * amplicon, then (+stride) the markup line, then (+2*stride) the aligned read,
 * each stats[r].aln_len bytes long, not NUL-terminated.  Synchronous. */
int nw_align_batch(nw_ctx* ctx, const char* reads, const int64_t* offsets, int64_t n,
                   char* aln_out, int64_t stride, nw_stat* stats);

/* Same three steps split for device-resident benchmarking: upload keeps the
 * batch in HBM, run launches the kernel on the context stream (async), sync
 * waits and returns the kernel time of the last run measured with HIP events
 * on that stream, download copies results to the host. */
int nw_batch_upload(nw_ctx* ctx, const char* reads, const int64_t* offsets, int64_t n);
/* nw_batch_upload for a batch in nw_align_ops_packed_lens' layout (2 bits per base by batch
 * position + exceptions + uint16 lengths; NW_OUT_OPS only): runs then execute the kernels of
 * the packed call on the resident batch (classify decodes the reads, rebuilds their offsets
 * from the lengths and writes the bytes of the reads that need the DP only): one launch of each
 * of the pipelined call's kernels over the whole batch (with nw_batch_set_lane_walk on, the lane
 * walk + stop summary the call's chunks of >= 65536 reads run; off, the wave walk its smaller
 * chunks run).  nw_batch_device_ops unpacks every read's bytes first. */
int nw_batch_upload_packed(nw_ctx* ctx, const uint8_t* packed, const int64_t* offsets, const uint16_t* lens, int64_t n,
                           const int64_t* exc_pos, const uint8_t* exc_byte, int64_t n_exc);
int nw_batch_run_async(nw_ctx* ctx);
int nw_batch_sync(nw_ctx* ctx, float* kernel_ms);
int nw_batch_download(nw_ctx* ctx, char* aln_out, int64_t stride, nw_stat* stats);
/* Sum over the uploaded batch of (read_len + 3*aln_len + 16): the algorithmic
 * bytes of the last run.  Valid after nw_batch_download or
 * nw_batch_algo_bytes computes it on device-side stats copied back. */
int64_t nw_batch_algo_bytes(nw_ctx* ctx);
/* Cells (sum of ref_len * read_len) of the uploaded batch. */
int64_t nw_batch_cells(const nw_ctx* ctx);
/* Launch geometry of the kernel that aligns the bulk of the batch: rows per
 * lane, waves per block, grid, LDS bytes per block, traceback storage
 * (0 = exact kernel, full traceback in LDS, 1 = exact kernel, full traceback in a
 * global slab, 5 = certified diagonal band: two reads per 16-lane row in packed
 * int16, traceback tiles in HBM). */
int nw_batch_geometry(const nw_ctx* ctx, int32_t* rows_per_lane, int32_t* waves_per_block,
                      int32_t* grid, int32_t* lds_bytes, int32_t* tb_mode);
/* Reads of the last run that the 16- and 32-diagonal band levels did not certify, plus a
 * skipped second level's reads (nw_batch_path_counts [3]; synchronises): the 128-diagonal
 * wide level's input; what it cannot certify either goes to the exact int32 kernel
 * (nw_batch_exact_reads). */
int64_t nw_batch_fallbacks(nw_ctx* ctx);
/* Device time of the last run split by kernel (synchronises): the first band
 * level's DP fill, its traceback walk, and the rest (sort, second level, exact
 * kernel).  With the exact kernel alone everything is reported as fill.  For
 * batches split into several passes the first two cover the first pass only. */
int nw_batch_kernel_times(nw_ctx* ctx, float* fill_ms, float* walk_ms, float* rest_ms);
/* Device-resident output of the last nw_batch_run_async (synchronises): the
 * [n][3][stride] alignment rows and the nw_stat array, valid until the next
 * upload / align call.  Lets the quantification (include/crispr_quant.h,
 * nwq_run_device with aln_len = &stats->aln_len, len_stride = 8) consume the
 * alignments without a round trip through host memory. */
int nw_batch_device_output(nw_ctx* ctx, void** d_aln, int64_t* stride, void** d_stats);
/* The same for an NW_OUT_OPS run (synchronises): the runs of every read (uint32), their
 * offsets (int64 [n + 1]: read r's runs are [d_ops_off[r], d_ops_off[r + 1])), the records
 * (nw_stat [n]), and the reads as the kernels aligned them (read r at d_reads +
 * d_offsets[r] - reads_bias, upper case), plus max_cols >= every alignment length (a
 * multiple of 16).  Valid until the next upload / align call.  The quantification's
 * nwq_run_device_ops consumes exactly these. */
int nw_batch_device_ops(nw_ctx* ctx, void** d_ops, void** d_ops_off, void** d_stats, void** d_reads, void** d_offsets,
                        int64_t* reads_bias, int64_t* max_cols);

/* Pooled batch (replaces one CRISPResso + needle process per amplicon,
 * CRISPRessoPooled.py:882-908): n_refs amplicons packed in `refs` with
 * ref_offsets[n_refs + 1]; read r is aligned against amplicon ref_of_read[r].
 * Outputs as nw_align_batch, in the callers' read order; `stride` at least
 * nw_required_stride_multi(ref_offsets, n_refs, longest read).  Synchronous: every
 * amplicon's tables are uploaded once, each amplicon's kernels are queued back to back.
 * Leaves the context without an uploaded batch (the nw_batch_* getters) and without a
 * reference (nw_set_reference before single-amplicon calls). */
int nw_align_multi(nw_ctx* ctx, const char* refs, const int64_t* ref_offsets, int32_t n_refs,
                   const char* reads, const int64_t* offsets, const int32_t* ref_of_read, int64_t n,
                   char* aln_out, int64_t stride, nw_stat* stats);
int64_t nw_required_stride_multi(const int64_t* ref_offsets, int32_t n_refs, int32_t max_read_len);
/* Pooled batch with ops output (nw_align_ops semantics; outputs in the caller's read
 * order): every amplicon's tables uploaded once, chunks of one amplicon each pipelined
 * through one set of streams.  Reads grouped by amplicon (ref_of_read non-decreasing)
 * are used in place, others are grouped on the host first.  Leaves the context without
 * a reference (nw_set_reference before nw_align_ops). */
int nw_align_multi_ops(nw_ctx* ctx, const char* refs, const int64_t* ref_offsets, int32_t n_refs, const char* reads,
                       const int64_t* offsets, const int32_t* ref_of_read, int64_t n, uint32_t* ops_out,
                       int64_t ops_cap, int64_t* ops_off, nw_stat* stats);
/* nw_align_multi_ops with the reads 2-bit packed (nw_align_ops_packed's layout): the
 * pooled C5 batch crosses PCIe at a quarter of the bytes.  Reads must be grouped by
 * amplicon (ref_of_read non-decreasing; NW_E_INVALID otherwise -- a packed batch is
 * not regrouped on the host). */
int nw_align_multi_ops_packed(nw_ctx* ctx, const char* refs, const int64_t* ref_offsets, int32_t n_refs,
                              const uint8_t* packed, const int64_t* offsets, const int32_t* ref_of_read, int64_t n,
                              const int64_t* exc_pos, const uint8_t* exc_byte, int64_t n_exc, uint32_t* ops_out,
                              int64_t ops_cap, int64_t* ops_off, nw_stat* stats);

/* Device time of the last nw_batch_run_async by phase of the band path (synchronises):
 * [0] classify + length sort, [1] nw_band_fill<16>, [2] nw_band_walk<16>, [3] the
 * 32-diagonal level, [4] the exact kernel + ops compaction.  Other paths: all in [4]. */
int nw_batch_phase_times(nw_ctx* ctx, float* ms5);
/* Whether nw_batch_run_async records the phase events nw_batch_phase_times and nw_batch_kernel_times
 * read (on != 0, the default).  Each is a timing event between two kernels, which writes back the L2's
 * dirty lines (~5-7 us per event on the pass's critical path): a timed resident pass turns them off;
 * both calls then return NW_E_STATE for that run. */
int nw_batch_set_phase_events(nw_ctx* ctx, int on);
/* Reads of the last run by path: [0] exact copies (no DP), [1] first band level,
 * [2] second band level, [3] the 128-diagonal wide level and the exact int32 kernel after
 * it (synchronises).  A chunk whose first level gave up on at most 1024 reads skips the
 * second level (direct hand-off; CRISPR_NW_DIRECT=0 disables it): those
 * reads count under [3]. */
int nw_batch_path_counts(nw_ctx* ctx, int64_t* counts4);
/* Of the reads in nw_batch_path_counts [3] (what the 16- and 32-diagonal levels did not
 * certify), those the 128-diagonal wide level did not certify either: the reads the exact
 * int32 kernel aligned (synchronises; -1 when nothing ran). */
int64_t nw_batch_exact_reads(nw_ctx* ctx);

/* Output mode of the upload/run API (NW_OUT_ROWS default).  Takes effect from
 * the next nw_batch_upload. */
int nw_batch_set_output(nw_ctx* ctx, int mode);
/* After an NW_OUT_OPS run: records, per-read run offsets (n + 1 entries; read r's
 * runs are ops_out[ops_off[r] .. ops_off[r + 1])) and the runs.  NW_E_CAPACITY when
 * ops_cap is short (ops_off is filled; ops_off[n] is the count needed). */
int nw_batch_download_ops(nw_ctx* ctx, uint32_t* ops_out, int64_t ops_cap, int64_t* ops_off, nw_stat* stats);

/* The call that replaces one `needle` pass end to end (CRISPRessoCORE.py:1791-1806:
 * FASTA in, alignments out; the SURVEY.md 8b nw_align_batch with ops output):
 * host reads in -> per-read records + traceback runs in host memory.  Chunks of
 * reads are pipelined over PCIe both ways and the kernels; only the runs cross back
 * (an exact copy is one run), nw_expand_ops rebuilds the strings on the host.
 * Host buffers should be pinned (nw_host_alloc / nw_host_register).  Synchronous.
 * Returns NW_E_CAPACITY when ops_cap is short (ops_off filled, ops_off[n] = needed).
 * ops_out[ops_off[n] .. ops_cap) is scratch: the call may write it (a chunk's runs are
 * copied back from an estimate of their count before the count is known).
 * ops_out = NULL: records and offsets only (a scores-only pass such as the HDR
 * repair alignment, CRISPRessoCORE.py:1808-1828 with just_score). */
int nw_align_ops(nw_ctx* ctx, const char* reads, const int64_t* offsets, int64_t n, uint32_t* ops_out,
                 int64_t ops_cap, int64_t* ops_off, nw_stat* stats);
/* nw_align_ops with the batch as 2 bits per base (what crosses PCIe is a quarter of
 * the bytes): base at batch position i (the offsets' units) in bits 2 (i % 4) of
 * packed[i / 4], A C T G = 0 1 2 3; every other byte of the reads (N, IUPAC codes, U,
 * '-', ...) listed in exc_pos (ascending) / exc_byte.  The kernels see the same bytes
 * as nw_align_ops on the text, but upper case (they compare case-insensitively; the
 * rows are rebuilt from the text by nw_expand_ops).  nw_pack_reads produces this. */
int nw_align_ops_packed(nw_ctx* ctx, const uint8_t* packed, const int64_t* offsets, int64_t n, const int64_t* exc_pos,
                        const uint8_t* exc_byte, int64_t n_exc, uint32_t* ops_out, int64_t ops_cap, int64_t* ops_off,
                        nw_stat* stats);
/* nw_align_ops_packed with every read's length as well (lens[r] = offsets[r + 1] -
 * offsets[r], at most 65535; nw_fastq_lens / nw_read_lengths16 produce them): the lengths
 * cross PCIe instead of the offsets (2 B per read instead of 8; the device rebuilds the
 * offsets from them and every 1024th offset).  NW_E_INVALID when a length differs from its
 * offsets' difference (checked for every read before any kernel runs). */
int nw_align_ops_packed_lens(nw_ctx* ctx, const uint8_t* packed, const int64_t* offsets, const uint16_t* lens, int64_t n,
                             const int64_t* exc_pos, const uint8_t* exc_byte, int64_t n_exc, uint32_t* ops_out,
                             int64_t ops_cap, int64_t* ops_off, nw_stat* stats);
/* The same for the pooled call (nw_align_multi_ops_packed). */
int nw_align_multi_ops_packed_lens(nw_ctx* ctx, const char* refs, const int64_t* ref_offsets, int32_t n_refs,
                                   const uint8_t* packed, const int64_t* offsets, const uint16_t* lens,
                                   const int32_t* ref_of_read, int64_t n, const int64_t* exc_pos, const uint8_t* exc_byte,
                                   int64_t n_exc, uint32_t* ops_out, int64_t ops_cap, int64_t* ops_off, nw_stat* stats);
/* lens[r] = offsets[r + 1] - offsets[r] as uint16 (host pool; nthreads > 0 caps its parts):
 * NW_E_UNSUPPORTED when a read is longer than 65535 (or offsets decrease). */
int nw_read_lengths16(const int64_t* offsets, int64_t n, uint16_t* lens, int32_t nthreads);
/* Pack reads[offsets[0] .. offsets[n]) for nw_align_ops_packed (host, nthreads; <= 0:
 * all cores): packed must hold bytes offsets[0] / 4 .. (offsets[n] + 3) / 4 (indexed by
 * batch position).  NW_E_CAPACITY when more than exc_cap exceptions (*n_exc = count). */
int nw_pack_reads(const char* reads, const int64_t* offsets, int64_t n, uint8_t* packed, int64_t* exc_pos,
                  uint8_t* exc_byte, int64_t exc_cap, int64_t* n_exc, int32_t nthreads);

/* nw_align_ops on the batch the last nw_align_ops of this context uploaded (still in
 * HBM: no upload), against the current reference -- the second pass of the same reads
 * (HDR amplicon, CRISPRessoCORE.py:1808-1828).  offsets / n must be that batch's. */
int nw_align_ops_resident(nw_ctx* ctx, const int64_t* offsets, int64_t n, uint32_t* ops_out, int64_t ops_cap,
                          int64_t* ops_off, nw_stat* stats);
/* CRISPResso's dual alignment in one call (CRISPRessoCORE.py:1808-1828: every read against the
 * amplicon, then against the expected HDR amplicon): the packed batch (nw_align_ops_packed_lens'
 * layout) crosses PCIe once; each read is aligned against the current reference (records, runs,
 * run offsets into stats / ops_out / ops_off as nw_align_ops_packed_lens) and against ref2 (into
 * stats2 / ops_out2 / ops_off2; ops_out2 may be null: records and run offsets only).  The second
 * pass's chunk of a read range runs as soon as that range is uploaded.  Results equal the two
 * separate calls'.  The context keeps its reference; the batch stays resident. */
int nw_align_dual_ops_packed_lens(nw_ctx* ctx, const char* ref2, int32_t ref2_len, const uint8_t* packed,
                                  const int64_t* offsets, const uint16_t* lens, int64_t n, const int64_t* exc_pos,
                                  const uint8_t* exc_byte, int64_t n_exc, uint32_t* ops_out, int64_t ops_cap,
                                  int64_t* ops_off, nw_stat* stats, uint32_t* ops_out2, int64_t ops_cap2,
                                  int64_t* ops_off2, nw_stat* stats2);
/* Last nw_align_ops: span of the uploads on the copy stream (h2d_ms); compute_ms = the device span
 * from the first upload to the last chunk's end (uploads included), or, with host timing on
 * (CRISPR_NW_HOST_TIMING=1), the sum of the chunks' kernel spans; bytes each way. */
int nw_ops_times(const nw_ctx* ctx, float* h2d_ms, float* compute_ms, int64_t* h2d_bytes, int64_t* d2h_bytes);

/* Page-locked host memory for the batch buffers (hipHostMalloc / hipHostRegister). */
int nw_host_alloc(int64_t bytes, void** out);
void nw_host_free(void* p);
int nw_host_register(void* p, int64_t bytes);
int nw_host_unregister(void* p);
/* Threads of the library's host pool (the call's length scan, FASTQ ingest, packing, the
 * DataFrame helpers): CRISPR_NW_HOST_THREADS when set, else the process's CPU affinity capped
 * by the cgroup quota and divided by LOCAL_WORLD_SIZE (crispresso_amd/placement.py binds a
 * rank and sets the variable).  Creates the pool on first use. */
int nw_host_threads(void);
/* A sequence whose exact copies among the reads (case-insensitive A C G T) take ONE alignment of
 * it against the amplicon, computed by the exact kernel during the call, instead of a DP each:
 * the HDR amplicon during the reference-amplicon pass of CRISPResso's dual alignment
 * (CRISPRessoCORE.py:1788-1828; len 0 clears it).  A resident pass against a new amplicon
 * (nw_align_ops_resident) uses the amplicon the batch was last aligned against the same way when
 * none is set.  Results are those of aligning every read; used when both sequences are A C G T,
 * of one length <= 256, and the input is packed. */
int nw_set_known(nw_ctx* ctx, const char* seq, int32_t len);
/* Resident passes (nw_batch_run_async): the first band level's lane walk and the stop summary
 * its fill writes (on != 0) -- what a pipelined call runs on its chunks of >= 65536 reads of one
 * amplicon -- instead of the wave-per-read walk (smaller chunks, pooled calls).  Off by default. */
int nw_batch_set_lane_walk(nw_ctx* ctx, int on);

/* The three alignment rows of n reads from their runs (host, nthreads threads;
 * <= 0: all cores): for read r at aln_out + r*3*stride the aligned amplicon, the
 * markup and the aligned read, stats[r].aln_len bytes each -- the bytes the kernels
 * write in NW_OUT_ROWS mode.  ref = the amplicon; reads/offsets as aligned.  Rows of
 * empty reads are left untouched.  Returns 0, or NW_E_INVALID when a read's runs do
 * not cover the amplicon and the read or exceed stride. */
int nw_expand_ops(const char* ref, int32_t ref_len, const char* reads, const int64_t* offsets, int64_t n,
                  const uint32_t* ops, const int64_t* ops_off, char* aln_out, int64_t stride, int32_t nthreads);

/* FASTQ(.gz) ingest (CRISPRessoCORE.py:1791-1797: gunzip | awk | sed 's/:/_/g', then
 * EMBOSS's FASTA reader): every record's name (first word of the header, ':' -> '_')
 * and the sequence bytes EMBOSS keeps (letters and * . ~ ? # + -), packed with n + 1
 * offsets.  The handle owns the buffers. */
typedef struct nw_fastq nw_fastq;
int nw_fastq_read(const char* path, nw_fastq** out);
int64_t nw_fastq_count(const nw_fastq* q);
const char* nw_fastq_seqs(const nw_fastq* q);
const int64_t* nw_fastq_offsets(const nw_fastq* q);
const char* nw_fastq_names(const nw_fastq* q, int64_t* bytes);   /* each name followed by '\n' */
void nw_fastq_free(nw_fastq* q);
/* nw_fastq_read keeping only the records whose Phred+33 qualities average >=
 * min_avg_quality with none < min_single_quality -- CRISPResso's read quality filter
 * (filter_se_fastq_by_qual, CRISPRessoCORE.py:270-308; --min_average_read_quality /
 * --min_single_bp_quality, 1547-1583).  Thresholds <= 0 both: no filter. */
int nw_fastq_read_filtered(const char* path, int32_t min_avg_quality, int32_t min_single_quality, nw_fastq** out);
int64_t nw_fastq_dropped(const nw_fastq* q);                    /* records the filter removed */
const uint8_t* nw_fastq_pass(const nw_fastq* q, int64_t* n);    /* every record's verdict (1 = kept), file order */
/* The handle's reads as nw_align_ops_packed takes them (nw_pack_reads' layout: 2 bits per
 * base by batch position = the nw_fastq_offsets positions, exceptions ascending) plus a
 * copy of the offsets, in page-locked host memory (pinned != 0: the upload runs at PCIe
 * rate; NW_E_NOMEM when the runtime cannot page-lock) or ordinary memory (pinned = 0).
 * Built once, in parallel, by the first call; the handle owns the buffers; a later call
 * with the other `pinned` returns NW_E_STATE.  Replaces the reference's FASTA pipe into
 * needle (CRISPRessoCORE.py:1791-1797) as the aligner's input. */
int nw_fastq_pack(nw_fastq* q, int32_t pinned, const uint8_t** packed, const int64_t** offsets, const int64_t** exc_pos,
                  const uint8_t** exc_byte, int64_t* n_exc);
/* After nw_fastq_pack: the reads' lengths as nw_align_ops_packed_lens takes them, in the
 * same kind of memory; NW_E_UNSUPPORTED (null) when a read is longer than 65535. */
int nw_fastq_lens(nw_fastq* q, const uint16_t** lens);
/* The FASTQ ingest's decompressor: a one-member gzip image decoded by `threads` threads
 * (ranges of the compressed bits decoded from block starts found in them, chained and
 * checked against the member's CRC-32 and size) into out[0 .. cap); *out_n = its size.
 * NW_E_UNSUPPORTED: not taken (several members, too small, no block starts found, damaged
 * data) -- nw_fastq_read then decodes on one thread; NW_E_CAPACITY: cap < *out_n. */
int nw_gunzip_parallel(const uint8_t* gz, int64_t n, int32_t threads, uint8_t* out, int64_t cap, int64_t* out_n);
/* The DataFrame's ID column (CRISPRessoCORE.py:1725) from nw_fastq_names' block (n names,
 * each followed by '\n'): ids = the names' bytes without the newlines, '_' -> ':'; name i
 * at [off[i], off[i + 1]) (off: n + 1 entries).  NW_E_UNSUPPORTED when a name holds
 * whitespace or a non-ASCII byte, or the block does not hold n names. */
int nw_names_to_ids(const uint8_t* raw, int64_t nbytes, int64_t n, uint8_t* ids, int64_t* off);

/* nw_expand_ops for the reads idx[0 .. m) only: read idx[q]'s rows at aln_out + q*3*stride. */
int nw_expand_ops_subset(const char* ref, int32_t ref_len, const char* reads, const int64_t* offsets,
                         const int64_t* idx, int64_t m, const uint32_t* ops, const int64_t* ops_off, char* aln_out,
                         int64_t stride, int32_t nthreads);
/* The rows of reads idx[0 .. m) from the runs, concatenated: read q's first
 * row_off[q + 1] - row_off[q] columns (<= its alignment length; the awidth cut) at
 * [row_off[q], row_off[q + 1]) of ref_rows / markup_rows / read_rows; read_chars[q] =
 * non-'-' bytes of that read-row span; ref_is_amplicon[q] = 1 when the amplicon row is
 * the amplicon itself (no gap in it, not cut).  The DataFrame hand-off's one pass. */
int nw_ops_rows_concat(const char* ref, int32_t ref_len, const char* reads, const int64_t* offsets, const int64_t* idx,
                       int64_t m, const uint32_t* ops, const int64_t* ops_off, const int64_t* row_off, char* ref_rows,
                       char* markup_rows, char* read_rows, int32_t* read_chars, uint8_t* ref_is_amplicon,
                       int32_t nthreads);
/* equal[r] = read r is byte for byte the amplicon (its three rows are the amplicon, a
 * row of '|' and the amplicon: the DataFrame shares one string for them).  Returns the
 * count. */
int64_t nw_reads_equal_ref(const char* ref, int32_t ref_len, const char* reads, const int64_t* offsets, int64_t n,
                           uint8_t* equal, int32_t nthreads);

/* Over the reads idx[0 .. m) (idx null: reads 0 .. m): rep[q] = the first q' whose read has
 * read idx[q]'s bytes (rep[q] == q for the first of each); returns the number of distinct
 * reads.  The alignment is a function of the read's bytes, so the DataFrame hand-off builds
 * the row strings of each distinct read once and shares them. */
int64_t nw_reads_first_copy(const char* reads, const int64_t* offsets, const int64_t* idx, int64_t m, int64_t* rep,
                            int32_t nthreads);

/* srspair text of n alignments (the blocks parse_needle_output consumes,
 * CRISPRessoCORE.py:1715-1765).  aname = amplicon id; bnames = n NUL-separated
 * read ids, concatenated.  Writes at most cap bytes; returns the number of
 * bytes the full text needs (call again with a bigger buffer if > cap).
 * awidth = needle -awidth3 (alignment columns per line). */
int64_t nw_format_srspair(char* buf, int64_t cap, const char* aname, const char* bnames,
                          float gap_open, float gap_extend, int32_t scale, int32_t awidth,
                          const char* aln, int64_t stride, const nw_stat* stats, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
