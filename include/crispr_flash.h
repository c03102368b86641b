/* crispr_flash.h -- C ABI of the MI355X paired-end read merge (FLASH 1.2.11 semantics).
 *
 * CRISPResso merges paired-end reads with the external FLASH program before the
 * alignment (CRISPResso/CRISPRessoCORE.py:1655-1677):
 *
 *     flash R1 R2 --allow-outies --max-overlap M --min-overlap m -f LEN -r AVG -s STD -z -d OUT
 *
 * This library call merges a batch of read pairs on the GPU with the algorithm the
 * test-infrastructure restatement oracle/flash_oracle.py states (read 2 reverse-
 * complemented; every overlap >= min_overlap scored by mismatch density over at most
 * max_overlap bases, ties by the mismatches' quality, then scan order; innies before
 * outies; merged overlap takes the higher-quality base).  The reference has no FFI
 * here (it runs a process); the binding a maintainer adds is crispresso_amd/flash.py
 * (ctypes), whose run_flash() writes FLASH's output files.
 */
#ifndef CRISPR_FLASH_H
#define CRISPR_FLASH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FLASH's options (flash --help): -m, -M, -x, -O, -p, -c. */
typedef struct nwf_params {
    int32_t min_overlap;           /* -m (default 10) */
    int32_t max_overlap;           /* -M (default 65) */
    float max_mismatch_density;    /* -x (default 0.25) */
    int32_t allow_outies;          /* -O */
    int32_t phred_offset;          /* -p (default 33) */
    int32_t cap_mismatch_quals;    /* -c */
} nwf_params;

enum { NWF_COMBINED = 1, NWF_OUTIE = 2 };

/* Merge n read pairs.  Pair i: read 1 = seq1/qual1[off1[i] .. off1[i+1]), read 2 =
 * seq2/qual2[off2[i] .. off2[i+1]) (as in the FASTQ files; qualities are ASCII).
 * Output (caller-owned host buffers): the merged read of pair i is written at
 * out_seq/out_qual + off1[i] + off2[i] (capacity len1 + len2), out_len[i] its
 * length (0: not combined), out_flags[i] NWF_COMBINED | NWF_OUTIE.  Bases other
 * than ACGT (any case) become N, as in FLASH.  kernel_ms (may be NULL) receives
 * the device time.  Returns 0, or a negative code (nwf_last_error() describes it):
 * -1 invalid arguments, -3 a read longer than 4096, -4 HIP error. */
int nwf_merge_batch(int device, const nwf_params* params, const uint8_t* seq1, const uint8_t* qual1,
                    const int64_t* off1, const uint8_t* seq2, const uint8_t* qual2, const int64_t* off2, int64_t n,
                    uint8_t* out_seq, uint8_t* out_qual, int32_t* out_len, int32_t* out_flags, float* kernel_ms);

/* Message of the last failed nwf_merge_batch call in this process. */
const char* nwf_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
