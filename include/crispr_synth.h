/*
 * crispr_synth.h -- synthetic read sets of SURVEY.md 8(d) (C2 / C4 mix), generated
 * natively for bench.py and the tests.  Not part of the needle-replacement boundary
 * (include/crispr_nw.h): the reference has no counterpart; it exists because the
 * C4 shards (12.5M reads per GPU) are too slow to draw in numpy within a bench run.
 *
 * mix[5] = weights of exact copy, 1-3 substitutions, one deletion (Geom(0.3) length,
 * 1-30, at La/2 +- 10), one insertion (1-10 random bases, at La/2 +- 10), 1 %-per-base
 * noise (crispresso_amd/synth.py C2_MIX: 0.6 0.2 0.1 0.05 0.05).  Read r depends only
 * on (amplicon, seed, r, mix): any range of a set is generated on its own.
 * nthreads <= 0: the library's host pool.
 */
#ifndef CRISPR_SYNTH_H
#define CRISPR_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* offsets[0 .. n] of reads first .. first + n - 1 of the set (offsets[0] = 0); returns
 * offsets[n] (total bases), or -1 on bad arguments. */
int64_t nw_synth_offsets(const char* amp, int32_t La, int64_t first, int64_t n, uint64_t seed, const double* mix,
                         int64_t* offsets, int32_t nthreads);
/* Those reads' bytes (A C G T) into buf[offsets[r] - offsets[0] ..]: offsets as
 * nw_synth_offsets returned them for the same first / n.  0, or -1 on bad arguments /
 * offsets that do not match. */
int nw_synth_reads(const char* amp, int32_t La, int64_t first, int64_t n, uint64_t seed, const double* mix,
                   const int64_t* offsets, char* buf, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
