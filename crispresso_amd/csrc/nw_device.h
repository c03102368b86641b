// nw_device.h -- definitions shared by the HIP kernel and the host launcher.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nw {

// Residue codes: 0..15 EDNAFULL (A T G C S W R Y K M B V H D N U),
// 16 = not in the matrix (scores 0 against everything).
constexpr int NCODE = 17;
constexpr int NCODE_PAD = 16;   // code used for columns past the end of a read

enum : int32_t { FLAG_EMPTY = 1 };
constexpr int kOpsSlot = 64;    // runs kept per read in its ops slot (more: spill area)
// nops[r] flag: read r's runs are in the row-major slot area (the walk / exact kernels:
// run q at ops[ops_stride * ops_slot + r * ops_slot + q]), not the column-major one (the
// classify / diagonal-pass records: run q at ops[q * ops_stride + r])
constexpr int32_t kNopsRows = 1 << 30;
// nops[r] flag: read r is a copy of the known sequence (KernelArgs::known2): its record and runs
// are the known alignment's (OpsKnown), filled in by the compaction
constexpr int32_t kNopsKnown = 1 << 29;

// Per-read record written by the kernel; layout matches nw_stat in include/crispr_nw.h.
struct Stat {
    int32_t aln_len, n_ident, n_sim, n_gaps, score, end_i, end_j, flags;
};

struct KernelArgs {
    const uint8_t* reads;      // packed read bytes
    const int64_t* offsets;    // n + 1 entries
    int64_t n;
    const int8_t* prof;        // [NCODE][64][RP] scaled EDNAFULL scores of each amplicon row
    const uint8_t* lut;        // [256] ascii -> code
    const uint8_t* amp;        // [La] amplicon bytes
    int32_t La;
    int32_t gap_open, gap_extend;   // scaled
    int32_t Lb_max;
    uint8_t* out;              // [n][3][stride]: aligned amplicon, markup, aligned read
    int64_t stride;
    Stat* stats;               // [n]
    uint8_t* tb_global;        // traceback slabs when they do not fit LDS
    int64_t tb_wave_bytes;
    // exact kernel: reads whose walk failed are appended here (never with full storage)
    int64_t* fallback_list;
    int32_t* fallback_count;
    // work list (full-storage kernel re-running the fallbacks); null = all reads
    const int64_t* work_list;
    const int32_t* work_count;
    int32_t work_lo;           // first work-list entry (or read, null list) this kernel takes (the one-wave
                               // kernel after the multi-wave one: entries [0, exact grid) are the multi-wave kernel's)
    const uint8_t* lut6;       // [256] ascii -> A T G C N pad in that order (0..5), 6 = other IUPAC code
    // certified diagonal-band kernels (nw_band.hip)
    const int32_t* band_order;     // read indices sorted by length; sorted positions 2g, 2g+1 = pair g
    int64_t band_pair_lo, band_pair_hi;   // pairs of this pass
    uint8_t* band_region;          // per-pair regions of the pass (band_stride bytes each)
    int64_t band_stride;
    int32_t band_words;            // traceback words per lane and pair
    int32_t band_summ;             // the first level's fill writes the stop summary the lane walk reads (nw_batch_set_lane_walk)
    int64_t* zero_ctl64;           // a resident pass: the ops compaction's control block, zeroed by classify (no memset launch)
    int32_t zero_ctl64_n;
    int32_t band_lb_cap;           // longest read the band kernels take; longer ones sort last
    int32_t band_maxsub;           // largest substitution score (scaled): the certificate's bound
    const uint32_t* band_tab;      // [17 amplicon codes (EDNAFULL, pad)][6][6 read codes] packed int16x2 score + 2 E
    const uint32_t* rowpos;        // [La] codes each amplicon row scores > 0 against (markup ':')
    int32_t* sort_key;             // [n] bucket of every read: length, band_lb_cap + 1 (longer), + 2 (exact copy)
    const int32_t* band_count;     // device: entries of band_order to align (sorted reads that need the DP,
                                   // or the previous level's redo count)
    unsigned long long* lb_status; // look-back words of the single-pass scans (band_lookback_words(n))
    int32_t* redo_list;            // reads a narrow first band could not certify (next level's band_order)
    int32_t* redo_count;
    uint8_t* redo_flags;           // [n] per sorted position: handed to the next level (compacted in order)
    // > 0: when the first level hands on at most this many reads (*redo_count), the second
    // level's kernels return at once and the exact kernel takes them too (its fallback list,
    // then the redo list): a few hundred reads cost the exact kernel's latency once, less
    // than the second level's fill + walk ahead of it.  Decided on the device per chunk.
    int32_t redo_direct;
    // > 0: a chunk whose sort found at most this many reads that need the DP (*band_count of the first
    // level's launches) sends them all past the 16-diagonal level: its fill and walk return at once, the
    // redo compaction takes every position, and (l1_skip <= redo_direct) the wide level aligns them -- a
    // chunk with few DP reads waits for one level's latency instead of three.  Decided on the device.
    int32_t l1_skip;
    int32_t band_from_work;    // the wide level: the band list is the exact kernel's work list (exact_work_read)
    int32_t* seed_info2;       // [n] the seeded reads' block facts for the refined certificate (seed2_pack; null: off)
    // ops output (include/crispr_nw.h nw_align_ops): instead of the three string rows,
    // every read's traceback runs (RUN_* << 28 | length, start -> end) go to its slot
    // ops[r * ops_slot ..]; a read with more runs than a slot holds writes them to the
    // spill area (bump-allocated words, the position in slot[0]).  null ops = rows.
    uint32_t* ops;
    int32_t ops_slot;
    int64_t ops_stride;            // slot layouts: column-major run q of read r at ops[q * ops_stride + r] (the
                                   // compaction reads consecutive reads' first runs as whole lines); row-major
                                   // (kNopsRows) at ops[ops_stride * ops_slot + r * ops_slot + q]
    int32_t* nops;                 // [n] runs per read (0: empty read)
    uint32_t* spill;
    int64_t spill_cap;             // words
    int32_t* ops_ctl;              // [0] spill words used, [1] error flag (spill area full)
    // exact multi-wave kernel (nw_exact.hip): [17 amplicon codes][4] dwords, the scaled
    // EDNAFULL scores against read codes 0..15 as int8 (byte j of dword q: code 4q + j)
    const uint32_t* sub16;
    // needle -endweight (the exact kernels only): an end gap of k residues costs
    // end_open + (k - 1) * end_extend (scaled) instead of nothing
    int32_t end_weight, end_open, end_extend;
    // the latency-bound kernels of a chunk's tail (second band level, exact kernels, the
    // scans) raise their waves' issue priority (s_setprio): they share the SIMDs with the
    // other chunk's bulk fill, and a chain waits for its tail
    int32_t tail_prio;
    // packed input (nw_align_ops_packed; band path): nw_band_classify decodes the chunk's reads
    // from the 2-bit stream, rebuilds their offsets from the lengths (pk_len), and writes the
    // bytes of the reads that need the DP -- the only bytes any later kernel reads -- with their
    // exception bytes.  Null pk_words: byte input (reads / offsets as uploaded).
    const uint32_t* pk_words;      // the stream's device copy: dword k = batch positions pk_pos0 + 16 k ..
    int64_t pk_pos0;               // a multiple of 16
    const int64_t* pk_exc_pos;     // the call's exceptions (positions ascending, bytes) ...
    const uint8_t* pk_exc_byte;
    int64_t pk_e0, pk_e1;          // ... searched in [pk_e0, pk_e1)
    const uint16_t* pk_len;        // call-indexed read lengths (null: the offsets are in place)
    const int64_t* pk_gbase;       // offset of read g * kLenGroup
    int64_t pk_call_lo;            // call index of the chunk's read 0
    // window seeds (packed classify): the amplicon's 2-bit stream and its A C G T 16-mers sorted by
    // (key, position) -- reads shorter than the amplicon that are an exact copy of one of its windows,
    // or one substitution from one, leave the DP (null amp2: off)
    const uint32_t* amp2;
    const uint32_t* seed_key;
    const uint16_t* seed_pos;
    int32_t n_seed;
    // seeded band: per read, the diagonals of its 16-mer blocks' exact hits
    // (seed_pack), written by the packed classify; null: off.  seed_keys: sort keys past the
    // length keys that order seeded reads by their hits' centre (the segment sort's key range)
    int32_t* seed_info;
    int32_t seed_keys;
    int32_t* seed_list;            // the segment sort's seeded reads (sorted), the wide level's list tail
    int32_t* seed_count;
    // the seeded list through the 32-diagonal level first: 1 on that level's launches
    // (its list, then the seeded list); it sets seed_flags[q] for the seeded list's entry q it leaves
    // to the wide level (clears it for a read it certified), and a compaction keeps those; 0: off
    int32_t seed_l2;
    uint8_t* seed_flags;
    // deferred certificates (packed classify, ops output): each classify wavefront queues its reads
    // that take the three-substitution or one-indel checks (64 entries per wavefront, its count in
    // cert_cnt) and nw_band_cert runs those checks on dense lists; null: classify runs them itself
    int32_t* cert_q;
    int32_t* cert_cnt;
    const uint32_t* cls_img;       // classify's LDS image of the amplicon (nw_host.cpp cls_image)
    int32_t cls_words;
    int32_t amp_acgt;              // every amplicon byte A C G T (either case)
    // known copies: the 2-bit words of a sequence of the amplicon's length whose
    // alignment against the amplicon is computed once (the previous amplicon of a resident batch:
    // the HDR pass's reads that are copies of the reference amplicon); classify flags the reads equal
    // to it (nops kNopsKnown) and the compaction gives them that alignment.  Null: off.
    const uint32_t* known2;
};

// Boundary value of a leading end gap of k residues (0: free end gaps, or k = 0) and
// the penalty of a trailing one.
__host__ __device__ inline int end_lead(const KernelArgs& a, int k) {
    return (a.end_weight && k > 0) ? -(a.end_open + (k - 1) * a.end_extend) : 0;
}
__host__ __device__ inline int end_trail(const KernelArgs& a, int k) { return -end_lead(a, k); }

// KernelArgs::redo_direct: the chunk's second band level is skipped (read on the device
// by the second level's kernels, the exact kernel and the ops counts alike).
__host__ __device__ inline bool redo_direct_taken(const KernelArgs& a) {
    return a.redo_direct > 0 && a.redo_count && *a.redo_count <= a.redo_direct;
}
__host__ __device__ inline bool l1_skipped(const KernelArgs& a) {
    return a.l1_skip > 0 && a.band_count && *a.band_count <= a.l1_skip;
}
// The exact kernel's work: entries [0, fallbacks) of the work list, then (direct) the redo list.
__host__ __device__ inline long long exact_work_count(const KernelArgs& a) {
    const long long nfb = a.work_list ? (long long)*a.work_count : a.n;
    return a.work_list && redo_direct_taken(a) ? nfb + *a.redo_count : nfb;
}
__host__ __device__ inline long long exact_work_read(const KernelArgs& a, long long wi) {
    if (!a.work_list) return wi;
    const long long nfb = *a.work_count;
    return wi < nfb ? a.work_list[wi] : (long long)a.redo_list[wi - nfb];
}

// Traceback storage of a kernel instantiation.
enum TbMode : int { TB_LDS_FULL = 0, TB_GLOBAL_FULL = 1, TB_DIAG = 5 };

struct LaunchCfg {
    int R;           // amplicon rows per lane
    int wpb;         // waves per block
    int grid;        // blocks
    int lds_bytes;   // dynamic LDS per block
    int tb_mode;     // TbMode
};

int rows_per_lane_for(int La);
int profile_rp(int R);
int lds_bytes_for(int R, int La, int Lb_max, int tb_mode, int wpb);
int tb_bytes_per_wave(int R, int Lb_max);
hipError_t launch(const KernelArgs& a, const LaunchCfg& c, hipStream_t s);

// band pair header flags: read A / B has a code outside A C G T N (BAD), or an N or a byte EDNAFULL
// does not score (NP: not a plain read for the walk's shortcuts)
enum : int32_t { REGION_BAD_A = 1, REGION_BAD_B = 2, REGION_NP_A = 8, REGION_NP_B = 16, REGION_SEEDED = 32 };
// seed_info word: bit 31 valid; the lowest and highest hit diagonal (d = j - i, + 1024, 11 bits
// each) and the number of 16-base blocks (7 bits)
__host__ __device__ inline int32_t seed_pack(int dmin, int dmax, int nb) {
    return (int32_t)(0x80000000u | (unsigned)(dmin + 1024) | ((unsigned)(dmax + 1024) << 11) | ((unsigned)nb << 22));
}
__host__ __device__ inline bool seed_valid(int32_t s) { return ((unsigned)s >> 31) != 0u; }
__host__ __device__ inline int seed_dmin(int32_t s) { return (int)((unsigned)s & 0x7ffu) - 1024; }
__host__ __device__ inline int seed_dmax(int32_t s) { return (int)(((unsigned)s >> 11) & 0x7ffu) - 1024; }
__host__ __device__ inline int seed_blocks(int32_t s) { return (int)(((unsigned)s >> 22) & 0x7fu); }
// seed_info2 word (reads whose blocks have at most one hit each, on at most 4 diagonals): bit 31
// valid; the blocks without a hit (7 bits), the most blocks on one diagonal (7 bits), the cheapest
// move between two blocks' diagonals in read order (16 bits, scaled score; 0xffff: one diagonal)
__host__ __device__ inline int32_t seed2_pack(int n0, int cmax, int shift) {
    return (int32_t)(0x80000000u | (unsigned)n0 | ((unsigned)cmax << 7) | ((unsigned)(shift < 0xffff ? shift : 0xffff) << 14));
}
__host__ __device__ inline bool seed2_valid(int32_t s) { return ((unsigned)s >> 31) != 0u; }
__host__ __device__ inline int seed2_n0(int32_t s) { return (int)((unsigned)s & 0x7fu); }
__host__ __device__ inline int seed2_cmax(int32_t s) { return (int)(((unsigned)s >> 7) & 0x7fu); }
__host__ __device__ inline int seed2_shift(int32_t s) { return (int)(((unsigned)s >> 14) & 0xffffu); }

// certified diagonal-band fill + walk (nw_band.hip): kBandDiags diagonals per read,
// two equal-length reads per 16-lane row, reads sorted by length on the device.
constexpr int kBandDiags = 32;
constexpr int kWideDiags = 128;   // the wide level: the narrower levels' give-ups before the exact kernel
int band_fill_lds_bytes(int La, int wpb, int W);
int band_walk_lds_bytes(int La, int wpb, int lb_max, int W);
int band_region_words(int La, int Lb_max, int W = kBandDiags);
int64_t band_region_bytes(int La, int Lb_max, int W);
bool band_pair_geometry(int La, int Lb, int* dlo);
hipError_t band_occupancy(int W, int fill_wpb, int walk_wpb, int fill_lds, int walk_lds, int* fill_blocks,
                          int* walk_blocks);
// classify + the segment sort (a.band_count <- reads that need the DP); `epoch`: a value
// not used by the previous look-back launch on a.lb_status
hipError_t launch_band_sort(const KernelArgs& a, unsigned epoch, hipStream_t s);
int64_t band_lookback_words(int64_t n);
hipError_t launch_band(int W, const KernelArgs& a, const LaunchCfg& fill, const LaunchCfg& walk, hipStream_t s,
                       hipEvent_t after_fill);
// 2-bit packed bases [b0, b1) (batch positions; device copy of the stream from byte
// pbyte0, 4-aligned) -> dst[pos - bias] bytes (A C T G), then exceptions [e0, e1)
// With `lens`: the same launch also rebuilds the chunk's offsets d_off[r_lo .. r_hi]
// (call-indexed, r_hi inclusive) from the reads' uint16 lengths and every kLenGroup-th
// offset (nw_align_ops_packed_lens: the 8-B offsets do not cross PCIe).
struct LenSeg {
    const uint16_t* len = nullptr;   // device: the call's read lengths (read r at len[r])
    const int64_t* gbase = nullptr;  // device: offset of read g * kLenGroup, per group g
    int64_t g0 = 0, ngroups = 0;     // the chunk's groups g0 .. g0 + ngroups - 1 (group g: reads [1024 g, 1024 g + 1024))
    int64_t r_lo = 0, r_hi = 0;      // offsets written: reads r_lo .. r_hi
    int64_t* d_off = nullptr;
};
constexpr int kLenGroup = 1024;
hipError_t launch_unpack(const uint32_t* packed, int64_t pbyte0, int64_t b0, int64_t b1, const int64_t* exc_pos,
                         const uint8_t* exc_byte, int64_t e0, int64_t e1, uint8_t* dst, int64_t bias, hipStream_t s,
                         const LenSeg* lens = nullptr);
// the first level's flagged positions -> a.redo_list (sorted order) and *a.redo_count;
// nmax >= the number of sorted positions (grid size)
hipError_t launch_redo_compact(const KernelArgs& a, int64_t nmax, unsigned epoch, hipStream_t s, bool pairs = false);

// exact int32 kernel for work lists (nw_exact.hip): one workgroup of exact_waves(La)
// wavefronts per read; traceback slots in LDS (tb_lds) or a per-block HBM slab of
// exact_slab_bytes at a.tb_global.  La <= 8192.
int exact_rows_per_lane(int La);
int exact_waves(int La);
int exact_lds_bytes(int La, int Lb_max, bool tb_lds);
int64_t exact_slab_bytes(int La, int Lb_max);
// cap: take work-list entries [0, min(count, grid)) only (the one-wave kernel the rest);
// a null work list = every read of the batch.
hipError_t launch_exact(const KernelArgs& a, int grid, int lds_bytes, bool tb_lds, int64_t slab_bytes, bool cap,
                        hipStream_t s);

// ops compaction (nw_ops.hip): per-read slots -> one contiguous run array, one launch.
// ctl (int64, kOpsCtl + 2): [0] running total after this chunk, [1] this chunk's base, [2]
// this chunk's total, [3] errors (1: staging full, 2: spill area full, from opsctl[1], 4: a
// look-back cut off); running over the call: [4] exact-kernel reads, [5] second band level
// reads of two-level chunks, [6] reads that needed the DP, [7] DP reads of chunks run on the
// second level alone, [8] reads that reached the exact kernel (after the wide level) (OpsCounts:
// the device counters of the chunk's kernels);
// [kOpsCtl], [kOpsCtl + 1]: the running base, read from [kOpsCtl + parity] and written to
// the other (chunk k: parity k & 1).
// status: band_lookback_words(n) look-back words; epoch: new per launch.  opsctl: the
// kernels' flags.  hctl: pinned host copy of ctl[0 .. kOpsCtl) written by the launch (or null).
constexpr int kOpsBlockReads = 1024;
constexpr int kOpsCtl = 9;
constexpr int kOpsCtlAll = kOpsCtl + 2;
struct OpsCounts {
    const int32_t* fallback;   // [0]: exact-kernel reads of the chunk, [3]: look-back error flag
    const int32_t* redo;       // second band level reads (null: one level)
    const int32_t* band;       // reads that needed the DP (null: not the band path)
    int32_t direct;            // KernelArgs::redo_direct of the chunk (0: off)
    int32_t one_level;         // the chunk ran the 32-diagonal level alone: its DP reads go to ctl[7]
    int32_t prio;              // raise the compaction's issue priority (KernelArgs::tail_prio)
    const int32_t* exact;      // the wide level's give-ups: the exact kernel's reads (null: no wide level)
    const int32_t* seeded;     // the seeded reads (to the wide level, or the second level first; null: none)
    const int32_t* seeded_l2;  // of those, the ones the 32-diagonal level left to the wide level (null: it took none)
    const int32_t* seed_pad;   // entries the segment sort added to pair up odd segments (counted in seeded)
};
// The call's last chunk: the compaction also writes the chunk's records, run offsets and runs
// straight into the caller's page-locked buffers (no copies and no host round trip after it).
// The known alignment (KernelArgs::known2): its record, run count (nops flags) and runs, as the
// exact kernel left them for one read in a 1-read layout (ops_stride 1).
struct OpsKnown {
    const Stat* stat;     // null: off
    const int32_t* nops;
    const uint32_t* slots;
    const uint32_t* spill;
    int32_t slot;
};
struct OpsHostOut {
    const int4* dstats;   // the chunk's records in HBM (2 int4 per nw_stat); null: off
    int4* hstats;         // the caller's records of the chunk's reads
    int64_t* hoff;        // the caller's run offsets of the chunk's reads
    uint32_t* hops;       // the caller's run array (the call's offsets; null: records only)
    int64_t hcap;         // its words
};
hipError_t launch_ops_compact(const int32_t* nops, const uint32_t* slots, int slot, int64_t stride, const uint32_t* spill, int64_t n,
                              unsigned long long* status, unsigned epoch, int parity, int64_t* ctl, int64_t* ops_off,
                              uint32_t* staging, int64_t staging_cap, int32_t* opsctl, const OpsCounts& cnt,
                              hipStream_t s, int64_t* hctl = nullptr, const OpsHostOut* host = nullptr,
                              Stat* stats = nullptr, const OpsKnown* known = nullptr);

}  // namespace nw
