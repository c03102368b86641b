// nw_band.hip -- certified diagonal-band DP: the default aligner path.
//
// The exact kernel (nw_kernel.hip) fills every cell of the La x Lb matrix.  A
// CRISPResso read is a near-copy of its amplicon, so its optimal alignments stay
// within a few diagonals of the main one.  These kernels fill only a band of
// kBD = 32 diagonals [dlo, dlo + 31] around [min(0, Lb - La), max(0, Lb - La)]
// and then PROVE that the result is the full DP's result:
//
//   A path that visits a cell on diagonal d = j - i has left |d| residues of one
//   sequence unpaired on the way there, so it pairs at most
//       min(Lb - d, La)  (d > 0)   or   min(Lb, La + d)  (d < 0)
//   residues, and every pair scores at most the matrix maximum (EDNAFULL: 5) while
//   gaps cost >= 0.  Hence every alignment touching a diagonal outside the band
//   scores at most UB = maxsub * max(min(Lb - dhi - 1, La), min(Lb, La + dlo - 1)).
//   If the best in-band score S > UB, every optimal alignment -- and every
//   alignment tied with one -- lies inside the band.  All values the traceback
//   compares (the predecessor states of an optimal path, the start cells of the
//   last row/column with score S, the open/extend choices along the path) are
//   then values of in-band paths, which the banded DP computes exactly; values it
//   under-estimates are strictly below S and below the compared optimum.  So the
//   banded traceback, with the same tie rules, is the full DP's
//   traceback, bit for bit.
//
// Reads that fail the certificate (S <= UB: chimeras, off-target, large indels),
// whose pair's lengths span more than the band, or that hold IUPAC codes other
// than N go to the exact int32 kernel's fallback list.
//
// Layout / schedule:
//   * reads are sorted by length on the device (nw_band_segsort: 4096-read segments
//     sorted in LDS, placed by look-back); DP-list positions (2g, 2g+1) form pair g,
//     packed in int16x2
//     (read A low, B high) on one band that holds both reads' start and end
//     diagonals; the sort keeps the wavefront's pairs at similar lengths;
//   * one read pair per 16-lane DPP row, 4 pairs per wavefront; lane q owns
//     diagonals d0 = dlo + 2q and d0 + 1; the wave sweeps anti-diagonals t = i + j
//     and at each step every lane computes one cell (the diagonal whose parity
//     matches t).  Predecessors: diag = own lane two steps back, up / left = own
//     lane or its row neighbour one step back (DPP row_shr:1 / row_shl:1; the row
//     edge reads -inf = outside the band).  Groups run at tau = t - dlo + kBK, so
//     the step parity is wave-uniform;
//   * biased recurrence: values carry + t * E (t = anti-diagonal step), so X = max(Mo,
//     X_left), Y = max(Mo, Y_up) with no "- extend"; the diagonal's + 2E is in
//     the score table; Mo = M - (O - E);
//   * 4 traceback bits per cell and read, 4 steps per dword (byte planes of the
//     sign bits); per pair region: header, the M of each
//     diagonal's last cell (= the last row / last column cells), bits in tiles
//     [words / 4][lanes][4 words]: the fill writes 16 steps of a pair's lanes as one
//     contiguous dwordx4 row, an M run of the walk reads 16 steps of its diagonal
//     pair with one dwordx4 per lane;
//   * nw_band_walk: one wavefront per read: start cell from the W captures,
//     certificate, the run-based walk of nw_common.h over the band, strings.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "nw_common.h"

#define NW_CAND 8            // classify: exact-copy candidates compared together
#define NW_BAND_WALK_CPL 1   // gap-run cells per lane and round (a gap run inside the band is < W <= 64 cells)

namespace nw {

namespace {

typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 as_v(unsigned u) { return __builtin_bit_cast(s16x2, u); }
__device__ __forceinline__ unsigned as_u(s16x2 v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ unsigned pk(int lo, int hi) { return ((unsigned)lo & 0xffffu) | ((unsigned)hi << 16); }
__device__ __forceinline__ int half(unsigned w, int h) { return (int)(short)(w >> (16 * h)); }
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// The fill keeps every value + kBias16 (unsigned, -inf = 0): max is v_pk_max_u16 and
// a DPP lane without a source reads 0 (bound_ctrl) -- no "old" operand to set up.
// Sums and differences are the same bits as in the signed domain.
constexpr int kBias16 = 16384;
__device__ __forceinline__ unsigned max2(unsigned a, unsigned b) {
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ unsigned add2(unsigned a, unsigned b) { return as_u(as_v(a) + as_v(b)); }
__device__ __forceinline__ unsigned sub2(unsigned a, unsigned b) { return as_u(as_v(a) - as_v(b)); }
// DPP within 16-lane rows by S lanes; a lane without a source reads 0 (= -inf:
// outside the band).  S = 2 when two read pairs share a row (interleaved lanes).
template <int S>
__device__ __forceinline__ unsigned row_shr(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x110 + S, 0xf, 0xf, true);
}
template <int S>
__device__ __forceinline__ unsigned row_shl(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x100 + S, 0xf, 0xf, true);
}
__device__ __forceinline__ unsigned and_or(unsigned a, unsigned m, unsigned c) {
    unsigned d;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(m), "v"(c));
    return d;
}
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) { return ~wave_max_u32(~v); }

// The range [lb, ub) of each of K keys among n sorted keys (LDS): branch-free binary searches in
// lockstep, one step per power of two from top (the largest <= n; wave-uniform), so every key's two
// probes of a step are in flight together (K = 8: 16 LDS loads per round trip, not one)
template <int K>
__device__ __forceinline__ void sorted_ranges(const unsigned* skey, int n, const unsigned* key, int* lb, int* ub) {
#pragma unroll
    for (int t = 0; t < K; ++t) lb[t] = ub[t] = 0;
    for (int step = n > 0 ? 1 << (31 - __builtin_clz((unsigned)n)) : 0; step > 0; step >>= 1) {
#pragma unroll
        for (int t = 0; t < K; ++t) {
            const int pl = lb[t] + step, pu = ub[t] + step;
            const unsigned kl = skey[min(pl, n) - 1], ku = skey[min(pu, n) - 1];
            lb[t] = pl <= n && kl < key[t] ? pl : lb[t];
            ub[t] = pu <= n && ku <= key[t] ? pu : ub[t];
        }
    }
}

}  // namespace

// ---- geometry shared by fill, walk and host --------------------------------------
// Band of a read pair: it must hold both reads' start (diagonal 0's neighbourhood)
// and end diagonals (Lb - La); the spare diagonals are split evenly.  An empty
// read imposes nothing.  False when the band cannot hold them or both are empty.
__host__ __device__ inline bool band_geometry2(int La, int LbA, int LbB, int* dlo, int W = kBandDiags) {
    int lo0 = 0, hi0 = 0;
    if (LbA > 0) { lo0 = min(lo0, LbA - La); hi0 = max(hi0, LbA - La); }
    if (LbB > 0) { lo0 = min(lo0, LbB - La); hi0 = max(hi0, LbB - La); }
    const int extra = W - (hi0 - lo0 + 1);
    *dlo = 0;
    if ((LbA <= 0 && LbB <= 0) || extra < 0) return false;
    *dlo = lo0 - extra / 2;
    return true;
}
__host__ __device__ inline bool band_geometry(int La, int Lb, int* dlo) { return band_geometry2(La, Lb, Lb, dlo); }

namespace {

// band of W diagonals: L = W / 2 lanes per read pair, PR pairs per 16-lane DPP row
// (interleaved: pair = lane % PR, q = lane / PR within the row), PW pairs per wavefront.
// W = kWideDiags (the wide level): one pair per wavefront, lane q = the lane, neighbours
// through the wave-wide DPP shifts (wave_shr:1 / wave_shl:1; lane 0 / 63 read -inf).
template <int W> struct BandGeo {
    static constexpr bool Wide = W > 32;
    static constexpr int L = W / 2;
    static constexpr int PR = Wide ? 1 : 16 / L;
    static constexpr int PW = Wide ? 1 : 4 * PR;
    static constexpr int CapBytes = W * 4;
    __device__ static int q_of(int lane) { return Wide ? lane : (lane & 15) / PR; }
    __device__ static int grp_of(int lane) { return Wide ? 0 : (lane >> 4) * PR + (lane & 15) % PR; }
    __device__ static int src_of(int p) { return Wide ? 0 : (p / PR) * 16 + p % PR; }   // lane q = 0 of pair p
    // the left / upper neighbour's value one step back (0 = -inf past the band's edge)
    __device__ static unsigned shr(unsigned v) {
        if constexpr (Wide) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);   // wave_shr:1
        else return row_shr<PR>(v);
    }
    __device__ static unsigned shl(unsigned v) {
        if constexpr (Wide) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);   // wave_shl:1
        else return row_shl<PR>(v);
    }
};
constexpr int kBK = 64;               // tau = t - dlo + kBK: >= 0 and even
constexpr int kAPad = 80;             // amplicon codes: index i + kAPad, i in [-17, La + 48] (wide level: [-66, La + 102])
constexpr int kJPad = 95;             // pair codes: index j + kJPad, j in [-48, La + 80] (wide: [-66, La + 196]); j = 1 is 4-aligned
constexpr int kPadCode = 5;           // lut6: A T G C N pad
constexpr int kTabRows = NCODE;       // amplicon rows: every EDNAFULL code (IUPAC too) + pad/unknown
constexpr int kTabBytes = 2448;       // [17][36] packed scores
constexpr int kHdrBytes = 48;         // {tau0, dlo, flags, -}, {ra, rb, LbA, LbB}, {offA, offB}
constexpr int kPairInactive = 4;      // header flag: the pair was not filled (walk: empty / fallback)

__host__ __device__ inline int band_acd_elems(int La) { return La + kAPad + 112; }
__host__ __device__ inline int band_pcs(int La, int W) { return align16(La + kJPad + (W > 32 ? 208 : 96)); }

}  // namespace

// reads longer than La + W - 1 never enter a level of W diagonals (KernelArgs::band_lb_cap)
__host__ __device__ inline int band_words(int La, int Lb_max, int W = kBandDiags) {
    const int Lbm = Lb_max < La + W - 1 ? Lb_max : La + W - 1;
    return (((La + Lbm + 80) / 4 + 2) + 3) & ~3;   // column length: whole dwordx4 of the walk
}
// Stop summary (the first level, KernelArgs::band_summ): after a pair's tiles, per lane (diagonal
// pair q) one byte per 16 words (64 steps, four tile rows) -- the OR of the block's "M < max"
// bits, read A's four sub-steps in the low nibble, read B's in the high -- padded to 16 bytes
// per lane.  A lane walk's M run skips the blocks whose bits for its read and diagonal are clear.
__host__ __device__ inline int band_summ_bytes(int NW) { return ((((NW + 15) >> 4) + 15) & ~15); }

__host__ __device__ inline int64_t band_region_stride(int La, int Lb_max, int W) {
    const int NW = band_words(La, Lb_max, W > kBandDiags ? W : kBandDiags);
    return ((int64_t)kHdrBytes + 4 * W + (int64_t)NW * (W / 2) * 4 + (int64_t)(W / 2) * band_summ_bytes(NW) + 255) &
           ~(int64_t)255;
}

// Sort key of every read: its length bucket, or cap + 2 for a read identical to the
// amplicon (case-insensitive, A C G T only).  Such a read needs no DP: its full
// diagonal scores S = maxsub * La, every other alignment pairs at most La - 1
// residues (S > UB of the one-diagonal band, the certificate above), so the
// alignment is the diagonal and the start cell the corner: this kernel writes its
// strings and record right away, and the sort keeps it out of the band passes.
// Wavefront batches of 64 reads, kCand compares in flight; 4 bytes per lane and compare:
// (byte | 0x20) folds case, the amplicon's folded dwords are 0 at non-ACGT bases.
__device__ __forceinline__ unsigned ld_dw(const uint8_t* p) { return *(const unsigned*)p; }

#ifndef NW_NO_SUB3
#define NW_NO_SUB3 0   // A/B builds only (scripts/diag/build_variant.sh): classify without the 3-substitution certificate
#endif
#ifndef NW_NO_INDEL1
#define NW_NO_INDEL1 0   // ... without the one-indel certificate
#endif
constexpr int kIndelMax = 10;   // classify's one-indel certificate: gaps of at most this many residues
constexpr int kCand = NW_CAND; // exact-copy candidates compared together (2 dword loads each in flight)

// Reads of the amplicon's length with ONE substitution (A C G T against A C G T; ops output,
// an A C G T amplicon of at most 256 bp) need no DP either.  With k mismatches on the main
// diagonal its sum is D = m (La - 1) - x for k = 1 (m = maxsub, x = -mismatch = 4 m / 5).  Any
// alignment with an internal gap pairs at most La - 1 residues and pays at least the gap
// open O: <= m (La - 1) - O < D when O > x (EMBOSS's 10 vs 4, scaled).  One without is a
// single diagonal d with free end gaps: |d| >= 2 pairs at most La - 2 residues (m (La - 2) <
// D as m > x); d = +1 / -1 score m p - x (La - 1 - p) for p matches of their La - 1 pairs,
// below D exactly when p <= La - 2: each needs one mismatch (shifted byte compares, ballots).
// So the diagonal is the unique optimum; along it M(i, i) = D_i >= m i - m - x >= X(i, i),
// Y(i, i) (<= m (i - 1) - O), so M wins every traceback tie: the record is the diagonal's,
// as the exact copy's.  ~8 % of C2's reads (a third of the 1-3 substitution
// class and of the 1 % noise class) leave the DP this way.
__device__ __forceinline__ unsigned zero_bytes(unsigned x) {   // 0x80 in each zero byte of x
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
}

// Packed input (KernelArgs::pk_words): the 4 bases at batch position p as bytes A C T G (an
// exception's place reads as A: its read is flagged).  The stream's dword k holds positions
// pk_pos0 + 16 k .. + 15, 2 bits each; the device copy has a spare dword past its end.
__device__ __forceinline__ unsigned pk_decode4(const KernelArgs& a, long long p) {
    const long long q = p - a.pk_pos0;
    const unsigned* w = a.pk_words + (q >> 4);
    const unsigned x = __builtin_amdgcn_alignbit(w[1], w[0], (unsigned)(2 * (q & 15))) & 0xffu;
    const unsigned sel = (x | (x << 6) | (x << 12) | (x << 18)) & 0x03030303u;   // one code per byte
    return __builtin_amdgcn_perm(0u, 0x47544341u, sel);   // 0 1 2 3 -> 'A' 'C' 'T' 'G'
}

// the low 8 bits of x (4 bases) as bytes A C T G
__device__ __forceinline__ unsigned pk_expand(unsigned x) {
    x &= 0xffu;
    return __builtin_amdgcn_perm(0u, 0x47544341u, (x | (x << 6) | (x << 12) | (x << 18)) & 0x03030303u);
}

// pk_decode4 at a 4-aligned position (the four bases sit in one stream dword: one load)
__device__ __forceinline__ unsigned pk_decode4_al(const KernelArgs& a, long long p) {
    const long long q = p - a.pk_pos0;
    const unsigned x = (a.pk_words[q >> 4] >> (unsigned)(2 * (q & 15))) & 0xffu;
    const unsigned sel = (x | (x << 6) | (x << 12) | (x << 18)) & 0x03030303u;
    return __builtin_amdgcn_perm(0u, 0x47544341u, sel);
}

// First exception at or after batch position `pos` in [pk_e0, pk_e1): a 64-ary search by one
// wavefront (every lane samples a pivot; ~3 dependent loads for a million exceptions).
__device__ inline long long exc_lower_bound(const KernelArgs& a, long long pos, int lane) {
    long long lo = a.pk_e0, hi = a.pk_e1;
    while (hi - lo > 64) {
        const long long step = (hi - lo + 63) / 64;
        const long long idx = lo + lane * step;
        const bool below = idx < hi && a.pk_exc_pos[idx] < pos;
        const int k = (int)__builtin_popcountll(__ballot(below));   // pivots below pos: lanes 0 .. k - 1
        const long long nlo = k == 0 ? lo : lo + (long long)(k - 1) * step + 1;
        hi = min(hi, lo + (long long)k * step);
        lo = nlo;
    }
    const long long idx = lo + lane;
    const bool below = idx < hi && a.pk_exc_pos[idx] < pos;
    return lo + (long long)__builtin_popcountll(__ballot(below));
}

// (classify and nw_band_cert) the bases 16 t + i < len of a 2-bit word (one bit per base)
__device__ __forceinline__ unsigned vmask16(int t, int len) {
    const int b = len - 16 * t;
    return b >= 16 ? 0x55555555u : (b <= 0 ? 0u : 0x55555555u >> (32 - 2 * b));
}
// 16 bases of the packed stream from batch position p
__device__ __forceinline__ unsigned pk_word16(const KernelArgs& a, long long p) {
    const long long q = p - a.pk_pos0;
    const unsigned* w = a.pk_words + (q >> 4);
    return __builtin_amdgcn_alignbit(w[1], w[0], (unsigned)(2 * (q & 15)));
}
// 16 bases of the amplicon from position p (its 2-bit words in LDS)
__device__ __forceinline__ unsigned amp_word16(const unsigned* amp2s, int p) {
    return __builtin_amdgcn_alignbit(amp2s[(p >> 4) + 1], amp2s[p >> 4], (unsigned)(2 * (p & 15)));
}
// A lane's read of the amplicon's length at batch position my_off: its 2-bit words shifted to base 0
// (rw[16] = 0; bases past the read are masked by the users); c: the lane holds such a read
__device__ __forceinline__ void load_read_words(const KernelArgs& a, bool c, long long my_off, unsigned (&rw)[17]) {
    const int nw = (a.La + 15) >> 4;   // <= 16
    const long long q0 = my_off - a.pk_pos0;
    const unsigned* src = a.pk_words + (q0 >> 4);
    const unsigned s2 = (unsigned)(2 * (q0 & 15));
    unsigned wd[17];
#pragma unroll
    for (int t = 0; t < 17; ++t) wd[t] = c && t <= nw ? src[t] : 0u;   // <= the read's last dword + 1
#pragma unroll
    for (int t = 0; t < 16; ++t) rw[t] = __builtin_amdgcn_alignbit(wd[t + 1], wd[t], s2);
    rw[16] = 0u;
}
// Its main diagonal against the amplicon's words (LDS): mismatches k, the first, second and last
// mismatching base (-1: none)
__device__ __forceinline__ void main_diag_mism(const unsigned (&rw)[17], const unsigned* amp2s, int La, int* k_, int* f_,
                                               int* f2_, int* l_) {
    const int nw = (La + 15) >> 4;
    int k = 0, f = -1, f2 = -1, l = -1;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        if (t >= nw) continue;
        const unsigned x = rw[t] ^ amp2s[t];
        const unsigned m = (x | (x >> 1)) & vmask16(t, La);
        k += __builtin_popcount(m);
        if (m != 0u && f >= 0 && f2 < 0) f2 = 16 * t + (__builtin_ctz(m) >> 1);
        if (m != 0u && f < 0) {
            f = 16 * t + (__builtin_ctz(m) >> 1);
            const unsigned m2 = m & (m - 1u);
            if (m2 != 0u) f2 = 16 * t + (__builtin_ctz(m2) >> 1);
        }
        if (m != 0u) l = 16 * t + ((31 - __builtin_clz(m)) >> 1);
    }
    *k_ = k;
    *f_ = f;
    *f2_ = f2;
    *l_ = l;
}

// The three-substitution certificate's per-read checks (i)-(iii) (classify, below; lanes s3: reads of the
// amplicon's length with three mismatches on the main diagonal, at bases f < f2 < l; the caller checked
// sub3_ok).  Called by the whole wavefront; fact: the wavefront's LDS for the diagonals' mismatch places
// (kSub3FactWords).  The diagonal loop stays rolled (its scans unrolled once: the kernel's code fits the
// instruction cache), the facts the pair test (ii) needs go through LDS.
constexpr int kSub3FactWords = 14 * 64;   // diagonals -3 .. 3: first two | last two mismatches, per lane
__device__ __forceinline__ bool cert_sub3(const KernelArgs& a, const unsigned* amp2s, const unsigned (&rw)[17], bool s3,
                                          int f, int f2, int l, long long my_off, unsigned* fact) {
    const int La = a.La, nw = (La + 15) >> 4, sc5 = a.band_maxsub / 5, lane = threadIdx.x & 63;
    const int m3 = a.band_maxsub, x3 = 4 * sc5, O3 = a.gap_open, D3 = 3 * (m3 + x3);
    // jogs (iii): diagonals +-1 against the 16 read bases from f + 1 (up to l - 1), one
    // word each from the packed stream (random sequence mismatches there; a read whose
    // diagonals +-1 match all 16 is left to the DP)
    bool jog_in[2] = {false, false};
    if (s3) {
        const int len = min(16, l - f - 1);
        const unsigned lm = len <= 0 ? 0u : (len >= 16 ? 0x55555555u : (0x55555555u >> (32 - 2 * len)));
        const unsigned rd = pk_word16(a, my_off + f + 1);
        const unsigned zp = rd ^ amp_word16(amp2s, f), zm = rd ^ amp_word16(amp2s, f + 2);   // d = +1 / -1
        jog_in[1] = ((zp | (zp >> 1)) & lm) != 0u;
        jog_in[0] = ((zm | (zm >> 1)) & lm) != 0u;
    }
    bool ok3 = s3;
    // per diagonal d = -5 .. 5: mismatches (capped at 3), the first two and the last two (read index;
    // last ones + 1) over the diagonal's pairs; (i) single diagonals 1 <= |d| <= 5 need more than
    // (3 (m + x) - m |d|) / (m + x) mismatches each
#pragma unroll 1
    for (int d = -5; d <= 5; ++d) {
        int a1 = f, a2 = f2, b1 = l + 1, b2 = f2 + 1;   // d = 0: the main diagonal's three (k == 3)
        if (d != 0) {
            const int sh = d > 0 ? d : -d;
            a1 = La; a2 = La; b1 = 0; b2 = 0;
            // the first two and the last two by scans from either end that stop once every lane has
            // found two (random sequence: within a word); the count up to 3 follows (3 when the
            // second-last lies past the second)
            auto word = [&](int t) -> unsigned {
                // d > 0: read base j = i + d against amplicon base i (words of i); d < 0: read
                // base j against amplicon base j - d (words of j)
                const unsigned am = d > 0 ? amp2s[t]
                                          : __builtin_amdgcn_alignbit(amp2s[t + 1], amp2s[t], (unsigned)(2 * sh));
                const unsigned rd = d > 0 ? __builtin_amdgcn_alignbit(rw[t + 1], rw[t], (unsigned)(2 * sh)) : rw[t];
                const unsigned z = rd ^ am;
                return (z | (z >> 1)) & vmask16(t, La - sh);
            };
            const int o0 = d > 0 ? d : 0;   // read index of a word's base 0, past 16 t
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                if (__ballot(s3 && a2 == La && t < nw) == 0ull) break;
                const unsigned mk = word(t);
                const int off = 16 * t + o0;
                if (mk != 0u && a1 == La) {
                    a1 = off + (__builtin_ctz(mk) >> 1);
                    const unsigned m2 = mk & (mk - 1u);
                    if (m2 != 0u) a2 = off + (__builtin_ctz(m2) >> 1);
                } else if (mk != 0u && a2 == La) {
                    a2 = off + (__builtin_ctz(mk) >> 1);
                }
            }
#pragma unroll
            for (int t = 15; t >= 0; --t) {
                if (__ballot(s3 && b2 == 0 && a1 < La) == 0ull) break;
                if (t >= nw) continue;
                const unsigned mk = word(t);
                const int off = 16 * t + o0;
                if (mk != 0u && b1 == 0) {
                    const int hb = 31 - __builtin_clz(mk);
                    b1 = off + (hb >> 1) + 1;
                    const unsigned mh = mk & ~(1u << hb);
                    if (mh != 0u) b2 = off + ((31 - __builtin_clz(mh)) >> 1) + 1;
                } else if (mk != 0u && b2 == 0) {
                    b2 = off + ((31 - __builtin_clz(mk)) >> 1) + 1;
                }
            }
            // (|d| >= 4: the score test needs one mismatch, no pair test reads the diagonal)
            const int cc = a1 == La ? 0 : (a2 == La ? 1 : (b2 > a2 ? 3 : 2));
            ok3 = ok3 && m3 * sh + (m3 + x3) * cc > D3;
        }
        if (d >= -3 && d <= 3) {
            fact[(d + 3) * 128 + lane] = (unsigned)a1 | ((unsigned)a2 << 16);
            fact[(d + 3) * 128 + 64 + lane] = (unsigned)b1 | ((unsigned)b2 << 16);
        }
    }
    // (ii) one gap, prefix on d1, suffix on d2 (|d| <= 3), with at most w_max mismatches in all: it exists
    // iff, in read coordinates, the prefix's mismatches on d1 end before the suffix's on d2 begin (the
    // suffix starts max(0, d2 - d1) read bases later: those are the gap's)
    unsigned fa[7], fb[7];
#pragma unroll
    for (int e = 0; e < 7; ++e) {
        fa[e] = fact[e * 128 + lane];
        fb[e] = fact[e * 128 + 64 + lane];
    }
#pragma unroll
    for (int e1 = 0; e1 < 7; ++e1) {
#pragma unroll
        for (int e2 = 0; e2 < 7; ++e2) {
            if (e1 == e2) continue;
            const int d1 = e1 - 3, d2 = e2 - 3, g = d2 > d1 ? d2 - d1 : d1 - d2;
            // unpaired residues of the amplicon (= of the read): its leading / trailing overhang
            // and the gap's residues when the gap is in the read (the diagonal falls)
            const int U = (d1 < 0 ? -d1 : 0) + (d2 > 0 ? d2 : 0) + (d1 > d2 ? d1 - d2 : 0);
            const int slack = D3 - m3 * U - O3 - (g - 1) * a.gap_extend;   // (m + x) w must not exceed it
            if (slack < 0) continue;
            const int wmax = slack / (m3 + x3);
            const int gb = d2 > d1 ? d2 - d1 : 0;   // read bases in the gap
            const int df1 = (int)(fa[e1] & 0xffffu), df2 = (int)(fa[e1] >> 16);
            const int dg1 = (int)(fb[e2] & 0xffffu), dg2 = (int)(fb[e2] >> 16);
            bool exists = dg1 - gb <= df1;
            if (wmax >= 1) exists = exists || dg2 - gb <= df1 || dg1 - gb <= df2;
            if (wmax >= 2) exists = true;   // (not reached with the gate's parameters: reject)
            ok3 = ok3 && !exists;
        }
    }
    // (iii) jogs through d = +-1: a mismatch of that diagonal in [f + 1, l - 1] (read index)
    return ok3 && l - f >= 2 && jog_in[0] && jog_in[1];
}

// The one-indel certificate (classify, below; lanes ci: reads of La -+ kab bases, 1 <= kab <= the
// certificate's largest gap, at batch position my_off).  True: certified, *gk_ the gap's read index q
// (runs M q, the gap, M the rest).  Called by the whole wavefront.
__device__ __forceinline__ bool cert_indel(const KernelArgs& a, const unsigned* amp2s, bool ci, long long my_off, int my_len,
                                           int* gk_) {
    const int La = a.La, n2 = (La + 15) / 16 + 2, sc5 = a.band_maxsub / 5;
    const int dl = my_len - La, kab = dl < 0 ? -dl : dl;
    const bool del = dl < 0;
    const int Ls = del ? my_len : La, Ll = del ? La : my_len;
    unsigned rw[18];
    {
        const long long q0 = my_off - a.pk_pos0;
        const unsigned* src = a.pk_words + (q0 >> 4);
        const unsigned s2 = (unsigned)(2 * (q0 & 15));
        const int nrw = (my_len + 15) >> 4;
        unsigned wd[18];
#pragma unroll
        for (int t = 0; t < 18; ++t) wd[t] = ci && t <= nrw ? src[t] : 0u;
#pragma unroll
        for (int t = 0; t < 17; ++t) rw[t] = __builtin_amdgcn_alignbit(wd[t + 1], wd[t], s2);
        rw[17] = 0u;
    }
    auto vmask = [](int t, int len) -> unsigned {   // bases 16 t + i < len
        const int b = len - 16 * t;
        return b >= 16 ? 0x55555555u : (b <= 0 ? 0u : 0x55555555u >> (32 - 2 * b));
    };
    const int mm = a.band_maxsub, xx = 4 * sc5;
    const int S = mm * Ls - a.gap_open - (kab - 1) * a.gap_extend;
    bool ok = false;
    int gk = 0;
    // the longer sequence l and the shorter s: the amplicon's words from LDS, the read's from
    // registers, picked per lane (deletion and insertion reads in one pass over the shifts)
    if (ci) {
        auto am = [&](int t) -> unsigned { return t < n2 ? amp2s[t] : 0u; };
        auto wl = [&](int t) -> unsigned { return del ? am(t) : rw[t]; };
        auto ws = [&](int t) -> unsigned { return del ? rw[t] : am(t); };
        bool o = true;
        // first and last mismatch of a shift (one side's sequence shifted by sh against the
        // other's, P positions): scans from either end that stop as soon as every lane has found
        // one (random sequence mismatches within a word; only the two diagonals of the
        // candidate run to the gap).  Mismatches: 0 (f == P), 1 (f == g - 1) or >= 2 -- all the
        // score test needs (its bound falls with the count)
        auto ends = [&](auto lw, auto rw2, int sh, int P, int* f, int* g) {
            int ff = P, gg = 0;
#pragma unroll
            for (int t = 0; t < 17; ++t) {
                if (__ballot(ff == P && 16 * t < P) == 0ull) break;
                const unsigned z = __builtin_amdgcn_alignbit(lw(t + 1), lw(t), (unsigned)(2 * sh)) ^ rw2(t);
                const unsigned mk = (z | (z >> 1)) & vmask(t, P);
                ff = (ff == P && mk != 0u) ? 16 * t + (int)(__builtin_ctz(mk) >> 1) : ff;
            }
#pragma unroll
            for (int t = 16; t >= 0; --t) {
                if (__ballot(gg == 0 && ff < P) == 0ull) break;   // (words past P: mk == 0)
                const unsigned z = __builtin_amdgcn_alignbit(lw(t + 1), lw(t), (unsigned)(2 * sh)) ^ rw2(t);
                const unsigned mk = (z | (z >> 1)) & vmask(t, P);
                gg = (gg == 0 && mk != 0u) ? 16 * t + (int)((31 - __builtin_clz(mk)) >> 1) + 1 : gg;
            }
            *f = ff;
            *g = gg;
        };
        auto cnt = [](int f, int g, int P) { return f == P ? 0 : (f == g - 1 ? 1 : 2); };
        // shifts sh = 0 .. kab + 3 of l; for sh <= kab the pair test G[s2] > F[s1] (s1 < s2) as a
        // running maximum of F: every earlier shift's for s2 < kab, shifts 1 .. kab - 1 for s2 =
        // kab (the pair (0, kab) is the candidate).  F / G are indices of s, P = Ls there.
        // the shifts past kab and the other side's need only enough mismatches for the score test
        // (the smallest c with m (P - c) - x c < S, 0 .. 2; more: the DP): forward scans that stop
        // once that many are found
        auto enough = [&](auto lw, auto rw2, int sh, int P) -> bool {
            int need = 0;
            while (need <= 2 && !(mm * (P - need) - xx * need < S)) ++need;
            int c = 0;
#pragma unroll
            for (int t = 0; t < 17; ++t) {
                if (__ballot(c < need && need <= 2 && 16 * t < P) == 0ull) break;
                const unsigned z = __builtin_amdgcn_alignbit(lw(t + 1), lw(t), (unsigned)(2 * sh)) ^ rw2(t);
                c += c < need ? __builtin_popcount((z | (z >> 1)) & vmask(t, P)) : 0;
            }
            return need <= 2 && c >= need;
        };
        int f0 = Ls, fmax_all = -1, fmax_1 = -1;
        for (int sh = 0; sh <= kab; ++sh) {
            int f, g;
            ends(wl, ws, sh, Ls, &f, &g);
            const int c = cnt(f, g, Ls);
            o = o && mm * (Ls - c) - xx * c < S;
            if (sh == 0) f0 = f;
            if (sh > 0) o = o && g > (sh == kab ? fmax_1 : fmax_all);
            if (sh == kab) gk = g;
            fmax_all = max(fmax_all, f);
            if (sh > 0) fmax_1 = max(fmax_1, f);
        }
        for (int sh = kab + 1; sh <= kab + 3; ++sh) o = o && enough(wl, ws, sh, Ll - sh);
        for (int sh = 1; sh <= 3; ++sh) o = o && enough(ws, wl, sh, Ls - sh);   // s shifted against l
        ok = ci && o && gk >= 1 && gk <= f0;
    }
    *gk_ = gk;
    return ok;
}

// Packed input: the bytes of the reads in dp (the lanes' reads at my_off, my_len; the whole wavefront)
// decoded into a.reads -- each read's own bytes exactly (neighbouring reads' bytes are never written by
// another read's wavefront: no races between blocks)
__device__ __forceinline__ void write_read_bytes(const KernelArgs& a, unsigned long long dp, long long my_off, int my_len) {
    const int lane = threadIdx.x & 63;
    // kWr reads at a time, lane l their dwords l, l + 64, ...: all their loads in flight
    // before any store (one read per round trip measured 2.7x the byte-input classify)
    constexpr int kWr = 8;
    uint8_t* dst = const_cast<uint8_t*>(a.reads);
    while (dp) {
        long long o[kWr], e[kWr];
        int rounds = 0;
#pragma unroll
        for (int t = 0; t < kWr; ++t) {
            o[t] = e[t] = 0;
            if (dp) {
                const int u = (int)__builtin_ctzll(dp);
                dp &= dp - 1;
                const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)my_off, u);
                const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(my_off >> 32), u);
                o[t] = (long long)(((unsigned long long)hi << 32) | lo);
                e[t] = o[t] + __builtin_amdgcn_readlane(my_len, u);
                const int span = (int)(e[t] - (o[t] & ~3ll));
                rounds = max(rounds, (span + 255) >> 8);
            }
        }
        for (int rd2 = 0; rd2 < rounds; ++rd2) {
            unsigned v[kWr];
#pragma unroll
            for (int t = 0; t < kWr; ++t) {
                const long long p = (o[t] & ~3ll) + 256 * rd2 + 4 * lane;
                v[t] = p < e[t] ? pk_decode4_al(a, p) : 0u;
            }
#pragma unroll
            for (int t = 0; t < kWr; ++t) {
                const long long p = (o[t] & ~3ll) + 256 * rd2 + 4 * lane;
                if (p >= e[t]) continue;
                if (p >= o[t] && p + 4 <= e[t]) {
                    *(unsigned*)(dst + p) = v[t];
                } else {
                    for (int b = 0; b < 4; ++b)
                        if (p + b >= o[t] && p + b < e[t]) dst[p + b] = (uint8_t)(v[t] >> (8 * b));
                }
            }
        }
    }
}


// (5 wavefronts per SIMD; forced to 6 / 8 with 31 / 60 VGPRs spilled it ran 0.188 / 0.223 vs 0.150 ms per resident
// pass in round 5)
#ifndef NW_CLASSIFY_WPE
#define NW_CLASSIFY_WPE 5
#endif
template <bool PK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NW_CLASSIFY_WPE))) void nw_band_classify(const KernelArgs a) {
    extern __shared__ unsigned amp_sh[];   // [nd] folded amplicon dwords (0 at non-ACGT), [nd] raw dwords
    constexpr int kRbw = 66;               // a window read's 16-base words (Lb < La <= 1024) + a zero word
    __shared__ unsigned s_rbw[4][kRbw];
    __shared__ unsigned s_known[18];       // the known sequence's 2-bit words (KernelArgs::known2; La <= 256)
    const int La = a.La, nd = (La + 3) / 4;
    // the chunk's counters (fallback / redo counts, spill bump and error flag): zeroed
    // here, the first kernel of the chain, instead of by memset launches
    if (blockIdx.x == 0 && threadIdx.x < 16) a.fallback_count[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x < 2 && a.ops) a.ops_ctl[threadIdx.x] = 0;
    if (blockIdx.x == 0 && a.zero_ctl64 && (int)threadIdx.x < a.zero_ctl64_n) a.zero_ctl64[threadIdx.x] = 0;
    // packed input, block b: the chunk's reads of call block B = call_lo / kPkBlock + b, [bl, bh)
    // (kPkBlock reads, one per thread; four blocks per group of kLenGroup lengths).  Its lengths'
    // loads go out before the image copy's barrier.
    constexpr int kPkBlock = 256;
    static_assert(kLenGroup % kPkBlock == 0, "blocks tile the length groups");
    const long long pB = a.pk_call_lo / kPkBlock + blockIdx.x;
    const long long pbl = max(0ll, pB * kPkBlock - a.pk_call_lo), pbh = min(a.n, (pB + 1) * kPkBlock - a.pk_call_lo);
    const long long pG = pB * kPkBlock / kLenGroup, pg0 = pG * kLenGroup;
    const long long prr = pB * kPkBlock + threadIdx.x - a.pk_call_lo;   // chunk-relative
    long long pk_l = 0, pk_pre = 0;   // this thread's read length; the group's lengths before the block (<= 3 per thread)
    if (PK && a.pk_len) {
        pk_l = prr < pbh ? (long long)a.pk_len[pB * kPkBlock + threadIdx.x] : 0ll;
        for (long long q = pg0 + threadIdx.x; q < pB * kPkBlock; q += kPkBlock) pk_pre += a.pk_len[q];
    }
    // the amplicon's folded and raw dwords and the window seeds: the host-built image, one copy
    // (the byte-input launch sizes LDS for the amplicon dwords only: no window seeds there)
    const int img_words = PK ? a.cls_words : 2 * nd;
    for (int k = threadIdx.x; k < img_words; k += blockDim.x) amp_sh[k] = a.cls_img[k];
    if (PK && a.known2 && threadIdx.x < 18) s_known[threadIdx.x] = threadIdx.x < (La + 15) / 16 ? a.known2[threadIdx.x] : 0u;
    __syncthreads();
    const int sc5 = a.band_maxsub / 5;
    // the one-substitution certificate (above): ops output, one 256-byte chunk, EDNAFULL's
    // 5 / -4 scaled, a gap open above the mismatch cost
    const bool amp_acgt_all = a.amp_acgt != 0;
    const bool sub1_ok = amp_acgt_all && a.ops && nd <= 64 && a.band_maxsub == 5 * sc5 && a.gap_open > 4 * sc5 &&
                         a.gap_extend >= 0;
    // two substitutions (x = 9/5 maxsub: a mismatch's loss against a match, D = m La - 2 x): with an
    // internal gap and <= La - 2 pairs O > 2 x - 2 m; La - 1 pairs and two gaps 2 O > 2 x - m, one gap
    // and a mismatch O > x - m; |d| >= 4 m (La - 4) < D: x < 2 m; d = +-1 / +-2 / +-3 need 2 / 1 / 1
    // mismatches (EDNAFULL); one gap, one end gap, no mismatch: excluded per read (below)
    const int mt2 = a.band_maxsub, xl = 9 * sc5;
    const bool sub2_ok = sub1_ok && 2 * a.gap_open > 2 * xl - mt2 && a.gap_open > 2 * xl - 2 * mt2 &&
                         a.gap_open > xl - mt2 && xl < 2 * mt2 && (2 * xl - mt2) / xl + 1 == 2 &&
                         (2 * xl - 2 * mt2) / xl + 1 == 1 && (2 * xl - 3 * mt2) / xl + 1 == 1;
    // one indel of k residues (below): certified for k <= indel_kmax, the largest k with m > (k - 1) E (no
    // alternative leaves a read or amplicon residue unpaired or mismatched), O > (k - 1) E (no alternative
    // with two internal gaps) and O + (k - 1) E < 4 m (no single diagonal pairing four residues fewer)
    int indel_kmax = 0;
    if (PK && !NW_NO_INDEL1 && sub1_ok && a.amp2)
        for (int k = 1; k <= kIndelMax; ++k) {
            const int p = (k - 1) * a.gap_extend;
            if (!(a.band_maxsub > p && a.gap_open > p && a.gap_open + p < 4 * a.band_maxsub)) break;
            indel_kmax = k;
        }
    // three substitutions (below): with D = m La - 3 (m + x), every alignment but the diagonal scores below
    // D when, beyond the per-read checks, x < m (|d| >= 6), 4 m + O, 2 m + 2 O and 3 O exceed 3 (m + x)
    // (one gap leaving 4 or more residues unpaired, two gaps leaving 2, three gaps) and a jog through a
    // neighbouring diagonal (two gaps, one residue of each sequence unpaired) with one mismatch scores below D
    const int m3 = a.band_maxsub, x3 = 4 * sc5, O3 = a.gap_open, D3 = 3 * (m3 + x3);
    const bool sub3_ok = !NW_NO_SUB3 && sub2_ok && x3 < m3 && 4 * m3 + O3 > D3 && 2 * m3 + 2 * O3 > D3 && 3 * O3 > D3 &&
                         m3 + 2 * O3 + (m3 + x3) > D3;
    const int lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
    const unsigned tail_mask = (La & 3) ? (0xffffffffu >> (8 * (4 - (La & 3)))) : 0xffffffffu;
    const int sd = (int)(a.stride / 4);
    // Window reads (packed input, ops output): a read shorter than the amplicon that equals one of its
    // windows amplicon[s, s + Lb) (A C G T, case-insensitive) scores m Lb, the most any alignment can
    // (pairs <= Lb, each <= m; a gap costs > 0), and every alignment that does is such a window: the
    // start-cell scan (last column bottom -> top) takes the largest such s, and along its diagonal M =
    // m j beats X, Y <= m j - O, so the traceback is the diagonal with free end gaps: s amplicon
    // residues before, La - s - Lb after.  One substitution (D = m (Lb - 1) - x): an alignment with an
    // internal gap pairs <= Lb residues and pays >= O, <= m Lb - O < D when O > m + x; a single
    // diagonal pairs its overlap P(d): P <= Lb - 2 scores <= m (Lb - 2) < D (m > x), P = Lb - 1 needs one
    // mismatch and P = Lb two (checked for every such diagonal, below) -- D is then the unique optimum
    // and M wins every tie along it (X, Y <= m j - O < m j - m - x <= M).  The window's offset comes from
    // the read's first (or, for a substitution there, last) 16 bases looked up among the amplicon's
    // sorted 16-mers (Profile::seed_key).
    unsigned* amp2s = amp_sh + 2 * nd;
    const int n2 = (La + 15) / 16 + 2, nseed = a.n_seed;
    unsigned* skey = amp2s + n2;
    uint16_t* spos = (uint16_t*)(skey + nseed);
    const bool win_ok = PK && amp_acgt_all && a.ops && a.band_maxsub == 5 * sc5 && a.gap_extend >= 0 && a.amp2 &&
                        a.gap_open > xl && nseed > 0 && La <= 1024;
    // 16 bases of the packed stream from batch position p, and of the amplicon from position p (LDS)
    auto rword = [&](long long p) -> unsigned {
        const long long q = p - a.pk_pos0;
        const unsigned* w = a.pk_words + (q >> 4);
        return __builtin_amdgcn_alignbit(w[1], w[0], (unsigned)(2 * (q & 15)));
    };
    auto aword = [&](int p) -> unsigned {
        return __builtin_amdgcn_alignbit(amp2s[(p >> 4) + 1], amp2s[p >> 4], (unsigned)(2 * (p & 15)));
    };
    // mismatches of read bases [roff + j0, + len) against amplicon [s, s + len), counted up to cap + 1:
    // 16 words (256 bases) per round with every load in flight before any compare
    auto mism = [&](long long roff, int j0, int s, int len, int cap) -> int {
        int cnt = 0;
        for (int w0 = 0; w0 < len && cnt <= cap; w0 += 256) {
            unsigned x[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) x[t] = w0 + 16 * t < len ? rword(roff + j0 + w0 + 16 * t) : 0u;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int w = w0 + 16 * t;
                if (w >= len) continue;
                unsigned y = x[t] ^ aword(s + w);
                if (len - w < 16) y &= (1u << (2 * (len - w))) - 1u;
                cnt += __builtin_popcount((y | (y >> 1)) & 0x55555555u);
            }
        }
        return cnt;
    };
    auto ham16 = [&](unsigned x, unsigned y) { const unsigned z = x ^ y; return __builtin_popcount((z | (z >> 1)) & 0x55555555u); };
    // a wavefront batch of the 64 reads r0 .. r0 + 63 (below r_end): lane u holds read r0 + u's
    // offset and length; exc: the reads holding an exception byte (packed input)
    auto batch = [&](long long r0, long long r_end, long long my_off, int my_len, bool exc) {
        const long long r = r0 + lane;
        unsigned long long cand = __ballot(my_len == La && !exc);   // reads of the amplicon's length
        unsigned long long exact = 0ull, sub1 = 0ull, sub2 = 0ull;
        unsigned long long pend3 = 0ull, pend_i = 0ull;   // queued for nw_band_cert (KernelArgs::cert_q)
        unsigned long long known = 0ull;   // copies of the known sequence (KernelArgs::known2)
        unsigned long long jog = 0ull;     // reads closer to the known sequence than to the amplicon (below)
        // compare kCand candidates at a time (their loads in flight together); when the read
        // fits one 256-byte chunk (La <= 256) its exact copy's rows are written right
        // away from the words already in registers
        const bool one_chunk = nd <= 64;
        unsigned long long emit_later = 0ull;
        if constexpr (PK) {
            // Packed input, ops output, an A C G T amplicon of at most 256 bp: one read per lane.  Its
            // 2-bit words (one shift of the stream's dwords) against the amplicon's give the
            // mismatches of the main diagonal; a read with one or two takes the certificates above
            // from the shifted diagonals' masks (the wave-per-candidate loop below decides the same
            // from byte compares).  Mismatch masks: one bit per base (bit 2 i of word t: base 16 t + i).
            if (a.ops && one_chunk && amp_acgt_all && a.amp2 && cand) {
                const bool c = ((cand >> lane) & 1ull) != 0ull;
                cand = 0ull;
                const int nw = (La + 15) >> 4;   // <= 16
                auto vmask = [](int t, int len) -> unsigned {   // bases 16 t + i < len
                    const int b = len - 16 * t;
                    return b >= 16 ? 0x55555555u : (b <= 0 ? 0u : 0x55555555u >> (32 - 2 * b));
                };
                unsigned rw[17];
                load_read_words(a, c, my_off, rw);
                int k, f, f2, l;   // mismatches of the main diagonal, first, second and last base
                main_diag_mism(rw, amp2s, La, &k, &f, &f2, &l);
                exact = __ballot(c && k == 0);
                const bool s1 = c && sub1_ok && k == 1, s2 = c && sub2_ok && k == 2;
                // diagonal d = sgn * sh (q <= La - 1 - sh): mismatches (counted up to 2), any at q >= qa, any at q <= qb
                auto shifted = [&](int sgn, int sh, int qa, int qb, int* tot, bool* ge, bool* le) {
                    int n = 0;
                    unsigned g = 0u, e = 0u;
#pragma unroll
                    for (int t = 0; t < 16; ++t) {
                        if (t >= nw) continue;
                        const unsigned am = sgn > 0 ? amp2s[t]
                                                    : __builtin_amdgcn_alignbit(amp2s[t + 1], amp2s[t], (unsigned)(2 * sh));
                        const unsigned rd = sgn > 0 ? __builtin_amdgcn_alignbit(rw[t + 1], rw[t], (unsigned)(2 * sh)) : rw[t];
                        const unsigned x = rd ^ am;
                        const unsigned m = (x | (x >> 1)) & vmask(t, La - sh);
                        n += __builtin_popcount(m);
                        g |= m & ~vmask(t, qa);      // bases >= qa
                        e |= m & vmask(t, qb + 1);   // bases <= qb
                    }
                    *tot = n;
                    *ge = g != 0u;
                    *le = e != 0u;
                };
                if (__ballot(s1 || s2)) {
                    // S_+-1 below D: one mismatch on each (k = 1); two substitutions at bases f < l: two on
                    // each, d = +1 one at q >= f and one at q <= l - 2, d = -1 at q >= f + 1 and q <= l - 1
                    int tp, tm;
                    bool gp, lp, gm, lm;
                    shifted(1, 1, f, l - 2, &tp, &gp, &lp);
                    shifted(-1, 1, f + 1, l - 1, &tm, &gm, &lm);
                    sub1 = __ballot(s1 && tp >= 1 && tm >= 1);
                    bool ok2 = s2 && tp >= 2 && tm >= 2 && gp && lp && gm && lm;
                    if (__ballot(ok2)) {   // d = +-2, +-3: one mismatch each
#pragma unroll
                        for (int sh = 2; sh <= 3; ++sh) {
                            int t2, t3;
                            bool x0, x1;
                            shifted(1, sh, 0, La, &t2, &x0, &x1);
                            shifted(-1, sh, 0, La, &t3, &x0, &x1);
                            ok2 = ok2 && t2 >= 1 && t3 >= 1;
                        }
                    }
                    sub2 = __ballot(ok2);
                }
                // Three substitutions (round 6; bases f < f2 < l of the main diagonal, D = m La - 3 (m + x)).
                // An alignment scores m (La - U) - (m + x) w - (its gaps' cost), U residues of each sequence
                // unpaired and w mismatches; below D when m U + (m + x) w + gaps > 3 (m + x).  Left open by
                // the gate above: (i) single diagonals 1 <= |d| <= 5 with too few mismatches (each must have
                // more than (3 (m + x) - m |d|) / (m + x)); (ii) one gap between diagonals d1 (prefix) and d2
                // (suffix), |d1|, |d2| <= 3, with at most w_max mismatches in all -- it exists iff, in read
                // coordinates, the prefix's mismatches on d1 end before the suffix's on d2 begin (the suffix
                // starts max(0, d2 - d1) read bases later: those are the gap's); (iii) a jog 0 -> +-1 -> 0
                // with no mismatch: its middle covers the read bases (f, l] (d = +1) / [f, l) (d = -1), so a
                // mismatch of that diagonal in [f + 1, l - 1] excludes both.  Then the diagonal is the unique
                // optimum and M beats X and Y along it (a tie would be a second alignment scoring D).  The checks
                // (cert_sub3) run in nw_band_cert, on the queued candidates.
                const bool s3 = c && sub3_ok && k == 3;
                pend3 = __ballot(s3);   // checked by nw_band_cert
                if (a.known2) {   // a copy of the known sequence that no certificate above took
                    int k2 = 0;
#pragma unroll
                    for (int t = 0; t < 16; ++t) {
                        if (t >= nw) continue;
                        const unsigned x = rw[t] ^ s_known[t];
                        k2 += __builtin_popcount((x | (x >> 1)) & vmask(t, La));
                    }
                    known = __ballot(c && k != 0 && k2 == 0) & ~(sub1 | sub2);
                    pend3 &= ~known;   // (a known copy takes its record from the known alignment)
                    // A read of the amplicon's length closer to the known sequence (the other pass's amplicon)
                    // than to this one: a variant of it carries the amplicons' difference -- C3's 10-base HDR
                    // block, two 10-base gaps against this amplicon, more than 16 diagonals hold.  It skips
                    // the first band level (its sort key marks it; nw_band_fill<16> leaves its pair inactive,
                    // the walk hands it to the 32-diagonal level) instead of failing there first.
                    jog = __ballot(c && k2 < k && k > 3) & ~(sub1 | sub2 | known);
                }
            }
        }
        while (cand) {
            int us[kCand];
            unsigned diff[kCand], raw[kCand];
#pragma unroll
            for (int t = 0; t < kCand; ++t) {
                us[t] = cand ? (int)__builtin_ctzll(cand) : -1;
                if (cand) cand &= cand - 1;
                diff[t] = 0u;
                raw[t] = 0u;
            }
            for (int c0 = 0; c0 < nd; c0 += 64) {
                const int k4 = c0 + lane;
                // every candidate's loads issued before any is used (branch-free: a missing
                // candidate re-reads candidate 0, lanes past the read re-read its last dword)
                const int kc = k4 < nd ? k4 : nd - 1;
                uint2 w[kCand];
                int sh[kCand];
#pragma unroll
                for (int t = 0; t < kCand; ++t) {
                    const int u = us[t] < 0 ? us[0] : us[t];
                    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)my_off, u);
                    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(my_off >> 32), u);
                    const long long off = (long long)(((unsigned long long)hi << 32) | lo);
                    if constexpr (PK) {   // the read's bytes 4 kc .. 4 kc + 3 from the 2-bit stream
                        const long long q0 = off - a.pk_pos0;   // wave-uniform: 64-bit math in SGPRs
                        const unsigned tq = (unsigned)(q0 & 15) + 4u * (unsigned)kc;
                        w[t] = *(const uint2*)(a.pk_words + (q0 >> 4) + (tq >> 4));
                        sh[t] = (int)(2 * (tq & 15));
                    } else {
                        w[t] = *(const uint2*)(a.reads + (off & ~3ll) + 4 * kc);   // 4-aligned dwordx2
                        sh[t] = (int)(off & 3);
                    }
                }
                const unsigned am = k4 < nd ? amp_sh[kc] : 0u;
                const unsigned msk = k4 < nd ? (k4 == nd - 1 ? tail_mask : 0xffffffffu) : 0u;
#pragma unroll
                for (int t = 0; t < kCand; ++t) {
                    if constexpr (PK) raw[t] = pk_expand(__builtin_amdgcn_alignbit(w[t].y, w[t].x, (unsigned)sh[t]));
                    else raw[t] = __builtin_amdgcn_alignbyte(w[t].y, w[t].x, sh[t]);
                    diff[t] |= ((raw[t] | 0x20202020u) ^ am) & msk;
                }
            }
#pragma unroll
            for (int t = 0; t < kCand; ++t) {
                if (us[t] < 0) continue;
                const unsigned long long anyd = __ballot(diff[t] != 0u);
                if (anyd != 0ull) {
                    // one or two substitutions (A C G T in the read): the certificates above
                    if (!sub1_ok) continue;
                    const unsigned zd = ~zero_bytes(diff[t]) & 0x80808080u;   // the lane's mismatching bytes
                    const int nzl = __builtin_popcount(zd);
                    const unsigned long long l2 = __ballot(nzl >= 2);
                    if (__ballot(nzl >= 3) || (l2 && __builtin_popcountll(anyd) > 1) || __builtin_popcountll(anyd) > 2)
                        continue;
                    const int ksub = l2 ? 2 : (int)__builtin_popcountll(anyd);
                    if (ksub == 2 && !sub2_ok) continue;
                    const unsigned rf = raw[t] | 0x20202020u;
                    bool bad = false;
                    for (unsigned z = zd; z; z &= z - 1) {
                        const unsigned cb = (rf >> ((int)__builtin_ctz(z) - 7)) & 0xffu;
                        bad = bad || !(cb == 'a' || cb == 'c' || cb == 'g' || cb == 't');
                    }
                    if (__ballot(bad)) continue;
                    // the shifted diagonals: d = +s pairs read byte q + s with amplicon byte q, d = -s
                    // read byte q with amplicon byte q + s (q <= La - 1 - s); mismatching bytes 0x80
                    const int k4 = lane, kc = k4 < nd ? k4 : nd - 1;   // one chunk (sub1_ok)
                    const unsigned rn = (unsigned)__shfl_down((int)raw[t], 1, 64);
                    const unsigned an = k4 + 1 < nd ? amp_sh[k4 + 1] : 0u;
                    const unsigned am0 = k4 < nd ? amp_sh[kc] : 0u;
                    const int q0 = 4 * k4;   // the lane's first byte
                    auto upto = [&](int qmax) -> unsigned {   // bytes q <= qmax of the lane
                        return qmax >= q0 + 3 ? 0x80808080u : (qmax < q0 ? 0u : (0x80808080u >> (8 * (q0 + 3 - qmax))));
                    };
                    auto mis = [&](int sgn, int sh) -> unsigned {
                        const unsigned x = sgn > 0 ? (__builtin_amdgcn_alignbyte(rn, raw[t], sh) | 0x20202020u) ^ am0
                                                   : rf ^ __builtin_amdgcn_alignbyte(an, am0, sh);
                        return ~zero_bytes(x) & upto(La - 1 - sh);
                    };
                    const unsigned p1m = mis(1, 1), m1m = mis(-1, 1);
                    if (ksub == 1) {
                        // S_+-1 = m p - x (La - 1 - p) is below D exactly when p <= La - 2: one
                        // mismatch on each shifted diagonal (two ballots, no sums)
                        if (__ballot(p1m != 0u) != 0ull && __ballot(m1m != 0u) != 0ull) sub1 |= 1ull << us[t];
                        continue;
                    }
                    // two substitutions at read bytes f < l: d = +-1 need two mismatches each, one at
                    // a read byte > f (no diagonal-0 prefix + one gap + shifted suffix scores above D)
                    // and one at a read byte < l (no shifted prefix + diagonal-0 suffix); d = +-2, +-3
                    // need one (S_d < D); |d| >= 4 and two or more gaps score below D by the checks in sub2_ok
                    const unsigned long long lz = __ballot(zd != 0u);
                    const int lf = (int)__builtin_ctzll(lz), ll = 63 - (int)__builtin_clzll(lz);
                    const int zf = __builtin_amdgcn_readlane((int)zd, lf), zl = __builtin_amdgcn_readlane((int)zd, ll);
                    const int f = 4 * lf + (__builtin_ctz((unsigned)zf) >> 3), l = 4 * ll + ((31 - __builtin_clz((unsigned)zl)) >> 3);
                    auto from = [&](int qmin) -> unsigned { return 0x80808080u & ~upto(qmin - 1); };   // bytes q >= qmin
                    auto two = [&](unsigned m) {   // at least two mismatching bytes over the wave
                        const unsigned long long b1 = __ballot(m != 0u);
                        return __ballot(__builtin_popcount(m) >= 2) != 0ull || __builtin_popcountll(b1) >= 2;
                    };
                    bool ok = two(p1m) && two(m1m);
                    // d = +1: read byte j = q + 1; d = -1: j = q
                    ok = ok && __ballot((p1m & from(f)) != 0u) && __ballot((p1m & upto(l - 2)) != 0u);
                    ok = ok && __ballot((m1m & from(f + 1)) != 0u) && __ballot((m1m & upto(l - 1)) != 0u);
                    ok = ok && __ballot(mis(1, 2) != 0u) && __ballot(mis(-1, 2) != 0u) && __ballot(mis(1, 3) != 0u) &&
                         __ballot(mis(-1, 3) != 0u);
                    if (ok) sub2 |= 1ull << us[t];
                    continue;
                }
                exact |= 1ull << us[t];
                if (a.ops) continue;   // ops output: the wave's exact copies are written together below
                if (!one_chunk) {
                    emit_later |= 1ull << us[t];
                    continue;
                }
                unsigned* o = (unsigned*)(a.out + (r0 + us[t]) * 3 * a.stride);
                if (lane < nd) {
                    o[lane] = amp_sh[nd + lane];
                    o[sd + lane] = 0x7c7c7c7cu;   // '|'
                    o[2 * sd + lane] = raw[t];
                }
                if (lane < 8) {
                    // the record (nw::Stat): aln_len, n_ident, n_sim, n_gaps, score, end_i, end_j, flags
                    const int v = lane == 3 || lane == 7 ? 0 : (lane == 4 ? a.band_maxsub * La : La);
                    ((int*)(a.stats + r0 + us[t]))[lane] = v;
                }
            }
        }
        // One indel (round 6; packed input, ops output, an A C G T amplicon of at most 256 bp, no exception
        // bytes): a read of La -+ k bases, 1 <= k <= indel_kmax.  Call the shorter of read and amplicon s
        // (Ls bases), the longer l; the candidate alignment pairs every residue of s, identically, with
        // one internal gap of k residues of l: S = m Ls - O - (k - 1) E.  Any alignment pairs <= Ls
        // residues; with u of s's residues unpaired, w mismatches and g the gap residues of one internal
        // gap it scores m (Ls - u - w) - x w - O - (g - 1) E, >= S only if m u + (m + x) w <= (k - g) E:
        // u = w = 0 (m > (k - 1) E), so the gap is in l (an l-gap of g <= k: an s-gap leaves s residues
        // unpaired); two or more internal gaps score <= m Ls - 2 O < S (O > (k - 1) E).  A one-gap
        // alignment with u = w = 0 pairs a prefix of s on diagonal shift s1 (l's residue i + s1 against
        // s's i) and the rest on s2 = s1 + g, 0 <= s1 < s2 <= k: it exists iff the last mismatch of
        // shift s2 precedes the first of s1 (G[s2] <= F[s1]); every such pair but (0, k) would score
        // >= S with a different alignment: none may exist.  No internal gap: a single shift pairs
        // P = min(Ls, Ll - s) residues (shifts of s, 1..3, pair Ls - s): each score m (P - c) - x c with
        // c mismatches must stay below S (shifts pairing 4 or more residues fewer do: O + (k - 1) E <
        // 4 m).  Then the optimal alignments are exactly (0, k) with the gap at any q in [G[k], F[0]]
        // (ties), all paired residues identical; the traceback from the corner (score S, first in the
        // scan) stays on the shift-k diagonal while M ties the gap state (M wins ties) and leaves it where
        // a mismatch precedes (q = G[k]): the gap is placed left-most, X when it is in the read, else Y.
        // Runs M q, gap k, M Ls - q; identities Ls, gaps k, length Ll.  Reads of C2's deletion and
        // insertion classes (~15 % of the reads) need no DP: the traceback fill and the wide level lose
        // their bulk (tests/test_gpu_indel.py: homopolymer and tandem-repeat indels against the oracle).
        // The checks (cert_indel) run in nw_band_cert, on the queued candidates.  A shorter read may instead be
        // a window of the amplicon (below; a read one certificate takes fails the other: a window scores m Lb,
        // an alignment with an internal gap less): one whose first and last 16 bases are the amplicon's ends
        // is queued at once, the others after the window check found none.
        bool ci_win = false;   // (a candidate the window check sees first)
        if constexpr (PK) {
            const int dl = my_len - La, kab = dl < 0 ? -dl : dl;
            const bool ci = indel_kmax > 0 && a.ops && one_chunk && amp_acgt_all && r < r_end && !exc && kab >= 1 &&
                            kab <= indel_kmax;
            if (ci && dl < 0 && my_len >= 16 && La >= 16)
                ci_win = pk_word16(a, my_off) != amp2s[0] ||
                         pk_word16(a, my_off + my_len - 16) != amp_word16(amp2s, La - 16);
            pend_i = __ballot(ci && !ci_win);   // checked by nw_band_cert
        }
        // window reads (above): an exact window at the largest offset, else one substitution
        unsigned long long win = 0ull;
        int win_s = 0, win_k = 0;
        if constexpr (PK) {
            if (win_ok) {
                bool cand_w = r < r_end && !exc && my_len >= 32 && my_len < La && !((pend_i >> lane) & 1ull);
                int best1 = -1;   // -2: an exact window at win_s; >= 0: an offset with one mismatch
                if (cand_w) {
                    // a window at s has the read's first 16 bases at s or its last 16 at s + Lb - 16 (one
                    // substitution cannot hit both); the other end word must then be within one mismatch
                    // -- one word compare rejects most offsets (reads with an indel) before the middle
                    const unsigned key0 = rword(my_off), key1 = rword(my_off + my_len - 16);
                    // their offsets among the amplicon's sorted 16-mers: [f, l), the last 8 at most
                    // (repeats: the DP)
                    const unsigned kk[2] = {key0, key1};
                    int lb[2], ub[2];
                    sorted_ranges<2>(skey, nseed, kk, lb, ub);
                    const int l0 = ub[0], f0 = max(lb[0], ub[0] - 8), l1 = ub[1], f1 = max(lb[1], ub[1] - 8);
                    for (int i = l0 - 1; i >= f0; --i) {   // offsets descending: the largest exact window first
                        const int s = spos[i];
                        if (s + my_len > La) continue;
                        const int he = ham16(key1, aword(s + my_len - 16));
                        if (he > 1) continue;
                        const int mm = he + mism(my_off, 16, s + 16, my_len - 32, 1 - he);
                        if (mm == 0) {
                            best1 = -2;
                            win_s = s;
                            break;
                        }
                        if (mm == 1 && best1 == -1) best1 = s;
                    }
                    if (best1 == -1)   // the substitution among the first 16 bases
                        for (int i = l1 - 1; i >= f1; --i) {
                            const int s = (int)spos[i] - (my_len - 16);
                            if (s < 0 || ham16(key0, aword(s)) != 1) continue;
                            if (mism(my_off, 16, s + 16, my_len - 32, 0) == 0) {
                                best1 = s;
                                break;
                            }
                        }
                    if (best1 >= 0) win_s = best1;
                    win_k = best1 >= 0 ? 1 : 0;
                    cand_w = best1 != -1;
                }
                win = __ballot(cand_w);
                // one substitution: every other full-overlap diagonal needs two mismatches, the two
                // diagonals pairing Lb - 1 residues one (the whole wave on each such read)
                // (the read's 16-base words go to LDS once per candidate: the offsets' compares read them
                // there, with no global round trip per offset)
                unsigned* rbw = s_rbw[threadIdx.x >> 6];
                for (unsigned long long need = __ballot(cand_w && win_k == 1); need; need &= need - 1) {
                    const int u = (int)__builtin_ctzll(need);
                    const int s1 = __builtin_amdgcn_readlane(win_s, u), Lb = __builtin_amdgcn_readlane(my_len, u);
                    const unsigned lo32 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)my_off, u);
                    const unsigned hi32 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(my_off >> 32), u);
                    const long long ro = (long long)(((unsigned long long)hi32 << 32) | lo32);
                    const int nwd = (Lb + 15) / 16 + 1;   // <= kRbw
                    for (int k = lane; k < nwd; k += 64) rbw[k] = 16 * k < Lb ? rword(ro + 16 * k) : 0u;
                    lds_fence();
                    // mismatches of read bases [j0, j0 + len) against amplicon [s, s + len), up to cap + 1
                    auto mism_l = [&](int j0, int s, int len, int cap) -> int {
                        int cnt = 0;
                        for (int w = 0; w < len && cnt <= cap; w += 16) {
                            const int p = j0 + w;
                            unsigned y = __builtin_amdgcn_alignbit(rbw[(p >> 4) + 1], rbw[p >> 4], (unsigned)(2 * (p & 15))) ^
                                         aword(s + w);
                            if (len - w < 16) y &= (1u << (2 * (len - w))) - 1u;
                            cnt += __builtin_popcount((y | (y >> 1)) & 0x55555555u);
                        }
                        return cnt;
                    };
                    bool bad = false;
                    for (int s2 = lane; s2 <= La - Lb; s2 += 64)
                        if (s2 != s1) bad = bad || mism_l(0, s2, Lb, 1) < 2;
                    if (lane == 0) bad = bad || mism_l(1, 0, Lb - 1, 0) < 1;            // d = +1
                    if (lane == 1) bad = bad || mism_l(0, La - Lb + 1, Lb - 1, 0) < 1;   // d = Lb - La - 1
                    if (__ballot(bad)) win &= ~(1ull << u);
                    lds_fence();   // every lane's reads of rbw before the next candidate's writes
                }
            }
            pend_i |= __ballot(ci_win && !((win >> lane) & 1ull));   // no window: the one-indel check
        }
        // Seeded band: a read the 16-diagonal band cannot hold (La - Lb >= 16, the
        // reference's own 151 bp reads on a 280 bp amplicon) and no window certificate took: the
        // diagonals of every exact hit of its disjoint 16-base blocks among the amplicon's 16-mers.
        // The wide level then centres its band on them and certifies it (nw_band_walk).  A block
        // with more than 8 hits (a repeat) leaves the read to the exact kernel.
        int32_t sinfo = 0, sinfo2 = 0;
        if constexpr (PK) {
            if (win_ok && a.seed_info && r < r_end && !exc && my_len >= 32 && La - my_len >= 16 &&
                !(((exact | sub1 | sub2 | win | known) >> lane) & 1ull)) {
                int dmin = 1 << 20, dmax = -(1 << 20);
                bool ok = true;
                const int nb = my_len >> 4;
                // the refined certificate's facts (nw_band_walk), for reads whose blocks have at most one
                // hit each: blocks without a hit, the blocks on each hit diagonal (at most 4), the
                // cheapest move between two blocks' diagonals in read order -- an increase of d = j - i
                // by D leaves D read bases unpaired: O + (D - 1) E + m D; a decrease: O + (|D| - 1) E
                int n0 = 0, nd = 0, shift = 0xffff;
                bool uniq = true;
                int dd0 = 0, dd1 = 0, dd2 = 0, dd3 = 0, dc0 = 0, dc1 = 0, dc2 = 0, dc3 = 0;
                for (int b0 = 0; b0 < nb && ok; b0 += 8) {   // eight blocks' words in flight together
                    unsigned keys[8];
#pragma unroll
                    for (int t = 0; t < 8; ++t) keys[t] = b0 + t < nb ? rword(my_off + 16 * (b0 + t)) : 0u;
                    int lbs[8], ubs[8];   // each block's hits among the amplicon's sorted 16-mers: [lb, ub)
                    sorted_ranges<8>(skey, nseed, keys, lbs, ubs);
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const int b = b0 + t;
                        if (b >= nb || !ok) continue;
                        const int l = ubs[t], f = lbs[t];
                        if (l - f > 8) ok = false;   // a repeat: more than 8 hits
                        for (int i = f; ok && i < l; ++i) {
                            const int d = 16 * b - (int)spos[i];
                            dmin = min(dmin, d);
                            dmax = max(dmax, d);
                        }
                        n0 += l == f;
                        uniq = uniq && l - f <= 1;
                        if (uniq && l - f == 1) {
                            const int d = 16 * b - (int)spos[f];
                            auto mv = [&](int d1) {
                                const int D = d - d1;
                                return D > 0 ? a.gap_open + (D - 1) * a.gap_extend + a.band_maxsub * D
                                             : a.gap_open + (-D - 1) * a.gap_extend;
                            };
                            const bool h0 = nd > 0 && dd0 == d, h1 = nd > 1 && dd1 == d, h2 = nd > 2 && dd2 == d,
                                       h3 = nd > 3 && dd3 == d;
                            if (nd > 0 && !h0) shift = min(shift, mv(dd0));
                            if (nd > 1 && !h1) shift = min(shift, mv(dd1));
                            if (nd > 2 && !h2) shift = min(shift, mv(dd2));
                            if (nd > 3 && !h3) shift = min(shift, mv(dd3));
                            dc0 += h0;
                            dc1 += h1;
                            dc2 += h2;
                            dc3 += h3;
                            if (!(h0 || h1 || h2 || h3)) {
                                if (nd == 0) { dd0 = d; dc0 = 1; }
                                else if (nd == 1) { dd1 = d; dc1 = 1; }
                                else if (nd == 2) { dd2 = d; dc2 = 1; }
                                else if (nd == 3) { dd3 = d; dc3 = 1; }
                                uniq = uniq && nd < 4;
                                ++nd;
                            }
                        }
                    }
                }
                if (ok && dmax >= dmin && dmax - dmin <= kWideDiags / 2 && nb < 128) {
                    sinfo = seed_pack(dmin, dmax, nb);
                    if (uniq) sinfo2 = seed2_pack(n0, max(max(dc0, dc1), max(dc2, dc3)), shift);
                }
            }
            if (a.seed_info && r < r_end) a.seed_info[r] = sinfo;
            if (a.seed_info2 && r < r_end) a.seed_info2[r] = sinfo2;
        }
        if (r < r_end)
            a.sort_key[r] = (((exact | sub1 | sub2 | win | known) >> lane) & 1ull)
                                ? a.band_lb_cap + 2
                                : (sinfo ? a.band_lb_cap + 3 +
                                               min(a.seed_keys - 1, max(0, ((seed_dmin(sinfo) + seed_dmax(sinfo)) / 2 + La) >> 2))
                                         : (my_len <= a.band_lb_cap && !((jog >> lane) & 1ull) ? my_len : a.band_lb_cap + 1));
        if (a.ops && r < r_end && ((win >> lane) & 1ull)) {
            // runs: s amplicon residues (Y), the window (M), the rest of the amplicon (Y)
            int q = 0;
            const long long sst = a.ops_stride;
            if (win_s > 0) a.ops[sst * q++ + r] = ((unsigned)RUN_Y << 28) | (unsigned)win_s;
            a.ops[sst * q++ + r] = ((unsigned)RUN_M << 28) | (unsigned)my_len;
            if (La - win_s - my_len > 0) a.ops[sst * q++ + r] = ((unsigned)RUN_Y << 28) | (unsigned)(La - win_s - my_len);
            a.nops[r] = q;
            int4* st = (int4*)(a.stats + r);
            st[0] = make_int4(La, my_len - win_k, my_len - win_k, La - my_len);   // aln_len, n_ident, n_sim, n_gaps
            st[1] = make_int4(a.band_maxsub * (my_len - win_k) - win_k * 4 * sc5, win_s + my_len, my_len, 0);
        }
        // a known copy: record and runs from the known alignment, by the compaction
        if (a.ops && r < r_end && ((known >> lane) & 1ull)) a.nops[r] = kNopsKnown;
        // ops output: every exact copy of the wave's 64 reads at once, lane u its own read's
        // record (2 x 16 B), its one M run of La columns (run 0 of its slot) and run count --
        // coalesced stores instead of three partial-line stores per copy
        if (a.ops && r < r_end && (((exact | sub1 | sub2) >> lane) & 1ull)) {
            // substitutions (0 .. 2; three: nw_band_cert; a mismatch scores -4 / 5 maxsub)
            const int k = (int)((sub1 >> lane) & 1ull) + 2 * (int)((sub2 >> lane) & 1ull);
            a.ops[r] = ((unsigned)RUN_M << 28) | (unsigned)La;
            a.nops[r] = 1;
            int4* st = (int4*)(a.stats + r);
            st[0] = make_int4(La, La - k, La - k, 0);   // aln_len, n_ident, n_sim, n_gaps
            st[1] = make_int4(a.band_maxsub * (La - k) - k * 4 * sc5, La, La, 0);   // score, end_i, end_j, flags
        }
        // the diagonal of every exact copy longer than one chunk: amplicon, '|' markup,
        // read; rows as dwords up to round4(La) (within the row stride)
        while (emit_later) {
            const int u = (int)__builtin_ctzll(emit_later);
            emit_later &= emit_later - 1;
            const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)my_off, u);
            const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(my_off >> 32), u);
            const long long off = (long long)(((unsigned long long)hi << 32) | lo);
            const uint8_t* base = a.reads + (off & ~3ll);
            unsigned* o = (unsigned*)(a.out + (r0 + u) * 3 * a.stride);
            for (int k4 = lane; k4 < nd; k4 += 64) {
                o[k4] = amp_sh[nd + k4];
                o[sd + k4] = 0x7c7c7c7cu;   // '|'
                o[2 * sd + k4] = __builtin_amdgcn_alignbyte(ld_dw(base + 4 * k4 + 4), ld_dw(base + 4 * k4), (int)(off & 3));
            }
            if (lane < 8) {
                // the record (nw::Stat): aln_len, n_ident, n_sim, n_gaps, score, end_i, end_j, flags
                const int v[8] = {La, La, La, 0, a.band_maxsub * La, La, La, 0};
                int x = 0;
#pragma unroll
                for (int t = 0; t < 8; ++t) x = lane == t ? v[t] : x;
                ((int*)(a.stats + r0 + u))[lane] = x;
            }
        }
        // packed input: the bytes of every read that needs the DP (the only reads a later kernel
        // reads), exactly its own bytes (neighbouring reads' bytes are never written by another
        // read's wave: no races between blocks); exception bytes follow (below)
        if constexpr (PK)
            write_read_bytes(a, __ballot(r < r_end && my_len > 0 &&
                                         !(((exact | sub1 | sub2 | win | known | pend3 | pend_i) >> lane) & 1ull)),
                             my_off, my_len);
        // deferred certificates (KernelArgs::cert_q): the wavefront's queued reads for nw_band_cert, the
        // three-substitution candidates from the front of its 64 entries, the one-indel ones from the back
        if constexpr (PK) {
            if (a.cert_q) {
                const unsigned long long lt = (1ull << lane) - 1ull;
                const long long slot = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
                if ((pend3 >> lane) & 1ull) a.cert_q[slot * 64 + __builtin_popcountll(pend3 & lt)] = (int32_t)r;
                if ((pend_i >> lane) & 1ull) a.cert_q[slot * 64 + 63 - __builtin_popcountll(pend_i & lt)] = (int32_t)r;
                if (lane == 0) a.cert_cnt[slot] = (int32_t)(__builtin_popcountll(pend3) | (__builtin_popcountll(pend_i) << 8));
            }
        }
    };
    if constexpr (!PK) {
        // wavefront batches of 64 reads, grid-strided
        for (long long r0 = ((long long)blockIdx.x * wpb + (threadIdx.x >> 6)) * 64; r0 < a.n;
             r0 += (long long)gridDim.x * wpb * 64) {
            const long long r = r0 + lane;
            const long long my_off = r < a.n ? a.offsets[r] : 0;
            const int my_len = r < a.n ? (int)(a.offsets[r + 1] - my_off) : -1;
            batch(r0, a.n, my_off, my_len, false);
        }
    } else {
        __shared__ long long s_off[kPkBlock + 1];
        __shared__ unsigned char s_exc[kPkBlock];
        __shared__ long long s_wsum[8];
        __shared__ long long s_x[2];
        const long long bl = pbl, bh = pbh;
        const int cnt = (int)(bh - bl), tid = threadIdx.x, wave = tid >> 6;
        int64_t* offs = const_cast<int64_t*>(a.offsets);
        if (a.pk_len) {
            // the offsets from the lengths (nw_align_ops_packed_lens): the group's base offset, the
            // lengths of the group's reads before this block (earlier chunks' included: they are uploaded
            // with the call's first lengths copy), an exclusive scan of the block's own
            const long long G = pG, rr = prr, l = pk_l;
            long long pre = pk_pre;
            long long inc = l;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const long long o = __shfl_up(inc, d, 64);
                const long long op = __shfl_xor(pre, d, 64);
                if (lane >= d) inc += o;
                pre += op;
            }
            if (lane == 63) s_wsum[wave] = inc;
            if (lane == 0) s_wsum[4 + wave] = pre;
            __syncthreads();
            long long o = a.pk_gbase[G] + inc - l + s_wsum[4] + s_wsum[5] + s_wsum[6] + s_wsum[7];
            for (int w2 = 0; w2 < wave; ++w2) o += s_wsum[w2];
            if (rr >= bl && rr < bh) {
                s_off[rr - bl] = o;
                offs[rr] = o;
            }
            if (rr == bh - 1) {   // the end of the block's last read (the chunk's last: offsets[n])
                s_off[cnt] = o + l;
                offs[bh] = o + l;
            }
        } else {
            for (int i = tid; i <= cnt; i += blockDim.x) s_off[i] = a.offsets[bl + i];
        }
        // reads holding exception bytes (not certifiable here; every one of them needs the DP)
        const bool any_exc = a.pk_e1 > a.pk_e0;
        for (int i = tid; i < kPkBlock; i += blockDim.x) s_exc[i] = 0;
        __syncthreads();
        long long x0 = 0, x1 = 0;
        if (any_exc) {
            if (wave == 0) {
                const long long lo_b = exc_lower_bound(a, s_off[0], lane);
                const long long hi_b = exc_lower_bound(a, s_off[cnt], lane);
                if (lane == 0) {
                    s_x[0] = lo_b;
                    s_x[1] = hi_b;
                }
            }
            __syncthreads();
            x0 = s_x[0];
            x1 = s_x[1];
            for (long long t = x0 + tid; t < x1; t += blockDim.x) {
                const long long p = a.pk_exc_pos[t];
                int lo_i = 0, hi_i = cnt - 1;   // the last read starting at or before p
                while (lo_i < hi_i) {
                    const int mid = (lo_i + hi_i + 1) >> 1;
                    if (s_off[mid] <= p) lo_i = mid;
                    else hi_i = mid - 1;
                }
                s_exc[lo_i] = 1;
            }
            __syncthreads();
        }
        const long long r0 = bl + 64 * wave;   // one batch per wavefront
        if (r0 < bh) {
            const long long r = r0 + lane;
            const long long my_off = r < bh ? s_off[r - bl] : 0;
            const int my_len = r < bh ? (int)(s_off[r - bl + 1] - my_off) : -1;
            batch(r0, bh, my_off, my_len, r < bh && s_exc[r - bl] != 0);
        } else if (a.cert_q && lane == 0) {
            a.cert_cnt[(long long)blockIdx.x * 4 + wave] = 0;   // (every wavefront's queue count is written)
        }
        if (any_exc && x1 > x0) {
            // after every wave's byte stores (completed: workgroup-scope release), the exception bytes
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            uint8_t* dst = const_cast<uint8_t*>(a.reads);
            for (long long t = x0 + tid; t < x1; t += blockDim.x) dst[a.pk_exc_pos[t]] = a.pk_exc_byte[t];
        }
    }
}

// ============================================================================
// Deferred certificates (KernelArgs::cert_q), between classify and the sort.  In classify each
// wavefront runs a check for all its 64 lanes when any lane needs it: the three-substitution and
// one-indel checks cost ~70 us of a 1M-read C2 pass there, for the ~20 % of reads that take them.
// Classify queues those reads instead (per wavefront: three-substitution candidates from the front of
// its 64 entries, one-indel candidates from the back, the two counts in cert_cnt) with the DP's sort
// key and no bytes; here one block gathers the queues of kCertSlots classify wavefronts into two dense
// lists in LDS and its wavefronts run the same checks (cert_sub3, cert_indel) 64 reads at a time.  A
// certified read gets its record, runs and the finished key; the others get their bytes for the DP.
// ============================================================================
constexpr int kCertSlots = 16;   // classify wavefronts per block (4 classify blocks)

__global__ __launch_bounds__(256) void nw_band_cert(const KernelArgs a, int nslots) {
    extern __shared__ unsigned c_amp2[];   // the amplicon's 2-bit words (classify's image from 2 nd)
    __shared__ int s_n3[kCertSlots], s_ni[kCertSlots], s_o3[kCertSlots + 1], s_oi[kCertSlots + 1];
    __shared__ int s_l3[kCertSlots * 64], s_li[kCertSlots * 64];
    __shared__ unsigned s_fact[4][kSub3FactWords];   // cert_sub3's per-wavefront facts
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long slot0 = (long long)blockIdx.x * kCertSlots;
    const int ns = (int)min<long long>(kCertSlots, nslots - slot0);
    if (tid < kCertSlots) {
        const int v = tid < ns ? a.cert_cnt[slot0 + tid] : 0;
        s_n3[tid] = v & 0xff;
        s_ni[tid] = v >> 8;
    }
    __syncthreads();
    if (tid == 0) {
        int x = 0, y = 0;
        for (int i = 0; i < kCertSlots; ++i) {
            s_o3[i] = x;
            s_oi[i] = y;
            x += s_n3[i];
            y += s_ni[i];
        }
        s_o3[kCertSlots] = x;
        s_oi[kCertSlots] = y;
    }
    __syncthreads();
    const int n3 = s_o3[kCertSlots], ni = s_oi[kCertSlots];
    if (n3 + ni == 0) return;   // (block-uniform)
    const int La = a.La, nd = (La + 3) / 4, n2 = (La + 15) / 16 + 2;
    for (int k = tid; k < n2; k += 256) c_amp2[k] = a.cls_img[2 * nd + k];
    for (int p = tid; p < ns * 64; p += 256) {
        const int sl = p >> 6, j = p & 63;
        if (j < s_n3[sl]) s_l3[s_o3[sl] + j] = a.cert_q[(slot0 + sl) * 64 + j];
        else if (j >= 64 - s_ni[sl]) s_li[s_oi[sl] + 63 - j] = a.cert_q[(slot0 + sl) * 64 + j];
    }
    __syncthreads();
    const int sc5 = a.band_maxsub / 5;
    const long long sst = a.ops_stride;
    // three substitutions: reads of the amplicon's length, three mismatches on the main diagonal
    for (int b = 64 * wave; b < n3; b += 256) {
        const bool v = b + lane < n3;
        const long long r = v ? s_l3[b + lane] : 0;
        const long long my_off = v ? a.offsets[r] : a.pk_pos0;
        unsigned rw[17];
        load_read_words(a, v, my_off, rw);
        int k, f, f2, l;
        main_diag_mism(rw, c_amp2, La, &k, &f, &f2, &l);
        const bool ok = cert_sub3(a, c_amp2, rw, v && k == 3, f, f2, l, my_off, s_fact[wave]);
        if (ok) {   // the diagonal with three substitutions (classify's record for them)
            a.ops[r] = ((unsigned)RUN_M << 28) | (unsigned)La;
            a.nops[r] = 1;
            int4* st = (int4*)(a.stats + r);
            st[0] = make_int4(La, La - 3, La - 3, 0);   // aln_len, n_ident, n_sim, n_gaps
            st[1] = make_int4(a.band_maxsub * (La - 3) - 3 * 4 * sc5, La, La, 0);   // score, end_i, end_j, flags
            a.sort_key[r] = a.band_lb_cap + 2;
        }
        write_read_bytes(a, __ballot(v && !ok), my_off, La);
    }
    // one indel: reads of La -+ k bases
    for (int b = 64 * wave; b < ni; b += 256) {
        const bool v = b + lane < ni;
        const long long r = v ? s_li[b + lane] : 0;
        const long long my_off = v ? a.offsets[r] : a.pk_pos0;
        const int my_len = v ? (int)(a.offsets[r + 1] - my_off) : La;
        int gk = 0;
        const bool ok = cert_indel(a, c_amp2, v, my_off, my_len, &gk);
        if (ok) {   // runs M q, the gap (X: residues of the read, Y: of the amplicon), M the rest of the shorter
            const bool del = my_len < La;
            const int Ls = del ? my_len : La, kab = del ? La - my_len : my_len - La;
            a.ops[r] = ((unsigned)RUN_M << 28) | (unsigned)gk;
            a.ops[sst + r] = ((unsigned)(del ? RUN_Y : RUN_X) << 28) | (unsigned)kab;
            a.ops[2 * sst + r] = ((unsigned)RUN_M << 28) | (unsigned)(Ls - gk);
            a.nops[r] = 3;
            int4* st = (int4*)(a.stats + r);
            st[0] = make_int4(Ls + kab, Ls, Ls, kab);   // aln_len, n_ident, n_sim, n_gaps
            st[1] = make_int4(a.band_maxsub * Ls - a.gap_open - (kab - 1) * a.gap_extend, La, my_len, 0);
            a.sort_key[r] = a.band_lb_cap + 2;
        }
        write_read_bytes(a, __ballot(v && !ok), my_off, my_len);
    }
}

// ============================================================================
// Length sort, one launch: segments of kSegReads reads, each sorted by key in LDS
// (stable: read order within a key), the reads that need the DP (every key but the
// exact-copy key) placed at the segment's base in the DP list -- an exclusive prefix of
// the segments' DP counts found by look-back (nw_common.h lookback_excl).  Pairs are
// consecutive DP-list positions: reads of one length within a segment (most of a
// CRISPResso segment shares the amplicon's length), so a pair's band holds both reads.
// Replaces a global counting sort (per-block histograms, two scans, scatter: four
// launches of ~8 us each per chunk).  The last segment writes the DP count (*band_count).
// ============================================================================
constexpr int kSegReads = 4096, kSegThreads = 1024, kSegWaves = kSegThreads / 64;

__host__ __device__ inline int segsort_lds_bytes(int lb_cap) { return 4 * (kSegWaves + 1) * (lb_cap + 3) + 4 * 32; }

__global__ __launch_bounds__(kSegThreads) void nw_band_segsort(const KernelArgs a, unsigned epoch) {
    extern __shared__ int seg_sm[];
    // keys: lengths 0 .. cap, cap + 1 (too long for the band), EX = cap + 2 (exact copy, no DP),
    // then the seeded reads' diagonal keys
    const int NB = a.band_lb_cap + 3 + a.seed_keys, EX = a.band_lb_cap + 2;
    int* cnt = seg_sm;                  // [kSegWaves][NB]: per-wave counts, then prefix over waves
    int* kbase = seg_sm + kSegWaves * NB;   // [NB]: bucket totals, then their exclusive prefix
    int* misc = kbase + NB;             // [0], [4] look-back results (band list, seeded list), [2] error, [16..31] wave sums
    const int KS = a.seed_list ? a.band_lb_cap + 3 : NB;   // keys >= KS: seeded reads (their own list)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int k = tid; k < kSegWaves * NB + NB; k += kSegThreads) seg_sm[k] = 0;
    if (tid < 32) misc[tid] = 0;
    __syncthreads();
    const long long r0 = (long long)blockIdx.x * kSegReads + 4 * tid;
    int key[4], rank[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const long long r = r0 + i;
        const int k = r < a.n ? a.sort_key[r] : EX;
        // lanes with the same key this round (11 key bits cover NB <= 2048)
        unsigned long long m = ~0ull;
#pragma unroll
        for (int bit = 0; bit < 11; ++bit) {
            const unsigned long long bb = __ballot((k >> bit) & 1);
            m &= ((k >> bit) & 1) ? bb : ~bb;
        }
        const unsigned long long below = m & ((1ull << lane) - 1ull);
        const int old = cnt[wave * NB + k];
        __builtin_amdgcn_wave_barrier();
        if (below == 0ull) cnt[wave * NB + k] = old + (int)__builtin_popcountll(m);
        lds_fence();
        key[i] = k;
        rank[i] = old + (int)__builtin_popcountll(below);
    }
    __syncthreads();
    // per key: prefix over the waves (in place) and the key's total
    for (int k = tid; k < NB; k += kSegThreads) {
        int run = 0;
        for (int w = 0; w < kSegWaves; ++w) {
            const int v = cnt[w * NB + k];
            cnt[w * NB + k] = run;
            run += v;
        }
        kbase[k] = k == EX ? 0 : run;
    }
    __syncthreads();
    // exclusive prefix of the key totals (thread t: keys [t * per, (t + 1) * per))
    const int per = (NB + kSegThreads - 1) / kSegThreads;
    const int k0 = tid * per, k1 = min(NB, k0 + per);
    int mine = 0;
    for (int k = k0; k < k1; ++k) mine += kbase[k];
    int incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) misc[16 + wave] = incl;
    __syncthreads();
    int before = 0, dp = 0;
#pragma unroll
    for (int w = 0; w < kSegWaves; ++w) {
        before += w < wave ? misc[16 + w] : 0;
        dp += misc[16 + w];
    }
    int run = before + incl - mine;
    for (int k = k0; k < k1; ++k) {
        const int v = kbase[k];
        kbase[k] = run;
        run += v;
    }
    __syncthreads();
    // the seeded keys are the tail of the key range: their prefix past the band list's total is
    // their place in the seeded list
    // the seeded list: an odd segment count gets its last entry twice (a pair of one read: the walks take
    // its first position), so every pair of that list lies within one segment's sorted run
    const int dpB = KS < NB ? kbase[KS] : dp, dpS0 = dp - dpB, dpS = dpS0 + (dpS0 & 1);
    if (wave == 0) {
        const unsigned base = lookback_excl(a.lb_status, blockIdx.x, epoch, (unsigned)dpB, &misc[2]);
        if (lane == 0) misc[0] = (int)base;
    } else if (wave == 1 && a.seed_list) {   // the seeded list: the look-back words after the band list's
        const unsigned base = lookback_excl(a.lb_status + gridDim.x + 1, blockIdx.x, epoch, (unsigned)dpS, &misc[2]);
        if (lane == 0) misc[4] = (int)base;
    }
    __syncthreads();
    const long long base = misc[0], baseS = misc[4];
    int32_t* order = const_cast<int32_t*>(a.band_order);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = key[i];
        if (k >= KS) {
            const int q = (kbase[k] - dpB) + cnt[wave * NB + k] + rank[i];
            a.seed_list[baseS + q] = (int32_t)(r0 + i);
            if (q == dpS0 - 1 && dpS != dpS0) {   // the segment's odd count padded to a pair
                a.seed_list[baseS + q + 1] = (int32_t)(r0 + i);
                atomicAdd(a.fallback_count + 9, 1);   // the path counters leave the padding out
            }
        }
        else if (k != EX) order[base + kbase[k] + cnt[wave * NB + k] + rank[i]] = (int32_t)(r0 + i);
    }
    if (tid == 0) {
        if (misc[2]) a.fallback_count[3] = 1;   // look-back cut off: the call reports an error
        if (blockIdx.x == gridDim.x - 1) {
            *const_cast<int32_t*>(a.band_count) = (int32_t)(base + dpB);
            if (a.seed_list) *a.seed_count = (int32_t)(baseS + dpS);
        }
    }
}

// ============================================================================
// Fill
// ============================================================================
// Overlap of diagonal d = j - i (pairs of the alignment that stays on it).
__device__ __forceinline__ int diag_pairs(int La, int Lb, int d) { return d >= 0 ? min(La, Lb - d) : min(Lb, La + d); }

// DP list of the traceback pass: band_order[0, *band_count).
// The wide level (a.band_from_work) reads the exact kernel's work list instead: the reads the
// narrower levels gave up on, then (direct hand-off) the first level's redo list; there
// a.band_count = a.work_count.
// The wide level's list ends with the seeded reads (the segment sort's seeded list, sorted by
// their hits' diagonals, so a pair's two reads share a band).
// The 32-diagonal level with the seeded list (KernelArgs::seed_l2 == 1): its own list (the redo
// list, none when the direct hand-off gave it to the wide level; as the only level, the sorted DP
// list), then, from the next even position, the seeded list -- an
// odd count before it leaves one hole (read by no walk), so no pair mixes a seeded read with another.
__device__ __forceinline__ long long l2_redo_n(const KernelArgs& a) {
    return redo_direct_taken(a) ? 0ll : (long long)*a.band_count;
}
__device__ __forceinline__ long long l2_seed0(const KernelArgs& a) { return (l2_redo_n(a) + 1) & ~1ll; }
__device__ __forceinline__ long long band_list_count(const KernelArgs& a) {
    if (a.band_from_work) return exact_work_count(a) + (a.seed_list ? (long long)*a.seed_count : 0ll);
    if (a.seed_l2 == 1) return l2_seed0(a) + (long long)*a.seed_count;
    return (long long)*a.band_count;
}
__device__ __forceinline__ long long band_list_read(const KernelArgs& a, long long k, long long nb) {
    if (a.band_from_work) {
        if (k < nb) return a.work_list[k];
        const long long nr = redo_direct_taken(a) ? (long long)*a.redo_count : 0ll;
        return k < nb + nr ? (long long)a.redo_list[k - nb] : (long long)a.seed_list[k - nb - nr];
    }
    if (a.seed_l2 == 1) {
        const long long nr = l2_redo_n(a), s0 = (nr + 1) & ~1ll;
        if (k >= s0) return (long long)a.seed_list[k - s0];
        if (k >= nr) --k;   // the hole: its pair's read A again (the pair holds one read)
    }
    return (long long)a.band_order[k];
}

// The traceback fill: a level's band list, its traceback bits into each pair's region (the walk
// follows).  (Round 6 removed the diagonal pass, a score-only fill over the reads of the
// amplicon's length ahead of this one: with the classify certificates taking nearly all of them,
// its sweep only lengthened the chain -- resident pass 0.536 -> 0.484 ms without it)
template <int W, bool SUMM = false>   // SUMM: the traceback fill also writes the stop summary (lane walk)
#define NW_FILL_WPE 6   // 5: no spills in the traceback fill but slower
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(NW_FILL_WPE))) void nw_band_fill(const KernelArgs a) {
    using G = BandGeo<W>;
    constexpr int kBL = G::L, kBPW = G::PW, kCapBytes = G::CapBytes;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // second level skipped: its reads go to the wide level (with the seeded list: that list alone)
    if (W == kBandDiags && redo_direct_taken(a) && a.seed_l2 != 1) return;
    if (W < kBandDiags && l1_skipped(a)) return;   // first level skipped (KernelArgs::l1_skip)
    if (W >= kBandDiags && a.tail_prio) __builtin_amdgcn_s_setprio(3);
    const int La = a.La;
    const int O = a.gap_open, E = a.gap_extend;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wpb = blockDim.x >> 6;
    const int q = G::q_of(lane), grp = G::grp_of(lane);
    const unsigned NEG2 = 0u;                    // -inf in the kBias16 domain
    const unsigned OE2 = pk(O - E, O - E);

    uint32_t* tab = (uint32_t*)smem;
    uint16_t* acd = (uint16_t*)(smem + kTabBytes);
    const int PCS = band_pcs(La, W);
    unsigned char* pcd_wave = smem + kTabBytes + align16(2 * band_acd_elems(La)) + wave * kBPW * PCS;
    unsigned char* pcd = pcd_wave + grp * PCS;
    unsigned char* lut6 = smem + kTabBytes + align16(2 * band_acd_elems(La)) + wpb * kBPW * PCS;
    // a tile row's four words per lane wait here (not in VGPRs) until its dwordx4 store
    unsigned* stage = (unsigned*)(lut6 + 256) + wave * 256 + 4 * lane;
    for (int k = tid; k < kTabRows * 36; k += blockDim.x) tab[k] = a.band_tab[k];
    for (int k = tid; k < 256; k += blockDim.x) lut6[k] = a.lut6[k];
    for (int k = tid; k < band_acd_elems(La); k += blockDim.x) {
        const int i = k - kAPad;   // row i = amplicon residue i - 1
        // the amplicon's EDNAFULL code (IUPAC codes included: their row of the table), pad outside
        const int c = (i >= 1 && i <= La) ? a.lut[a.amp[i - 1]] : NCODE_PAD;
        // the score table's LDS address is folded in: a0 + j0 is the entry's LDS address
        acd[k] = (uint16_t)(c * 36 * 4 + (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)tab);
    }
    __syncthreads();

    // byte-plane masks of the sign bits (SGPRs: v_and_or_b32 takes no literal)
    unsigned mT[4], mU[4];
    asm volatile("s_mov_b32 %0, 0x01010101" : "=s"(mT[0]));
    asm volatile("s_mov_b32 %0, 0x02020202" : "=s"(mT[1]));
    asm volatile("s_mov_b32 %0, 0x04040404" : "=s"(mT[2]));
    asm volatile("s_mov_b32 %0, 0x08080808" : "=s"(mT[3]));
    asm volatile("s_mov_b32 %0, 0x10101010" : "=s"(mU[0]));
    asm volatile("s_mov_b32 %0, 0x20202020" : "=s"(mU[1]));
    asm volatile("s_mov_b32 %0, 0x40404040" : "=s"(mU[2]));
    asm volatile("s_mov_b32 %0, 0x80808080" : "=s"(mU[3]));

    // the band list: wave work items of kBPW pairs each
    const int NW = a.band_words;
    const long long nb = (long long)*a.band_count;
    const long long count = band_list_count(a);
    const long long pair_lo = a.band_pair_lo;
    const long long pair_hi = min(a.band_pair_hi, (count + 1) / 2);
    const long long npB = pair_hi - pair_lo;
    const long long nB = npB > 0 ? (npB + kBPW - 1) / kBPW : 0ll;
    auto body = [&](long long wv) __attribute__((always_inline)) {
        const long long g = pair_lo + wv * kBPW + grp;
        int dlo = 0;
        bool act = false;
        long long offA = 0, offB = 0, ra = 0, rb = 0;
        int LbA = 0, LbB = 0;
        bool seeded = false;
        if (g < pair_hi) {
            ra = band_list_read(a, 2 * g, nb);
            rb = (2 * g + 1 < count) ? band_list_read(a, 2 * g + 1, nb) : ra;
            offA = a.offsets[ra];
            offB = a.offsets[rb];
            LbA = (int)(a.offsets[ra + 1] - offA);
            LbB = (int)(a.offsets[rb + 1] - offB);
            act = LbA <= a.band_lb_cap && LbB <= a.band_lb_cap && band_geometry2(La, LbA, LbB, &dlo, W);
            // the first level (16 diagonals) leaves a pair with a read classify keyed past the band's lengths
            // -- one that needs more diagonals (a known sequence's variant: nw_band_classify) -- to the next
            if constexpr (W < kBandDiags) act = act && a.sort_key[ra] <= a.band_lb_cap && a.sort_key[rb] <= a.band_lb_cap;
            if constexpr (W >= kBandDiags) {
                // seeded reads (both of the pair): the band centred on their hits' diagonals
                if (a.seed_info) {
                    const int32_t sa = a.seed_info[ra], sb = a.seed_info[rb];
                    const int lo = min(seed_dmin(sa), seed_dmin(sb)), hi = max(seed_dmax(sa), seed_dmax(sb));
                    const int sdlo = lo - (W - (hi - lo + 1)) / 2;
                    // the second level's LDS code pads hold columns j >= -(kJPad - 1) and rows i < La + 112
                    // (the sweep's first and last steps): narrower than the wide level's
                    const bool pads_ok = W > kBandDiags || (sdlo >= -2 * (kJPad - 3) && max(LbA, LbB) - sdlo < La + 200);
                    if (seed_valid(sa) && seed_valid(sb) && hi - lo + 1 <= W - 2 && LbA <= a.band_lb_cap &&
                        LbB <= a.band_lb_cap && sdlo <= kBK && sdlo + W - 1 >= 1 - La && pads_ok) {
                        dlo = sdlo;   // (tau = t - dlo + kBK stays >= 0)
                        act = true;
                        seeded = true;
                    }
                }
            }
        }
        if (!act) {   // neutral geometry, nothing stored
            band_geometry2(La, La, La, &dlo, W);
            LbA = LbB = 0;
        }
        const int Lmax = max(LbA, LbB);

        // pair codes of the wavefront's pairs' columns (j = 1..Lb real, the rest pad):
        // all 64 lanes stage one pair at a time, 4 columns per lane from coalesced dword
        // loads of both reads (all pairs' loads issued before any is used)
        for (int k4 = lane; k4 < kBPW * PCS / 4; k4 += 64) ((unsigned*)pcd_wave)[k4] = 0x8c8c8c8cu;   // pad pair
        const int Lw = (int)wave_max_u32((unsigned)Lmax);
        unsigned bad_mask = 0u;   // bit p: pair p has a read A / B code outside A C G T N (bits 0-15 / 16-31)
        unsigned pad_mask = 0u;   // the same for bytes EDNAFULL does not score ('-', '*', ...: the walk's gap columns)
        unsigned n_mask = 0u;     // the same for N
        constexpr int kSub = kBPW < 4 ? kBPW : 4;   // pairs staged together (loads in flight)
        for (int c0 = 0; c0 < Lw; c0 += 256)
        for (int p0 = 0; p0 < kBPW; p0 += kSub) {
            const int k4 = (c0 >> 2) + lane;
            unsigned wA[kSub], wB[kSub];
            int lenA[kSub], lenB[kSub];
#pragma unroll
            for (int pp = 0; pp < kSub; ++pp) {
                const int p = p0 + pp;
                const int src = G::src_of(p);   // lane q = 0 of pair p
                const unsigned oAl = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)offA, src);
                const unsigned oAh = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(offA >> 32), src);
                const unsigned oBl = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)offB, src);
                const unsigned oBh = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(offB >> 32), src);
                lenA[pp] = __builtin_amdgcn_readlane(LbA, src);
                lenB[pp] = __builtin_amdgcn_readlane(LbB, src);
                const long long oA = (long long)(((unsigned long long)oAh << 32) | oAl);
                const long long oB = (long long)(((unsigned long long)oBh << 32) | oBl);
                wA[pp] = wB[pp] = 0u;
                if (4 * k4 < lenA[pp]) {
                    const uint8_t* b = a.reads + (oA & ~3ll) + 4 * k4;
                    wA[pp] = __builtin_amdgcn_alignbyte(*(const unsigned*)(b + 4), *(const unsigned*)b, (int)(oA & 3));
                }
                if (4 * k4 < lenB[pp]) {
                    const uint8_t* b = a.reads + (oB & ~3ll) + 4 * k4;
                    wB[pp] = __builtin_amdgcn_alignbyte(*(const unsigned*)(b + 4), *(const unsigned*)b, (int)(oB & 3));
                }
            }
#pragma unroll
            for (int pp = 0; pp < kSub; ++pp) {
                const int p = p0 + pp;
                const int Lm = max(lenA[pp], lenB[pp]);
                bool bA = false, bB = false, zA = false, zB = false, nnA = false, nnB = false;
                if (4 * k4 < Lm) {
                    unsigned packed = 0u;
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const int j0 = 4 * k4 + b;   // 0-based column
                        int cA = j0 < lenA[pp] ? lut6[(wA[pp] >> (8 * b)) & 0xffu] : kPadCode;
                        int cB = j0 < lenB[pp] ? lut6[(wB[pp] >> (8 * b)) & 0xffu] : kPadCode;
                        // lut6: 5 = pad / not in EDNAFULL (scores 0, as EMBOSS does); 6 = IUPAC code
                        bA = bA || cA > kPadCode;
                        bB = bB || cB > kPadCode;
                        zA = zA || (j0 < lenA[pp] && cA == kPadCode);
                        zB = zB || (j0 < lenB[pp] && cB == kPadCode);
                        nnA = nnA || (j0 < lenA[pp] && cA == 4);   // N
                        nnB = nnB || (j0 < lenB[pp] && cB == 4);
                        cA = min(cA, kPadCode);
                        cB = min(cB, kPadCode);
                        packed |= (unsigned)((cA * 6 + cB) * 4) << (8 * b);
                    }
                    *(unsigned*)(pcd_wave + p * PCS + kJPad + 1 + 4 * k4) = packed;
                }
                // ballots with every lane active: bad_mask must be the same in all lanes
                // (pair p's header is written by its own q = 0 lane)
                if (__ballot(bA)) bad_mask |= 1u << p;
                if (__ballot(bB)) bad_mask |= 1u << (16 + p);
                if (__ballot(zA)) pad_mask |= 1u << p;
                if (__ballot(zB)) pad_mask |= 1u << (16 + p);
                if (__ballot(nnA)) n_mask |= 1u << p;
                if (__ballot(nnB)) n_mask |= 1u << (16 + p);
            }
        }
        const unsigned npm = n_mask | pad_mask;   // N, or a byte EDNAFULL does not score (the walk's plain reads have neither)
        const int flags = (((bad_mask >> grp) & 1u) ? REGION_BAD_A : 0) | (((bad_mask >> (16 + grp)) & 1u) ? REGION_BAD_B : 0) |
                          (((npm >> grp) & 1u) ? REGION_NP_A : 0) | (((npm >> (16 + grp)) & 1u) ? REGION_NP_B : 0);

        // wave-uniform tau range; per lane: boundary and capture steps
        const unsigned tlo = act ? (unsigned)(kBK - dlo) : 0xffffffffu;
        const unsigned thi = act ? (unsigned)(kBK - dlo + La + Lmax) : 0u;
        const unsigned dmax = (unsigned)(-dlo > dlo + W - 1 ? -dlo : dlo + W - 1);
        const unsigned tpro = act ? (unsigned)(kBK - dlo) + dmax + 1 : 0u;
        const int tau0 = (int)(wave_min_u32(tlo) & ~3u);
        const int tau_end = (int)wave_max_u32(thi);
        const int tau_pro = (int)wave_max_u32(tpro);
        lds_fence();
        unsigned char* region = a.band_region + (g - pair_lo) * a.band_stride;
        if (q == 0 && g < pair_hi) {
            // everything the walk needs to find the pair's reads: one 48-byte load
            int4* hp = (int4*)region;
            hp[0] = make_int4(tau0, dlo, flags | (act ? 0 : kPairInactive) | (seeded ? REGION_SEEDED : 0), 0);
            hp[1] = make_int4((int)ra, (int)rb, (int)(a.offsets[ra + 1] - offA), (int)(a.offsets[rb + 1] - offB));
            hp[2] = make_int4((int)(unsigned)offA, (int)(offA >> 32), (int)(unsigned)offB, (int)(offB >> 32));
        }
        if (tau_end == 0) return;   // no active group in this wavefront

        const int d0 = dlo + 2 * q;
        int tb[2], te[2], teB[2];
        unsigned bval[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int d = d0 + p;
            const int ad = d < 0 ? -d : d;
            tb[p] = kBK - dlo + ad;
            bval[p] = pk(E * ad + kBias16, E * ad + kBias16);
            const int ilo = 1 - d > 1 ? 1 - d : 1;
            // step at which diagonal d reaches read A's / read B's last row or column
            const int ieA = La < LbA - d ? La : LbA - d, ieB = La < LbB - d ? La : LbB - d;
            te[p] = (LbA > 0 && ieA >= ilo) ? kBK - dlo + 2 * ieA + d : -1;
            teB[p] = (LbB > 0 && ieB >= ilo) ? kBK - dlo + 2 * ieB + d : -1;
        }
        // capture window: the steps at which some lane's diagonal reaches the last row
        // or column; blocks before it skip the capture selects
        const int te_lo = (int)wave_min_u32(min(min((unsigned)te[0], (unsigned)te[1]),
                                                min((unsigned)teB[0], (unsigned)teB[1])));
        unsigned* bits = (unsigned*)(region + kHdrBytes + kCapBytes) + 4 * q;   // this lane's slot of each tile
        // the stop summary (band_summ): the OR of a 16-word block's words (accumulated in LDS at each
        // row's store, next to the row's stage), one byte per block, gathered in LDS 16 blocks at a
        // time and stored as one 16-byte line piece per lane (byte stores spread over the pass had
        // cost +0.12 GB of partial-line writes)
        constexpr bool summ_on = SUMM;
        unsigned* sum_lds = (unsigned*)(lut6 + 256) + wpb * 256 + wave * 320 + lane;   // the block's OR
        unsigned* sum_chunk = (unsigned*)(lut6 + 256) + wpb * 256 + wave * 320 + 64 + 4 * lane;   // 16 blocks' bytes
        if (summ_on) {
            *sum_lds = 0u;
            *(uint4*)sum_chunk = make_uint4(0u, 0u, 0u, 0u);
        }
        auto summ_flush = [&](int b) {   // the chunk holding block b, to the pair's summary
            unsigned char* sp = (unsigned char*)(bits - 4 * q) + (size_t)NW * (W / 2) * 4 + q * band_summ_bytes(NW);
            *(uint4*)(sp + (b & ~15)) = *(const uint4*)sum_chunk;
            *(uint4*)sum_chunk = make_uint4(0u, 0u, 0u, 0u);
        };
        auto summ_put = [&](int b, unsigned x) {   // block b's byte; the chunk goes out with its last block
            ((unsigned char*)sum_chunk)[b & 15] = (unsigned char)(((x >> 20) & 0xfu) | (((x >> 28) & 0xfu) << 4));
            if ((b & 15) == 15) summ_flush(b);
        };

        unsigned Hp0 = pk(kBias16, kBias16), Hp1 = Hp0, MoP = NEG2, XP = NEG2, YP = NEG2;
        unsigned cap0 = NEG2, cap1 = NEG2, capB0 = NEG2, capB1 = NEG2;   // read A's (low) / B's (high half)
        // LDS code cursors of the block starting at tau4: rows i0, i0 + 1; columns j0 .. j0 + 2
        auto ibase = [&](int tau4) { return (tau4 - kBK) / 2 - q; };
        const uint16_t* ap = acd + kAPad + ibase(tau0);
        const unsigned char* jp = pcd + kJPad + (ibase(tau0) + dlo + 2 * q);
        auto load_scores = [&](unsigned* s) {
            const int a0 = ap[0], a1 = ap[1];
            const int j0 = jp[0], j1 = jp[1], j2 = jp[2];
            using LdsU = const __attribute__((address_space(3))) unsigned;
            s[0] = *(LdsU*)(uintptr_t)(a0 + j0);
            s[1] = *(LdsU*)(uintptr_t)(a0 + j1);
            s[2] = *(LdsU*)(uintptr_t)(a1 + j1);
            s[3] = *(LdsU*)(uintptr_t)(a1 + j2);
            ap += 2;   // rows and columns both advance by 2 per 4 steps
            jp += 2;
        };
        unsigned sc[4], sn[4];
        load_scores(sc);

        auto step = [&](int tau, auto Uc, auto PROc, auto CAPc, const unsigned* scr, unsigned& acc) {
            constexpr int U = decltype(Uc)::value;
            constexpr int P = U & 1;
            constexpr bool PRO = decltype(PROc)::value;
            constexpr bool CAP = decltype(CAPc)::value;
            unsigned X, Y, d1 = 0u, d2 = 0u;
            if constexpr (P == 0) {
                // up = own diagonal d0 + 1 one step back; left = lane q-1's d0 - 1
                const unsigned Ml = G::shr(MoP), Xl = G::shr(XP);
                X = max2(Ml, Xl);
                d2 = sub2(Xl, Ml);     // sign: X opens (open > extend)
                Y = max2(MoP, YP);
                d1 = sub2(YP, MoP);    // sign: Y opens
            } else {
                // up = lane q+1's d0 one step back; left = own diagonal d0
                const unsigned Mu = G::shl(MoP), Yu = G::shl(YP);
                Y = max2(Mu, Yu);
                d1 = sub2(Yu, Mu);
                X = max2(MoP, XP);
                d2 = sub2(XP, MoP);
            }
            unsigned M = add2(P ? Hp1 : Hp0, scr[U]);
            const unsigned mxy = max2(X, Y);
            unsigned H = max2(M, mxy);
            if constexpr (PRO) {
                if (tau == tb[P]) {   // DP boundary cell (row 0 / column 0): M = 0, X = Y = -inf
                    M = bval[P];
                    H = M;
                    X = NEG2;
                    Y = NEG2;
                }
            }
            if constexpr (P == 0) Hp0 = H; else Hp1 = H;
            MoP = sub2(M, OE2);
            XP = X;
            YP = Y;
            if constexpr (CAP) {
                if constexpr (P == 0) {
                    cap0 = tau == te[0] ? M : cap0;
                    capB0 = tau == teB[0] ? M : capB0;
                } else {
                    cap1 = tau == te[1] ? M : cap1;
                    capB1 = tau == teB[1] ? M : capB1;
                }
            }
            const unsigned d3 = sub2(X, Y);     // sign: Y > X (X wins an X == Y tie)
            const unsigned d4 = sub2(M, mxy);   // sign: M < max(X, Y)
            const unsigned tt = __builtin_amdgcn_perm(d2, d1, 0x0B0A0908u);
            const unsigned uu = __builtin_amdgcn_perm(d4, d3, 0x0B0A0908u);
            acc = and_or(tt, mT[U], acc);
            acc = and_or(uu, mU[U], acc);
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        // one block = 4 steps = one bit word; the next block's scores load meanwhile
        // (into the other buffer: blocks go in pairs, so no register copies)
        auto block = [&](int tau4, auto PROc, auto CAPc, const unsigned* cur, unsigned* nxt) {
            load_scores(nxt);
            unsigned acc = 0u;
            step(tau4, I0{}, PROc, CAPc, cur, acc);
            step(tau4 + 1, I1{}, PROc, CAPc, cur, acc);
            step(tau4 + 2, I2{}, PROc, CAPc, cur, acc);
            step(tau4 + 3, I3{}, PROc, CAPc, cur, acc);
            return acc;
        };
        // four blocks = one tile row: words w .. w + 3 of every lane (w % 4 == 0)
        // a block pair (8 steps) is half a tile row; its words wait in LDS and the
        // second half stores the row (the phases may split a row: the stage carries it)
        auto flush = [&](int tau4) {
            asm volatile("" ::: "memory");
            const int w = ((tau4 - tau0) >> 2) & ~3;
            const uint4 row = *(const uint4*)stage;
            if (act && w < NW) *(uint4*)(bits + w * kBL) = row;
            if (summ_on) {
                const unsigned x = *sum_lds | row.x | row.y | row.z | row.w;
                const bool last = ((w >> 2) & 3) == 3;   // the block's fourth row: its summary byte
                if (last && act && (w >> 4) <= ((NW - 1) >> 4)) summ_put(w >> 4, x);   // a block with stored words
                *sum_lds = last ? 0u : x;
            }
        };
        auto pair8 = [&](int tau4, auto PROc, auto CAPc) {
            const int h2 = ((tau4 - tau0) >> 2) & 2;
            stage[h2] = block(tau4, PROc, CAPc, sc, sn);
            stage[h2 + 1] = block(tau4 + 4, PROc, CAPc, sn, sc);
            if (h2) flush(tau4);
        };
        // phases in whole block pairs (8 steps) from tau0: prologue (boundary cells,
        // captures of short reads), bulk, capture window to tau_end (may run up to 7
        // steps past it: cells outside the matrix, bits beyond NW not stored)
        auto up8 = [&](int t) { return tau0 + ((t - tau0 + 7) & ~7); };
        const int p1 = up8(tau_pro);
        const int p2 = max(p1, tau0 + ((te_lo - tau0) & ~7));
        int tau4 = tau0;
        for (; tau4 < p1; tau4 += 8) {
            pair8(tau4, std::true_type{}, std::true_type{});
        }
        for (; tau4 < p2; tau4 += 8) {
            pair8(tau4, std::false_type{}, std::false_type{});
        }
        for (; tau4 <= tau_end; tau4 += 8) {
            pair8(tau4, std::false_type{}, std::true_type{});
        }
        if (((tau4 - tau0) >> 2) & 2) flush(tau4 - 8);   // a half row left: its other half is past tau_end
        if (summ_on) {   // the last block, unless its fourth row stored it (every block up to the last word is written)
            const int wl = ((tau4 - tau0) >> 2) - 1;
            const int bl = min(wl >> 4, (NW - 1) >> 4);   // the last block with stored words
            if (act && wl >= 0) {
                // its byte unless its fourth row put it (the block ends past the computed words), then its chunk
                const bool open = (wl >> 4) <= bl && ((wl >> 2) & 3) != 3;
                if (open) ((unsigned char*)sum_chunk)[bl & 15] =
                    (unsigned char)(((*sum_lds >> 20) & 0xfu) | (((*sum_lds >> 28) & 0xfu) << 4));
                if (open || (bl & 15) != 15) summ_flush(bl);
            }
        }
        if (act) {
            unsigned* caps = (unsigned*)(region + kHdrBytes);
            caps[2 * q] = (cap0 & 0xffffu) | (capB0 & 0xffff0000u);
            caps[2 * q + 1] = (cap1 & 0xffffu) | (capB1 & 0xffff0000u);
        }
    };
    for (long long wv = (long long)blockIdx.x * wpb + wave; wv < nB; wv += (long long)gridDim.x * wpb) body(wv);
}

// ============================================================================
// Walk + emit: one wavefront per read (sorted order), latency-bound.
// ============================================================================
// The run-based traceback (nw_common.h walk_runs_wide) specialised per run type (the state
// is wave-uniform, so each round takes one scalar branch): an M run follows one diagonal
// (its band membership is uniform, tau falls by 2 per cell); X / Y runs move along a
// row / column.  Each
// lane tests CPL cells; the round's first stop is found with one ballot.  `word(tau,
// kd)` returns the band dword of anti-diagonal step tau (relative to the stored
// range) and band diagonal kd; bit positions of read h at sub-step s: Y opens hb,
// Y > X hb + 4, X opens 16 + hb, M < max(X, Y) 20 + hb, with hb = 8 h + s.
// tot (optional): [0] M columns, [1] gap columns, [2] the paid gaps' cost (runs opened inside the
// matrix: O + (k - 1) E; the end overhangs are free) -- a plain read's record without band_emit.
template <int CPL, int W>
__device__ int band_walk_runs2(const unsigned* bits, int NW, int La, int Lb, int ei, int ej, int dlo, int tb0, int h,
                               unsigned* runs, int cap, int lane, int gO = 0, int gE = 0, int* tot = nullptr) {
    int nruns = 0, last_type = -1;
    bool full = false;
    int tm = 0, tg = 0, tp = 0;
    auto push = [&](int type, int n, bool paid = false) {
        if (n <= 0) return;
        if (type == RUN_M) tm += n; else tg += n;
        if (paid) tp += (type == last_type ? 0 : gO - gE) + n * gE;
        if (type == last_type) {
            if (lane == 0) runs[nruns - 1] += (unsigned)n;
        } else if (nruns < cap) {
            if (lane == 0) runs[nruns] = ((unsigned)type << 28) | (unsigned)n;
            ++nruns;
            last_type = type;
        } else {
            full = true;
        }
    };
    // the state machine is wave-uniform: keep its inputs in SGPRs so every branch
    // below is a scalar branch (values loaded through VGPRs are not provably uniform)
    La = __builtin_amdgcn_readfirstlane(La);
    Lb = __builtin_amdgcn_readfirstlane(Lb);
    ei = __builtin_amdgcn_readfirstlane(ei);
    ej = __builtin_amdgcn_readfirstlane(ej);
    dlo = __builtin_amdgcn_readfirstlane(dlo);
    tb0 = __builtin_amdgcn_readfirstlane(tb0);
    NW = __builtin_amdgcn_readfirstlane(NW);
    h = __builtin_amdgcn_readfirstlane(h);
    if (ei == La && ej < Lb) push(RUN_X, Lb - ej);
    else if (ej == Lb && ei < La) push(RUN_Y, La - ei);
    constexpr int WR = 64 * CPL;
    constexpr int WM = 64 * 8;   // M rounds: 8 cells per lane from one dwordx4
    int i = __builtin_amdgcn_readfirstlane(ei), j = __builtin_amdgcn_readfirstlane(ej), state = RUN_M;
    const int hb = 8 * h;
    while (i > 0 && j > 0) {
        nruns = __builtin_amdgcn_readfirstlane(nruns);   // uniform (see above)
        last_type = __builtin_amdgcn_readfirstlane(last_type);
        int k0;            // cells of the current run before the stop (the run is k0 + 1 long)
        int nb = RUN_M;    // M runs: the state the stop cell continues in
        if (state == RUN_M) {
            // cells (i-1-k, j-1-k), 1-based, all on diagonal kd = j - i - dlo: one column.
            // Lane l reads the 4 words [W0 - 4l, W0 - 4l + 3] (16 steps, 8 cells of the
            // run's parity): cell u has tau = 4 (W0 - 4l) + 14 + p - 2u, run index k_l + u.
            const int kd = j - i - dlo;
            if ((unsigned)kd >= (unsigned)W) return -1;
            const int lim = min(i, j) - 1;          // k < lim: cell inside the matrix
            const int t0 = i + j - 4 + tb0;         // tau of cell k = 0
            const int p = t0 & 1;
            const int W0 = (t0 >> 2) & ~3;
            const int tl = min(max((W0 >> 2) - lane, 0), (NW >> 2) - 1);   // lane's tile row
            const int k0l = (t0 - p - 4 * W0 - 14) >> 1;   // lane 0's k of cell u = 0, in [-7, 0]
            const int kl = k0l + 8 * lane;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);   // lanes past the matrix edge stop without a load
            if (kl < lim) v = *(const uint4*)(bits + tl * (2 * W) + 4 * (kd >> 1));
            const int se = 20 + hb + 2 + p, so = 20 + hb + p;   // "M < max" bit of even / odd u
            unsigned nm = 0u;
            nm |= ((v.w >> se) & 1u) | (((v.w >> so) & 1u) << 1);
            nm |= (((v.z >> se) & 1u) << 2) | (((v.z >> so) & 1u) << 3);
            nm |= (((v.y >> se) & 1u) << 4) | (((v.y >> so) & 1u) << 5);
            nm |= (((v.x >> se) & 1u) << 6) | (((v.x >> so) & 1u) << 7);
            const int sz = min(max(-kl, 0), 8), sl = min(max(lim - kl, 0), 8);
            const unsigned ge0 = (0xffu << sz) & 0xffu, gel = (0xffu << sl) & 0xffu;
            const unsigned stop = (nm | gel) & ge0;
            const unsigned long long m = __ballot(stop != 0u);
            if (m == 0) {   // cells k < k0l + WM tested (k0l <= 0)
                push(RUN_M, WM + k0l);
                i -= WM + k0l;
                j -= WM + k0l;
                continue;
            }
            const int L = (int)__builtin_ctzll(m);
            const unsigned sL = (unsigned)__builtin_amdgcn_readlane((int)stop, L);
            const int u0 = (int)__builtin_ctz(sL);
            k0 = k0l + 8 * L + u0;
            const int q = u0 >> 1;
            const unsigned wq = (unsigned)__builtin_amdgcn_readlane(
                (int)(q == 0 ? v.w : (q == 1 ? v.z : (q == 2 ? v.y : v.x))), L);
            nb = ((wq >> (4 + hb + ((u0 & 1) ? p : 2 + p))) & 1u) ? RUN_Y : RUN_X;
            push(RUN_M, k0 + 1);
            i -= k0 + 1;
            j -= k0 + 1;
            state = nb;
        } else {
            // X: cells (i, j-k), diagonal kd = j - k - i - dlo; Y: cells (i-k, j), kd = j - i + k - dlo
            const bool isX = state == RUN_X;
            const int lim = isX ? j : i;             // k < lim: inside the matrix
            const int kd0 = j - i - dlo;
            const int t0 = i + j - 2 + tb0;          // tau of cell k = 0
            const int bit = isX ? 16 : 0;            // "opens" bit of the run's gap type
            unsigned stop = 0u, oob = 0u;
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                const int kk = lane * CPL + u;
                const int kd = isX ? kd0 - kk : kd0 + kk;
                const int tau = t0 - kk;
                const bool out = (unsigned)kd >= (unsigned)W;
                const int wd = min(max(tau, 0) >> 2, NW - 1);
                const unsigned w = (kk < lim && !out) ? bits[(wd >> 2) * (2 * W) + 4 * ((kd & (W - 1)) >> 1) + (wd & 3)]
                                                      : 0u;   // cells that stop anyway: no load
                const bool opens = ((w >> (bit + hb + (tau & 3))) & 1u) != 0u;
                const bool valid = kk < lim;
                stop |= (unsigned)(!valid || out || opens) << u;
                oob |= (unsigned)(valid && out) << u;
            }
            const unsigned long long m = __ballot(stop != 0u);
            if (m == 0) {
                push(state, WR, true);
                if (isX) j -= WR; else i -= WR;
                continue;
            }
            const int L = (int)__builtin_ctzll(m);
            const unsigned sL = (unsigned)__builtin_amdgcn_readlane((int)stop, L);
            const int u0 = (int)__builtin_ctz(sL);
            if (((unsigned)__builtin_amdgcn_readlane((int)oob, L) >> u0) & 1u) return -1;
            k0 = L * CPL + u0;
            push(state, k0 + 1, true);
            if (isX) j -= k0 + 1; else i -= k0 + 1;
            state = RUN_M;
        }
        if (full) return -1;
    }
    if (i > 0) push(RUN_Y, i);
    if (j > 0) push(RUN_X, j);
    if (tot) {
        tot[0] = tm;
        tot[1] = tg;
        tot[2] = tp;
    }
    return full ? -1 : nruns;
}

constexpr int kBandReadCap = 1280;   // >= the band length cap (La + 31, La <= 1024): every walked read fits
// lut, amplicon bytes, markup rows, the EDNAFULL score rows (17 x 16 int8: the
// single-diagonal test)
__host__ __device__ inline int band_walk_shared_bytes(int La) { return 256 + align16(La + 16) + align16(4 * La) + 17 * 16; }
constexpr int kBandRunsCap = 256;     // traceback runs per read (more: the read goes to the next level)
__host__ __device__ inline int band_walk_row(int La, int lb_max) { return (La + lb_max + 15) & ~15; }   // = stride_for()
__host__ __device__ inline int band_walk_rcap(int lb_max) { return min(kBandReadCap, (lb_max + 255) & ~255); }
// a pair's header and W captures, whole 64-dword DMA loads
__host__ __device__ constexpr int band_walk_hdr_slot(int W) { return 64 * ((kHdrBytes / 4 + W + 63) / 64); }
// per wave: runs, two read-byte buffers and two header slots (one read ahead), the three output rows
__host__ __device__ inline int band_walk_wave_bytes(int La, int lb_max, int W) {
    return kBandRunsCap * 4 + 2 * (band_walk_rcap(lb_max) + 256) + 2 * 4 * band_walk_hdr_slot(W) +
           3 * band_walk_row(La, lb_max);
}

// emit_alignment (nw_common.h) with the three rows built in LDS (byte writes) and
// written out as dwordx4 rows: 16 B per lane instead of a byte store per column.
// The rows are padded to 16 B; the host reads aln_len columns of each.
template <bool ROWS, class Score>
__device__ void band_emit(const unsigned* runs, int nruns, const unsigned char* amp, const unsigned char* raw,
                          const unsigned char* lut, const Score& sim_score, unsigned char* rows, int row,
                          unsigned char* o_ref, int64_t stride, int score, int ei, int ej, Stat* st, int lane) {
    int col = 0, ia = 0, jb = 0;
    int n_id = 0, n_sim = 0, n_gap = 0;
    for (int q = nruns - 1; q >= 0; --q) {
        const unsigned rc = (unsigned)__builtin_amdgcn_readfirstlane((int)runs[q]);
        const int type = (int)(rc >> 28);
        const int n = (int)(rc & 0x0fffffffu);
        if (type == RUN_M) {
            int same = 0;   // columns with identical bytes (not '-'): '|', identical and similar
            for (int c0 = 0; c0 < n; c0 += 64) {   // uniform trip count: scalar loop
                const int p = c0 + lane;
                if (p < n) {
                    const unsigned char ca = amp[ia + p], cb = raw[jb + p];
                    unsigned char mk = '|';
                    if (ca != cb || ca == '-') {   // rare: a mismatch, a case difference or an input '-'
                        mk = ' ';
                        if (ca == '-' || cb == '-') {   // an input '-' counts as a gap (CORE:1846)
                            ++n_gap;
                        } else {
                            const bool id = upcase(ca) == upcase(cb);
                            const bool sim = id || sim_score(ia + p, (int)lut[cb]) > 0;
                            mk = id ? '|' : (sim ? ':' : '.');
                            n_id += id;
                            n_sim += sim;
                        }
                    } else {
                        ++same;
                    }
                    if constexpr (ROWS) {
                        rows[col + p] = ca;
                        rows[row + col + p] = mk;
                        rows[2 * row + col + p] = cb;
                    }
                }
            }
            n_id += same;
            n_sim += same;
        } else if constexpr (!ROWS) {   // gap run: n gap columns
            if (lane == 0) n_gap += n;
        } else {   // gap run: every column is a gap
            const unsigned char* src = type == RUN_X ? raw + jb : amp + ia;
            unsigned char* dst = rows + (type == RUN_X ? 2 * row : 0) + col;
            unsigned char* gap = rows + (type == RUN_X ? 0 : 2 * row) + col;
            for (int c0 = 0; c0 < n; c0 += 64) {
                const int p = c0 + lane;
                if (p < n) {
                    dst[p] = src[p];
                    rows[row + col + p] = ' ';
                    gap[p] = '-';
                    ++n_gap;
                }
            }
        }
        col += n;
        if (type != RUN_X) ia += n;
        if (type != RUN_Y) jb += n;
    }
    if constexpr (ROWS) lds_fence();
    for (int c = 16 * lane; ROWS && c < col; c += 1024) {
        const uint4 r0 = *(const uint4*)(rows + c), r1 = *(const uint4*)(rows + row + c),
                    r2 = *(const uint4*)(rows + 2 * row + c);
        *(uint4*)(o_ref + c) = r0;
        *(uint4*)(o_ref + stride + c) = r1;
        *(uint4*)(o_ref + 2 * stride + c) = r2;
    }
    if (col < 1024) {
        const unsigned t = wave_sum_u32((unsigned)n_id | ((unsigned)n_sim << 10) | ((unsigned)n_gap << 20));
        n_id = (int)(t & 1023u);
        n_sim = (int)((t >> 10) & 1023u);
        n_gap = (int)(t >> 20);
    } else {
        n_id = wave_sum(n_id);
        n_sim = wave_sum(n_sim);
        n_gap = wave_sum(n_gap);
    }
    if (lane == 0) {
        Stat s;
        s.aln_len = col;
        s.n_ident = n_id;
        s.n_sim = n_sim;
        s.n_gaps = n_gap;
        s.score = score;
        s.end_i = ei;
        s.end_j = ej;
        s.flags = 0;
        *st = s;
    }
}


// True when every single-diagonal alignment outside [dlo, dhi] whose overlap could
// reach `score` (maxsub * P(d) >= score) scores below it.  A score table lookup per
// pair: amplicon / read bytes in LDS, the amplicon's EDNAFULL code (lut) and the read's
// 6-code (lut6), scores from band_tab (packed with + 2E, entry [x][y][y]).
__device__ bool band_single_diagonals_below(const KernelArgs& a, const unsigned char* amp, const unsigned char* rd,
                                            int La, int Lb, int dlo, int dhi, int score, int lane) {
    const int E2 = 2 * a.gap_extend;
    for (int side = 0; side < 2; ++side) {
        for (int k = 1;; ++k) {
            const int d = side == 0 ? dhi + k : dlo - k;
            const int P = diag_pairs(La, Lb, d);
            if (P <= 0 || a.band_maxsub * P < score) break;
            const int i0 = d >= 0 ? 0 : -d, j0 = d >= 0 ? d : 0;   // 0-based first pair
            int sum = 0;
            for (int t = lane; t < P; t += 64) {
                const int x = a.lut[amp[i0 + t]], y = a.lut6[rd[j0 + t]];
                const unsigned w = a.band_tab[x * 36 + (y < 6 ? y : 5) * 7];
                sum += (int)(short)(w & 0xffffu) - E2;
            }
            if (wave_sum(sum) >= score) return false;
        }
    }
    return true;
}

// The first level's walk, one read per lane (ops output): 64 consecutive list positions per
// wavefront, each lane its own read's header, start cell, certificate and traceback
// (band_walk_runs2's rules cell for cell, the state machine in VGPRs: the wave-per-read walk
// spends ~430 scalar instructions per read on it), its record from the runs and the score
// (plain reads), its runs into its slot.  What a lane cannot finish -- the refined certificate
// (sums over the band's neighbour diagonals), reads with codes outside A C G T, more than
// kLaneRuns runs -- goes to `defer(k)`, the wave-per-read body, one read at a time.
constexpr int kLaneRuns = 8;   // runs per lane in LDS ([kLaneRuns][64] dwords at the wave's area)
#define NW_MIS_UNROLL 8   // dword compares in flight per lane in count_mis (4: walk 0.086 ms, 8: 0.079, 16: 0.081)
constexpr int kMRows = 2;   // tile rows per M round of the lane walk (<= 4: 32 cells)
// The lane walk (with the stop summary its fill writes) pays on one long list: the kernel-resident
// pass, walk<16> 0.189 -> 0.092 ms (fill<16> +13 us for the summary).  A pipelined call runs it on
// its chunks of >= 65536 reads of one amplicon (the call's time the same, C2 1.961 vs 1.954 ms; its
// kernels faster); the pooled call's small chunks keep the wave walk (C5 17.15 vs 16.61 ms with the
// lane walk on every chunk, in-process A/Bs).  KernelArgs::band_summ selects it per launch.
// (Running it twice -- the certificates alone, then, while the next levels ran on a side stream, the
// walk of what they kept -- measured no gain: resident pass 0.700-0.703 vs 0.690-0.700 ms, C2 call
// 1.951 vs 1.956 ms; the walk and the wide level slowed each other to the serial sum)
template <int W, class Defer>
__device__ void walk_lanes(const KernelArgs& a, long long klo, long long khi, unsigned char* wb,
                           const unsigned char* amp_lds, bool amp_acgt, int sc5, const Defer& defer) {
    constexpr int kCapBytes = BandGeo<W>::CapBytes;
    const int La = a.La, E = a.gap_extend, O = a.gap_open, m = a.band_maxsub, NW = a.band_words;
    const int lane = threadIdx.x & 63, wpb = blockDim.x >> 6, wave = threadIdx.x >> 6;
    const int rcap = band_walk_rcap(a.Lb_max);
    unsigned* lruns = (unsigned*)wb;   // [kLaneRuns][64]: lane's run q at lruns[64 q + lane]
    const long long ng = (khi - klo + 63) >> 6;
    for (long long g = (long long)blockIdx.x * wpb + wave; g < ng; g += (long long)gridDim.x * wpb) {
        const long long k = klo + 64 * g + lane;
        const bool live = k < khi;
        // 0: done, 1: the wave path, 2: redo list (retry), 3: fallback list
        int fate = 0;
        long long rd = 0;
        if (live) {
            const unsigned char* region = a.band_region + ((k >> 1) - a.band_pair_lo) * a.band_stride;
            const int4 hdr = *(const int4*)region, hr = *(const int4*)(region + 16), ho = *(const int4*)(region + 32);
            const int h = (int)(k & 1);
            rd = h ? hr.y : hr.x;
            const int Lb = h ? hr.w : hr.z;
            if (a.redo_flags) a.redo_flags[k] = 0;
            if (Lb <= 0) {
                Stat z = {};
                z.flags = FLAG_EMPTY;
                a.stats[rd] = z;
                a.nops[rd] = 0;
            } else if (hdr.z & kPairInactive) {
                fate = 2;
            } else if (Lb > rcap) {
                fate = 3;
            } else {
                const int dlo = hdr.y, tau0 = hdr.x;
                // start cell: the largest end key over the band's diagonals (their last cells)
                const uint4* capw = (const uint4*)(region + kHdrBytes);
                unsigned k32 = 0u;
#pragma unroll
                for (int c4 = 0; c4 < W / 4; ++c4) {
                    const uint4 q4 = capw[c4];
                    const unsigned cv[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int d = dlo + 4 * c4 + e;
                        const int iend = La < Lb - d ? La : Lb - d;
                        const int ilo = 1 - d > 1 ? 1 - d : 1;
                        if (iend >= ilo) {
                            const int v = half(cv[e], h) - kBias16 - E * (2 * iend + d);
                            const int jend = iend + d;
                            const unsigned kk = (iend == La && jend == Lb) ? end_key32(v, 3, 0)
                                                : (jend == Lb ? end_key32(v, 2, iend - 1) : end_key32(v, 1, jend - 1));
                            k32 = kk > k32 ? kk : k32;
                        }
                    }
                }
                int score, ei, ej;
                decode_end(end_key_widen(k32), La, Lb, &score, &ei, &ej);
                const int dhi = dlo + W - 1;
                int pmax = -1;
                if (dhi < Lb - 1) pmax = max(pmax, min(Lb - dhi - 1, La));
                if (dlo > 1 - La) pmax = max(pmax, min(Lb, La + dlo - 1));
                const bool certified = pmax < 0 || score > m * pmax;
                const bool bad_code = (hdr.z & (h ? REGION_BAD_B : REGION_BAD_A)) != 0;
                const bool plain = amp_acgt && !(hdr.z & (h ? (REGION_BAD_B | REGION_NP_B) : (REGION_BAD_A | REGION_NP_A)));
                const int nd = min(ei, ej);
                const long long off = h ? (long long)(((unsigned long long)(unsigned)ho.w << 32) | (unsigned)ho.z)
                                        : (long long)(((unsigned long long)(unsigned)ho.y << 32) | (unsigned)ho.x);
                // mismatches of amplicon bytes [ia, ia + n) against read bytes [jb, jb + n) (plain: A C G T,
                // case folded), dword compares
                auto count_mis = [&](int ia, int jb, int n) -> int {
                    int c = 0;
                    const unsigned char* rp = a.reads + off + jb;
                    const int ra = (int)((uintptr_t)rp & 3), aa = ia & 3;
                    const unsigned* rw = (const unsigned*)(rp - ra);
                    const unsigned* aw = (const unsigned*)(amp_lds + (ia - aa));
                    unsigned rlo = rw[0], alo = aw[0];
#pragma unroll NW_MIS_UNROLL
                    for (int t = 0; t < n; t += 4) {
                        const unsigned rhi = rw[(t >> 2) + 1], ahi = aw[(t >> 2) + 1];
                        unsigned x = (__builtin_amdgcn_alignbyte(rhi, rlo, ra) ^ __builtin_amdgcn_alignbyte(ahi, alo, aa)) &
                                     0xdfdfdfdfu;
                        if (n - t < 4) x &= 0xffffffffu >> (8 * (4 - (n - t)));
                        c += 4 - __builtin_popcount(zero_bytes(x));
                        rlo = rhi;
                        alo = ahi;
                    }
                    return c;
                };
                bool cert = certified;
                if (!certified && !bad_code && score > m * pmax - O) {
                    // the refined certificate (band_single_diagonals_below): every single diagonal beyond the
                    // band whose overlap could reach the score sums below it -- a plain read's diagonal d
                    // sums to m P - 9 sc5 mis_d; other reads: the wave path
                    if (!plain) {
                        fate = 1;
                    } else {
                        cert = true;
                        for (int side = 0; side < 2 && cert; ++side) {
                            for (int kq = 1;; ++kq) {
                                const int d = side == 0 ? dhi + kq : dlo - kq;
                                const int P = diag_pairs(La, Lb, d);
                                if (P <= 0 || m * P < score) break;
                                const int i0 = d >= 0 ? 0 : -d, j0 = d >= 0 ? d : 0;
                                if (m * P - 9 * sc5 * count_mis(i0, j0, P) >= score) {
                                    cert = false;
                                    break;
                                }
                            }
                        }
                    }
                }
                if (fate != 0) {
                } else if (bad_code || !cert) {
                    fate = bad_code ? 3 : 2;
                } else if (!plain || nd >= 1024) {
                    fate = 1;
                } else {
                    // (no single-diagonal fast path here: when the start cell's diagonal sums to the score the
                    // walk's M rounds follow that diagonal to the edge -- M wins every tie on it -- and the record
                    // from the runs equals the diagonal's; a compare of every pair would cost as many rounds)
                    int nr = 0, tm = 0, tg = 0, tp = 0, last = -1;
                    bool over = false;
                    auto push = [&](int type, int n, bool paid) {
                        if (n <= 0) return;
                        if (type == RUN_M) tm += n; else tg += n;
                        if (paid) tp += (type == last ? 0 : O - E) + n * E;
                        if (type == last) {
                            lruns[64 * (nr - 1) + lane] += (unsigned)n;
                        } else if (nr < kLaneRuns) {
                            lruns[64 * nr + lane] = ((unsigned)type << 28) | (unsigned)n;
                            ++nr;
                            last = type;
                        } else {
                            over = true;
                        }
                    };
                    if (ei == La && ej < Lb) push(RUN_X, Lb - ej, false);
                    else if (ej == Lb && ei < La) push(RUN_Y, La - ei, false);
                    Stat r;
                    r.score = score;
                    r.end_i = ei;
                    r.end_j = ej;
                    r.flags = 0;
                    {
                        // band_walk_runs2, one lane: M runs scan kMRows tile rows (8 cells of their diagonal
                        // each) per round, X / Y runs 8 cells per round; the same stop rules
                        const unsigned* bits = (const unsigned*)(region + kHdrBytes + kCapBytes);
                        const int tb0 = kBK - dlo + 2 - tau0, hb = 8 * h;
                        int i = ei, j = ej, state = RUN_M, kc = 0;   // kc: cells of the current run so far
                        bool fail = false;
                        // the stop summary (band_summ_bytes): 16 blocks' bytes of one diagonal pair per load,
                        // kept while the M runs stay on that pair and chunk
                        const unsigned char* summ = (const unsigned char*)bits + (size_t)NW * (W / 2) * 4;
                        const int NBp = band_summ_bytes(NW);
                        int skey = -1;
                        uint4 sv = make_uint4(0u, 0u, 0u, 0u);
                        for (int guard = 0; i > 0 && j > 0 && !over && !fail; ++guard) {
                            if (guard > 4 * (La + Lb + 64)) {
                                fate = 1;
                                break;
                            }
                            if (state == RUN_M) {
                                const int kd = j - i - dlo;
                                if ((unsigned)kd >= (unsigned)W) {
                                    fail = true;
                                    break;
                                }
                                const int lim = min(i, j) - 1;
                                const int tc = i + j - 4 + tb0 - 2 * kc;   // tau of the next cell to test
                                const int r0 = tc >> 4, NR = NW >> 2;
                                if (tc >= 0 && r0 < NR) {
                                    // the first block at or below tc's with an "M < max" bit of this read on this
                                    // diagonal (tau parity p: sub-steps p, p + 2); the cells above it are clear
                                    const int b = tc >> 6, pq = kd >> 1;
                                    const unsigned shb = 4 * h + (tc & 1);
                                    int bf = -1;
                                    for (int ch = b >> 4; ch >= 0 && bf < 0; --ch) {
                                        if (skey != pq * 64 + ch) {
                                            sv = *(const uint4*)(summ + pq * NBp + 16 * ch);
                                            skey = pq * 64 + ch;
                                        }
                                        const unsigned sw[4] = {sv.x, sv.y, sv.z, sv.w};
                                        unsigned m16 = 0u;
#pragma unroll
                                        for (int e = 0; e < 4; ++e) {
                                            const unsigned t = (sw[e] >> shb) & 0x05050505u;
                                            const unsigned nz = (t + 0x7f7f7f7fu) & 0x80808080u;   // bytes with a bit
                                            m16 |= (((nz >> 7) & 1u) | ((nz >> 14) & 2u) | ((nz >> 21) & 4u) | ((nz >> 28) & 8u))
                                                   << (4 * e);
                                        }
                                        const int top = ch == (b >> 4) ? (b & 15) : 15;
                                        const unsigned cand = m16 & ((2u << top) - 1u);
                                        if (cand) bf = 16 * ch + 31 - __builtin_clz(cand);
                                    }
                                    if (bf < b) {   // skip the clear blocks (to the matrix edge when none is flagged)
                                        const int tstop = bf < 0 ? -1 : 64 * bf + 63;
                                        const int cnt = (tc - tstop + 1) >> 1;   // cells with tau > tstop
                                        const int L = lim - kc;
                                        if (cnt > L) {   // the run reaches the matrix edge first
                                            const int run = kc + max(L, 0) + 1;
                                            push(RUN_M, run, false);
                                            i -= run;
                                            j -= run;
                                            kc = 0;
                                        } else {
                                            kc += cnt;
                                        }
                                        continue;
                                    }
                                }
                                // kMRows tile rows per round (8 cells of the diagonal each), their loads together
                                uint4 v[kMRows];
#pragma unroll
                                for (int q = 0; q < kMRows; ++q)
                                    v[q] = r0 - q >= 0 && r0 - q < NR ? *(const uint4*)(bits + (r0 - q) * (2 * W) + 4 * (kd >> 1))
                                                                      : make_uint4(0u, 0u, 0u, 0u);
                                // the rows' cells of this diagonal in decreasing tau, from the "M < max" bits of its
                                // parity (s = p: bit sh, s = p + 2: bit sh + 2 of each word)
                                const int p = tc & 1;
                                const unsigned sh = 20 + hb + p;
                                unsigned long long all = 0ull, oddr = 0ull;
#pragma unroll
                                for (int q = 0; q < kMRows; ++q) {
                                    const unsigned w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
                                    unsigned mm = 0u;
#pragma unroll
                                    for (int e = 0; e < 4; ++e) {
                                        const unsigned t = w[e] >> sh;
                                        mm |= (((t >> 2) & 1u) | ((t & 1u) << 1)) << (2 * (3 - e));
                                    }
                                    all |= (unsigned long long)mm << (8 * q);
                                    // a cell of the matrix outside the stored steps: the wave path's clamps decide
                                    if (r0 - q < 0 || r0 - q >= NR) oddr |= 0xffull << (8 * q);
                                }
                                constexpr int kCells = 8 * kMRows;
                                const int c0 = (16 * r0 + 14 + p - tc) >> 1;   // cell tc's place in row r0 (0 .. 7)
                                const int ncell = kCells - c0;
                                const unsigned cells = (unsigned)((1ull << ncell) - 1ull);
                                const unsigned nm = (unsigned)(all >> c0) & cells;
                                const int L = lim - kc;   // cells u < L are inside the matrix
                                const unsigned inm = L <= 0 ? 0u : (L >= ncell ? cells : (1u << L) - 1u);
                                const unsigned stop = nm | (cells & ~inm);
                                const unsigned odd = (unsigned)(oddr >> c0) & inm;
                                const unsigned upto = stop ? (unsigned)((2ull << __builtin_ctz(stop)) - 1ull) : 0xffffffffu;
                                if (odd & upto) {
                                    fate = 1;
                                    break;
                                }
                                if (stop) {
                                    const int u0 = __builtin_ctz(stop);
                                    const int run = kc + u0 + 1;
                                    push(RUN_M, run, false);
                                    i -= run;
                                    j -= run;
                                    const int ts = tc - 2 * u0;   // the stop cell: "Y > X" picks the gap it continues in
                                    uint4 vs = v[0];
#pragma unroll
                                    for (int q = 1; q < kMRows; ++q) vs = (ts >> 4) == r0 - q ? v[q] : vs;
                                    const int qs = (ts >> 2) & 3;
                                    const unsigned ws = qs == 0 ? vs.x : (qs == 1 ? vs.y : (qs == 2 ? vs.z : vs.w));
                                    state = ((ws >> (4 + hb + (ts & 3))) & 1u) ? RUN_Y : RUN_X;
                                    kc = 0;
                                } else {
                                    kc += ncell;
                                }
                            } else {
                                const bool isX = state == RUN_X;
                                const int lim = isX ? j : i;
                                const int kd0 = j - i - dlo;
                                const int t0 = i + j - 2 + tb0;
                                const int bit = isX ? 16 : 0;
                                unsigned stop = 0u, oob = 0u;
#pragma unroll
                                for (int u = 0; u < 8; ++u) {
                                    const int kk = kc + u;
                                    const int kd = isX ? kd0 - kk : kd0 + kk;
                                    const int tau = t0 - kk;
                                    const bool out = (unsigned)kd >= (unsigned)W;
                                    const int wd = min(max(tau, 0) >> 2, NW - 1);
                                    const bool valid = kk < lim;
                                    const unsigned w = (valid && !out)
                                                           ? bits[(wd >> 2) * (2 * W) + 4 * ((kd & (W - 1)) >> 1) + (wd & 3)]
                                                           : 0u;
                                    const bool opens = ((w >> (bit + hb + (tau & 3))) & 1u) != 0u;
                                    stop |= (unsigned)(!valid || out || opens) << u;
                                    oob |= (unsigned)(valid && out) << u;
                                }
                                if (stop) {
                                    const int u0 = __builtin_ctz(stop);
                                    if ((oob >> u0) & 1u) {
                                        fail = true;
                                        break;
                                    }
                                    const int run = kc + u0 + 1;
                                    push(state, run, true);
                                    if (isX) j -= run; else i -= run;
                                    state = RUN_M;
                                    kc = 0;
                                } else {
                                    kc += 8;
                                }
                            }
                        }
                        if (fate == 0) {
                            if (fail) {
                                fate = 2;
                            } else {
                                if (i > 0) push(RUN_Y, i, false);
                                if (j > 0) push(RUN_X, j, false);
                                // a plain read's record from its runs and score: m id - x (M - id) - paid gaps
                                const int idn = score + tp + 4 * sc5 * tm;
                                if (over || idn < 0 || idn % (9 * sc5) != 0) {
                                    fate = 1;
                                } else {
                                    r.aln_len = tm + tg;
                                    r.n_ident = idn / (9 * sc5);
                                    r.n_sim = r.n_ident;
                                    r.n_gaps = tg;
                                }
                            }
                        }
                    }
                    if (fate == 0 && over) fate = 1;
                    if (fate == 0) {
                        // store_ops for one lane: its runs start -> end into its slot (or the spill area)
                        uint32_t* dst = a.ops + a.ops_stride * a.ops_slot + rd * a.ops_slot;
                        int32_t flag = kNopsRows;
                        bool lost = false;
                        if (nr > a.ops_slot) {
                            flag = 0;
                            const int pos = atomicAdd(a.ops_ctl, nr);
                            if ((long long)pos + nr > a.spill_cap) {
                                atomicOr(a.ops_ctl + 1, 1);
                                a.nops[rd] = 0;
                                lost = true;
                            } else {
                                a.ops[rd] = (uint32_t)pos;
                                dst = a.spill + pos;
                            }
                        }
                        if (!lost) {
                            a.nops[rd] = nr | flag;
                            for (int q = 0; q < nr; ++q) dst[q] = lruns[64 * (nr - 1 - q) + lane];
                        }
                        a.stats[rd] = r;
                    }
                }
            }
        }
        // the lists: one atomic per list and wavefront (redo flags instead when the level keeps them)
        const unsigned long long to_redo = __ballot(fate == 2 && !a.redo_flags), to_fb = __ballot(fate == 3);
        if (fate == 2 && a.redo_flags) a.redo_flags[k] = 1;
        if (to_redo) {
            int base = 0;
            if (lane == 0) base = atomicAdd(a.redo_count, (int)__builtin_popcountll(to_redo));
            base = __builtin_amdgcn_readfirstlane(base);
            if ((to_redo >> lane) & 1ull) a.redo_list[base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(to_redo >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)to_redo, 0u))] = (int)rd;
        }
        if (to_fb) {
            int base = 0;
            if (lane == 0) base = atomicAdd(a.fallback_count, (int)__builtin_popcountll(to_fb));
            base = __builtin_amdgcn_readfirstlane(base);
            if ((to_fb >> lane) & 1ull) a.fallback_list[base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(to_fb >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)to_fb, 0u))] = rd;
        }
        // the wave path for the rest, one read at a time (its LDS buffers overlay lruns: read above)
        lds_fence();
        for (unsigned long long dq = __ballot(fate == 1); dq; dq &= dq - 1) {
            const int u = (int)__builtin_ctzll(dq);
            const long long ku = klo + 64 * g + u;
            defer(ku);
            lds_fence();
        }
    }
}

// W < kBandDiags: a first level; reads it cannot certify go to the redo list of the
// next (wider) level.  W >= kBandDiags: they go to the fallback list (W = kBandDiags: the
// wide level's input; the wide level: the exact int32 kernel's).
template <int W, bool LN = false>   // LN: the lane walk (walk_lanes) first, W < kBandDiags, ops output
#define NW_WALK_WPE 6
#define NW_WALK_LANE_WPE 4   // the lane walk: 116 VGPRs, no spills (5: 96 with 11 spilled, walk 0.091 vs 0.085 ms); a resident pass runs ~9 of its wavefronts per CU
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(LN ? NW_WALK_LANE_WPE : NW_WALK_WPE))) void nw_band_walk(const KernelArgs a) {
    using G = BandGeo<W>;
    constexpr int kCapBytes = G::CapBytes;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // second level skipped: its reads go to the wide level (with the seeded list: that list alone)
    if (W == kBandDiags && redo_direct_taken(a) && a.seed_l2 != 1) return;
    if (W < kBandDiags && l1_skipped(a)) return;   // first level skipped (KernelArgs::l1_skip)
    if (W >= kBandDiags && a.tail_prio) __builtin_amdgcn_s_setprio(3);
    constexpr int CW = W > 64 ? W / 64 : 1;   // captures (band diagonals) per lane
    const int La = a.La, E = a.gap_extend;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wpb = blockDim.x >> 6;
    // Reads handed on (next level's redo list, or the exact kernel's list) wait in a
    // lane of the wavefront (entry p in lane p) and go out 64 at a time: one atomic
    // per 64 reads and one coalesced store (a per-read atomic on one counter serialises
    // when most reads are handed on, e.g. the HDR pass).  Called wave-uniformly.
    int redo_n = 0, fb_n = 0;
    int redo_v = 0;
    long long fb_v = 0;
    auto flush_redo = [&]() {
        int base = 0;
        if (lane == 0) base = atomicAdd(a.redo_count, redo_n);
        base = __builtin_amdgcn_readfirstlane(base);
        if (lane < redo_n) a.redo_list[base + lane] = redo_v;
        redo_n = 0;
    };
    auto flush_fb = [&]() {
        int base = 0;
        if (lane == 0) base = atomicAdd(a.fallback_count, fb_n);
        base = __builtin_amdgcn_readfirstlane(base);
        if (lane < fb_n) a.fallback_list[base + lane] = fb_v;
        fb_n = 0;
    };
    // the second level over the seeded list (seed_l2 == 1): positions from l2_s0 on are seeded reads
    const bool l2s = W == kBandDiags && a.seed_l2 == 1;
    const long long l2_nr = l2s ? l2_redo_n(a) : 0ll;
    const long long l2_s0 = l2s ? (l2_nr + 1) & ~1ll : (1ll << 62);
    auto seed_done = [&](long long k) {   // a seeded read's record and runs are out
        if (k >= l2_s0 && lane == 0) a.seed_flags[k - l2_s0] = 0;
    };
    auto give_up = [&](long long k, long long rd, bool retry) {
        if (k >= l2_s0) {   // a seeded read: to the wide level, in the seeded list's order (compaction)
            if (lane == 0) a.seed_flags[k - l2_s0] = 1;
            return;
        }
        if (W < kBandDiags && retry && a.redo_flags) {
            // the next level's list keeps the sorted order (nw_band_redo_* compaction):
            // its pairs are reads of similar length, as on this level
            if (lane == 0) a.redo_flags[k] = 1;
        } else if (W < kBandDiags && retry) {
            if (lane == redo_n) redo_v = (int)rd;
            if (++redo_n == 64) flush_redo();
        } else {
            if (lane == fb_n) fb_v = rd;
            if (++fb_n == 64) flush_fb();
        }
    };
    unsigned char* lut_lds = smem;
    unsigned char* amp_lds = smem + 256;
    unsigned* rowpos = (unsigned*)(smem + 256 + align16(La + 16));
    unsigned* sub_lds = rowpos + align16(4 * La) / 4;   // [17][4]: EDNAFULL(a, b) * scale, int8, b = 0..15
    for (int k = tid; k < 256; k += blockDim.x) lut_lds[k] = a.lut[k];
    for (int k = tid; k < La; k += blockDim.x) {
        amp_lds[k] = a.amp[k];
        rowpos[k] = a.rowpos[k];
    }
    for (int k = tid; k < 17 * 4; k += blockDim.x) sub_lds[k] = a.sub16[k];
    int acgt = 1;
    for (int k = tid; k < La; k += blockDim.x) {
        const unsigned char c = upcase(a.amp[k]);
        acgt &= c == 'A' || c == 'C' || c == 'G' || c == 'T';
    }
    // a plain read (A C G T against an A C G T amplicon, EDNAFULL): every pair scores +m or -x
    // (x = 4 m / 5), so a diagonal's sum, and an alignment's identities, follow from its score
    const int sc5 = a.band_maxsub / 5;
    const bool amp_acgt = __syncthreads_and(acgt) && a.band_maxsub == 5 * sc5;
    // substitution score of amplicon byte x against read byte y (0 for codes outside EDNAFULL)
    auto sub_of = [&](unsigned char x, unsigned char y) {
        const int cx = lut_lds[x], cy = lut_lds[y];
        return cy < 16 ? (int)(signed char)(sub_lds[cx * 4 + (cy >> 2)] >> (8 * (cy & 3))) : 0;
    };
    const int row = band_walk_row(La, a.Lb_max);   // columns <= La + Lb
    const int rcap = band_walk_rcap(a.Lb_max);
    constexpr int kSlot = band_walk_hdr_slot(W);   // dwords of a pair header + captures slot
    unsigned char* wb = smem + band_walk_shared_bytes(La) + wave * band_walk_wave_bytes(La, a.Lb_max, W);
    unsigned* runs = (unsigned*)wb;
    unsigned char* rbufs = wb + kBandRunsCap * 4;               // [2][rcap + 256]: read bytes (DMA)
    unsigned* hbufs = (unsigned*)(rbufs + 2 * (rcap + 256));    // [2][kSlot]: pair header + captures (DMA)
    unsigned char* rows = (unsigned char*)(hbufs + 2 * kSlot);

    const long long count = band_list_count(a);
    const long long klo = 2 * a.band_pair_lo;
    const long long khi = 2 * a.band_pair_hi < count ? 2 * a.band_pair_hi : count;
    // Per read, everything it needs from memory before its walk -- the pair header (reads,
    // lengths, offsets, geometry), the W captures and the read's bytes -- lands in LDS by DMA
    // ahead of it: read k's bytes (and read k + kstep's header) go out right after read
    // k - kstep's wait, so they travel during that read's walk; read k's own wait (vmcnt 0)
    // then finds them landed, and only the walk's rounds wait on memory.
    const long long kstep = (long long)gridDim.x * wpb;
    auto region_of = [&](long long k) { return a.band_region + ((k >> 1) - a.band_pair_lo) * a.band_stride; };
    auto load_hdr = [&](long long kk, unsigned* dst) {   // header and captures: the region's first kSlot dwords
        const unsigned char* rg = region_of(kk);
#pragma unroll
        for (int m = 0; m < kSlot; m += 64)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(rg + 4 * (m + lane)),
                                             (__attribute__((address_space(3))) void*)(dst + m), 4, 0, 0);
    };
    auto uni = [](int4 v) {   // the header is wave-uniform: SGPRs, scalar branches
        return make_int4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                         __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
    };
    // read kk's length and byte offset from its header slot (kk & 1: read B of the pair)
    auto read_of = [&](const unsigned* hb, long long kk, int* Lb, long long* off) {
        const int4 hr = uni(*(const int4*)(hb + 4)), ho = uni(*(const int4*)(hb + 8));
        const bool hB = (kk & 1) != 0;
        *Lb = hB ? hr.w : hr.z;
        *off = hB ? (long long)(((unsigned long long)(unsigned)ho.w << 32) | (unsigned)ho.z)
                  : (long long)(((unsigned long long)(unsigned)ho.y << 32) | (unsigned)ho.x);
    };
    auto load_bytes = [&](long long off, int Lb, unsigned char* dst) {   // Lb <= rcap
        const unsigned char* raw = a.reads + off;
        const int ms = (int)((uintptr_t)raw & 3);
        for (int m = 0; m < Lb + ms; m += 256)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(raw - ms + m + 4 * lane),
                                             (__attribute__((address_space(3))) void*)(dst + m), 4, 0, 0);
    };
    // read k once its header (hb: pair header + captures) and bytes (rbuf) are in LDS and have landed
    auto process = [&](long long k, const int4 hdr, const int4 hr, const unsigned* cw, int h, long long rd, int Lb,
                       long long off, unsigned char* rbuf) {
        if (W < kBandDiags && a.redo_flags && lane == 0) a.redo_flags[k] = 0;   // give_up may set it
        // a pair of one read (the seeded list's padding, the 32-diagonal level's hole): its first position
        if (W >= kBandDiags && (k & 1) && hr.x == hr.y) {
            seed_done(k);   // (its flag: the pair's first position decides)
            return;
        }
        if (Lb <= 0) {
            if (lane == 0) {
                Stat z = {};
                z.flags = FLAG_EMPTY;
                a.stats[rd] = z;
                if (a.ops) a.nops[rd] = 0;
            }
            return;
        }
        if (hdr.z & kPairInactive) {   // too long, or the pair's lengths do not fit the band
            give_up(k, rd, true);
            return;
        }
        const int dlo = hdr.y;
        const unsigned char* region = region_of(k);
        if (Lb > rcap) {   // not reached: rcap covers the band length cap
            give_up(k, rd, false);
            return;
        }
        const int mis = (int)((uintptr_t)(a.reads + off) & 3);
        const int tau0 = hdr.x;
        // start cell: the last cell of each band diagonal is on the last row or column
        unsigned k32 = 0u;
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            if (lane + 64 * c >= W) continue;
            const int d = dlo + lane + 64 * c;
            const int iend = La < Lb - d ? La : Lb - d;
            const int ilo = 1 - d > 1 ? 1 - d : 1;
            if (iend >= ilo) {
                const int v = half(cw[c], h) - kBias16 - E * (2 * iend + d);
                const int jend = iend + d;
                const unsigned kk = (iend == La && jend == Lb) ? end_key32(v, 3, 0)
                                    : (jend == Lb ? end_key32(v, 2, iend - 1) : end_key32(v, 1, jend - 1));
                k32 = kk > k32 ? kk : k32;
            }
        }
        int score, ei, ej;
        decode_end(end_key_widen(wave_max_u32(k32)), La, Lb, &score, &ei, &ej);
        score = __builtin_amdgcn_readfirstlane(score);
        ei = __builtin_amdgcn_readfirstlane(ei);
        ej = __builtin_amdgcn_readfirstlane(ej);
        // certificate: every alignment leaving the band scores <= UB < score
        const int dhi = dlo + W - 1;
        int pmax = -1;
        if (dhi < Lb - 1) pmax = max(pmax, min(Lb - dhi - 1, La));
        if (dlo > 1 - La) pmax = max(pmax, min(Lb, La + dlo - 1));
        bool certified = pmax < 0 || score > a.band_maxsub * pmax;
        const bool bad_code = (hdr.z & (h ? REGION_BAD_B : REGION_BAD_A)) != 0;
        if (W >= kBandDiags && (hdr.z & REGION_SEEDED) && !certified) {
            // Seeded band: every exact hit of the read's nb disjoint 16-base blocks
            // lies on diagonals [smin, smax] inside the band.  An alignment with a cell outside the
            // band either has a block paired as an exact match -- on one of those diagonals, so its
            // gaps shift it by >= dexit diagonals: it scores <= m Lb - O - (dexit - 1) E -- or has
            // none: each block then loses >= m (an unpaired base, a mismatch, or a gap opened
            // inside it, O >= m), <= m (Lb - nb).  Plain reads and amplicon, EDNAFULL 5 / -4.
            const int32_t si = a.seed_info[rd];
            const int smin = seed_dmin(si), smax = seed_dmax(si), nb = seed_blocks(si);
            const int dexit = min(smin - dlo + 1, dhi - smax + 1);
            const int m = a.band_maxsub;
            const bool plainr = amp_acgt && !(hdr.z & (h ? (REGION_BAD_B | REGION_NP_B) : (REGION_BAD_A | REGION_NP_A)));
            const bool pen_ok = a.gap_open >= m && a.gap_open >= a.gap_extend && a.gap_extend >= 0;
            certified = plainr && seed_valid(si) && dexit >= 1 && pen_ok && score > m * (Lb - nb) &&
                        score > m * Lb - a.gap_open - (dexit - 1) * a.gap_extend;
            const int32_t si2 = a.seed_info2 ? a.seed_info2[rd] : 0;
            if (!certified && plainr && seed_valid(si) && seed2_valid(si2) && dexit >= 1 && pen_ok) {
                // Refined (round 5): a block not paired as an exact match loses >= m when it can sit
                // in a free end gap (the first and the last block), else >= w = min(m + x, O, m + O / 2)
                // -- a mismatch, a deletion opened inside it, or unpaired bases in an insertion whose
                // open it shares with at most one neighbouring block.  An alignment with a cell outside
                // the band pairs (a) no block exactly: every block loses; (b) blocks on one diagonal only:
                // the others lose and it moves >= d_exit diagonals; (c) blocks on two diagonals: it also
                // pays the cheapest move between them (seed_info2).  S above all three bounds.
                const int x = 4 * (m / 5), O = a.gap_open;
                const int w = min(min(m + x, O), m + O / 2);
                auto lose = [&](int k) { return w * max(0, k - 2) + m * min(k, 2); };
                const int ex = O + (dexit - 1) * a.gap_extend;
                const int ba = lose(nb);
                const int bb = ex + lose(max(0, nb - seed2_cmax(si2)));
                const int bc = seed2_shift(si2) >= 0xffff ? (1 << 30) : ex + seed2_shift(si2) + lose(seed2_n0(si2));
                const int loss = m * Lb - score;
                certified = loss < ba && loss < bb && loss < bc;
            }
        }
        if (!certified && !bad_code && score > a.band_maxsub * pmax - a.gap_open) {
            // Refined bound: an alignment leaving the band with an internal gap pays at
            // least the gap open, so it scores <= maxsub * pmax - O < score; one without
            // internal gaps is a single diagonal d (free end gaps), paired over its whole
            // overlap P(d): its score S_d is computed exactly, for the few diagonals beyond
            // the band with maxsub * P(d) >= score (P falls by one per diagonal: at most
            // about two per side, as score > maxsub * (pmax - 2)).
            certified = band_single_diagonals_below(a, amp_lds, rbuf + mis, La, Lb, dlo, dhi, score, lane);
        }
        if (bad_code || !certified) {
            give_up(k, rd, !bad_code);   // IUPAC codes: no band helps
            return;
        }
        // Single-diagonal fast path: when the start cell's score equals the plain sum of
        // substitution scores down its diagonal to the matrix edge, D(ei, ej), the
        // traceback is that diagonal (M(i, j) >= D(i, j) everywhere, so H = M = D on
        // each of its cells, and M wins ties), with the end gaps around it: no band bits
        // are read.  Reads with substitutions only (most non-identical reads) take it.
        int nruns;
        const int nd = min(ei, ej);
        const bool plain = amp_acgt && !(hdr.z & (h ? (REGION_BAD_B | REGION_NP_B) : (REGION_BAD_A | REGION_NP_A)));
        // a plain read's diagonal sums to m nd - (m + x) k for its k mismatches: a score not of that
        // form cannot be the diagonal's (reads with an indel: the test's loop is skipped)
        const int dres = a.band_maxsub * nd - score;
        const bool maybe_diag = !plain || (dres >= 0 && dres % (9 * sc5) == 0);
        int dsum = 0;
        unsigned cnt = 0u;   // identical | similar << 10 | gap columns << 20 of the diagonal (band_emit's counts)
        for (int t = lane; maybe_diag && t < nd; t += 64) {
            const unsigned char ca = amp_lds[ei - 1 - t], cb = rbuf[mis + ej - 1 - t];
            const int sc = sub_of(ca, cb);
            dsum += sc;
            const bool gapc = ca == '-' || cb == '-';   // an input '-' prints as a gap (CORE:1846)
            const bool id = !gapc && upcase(ca) == upcase(cb);
            const bool sim = !gapc && (id || sc > 0);
            cnt += (unsigned)id | ((unsigned)sim << 10) | ((unsigned)gapc << 20);
        }
        const bool diag = maybe_diag && wave_sum(dsum) == score;
        if (diag) {
            const bool endg = (ei == La && ej < Lb) || (ej == Lb && ei < La);
            const int lead = max(ei, ej) - nd;   // leading gap run (Y when ei > nd, X when ej > nd)
            if (lane == 0) {
                int q = 0;
                if (ei == La && ej < Lb) runs[q++] = ((unsigned)RUN_X << 28) | (unsigned)(Lb - ej);
                else if (ej == Lb && ei < La) runs[q++] = ((unsigned)RUN_Y << 28) | (unsigned)(La - ei);
                runs[q++] = ((unsigned)RUN_M << 28) | (unsigned)nd;
                if (ei > nd) runs[q++] = ((unsigned)RUN_Y << 28) | (unsigned)(ei - nd);
                else if (ej > nd) runs[q++] = ((unsigned)RUN_X << 28) | (unsigned)(ej - nd);
            }
            nruns = 1 + (int)endg + (lead > 0);
            if (a.ops && nd < 1024) {
                // ops output: the record comes from the diagonal's counts; no emit pass
                lds_fence();
                store_ops(a, rd, runs, nruns, lane);
                const unsigned t = wave_sum_u32(cnt);
                if (lane == 0) {
                    const int endlen = endg ? (ei == La ? Lb - ej : La - ei) : 0;
                    Stat r;
                    r.aln_len = nd + endlen + lead;
                    r.n_ident = (int)(t & 1023u);
                    r.n_sim = (int)((t >> 10) & 1023u);
                    r.n_gaps = (int)(t >> 20) + endlen + lead;
                    r.score = score;
                    r.end_i = ei;
                    r.end_j = ej;
                    r.flags = 0;
                    a.stats[rd] = r;
                }
                lds_fence();
                seed_done(k);
                return;
            }
        } else {
            const unsigned* bits = (const unsigned*)(region + kHdrBytes + kCapBytes);
            const int tb0 = kBK - dlo + 2 - tau0;
            int tot[3];
            nruns = band_walk_runs2<NW_BAND_WALK_CPL, W>(bits, a.band_words, La, Lb, ei, ej, dlo, tb0, h, runs,
                                                         kBandRunsCap, lane, a.gap_open, a.gap_extend, tot);
            // ops output, plain read: the record from the runs and the score (score = m id - x (M - id) -
            // paid gaps), no emit pass; similar pairs are the identical ones
            const int idn = score + tot[2] + 4 * sc5 * tot[0];
            if (a.ops && plain && nruns >= 0 && idn >= 0 && idn % (9 * sc5) == 0) {
                lds_fence();
                store_ops(a, rd, runs, nruns, lane);
                if (lane == 0) {
                    Stat r;
                    r.aln_len = tot[0] + tot[1];
                    r.n_ident = idn / (9 * sc5);
                    r.n_sim = r.n_ident;
                    r.n_gaps = tot[1];
                    r.score = score;
                    r.end_i = ei;
                    r.end_j = ej;
                    r.flags = 0;
                    a.stats[rd] = r;
                }
                lds_fence();
                seed_done(k);
                return;
            }
        }
        if (nruns < 0) {
            give_up(k, rd, true);
            return;
        }
        lds_fence();
        auto sim = [&](int ai, int code) { return (int)((rowpos[ai] >> code) & 1u); };
        if (a.ops) {
            store_ops(a, rd, runs, nruns, lane);
            band_emit<false>(runs, nruns, amp_lds, rbuf + mis, lut_lds, sim, rows, row, nullptr, 0, score, ei, ej,
                             a.stats + rd, lane);
        } else {
            band_emit<true>(runs, nruns, amp_lds, rbuf + mis, lut_lds, sim, rows, row, a.out + rd * 3 * a.stride, a.stride,
                            score, ei, ej, a.stats + rd, lane);
        }
        lds_fence();
        seed_done(k);
    };
    if constexpr (LN && W < kBandDiags) {
        if (a.ops) {
            walk_lanes<W>(a, klo, khi, wb, amp_lds, amp_acgt, sc5, [&](long long kq) {
                // a read the lane walk leaves to the wave path: its header, captures and bytes into
                // LDS, then the per-read body
                load_hdr(kq, hbufs);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int4 hdr = uni(*(const int4*)hbufs), hr = uni(*(const int4*)(hbufs + 4));
                unsigned cw[CW];
#pragma unroll
                for (int c = 0; c < CW; ++c) cw[c] = lane + 64 * c < W ? hbufs[kHdrBytes / 4 + lane + 64 * c] : 0u;
                const int h = (int)(kq & 1);
                const long long rd = h ? hr.y : hr.x;
                int Lb;
                long long off;
                read_of(hbufs, kq, &Lb, &off);
                if (Lb > 0 && Lb <= rcap) load_bytes(off, Lb, rbufs);
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                process(kq, hdr, hr, cw, h, rd, Lb, off, rbufs);
            });
            if (redo_n) flush_redo();
            if (fb_n) flush_fb();
            return;
        }
    }
    long long k = klo + (long long)blockIdx.x * wpb + wave;
    int it = 0;   // parity of the slots holding read k's header and bytes
    if (k < khi) {   // the pipeline's start: read k's header, then its bytes and the next header
        load_hdr(k, hbufs);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int Lb0;
        long long off0;
        read_of(hbufs, k, &Lb0, &off0);
        if (Lb0 > 0 && Lb0 <= rcap) load_bytes(off0, Lb0, rbufs);
        if (k + kstep < khi) load_hdr(k + kstep, hbufs + kSlot);
    }
    for (; k < khi; k += kstep, it ^= 1) {
        const unsigned* hb = hbufs + it * kSlot;   // landed: the previous read's wait
        unsigned char* rbuf = rbufs + it * (rcap + 256);
        const int4 hdr = uni(*(const int4*)hb), hr = uni(*(const int4*)(hb + 4));
        unsigned cw[CW];
#pragma unroll
        for (int c = 0; c < CW; ++c) cw[c] = lane + 64 * c < W ? hb[kHdrBytes / 4 + lane + 64 * c] : 0u;
        const int h = (int)(k & 1);
        const long long rd = h ? hr.y : hr.x;
        int Lb;
        long long off;
        read_of(hb, k, &Lb, &off);
        // every load issued for this read has landed (its bytes, the next read's header), and the
        // header reads above are done (lgkmcnt); the next read's bytes and the header after it go
        // out now, into the slots the previous read used and this read's header slot
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if (k + kstep < khi) {
            unsigned* hn = hbufs + (it ^ 1) * kSlot;
            int Lbn;
            long long offn;
            read_of(hn, k + kstep, &Lbn, &offn);
            if (Lbn > 0 && Lbn <= rcap) load_bytes(offn, Lbn, rbufs + (it ^ 1) * (rcap + 256));
            if (k + 2 * kstep < khi) load_hdr(k + 2 * kstep, hbufs + it * kSlot);   // this read's header is in registers
        }
        process(k, hdr, hr, cw, h, rd, Lb, off, rbuf);
    }
    if constexpr (W > kBandDiags) {
        // the wide level's list entries past its region's capacity: straight to the exact kernel
        const long long nb = (long long)*a.band_count;
        for (long long k2 = khi + (long long)blockIdx.x * wpb + wave; k2 < count; k2 += kstep)
            if (!((k2 & 1) && band_list_read(a, k2 - 1, nb) == band_list_read(a, k2, nb))) give_up(k2, band_list_read(a, k2, nb), false);
    }
    if (redo_n) flush_redo();
    if (fb_n) flush_fb();
}

// ============================================================================
// Redo list of the second level: the sorted positions the first level flagged,
// compacted in sorted order (block sums, one scan block, scatter): no atomics,
// deterministic, and consecutive entries (the second level's pairs) have similar
// lengths.  Positions [0, *band_count) are the first level's.
// ============================================================================
constexpr int kRedoBlock = 1024;   // positions per block (256 threads x 4)

__device__ int block_excl_scan_i32(int v, int* total) {
    __shared__ int wsum[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        before += w < wave ? wsum[w] : 0;
        all += wsum[w];
    }
    __syncthreads();
    *total = all;
    return before + incl - v;
}

// One launch: flags of block b's 1024 positions, its exclusive prefix by look-back,
// scatter; the last block writes the count (*redo_count).  pairs: positions 2q, 2q + 1 are kept
// together when either is flagged (the seeded list's pairs stay pairs).
__global__ __launch_bounds__(256) void nw_band_redo_compact(const KernelArgs a, unsigned epoch, int pairs) {
    __shared__ int sh[2];
    if (a.tail_prio) __builtin_amdgcn_s_setprio(3);
    const long long nb = *a.band_count;
    const long long n = band_list_count(a);
    const long long k0 = (long long)blockIdx.x * kRedoBlock + threadIdx.x * 4;
    int f[4], s = 0;
    const bool all = l1_skipped(a);   // the first level was skipped: every position goes on
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        f[t] = k0 + t < n ? (all ? 1 : a.redo_flags[k0 + t]) : 0;
    }
    if (pairs) {   // (k0 is even: positions k0 .. k0 + 3 are two whole pairs)
        f[0] = f[1] = f[0] | f[1];
        f[2] = f[3] = f[2] | f[3];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        f[t] = f[t] && k0 + t < n;
        s += f[t];
    }
    if (threadIdx.x == 0) sh[1] = 0;
    int total;
    const int local = block_excl_scan_i32(s, &total);
    if (threadIdx.x < 64) {
        const unsigned e = lookback_excl(a.lb_status, blockIdx.x, epoch, (unsigned)total, &sh[1]);
        if (threadIdx.x == 0) sh[0] = (int)e;
    }
    __syncthreads();
    long long pos = sh[0] + local;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        if (f[t]) a.redo_list[pos++] = (int32_t)band_list_read(a, k0 + t, nb);
    if (threadIdx.x == 0) {
        if (sh[1]) a.fallback_count[3] = 1;
        if (blockIdx.x == gridDim.x - 1) *a.redo_count = (int32_t)(sh[0] + total);
    }
}

hipError_t launch_redo_compact(const KernelArgs& a, int64_t nmax, unsigned epoch, hipStream_t s, bool pairs) {
    const int nblk = (int)std::max<int64_t>(1, (nmax + kRedoBlock - 1) / kRedoBlock);
    hipLaunchKernelGGL(nw_band_redo_compact, dim3(nblk), dim3(256), 0, s, a, epoch, pairs ? 1 : 0);
    return hipGetLastError();
}

// ---- host-side helpers -------------------------------------------------------
int band_fill_lds_bytes(int La, int wpb, int W) {
    const int pw = W == 16 ? BandGeo<16>::PW : W == 32 ? BandGeo<32>::PW : BandGeo<kWideDiags>::PW;
    return kTabBytes + align16(2 * band_acd_elems(La)) + wpb * pw * band_pcs(La, W) + 256 + wpb * 1024 +
           (W == 16 ? wpb * 1280 : 0);   // + the stop summary's per-lane accumulators and 16-block chunks
}
int band_walk_lds_bytes(int La, int wpb, int lb_max, int W) {
    return band_walk_shared_bytes(La) + wpb * band_walk_wave_bytes(La, lb_max, W);
}
int band_region_words(int La, int Lb_max, int W) { return band_words(La, Lb_max, W > kBandDiags ? W : kBandDiags); }
int64_t band_region_bytes(int La, int Lb_max, int W) { return band_region_stride(La, Lb_max, W); }
bool band_pair_geometry(int La, int Lb, int* dlo) { return band_geometry(La, Lb, dlo); }

hipError_t band_occupancy(int W, int fill_wpb, int walk_wpb, int fill_lds, int walk_lds, int* fill_blocks,
                          int* walk_blocks) {
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        fill_blocks,
        W == 16 ? (const void*)nw_band_fill<16>
                : (W == 32 ? (const void*)nw_band_fill<32> : (const void*)nw_band_fill<kWideDiags>),
        64 * fill_wpb, fill_lds);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        walk_blocks,
        W == 16 ? (const void*)nw_band_walk<16> : (W == 32 ? (const void*)nw_band_walk<32> : (const void*)nw_band_walk<kWideDiags>),
        64 * walk_wpb, walk_lds);
}

// classify (exact copies, sort keys) then the segment sort; a.band_count receives the
// DP count, a.lb_status holds ceil(n / kSegReads) look-back words
hipError_t launch_band_sort(const KernelArgs& a, unsigned epoch, hipStream_t s) {
    if (a.pk_words) {   // one block per call block of 256 reads the chunk touches
        const int64_t g0 = a.pk_call_lo / 256, g1 = (a.pk_call_lo + a.n - 1) / 256;
        const size_t lds = (size_t)(8 * ((a.La + 3) / 4)) +
                           (a.amp2 ? (size_t)(4 * ((a.La + 15) / 16 + 2) + 6 * a.n_seed + 16) : 0);
        hipLaunchKernelGGL(nw_band_classify<true>, dim3((unsigned)(g1 - g0 + 1)), dim3(256), lds, s, a);
        if (a.cert_q) {   // its four wavefronts' queues per block
            const int nslots = (int)(4 * (g1 - g0 + 1));
            hipLaunchKernelGGL(nw_band_cert, dim3((unsigned)((nslots + kCertSlots - 1) / kCertSlots)), dim3(256),
                               (size_t)(4 * ((a.La + 15) / 16 + 2)), s, a, nslots);
        }
    } else {
        hipLaunchKernelGGL(nw_band_classify<false>, dim3(std::max(1, std::min(2048, (int)((a.n + 255) / 256)))),
                           dim3(256), (size_t)(8 * ((a.La + 3) / 4)), s, a);
    }
    const int nseg = (int)std::max<int64_t>(1, (a.n + kSegReads - 1) / kSegReads);
    hipLaunchKernelGGL(nw_band_segsort, dim3(nseg), dim3(kSegThreads), (size_t)segsort_lds_bytes(a.band_lb_cap + a.seed_keys), s, a,
                       epoch);
    return hipGetLastError();
}
// words of the single-pass scans over n reads: the largest of the segment sort's two lists
// (the seeded list after the band list's ceil(n / kSegReads) + 1 words), the redo and ops
// compactions (1024-read blocks)
int64_t band_lookback_words(int64_t n) {
    const int64_t seg = std::max<int64_t>(1, (n + kSegReads - 1) / kSegReads);
    return std::max<int64_t>(std::max<int64_t>(1, (n + 1023) / 1024) + 1, 2 * seg + 2);   // band list, seeded list
}

hipError_t launch_band(int W, const KernelArgs& a, const LaunchCfg& fill, const LaunchCfg& walk, hipStream_t s,
                       hipEvent_t after_fill) {
    // the lane walk (and the stop summary its fill writes for it) when the context asked for it
    KernelArgs al = a;
    al.band_summ = W == 16 && a.ops && a.band_summ;
    if (al.band_summ)
        hipLaunchKernelGGL((nw_band_fill<16, true>), dim3(fill.grid), dim3(64 * fill.wpb), fill.lds_bytes, s, al);
    else if (W == 16)
        hipLaunchKernelGGL((nw_band_fill<16>), dim3(fill.grid), dim3(64 * fill.wpb), fill.lds_bytes, s, a);
    else if (W == 32)
        hipLaunchKernelGGL((nw_band_fill<32>), dim3(fill.grid), dim3(64 * fill.wpb), fill.lds_bytes, s, a);
    else
        hipLaunchKernelGGL((nw_band_fill<kWideDiags>), dim3(fill.grid), dim3(64 * fill.wpb), fill.lds_bytes, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (after_fill && (e = hipEventRecord(after_fill, s)) != hipSuccess) return e;
    if (al.band_summ)
        hipLaunchKernelGGL((nw_band_walk<16, true>), dim3(walk.grid), dim3(64 * walk.wpb), walk.lds_bytes, s, al);
    else if (W == 16)
        hipLaunchKernelGGL(nw_band_walk<16>, dim3(walk.grid), dim3(64 * walk.wpb), walk.lds_bytes, s, a);
    else if (W == 32)
        hipLaunchKernelGGL(nw_band_walk<32>, dim3(walk.grid), dim3(64 * walk.wpb), walk.lds_bytes, s, a);
    else
        hipLaunchKernelGGL(nw_band_walk<kWideDiags>, dim3(walk.grid), dim3(64 * walk.wpb), walk.lds_bytes, s, a);
    return hipGetLastError();
}

}  // namespace nw
