// nw_stream.hip -- streaming wavefront fill + separate traceback kernel.
//
// Same recurrence, tie rules and output as nw_kernel.hip / nw_pair.hip.  The
// pair kernel pays a 63-column ramp-up/ramp-down per pair of reads (lane l
// starts l columns after lane 0), ~20 % of its DP steps at 250 bp.  Here the
// pairs of one wavefront follow each other in a single stream of columns:
//
//   * pair q occupies stream columns [S_q, S_q + span_q); both reads are
//     right-aligned in it (read h starts at column pad_h = span_q - Lb_h), so the
//     columns before a shorter read are neutral pad columns (see nw_pair.hip:
//     they leave a lane in the boundary state) and both reads end on the pair's
//     last column;
//   * lane l works on stream column T - l at step T; when that column is the
//     first of its next pair, the lane stores its last-column scores of the
//     finished pair (the "captures"), resets to the boundary state and loads the
//     next pair's band geometry -- one event per lane and pair, no ramp;
//   * the traceback band, the captures and the last amplicon row go to a
//     per-pair region in HBM (7-16 KB per pair; 288 GB leave room for millions
//     of pairs), so the fill kernel holds no traceback in LDS and its occupancy
//     is register-limited;
//   * nw_stream_walk (one wavefront per read, latency-bound, high occupancy)
//     finds the start cell, walks the band and writes the strings.  Reads whose
//     walk leaves the band go to the fallback list of the exact int32 kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_common.h"

#ifndef NW_FILL_WAVES_PER_SIMD
#define NW_FILL_WAVES_PER_SIMD 5   // register budget of the fill kernel (occupancy)
#endif
#ifndef NW_WALK_CPL
#define NW_WALK_CPL 2              // walk cells tested per lane per ballot
#endif
#ifndef NW_WALK_WAVES_PER_SIMD
#define NW_WALK_WAVES_PER_SIMD 8   // the walk is latency-bound: as many waves as fit
#endif

namespace nw {

namespace {

typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 as_v(unsigned u) { return __builtin_bit_cast(s16x2, u); }
__device__ __forceinline__ unsigned as_u(s16x2 v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ unsigned pk(int lo, int hi) { return ((unsigned)lo & 0xffffu) | ((unsigned)hi << 16); }
__device__ __forceinline__ int half(unsigned w, int h) { return (int)(short)(w >> (16 * h)); }

__device__ __forceinline__ unsigned dpp_shr1(unsigned old, unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}

// d = (a & m) | c as one VOP3 (the compiler prefers and+and+or3 = 3 ops for two terms)
__device__ __forceinline__ unsigned and_or(unsigned a, unsigned m, unsigned c) {
    unsigned d;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(m), "v"(c));
    return d;
}

constexpr int kRing = 256;         // staged columns per read (power of two)
constexpr int kRingAlloc = kRing + 4;   // + mirror of the first entries (4-step unroll)
constexpr int kDescQ = 16;         // pair descriptors per wave (ring)
constexpr int kStage = 64;         // steps between two staging points
constexpr int kChunk = 2;          // pairs per dequeue

}  // namespace

// ---- per-pair region in HBM --------------------------------------------------
__host__ __device__ inline StreamRegion stream_region(int R, int band_slots, int Lb_max) {
    const int NG = ((R + 3) & ~3) / 4;
    StreamRegion g;
    g.bits = 0;
    g.caps = (int64_t)band_slots * 64 * NG * 4;
    g.last = g.caps + (int64_t)64 * R * 4;
    const int64_t span_cap = (Lb_max > kStreamMinSpan ? Lb_max : kStreamMinSpan) + 8;
    g.flags = g.last + 4 * span_cap;
    g.stride = (g.flags + 4 + 255) & ~(int64_t)255;
    return g;
}

// Band of a pair in the stream (pair-relative column c, padded row g = ai + F):
// slot = c - lane * R - dlo; stored at word (((lane / 8) * slots + slot) * 8 + lane % 8) * NG.  Returns false when the pair has no read or the
// band cannot hold both reads' start and end diagonals.
__host__ __device__ inline bool stream_pair_band(int La, int R, int F, int slots, int LbA, int LbB, int* span,
                                                 int* dlo) {
    const int Lmax = LbA > LbB ? LbA : LbB;
    *span = 0;
    *dlo = 0;
    if (Lmax <= 0) return false;
    // spans are multiples of 4: every pair starts at the same column phase (mod 4)
    const int sp = ((Lmax > kStreamMinSpan ? Lmax : kStreamMinSpan) + 3) & ~3;
    int lo = 1 << 30, hi = -(1 << 30);
    const int Lb[2] = {LbA, LbB};
    for (int h = 0; h < 2; ++h) {
        if (Lb[h] <= 0) continue;
        const int pad = sp - Lb[h];
        const int a = (Lb[h] - La < 0 ? Lb[h] - La : 0) + pad;
        const int b = (Lb[h] - La > 0 ? Lb[h] - La : 0) + pad;
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    *span = sp;
    const int room = slots - (hi - lo) - R;
    if (room < 0) return false;
    *dlo = lo - room / 2 - F;
    return true;
}

template <int R> struct SGeo {
    static constexpr int R4 = (R + 3) & ~3;
    static constexpr int PB = 2 * R4;
    static constexpr int NG = R4 / 4;
};

__host__ __device__ inline int stream_shared_bytes(int R, bool PT) {
    const int PB = 2 * ((R + 3) & ~3);
    return PT ? kPairCodes * kPairCodes * 64 * 16 + 256 : align16(NCODE * 64 * PB) + 256;
}
__host__ __device__ inline int stream_wave_bytes() {
    return align16(2 * 2 * kRingAlloc) + kDescQ * 48;
}

template <class T, int N>
struct SArr { T v[N]; };

template <int R>
__device__ __forceinline__ void sload_prof(const unsigned char* p, SArr<unsigned, SGeo<R>::R4 / 2>& out) {
#pragma unroll
    for (int q = 0; q < SGeo<R>::R4 / 4; ++q) {
        const uint2 v = ((const uint2*)p)[q];
        out.v[2 * q] = v.x;
        out.v[2 * q + 1] = v.y;
    }
}

// ============================================================================
// Fill: one continuous stream of read pairs per wavefront.
// ============================================================================
// PT: scores from the pair-code table (one ds_read_b128 per column gives the
// packed scores of both reads for the lane's 4 rows) instead of two per-read
// profile rows merged with v_perm.
template <int R, bool PT>
__global__ __launch_bounds__(640, NW_FILL_WAVES_PER_SIMD) void nw_stream_fill(const KernelArgs args) {
    static_assert(!PT || R <= 4, "pair table holds 4 rows per lane");
    constexpr int R4 = SGeo<R>::R4;
    constexpr int PB = SGeo<R>::PB;
    constexpr int NG = SGeo<R>::NG;
    constexpr int LB = PT ? 16 : PB;    // score bytes per lane and column code
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int La = args.La;
    const int O = args.gap_open, E = args.gap_extend;
    const unsigned E2 = pk(E, E);
    const unsigned NEG2 = pk(-16384, -16384);
    // Biased recurrence: every value of cell (r, c) (r = padded row + 1, c = pair
    // column + 1; 0 = the DP boundary) carries + (r + c) * E.  A horizontal or
    // vertical step then adds E, so X = max(Mo_left, X_left) and Y = max(Mo_up,
    // Y_up) need no "- extend"; the diagonal step's + 2E is in the score table
    // (prof_fill / ptab), and Mo = M - (O - E).  Traceback differences are
    // unchanged (both operands carry the same bias); the walk removes the bias
    // from captures and last row.  Boundary: H(r, 0) = r E, H(0, c) = c E.
    const unsigned OE2 = pk(O - E, O - E);
    const unsigned EmO2 = pk(E - O, E - O);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    unsigned char* prof_lds = smem;
    const int prof_bytes = PT ? kPairCodes * kPairCodes * 64 * 16 : NCODE * 64 * PB;
    unsigned char* lut_lds = smem + align16(prof_bytes);
    const int4* prof_src = PT ? (const int4*)args.ptab : (const int4*)args.prof_fill;
    for (int q = tid; q < prof_bytes / 16; q += blockDim.x) ((int4*)prof_lds)[q] = prof_src[q];
    for (int q = tid; q < 256; q += blockDim.x) lut_lds[q] = PT ? args.lut6[q] : args.lut[q];
    __syncthreads();

    unsigned char* wbase = smem + stream_shared_bytes(R, PT) + wave * stream_wave_bytes();
    unsigned short* ringA = (unsigned short*)wbase;
    unsigned short* ringB = ringA + kRingAlloc;
    int4* desc = (int4*)(wbase + align16(2 * 2 * kRingAlloc));   // [kDescQ][3]

    const int slots = args.band_slots;
    const int nl = (La + R - 1) / R;
    const int F = nl * R - La;
    const int lr = nl - 1;
    const int prof_lane = lane * LB;
    const unsigned short pad_coff = (unsigned short)(PT ? (kPairCodes * kPairCodes - 1) * 64 * 16
                                                         : NCODE_PAD * 64 * PB);
    const long long npairs = (args.n + 1) / 2;
    const StreamRegion reg = stream_region(R, slots, args.Lb_max);
    constexpr int BIG = 1 << 29;

    // ---- wave-uniform stream state ----
    int q_count = 0;           // pairs appended so far
    // The stream starts at column S0 = -lr mod 4: pair starts are then = -lr
    // (mod 4), so lane lr (the last amplicon row) changes pairs only on the first
    // of every 4 steps and stores its last-row words 4 at a time.
    const int S0 = (4 - (lr & 3)) & 3;
    int S_tail = S0;           // first stream column after the appended pairs
    bool exhausted = false;
    long long cur = 0, cur_end = 0;   // dequeued pair range being appended
    long long next_chunk = 0;
    if (lane == 0) next_chunk = atomicAdd(args.work_counter, 1);
    next_chunk = __shfl(next_chunk, 0, 64);

    // Appends pairs (skipping empty / band-less ones, which the walk kernel
    // handles) until the stream covers column `need` or the queue is empty.
    auto append = [&](int need) {
        while (!exhausted && S_tail <= need) {
            if (cur >= cur_end) {
                const long long c0 = next_chunk * kChunk;
                if (c0 >= npairs) { exhausted = true; break; }
                cur = c0;
                cur_end = min(npairs, c0 + kChunk);
                long long nc = 0;
                if (lane == 0) nc = atomicAdd(args.work_counter, 1);
                next_chunk = __shfl(nc, 0, 64);
            }
            const long long p = cur++;
            const long long ra = 2 * p, rb = 2 * p + 1;
            const long long offA = args.offsets[ra];
            const int LbA = (int)(args.offsets[ra + 1] - offA);
            long long offB = 0;
            int LbB = 0;
            if (rb < args.n) { offB = args.offsets[rb]; LbB = (int)(args.offsets[rb + 1] - offB); }
            int span, dlo;
            if (!stream_pair_band(La, R, F, slots, LbA, LbB, &span, &dlo)) continue;
            if (PT && lane == 0) *(int*)(args.region + p * reg.stride + reg.flags) = 0;
            if (lane == 0) {
                int4* d = desc + (q_count & (kDescQ - 1)) * 3;
                d[0] = make_int4(S_tail, span, dlo, (int)p);
                d[1] = make_int4(span - LbA, span - LbB, LbA, LbB);
                d[2] = make_int4((int)(unsigned)offA, (int)(offA >> 32), (int)(unsigned)offB, (int)(offB >> 32));
            }
            S_tail += span;
            ++q_count;
        }
        // the stream state is wave-uniform: keep it in SGPRs
        S_tail = __builtin_amdgcn_readfirstlane(S_tail);
        q_count = __builtin_amdgcn_readfirstlane(q_count);
        exhausted = __builtin_amdgcn_readfirstlane((int)exhausted) != 0;
        lds_fence();
    };

    // ---- column staging: read bytes -> profile offsets in the ring ----
    int sq = 0;                 // pair of this lane's staged column (monotone)
    unsigned ldA = 0, ldB = 0;  // bytes loaded for the next block
    int ldP = -1;               // their pair (PT: flagged when a byte is outside the table)
    auto stage_load = [&](int c0) {
        const int c = c0 + lane;
        unsigned vA = 0, vB = 0;
        ldP = -1;
        if (c < S_tail) {
            while (sq + 1 < q_count && c >= desc[((sq + 1) & (kDescQ - 1)) * 3].x) ++sq;
            const int4* d = desc + (sq & (kDescQ - 1)) * 3;
            const int4 d0 = d[0], d1 = d[1], d2 = d[2];
            const int jj = c - d0.x;
            const int jA = jj - d1.x, jB = jj - d1.y;
            const long long oA = (long long)(((unsigned long long)(unsigned)d2.y << 32) | (unsigned)d2.x);
            const long long oB = (long long)(((unsigned long long)(unsigned)d2.w << 32) | (unsigned)d2.z);
            if ((unsigned)jA < (unsigned)d1.z) vA = args.reads[oA + jA];
            if ((unsigned)jB < (unsigned)d1.w) vB = args.reads[oB + jB];
            ldP = d0.w;
        }
        ldA = vA;
        ldB = vB;
    };
    auto stage_write = [&](int c0) {
        const int idx = (c0 + lane) & (kRing - 1);
        if constexpr (PT) {
            int ca = lut_lds[ldA], cb = lut_lds[ldB];
            if (ca >= kPairCodes || cb >= kPairCodes) {
                // a code the table does not hold: the read goes to the exact fallback
                atomicOr((int*)(args.region + (long long)ldP * reg.stride + reg.flags),
                         (ca >= kPairCodes ? REGION_BAD_A : 0) | (cb >= kPairCodes ? REGION_BAD_B : 0));
                ca = ca >= kPairCodes ? kPairCodes - 1 : ca;
                cb = cb >= kPairCodes ? kPairCodes - 1 : cb;
            }
            const unsigned short o = (unsigned short)((ca * kPairCodes + cb) * 64 * 16);
            ringA[idx] = o;
            if (idx < kRingAlloc - kRing) ringA[kRing + idx] = o;
        } else {
            const unsigned short oA = (unsigned short)(lut_lds[ldA] * 64 * PB);
            const unsigned short oB = (unsigned short)(lut_lds[ldB] * 64 * PB);
            ringA[idx] = oA;
            ringB[idx] = oB;
            if (idx < kRingAlloc - kRing) { ringA[kRing + idx] = oA; ringB[kRing + idx] = oB; }
        }
    };

    // ---- prologue ----
    for (int q = lane; q < kRingAlloc; q += 64) { ringA[q] = pad_coff; ringB[q] = pad_coff; }
    append(3 * kStage - 1);
    if (q_count == 0) return;
    stage_load(0);
    stage_write(0);
    stage_load(kStage);
    stage_write(kStage);
    stage_load(2 * kStage);
    lds_fence();

    // ---- per-lane DP state ----
    // boundary column of this lane's rows: H(r, 0) = r E for r = lane R + k + 1;
    // laneH = H(lane R, 0), the diagonal of the lane's top row at its first column
    const unsigned laneH = pk(lane * R * E, lane * R * E);
    unsigned kH[R];
#pragma unroll
    for (int k = 0; k < R; ++k) kH[k] = pk((k + 1) * E, (k + 1) * E);
    unsigned Mol[R], Xl[R], Hold[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        Hold[k] = as_u(as_v(laneH) + as_v(kH[k]));
        Mol[k] = as_u(as_v(Hold[k]) + as_v(EmO2));
        Xl[k] = NEG2;
    }
    unsigned sMo = EmO2, sY = NEG2, sH = 0u;
    // lane 0's DPP "old" operands carry the top boundary row: rMo + E = Mo(0, c)
    // and rH = H(0, c - 1) at its current column c, advanced by E every step
    unsigned rMo = EmO2, rY = NEG2, rH = laneH;
    // Pair changes.  evT = step at which this lane's column is the first of its
    // next pair.  The next pair's pointers (n_*) are prepared for all lanes at
    // once at the staging point before that step (one change per lane and
    // 64-step block, span >= 64), so the change itself is a capture store,
    // register moves and the reset.  Before the first pair and after the last
    // one the captures / last row go to scratch words after the last region.
    unsigned char* region = args.region;
    unsigned* const lr_dummy = (unsigned*)(args.region + npairs * reg.stride);
    unsigned* const caps_dummy = lr_dummy + 256;
    int qi = -1;                   // this lane's latest prepared pair (count index)
    int evT = S0 + lane;
    int slot = -BIG;
    unsigned* bitp = nullptr;      // band word of the current column (used while 0 <= slot < slots)
    unsigned* lrp = lr_dummy;      // last-row word of the current column (lane lr)
    unsigned* capp = caps_dummy;   // this lane's captures
    int n_evT = -1, n_slot = -BIG;
    unsigned *n_bitp = nullptr, *n_lrp = lr_dummy, *n_capp = caps_dummy;
    auto prep_events = [&](int T0) {
        if (evT >= T0 && evT < T0 + kStage) {
            const int q = qi + 1;
            const bool more = q < q_count;
            const int4 d0 = desc[(q & (kDescQ - 1)) * 3];
            unsigned char* base = region + (long long)d0.w * reg.stride;
            n_evT = more ? d0.x + d0.y + lane : -1;
            n_slot = (more && lane < nl) ? -lane * R - d0.z : -BIG;
            // band words grouped by 8 lanes: [lane / 8][slot][lane % 8] -- a 128-B
            // line (4 slots x 8 lanes) is written within ~38 steps, so it is
            // complete while still in L2, and a diagonal of the walk reads ~8 lines
            n_bitp = (unsigned*)(base + reg.bits) + (((long long)(lane >> 3) * slots + n_slot) * 8 + (lane & 7)) * NG;
            n_capp = more ? (unsigned*)(base + reg.caps) + lane * R : caps_dummy;
            n_lrp = more ? (unsigned*)(base + reg.last) : lr_dummy;
            qi = q;
        }
    };
    prep_events(0);

    // scores of the next column: PT -> 4 packed dwords in pa; else each read's
    // R4 int16 profile scores in pa / pb
    constexpr int SN = PT ? R4 : R4 / 2;
    using Buf = SArr<unsigned, SN>;
    auto load_scores = [&](int ridx, Buf& oa, Buf& ob) {
        if constexpr (PT) {
            const uint4 v = *(const uint4*)(prof_lds + ringA[ridx] + prof_lane);
            oa.v[0] = v.x; oa.v[1] = v.y; oa.v[2] = v.z; oa.v[3] = v.w;
        } else {
            sload_prof<R>(prof_lds + ringA[ridx] + prof_lane, *(SArr<unsigned, R4 / 2>*)&oa);
            sload_prof<R>(prof_lds + ringB[ridx] + prof_lane, *(SArr<unsigned, R4 / 2>*)&ob);
        }
    };
    Buf pa0, pb0, pa1, pb1;
    load_scores((-lane) & (kRing - 1), pa0, pb0);

    // byte-plane masks of the sign bits, forced into SGPRs so that each row's
    // merge is two v_and_or_b32 (VOP3 takes no literal on gfx9)
    unsigned mT[4], mU[4];
    asm volatile("s_mov_b32 %0, 0x01010101" : "=s"(mT[0]));
    asm volatile("s_mov_b32 %0, 0x02020202" : "=s"(mT[1]));
    asm volatile("s_mov_b32 %0, 0x04040404" : "=s"(mT[2]));
    asm volatile("s_mov_b32 %0, 0x08080808" : "=s"(mT[3]));
    asm volatile("s_mov_b32 %0, 0x10101010" : "=s"(mU[0]));
    asm volatile("s_mov_b32 %0, 0x20202020" : "=s"(mU[1]));
    asm volatile("s_mov_b32 %0, 0x40404040" : "=s"(mU[2]));
    asm volatile("s_mov_b32 %0, 0x80808080" : "=s"(mU[3]));

    unsigned lrv[3] = {0u, 0u, 0u};   // last-row words of sub-steps 0..2 (lane lr)
    auto step = [&](int T, int ridx, int sub, const Buf& pa, const Buf& pb, Buf& pn_a, Buf& pn_b) {
        if (T == evT) {
            // this lane's column is the first of its next pair
#pragma unroll
            for (int k = 0; k < R; ++k) capp[k] = Mol[k];
            evT = n_evT;
            slot = n_slot;
            bitp = n_bitp;
            capp = n_capp;
            lrp = n_lrp;
#pragma unroll
            for (int k = 0; k < R; ++k) {
                Hold[k] = as_u(as_v(laneH) + as_v(kH[k]));
                Mol[k] = as_u(as_v(Hold[k]) + as_v(EmO2));
                Xl[k] = NEG2;
            }
            rH = laneH;   // diagonal of the top row at the pair's first column: the boundary
            rMo = EmO2;   // lane 0: Mo(0, 1) - E
        }
        rMo = dpp_shr1(as_u(as_v(rMo) + as_v(E2)), sMo);
        rY = dpp_shr1(rY, sY);
        load_scores(ridx, pn_a, pn_b);
        unsigned acc[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] = 0u;
        // rH = H of the row above at the previous column (the diagonal of row 0)
        s16x2 Hd = as_v(rH), Mou = as_v(rMo), Yu = as_v(rY);
#pragma unroll
        for (int k = 0; k < R; ++k) {
            s16x2 sc;
            if constexpr (PT) {
                sc = as_v(pa.v[k]);
            } else {
                const unsigned sel = (k & 1) ? 0x07060302u : 0x05040100u;
                sc = as_v(__builtin_amdgcn_perm(pb.v[k >> 1], pa.v[k >> 1], sel));
            }
            const s16x2 M = Hd + sc;
            const s16x2 X = __builtin_elementwise_max(as_v(Mol[k]), as_v(Xl[k]));
            const s16x2 Y = __builtin_elementwise_max(Mou, Yu);
            const s16x2 mxy = __builtin_elementwise_max(X, Y);
            const s16x2 H = __builtin_elementwise_max(M, mxy);
            // sign bits (nw_common.h walk_runs): Y opens (open > extend), X opens,
            // X > Y, M < max(X, Y) -- ties extend gaps and stay on the diagonal
            const unsigned d1 = as_u(Yu - Mou);
            const unsigned d2 = as_u(as_v(Xl[k]) - as_v(Mol[k]));
            const unsigned d3 = as_u(Y - X);
            const unsigned d4 = as_u(M - mxy);
            const unsigned tt = __builtin_amdgcn_perm(d2, d1, 0x0B0A0908u);
            const unsigned uu = __builtin_amdgcn_perm(d4, d3, 0x0B0A0908u);
            acc[k >> 2] = and_or(tt, mT[k & 3], acc[k >> 2]);
            acc[k >> 2] = and_or(uu, mU[k & 3], acc[k >> 2]);
            const s16x2 Mo = M - as_v(OE2);
            Hd = as_v(Hold[k]);
            Hold[k] = as_u(H);
            Mol[k] = as_u(Mo);
            Xl[k] = as_u(X);
            Mou = Mo;
            Yu = Y;
        }
        sMo = as_u(Mou);
        sY = as_u(Yu);
        // the row above's H at this column, for the next step (reads the previous
        // step's sH; done after its use as the diagonal, so rH needs no copy)
        rH = dpp_shr1(as_u(as_v(rH) + as_v(E2)), sH);
        sH = Hold[R - 1];
        if ((unsigned)slot < (unsigned)slots) {
#pragma unroll
            for (int g = 0; g < NG; ++g) bitp[g] = acc[g];
        }
        ++slot;
        bitp += 8 * NG;
        if (sub < 3) {
            lrv[sub] = sMo;
        } else if (lane == lr) {
            *(uint4*)lrp = make_uint4(lrv[0], lrv[1], lrv[2], sMo);
            lrp += 4;
        }
    };

    int T = 0;
    for (;;) {
        if (T > 0) {
            append(T + 3 * kStage - 1);
            stage_write(T + kStage);
            stage_load(T + 2 * kStage);
            prep_events(T);
        }
        const int Tend = __builtin_amdgcn_readfirstlane(exhausted ? S_tail + lr : (1 << 30));
        const int nb = __builtin_amdgcn_readfirstlane(min(kStage, Tend - T + 1));
        int u = 0;
        for (; u + 3 < nb; u += 4) {
            const int ridx = (T + u + 1 - lane) & (kRing - 1);
            step(T + u, ridx, 0, pa0, pb0, pa1, pb1);
            step(T + u + 1, ridx + 1, 1, pa1, pb1, pa0, pb0);
            step(T + u + 2, ridx + 2, 2, pa0, pb0, pa1, pb1);
            step(T + u + 3, ridx + 3, 3, pa1, pb1, pa0, pb0);
        }
        if (u < nb) {
            // only at the end of the stream: nb = Tend - T + 1 = 1 (mod 4), the last
            // step is lane lr's final pair change
            step(T + u, (T + u + 1 - lane) & (kRing - 1), 0, pa0, pb0, pa1, pb1);
            break;
        }
        T += kStage;
        if (T > Tend) break;
    }
}

// ============================================================================
// Walk + emit: one wavefront per read, latency-bound.  Per read the dependent
// global round trips are: record offsets; {flags, captures, last row, the read's
// bytes DMA'd into LDS} together; ~1-3 walk ballots over the band (256 cells
// each); then the strings are built from LDS only.
// ============================================================================
constexpr int kWalkReadCap = 1024;   // reads up to this length are staged in LDS for the emit

__host__ __device__ inline int walk_shared_bytes(int La) { return 256 + align16(La + 16) + align16(4 * La); }
__host__ __device__ inline int walk_wave_bytes() { return kStreamRunsCap * 4 + kWalkReadCap + 256; }

template <int R>
__global__ __launch_bounds__(512, NW_WALK_WAVES_PER_SIMD) void nw_stream_walk(const KernelArgs args) {
    constexpr int R4 = SGeo<R>::R4;
    constexpr int NG = SGeo<R>::NG;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int La = args.La;
    const int O = args.gap_open, E = args.gap_extend;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wpb = blockDim.x >> 6;
    const int nl = (La + R - 1) / R;
    const int F = nl * R - La;
    const short* prof16 = (const short*)args.prof;

    // block-shared: ascii->code, amplicon bytes, per amplicon row the codes it scores > 0 against
    unsigned char* lut_lds = smem;
    unsigned char* amp_lds = smem + 256;
    unsigned* rowpos = (unsigned*)(smem + 256 + align16(La + 16));
    for (int q = tid; q < 256; q += blockDim.x) lut_lds[q] = args.lut[q];
    for (int q = tid; q < La; q += blockDim.x) {
        amp_lds[q] = args.amp[q];
        const int g = q + F;
        unsigned m = 0;
        for (int code = 0; code < NCODE; ++code)
            m |= (prof16[(size_t)code * 64 * R4 + (g / R) * R4 + g % R] > 0 ? 1u : 0u) << code;
        rowpos[q] = m;
    }
    __syncthreads();
    unsigned char* wb = smem + walk_shared_bytes(La) + wave * walk_wave_bytes();
    unsigned* runs = (unsigned*)wb;
    unsigned char* rbuf = wb + kStreamRunsCap * 4;

    const int slots = args.band_slots;
    const StreamRegion reg = stream_region(R, slots, args.Lb_max);
    // int16 scores; positions (row or column) below 2^14 -> 32-bit start-cell keys
    const bool small_keys = La < 16384 && args.Lb_max < 16384;

    for (long long rd = (long long)blockIdx.x * wpb + wave; rd < args.n; rd += (long long)gridDim.x * wpb) {
        const long long p = rd >> 1;
        const int h = (int)(rd & 1);
        const long long ra = 2 * p, rb = 2 * p + 1;
        const long long offA = args.offsets[ra], offB1 = args.offsets[ra + 1];
        const int LbA = (int)(offB1 - offA);
        const int LbB = rb < args.n ? (int)(args.offsets[rb + 1] - offB1) : 0;
        const int Lb = h ? LbB : LbA;
        if (Lb <= 0) {
            if (lane == 0) { Stat z = {}; z.flags = FLAG_EMPTY; args.stats[rd] = z; }
            continue;
        }
        int span, dlo;
        if (!stream_pair_band(La, R, F, slots, LbA, LbB, &span, &dlo)) {
            if (lane == 0) args.fallback_list[atomicAdd(args.fallback_count, 1)] = rd;
            continue;
        }
        const int pad = span - Lb;
        const unsigned char* base = args.region + p * reg.stride;
        const unsigned* bits = (const unsigned*)(base + reg.bits);
        const unsigned* caps = (const unsigned*)(base + reg.caps);
        const unsigned* last = (const unsigned*)(base + reg.last);
        const unsigned char* raw = args.reads + (h ? offB1 : offA);

        // ---- one round of loads: read bytes -> LDS, flags, captures, last row ----
        // LDS-DMA writes one dword per lane: copy from the 4-byte-aligned address
        // below the read (the reads buffer is padded) and index by the misalignment
        const bool cached = Lb <= kWalkReadCap;
        const int mis = (int)((uintptr_t)raw & 3);
        if (cached) {
            const unsigned char* src = raw - mis;
            for (int m = 0; m < Lb + mis; m += 256)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + m + 4 * lane),
                                                 (__attribute__((address_space(3))) void*)(rbuf + m), 4, 0, 0);
        }
        const int flags = args.ptab ? *(const int*)(base + reg.flags) : 0;
        // the fill's Mo of cell (r, c) is M - O + E + (r + c) E (biased recurrence):
        // captures are column c = span, row r = g + 1; the last row is r = nl R,
        // column c = pad + q + 1
        const int capb = O - E - (1 + span) * E;
        const int lastb = O - E - (nl * R + pad + 1) * E;
        long long key;
        if (small_keys) {
            // 32-bit keys, DPP max: score (int16) | class | position
            unsigned k32 = 0;
            if (lane < nl) {
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const int ai = lane * R + k - F;
                    if (ai >= 0) {
                        const int v = half(caps[lane * R + k], h) + capb - (lane * R + k) * E;
                        const unsigned kk = (ai == La - 1) ? end_key32(v, 3, 0) : end_key32(v, 2, ai);
                        k32 = kk > k32 ? kk : k32;
                    }
                }
            }
#pragma unroll 4
            for (int q = lane; q < Lb - 1; q += 64) {
                const unsigned kk = end_key32(half(last[pad + q], h) + lastb - q * E, 1, q);
                k32 = kk > k32 ? kk : k32;
            }
            key = end_key_widen(wave_max_u32(k32));
        } else {
            key = -0x7fffffffffffffffll - 1;
            if (lane < nl) {
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const int ai = lane * R + k - F;
                    if (ai >= 0) {
                        const int v = half(caps[lane * R + k], h) + capb - (lane * R + k) * E;
                        const long long kk = (ai == La - 1) ? end_key(v, 3, 0) : end_key(v, 2, ai);
                        key = kk > key ? kk : key;
                    }
                }
            }
            for (int q = lane; q < Lb - 1; q += 64) {
                const long long kk = end_key(half(last[pad + q], h) + lastb - q * E, 1, q);
                key = kk > key ? kk : key;
            }
            key = wave_max_i64(key);
        }
        int score, ei, ej;
        decode_end(key, La, Lb, &score, &ei, &ej);
        if (flags & (h ? REGION_BAD_B : REGION_BAD_A)) {
            // a code outside the pair table: the fill's scores are not this read's
            if (lane == 0) args.fallback_list[atomicAdd(args.fallback_count, 1)] = rd;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            continue;
        }
        if (args.debug_mode == 1) {
            if (lane == 0) { Stat z = {}; z.score = score; z.end_i = ei; z.end_j = ej; args.stats[rd] = z; }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            continue;
        }

        // ---- walk ----
        auto nib = [&](int ai, int bjj, bool* oob) -> unsigned {
            const int g = ai + F;
            const int ln = g / R, k = g - ln * R;
            const int s = bjj + pad - ln * R - dlo;
            if ((unsigned)s >= (unsigned)slots) { *oob = true; return 0u; }
            *oob = false;
            const unsigned w = bits[((((size_t)(ln >> 3) * slots + s) << 3) + (ln & 7)) * NG + (k >> 2)];
            const int kk = k & 3;
            const int hb = 8 * h + kk, lb = 8 * h + 4 + kk;
            const unsigned yext = (w >> hb) & 1u, bX = (w >> lb) & 1u;
            const unsigned xext = (w >> (16 + hb)) & 1u, bM = (w >> (16 + lb)) & 1u;
            return bM | (bX << 1) | (xext << 2) | (yext << 3);
        };
        const int nruns = walk_runs_wide<NW_WALK_CPL>(nib, La, Lb, ei, ej, runs, kStreamRunsCap, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // read bytes landed in LDS
        if (nruns < 0) {
            if (lane == 0) args.fallback_list[atomicAdd(args.fallback_count, 1)] = rd;
            continue;
        }
        lds_fence();
        if (args.debug_mode == 2) {
            if (lane == 0) { Stat z = {}; z.score = score; z.aln_len = nruns; args.stats[rd] = z; }
            continue;
        }
        auto sim = [&](int ai, int code) { return (int)((rowpos[ai] >> code) & 1u); };
        if (args.ops) store_ops(args, rd, runs, nruns, lane);
        emit_alignment(runs, nruns, amp_lds, cached ? rbuf + mis : raw, lut_lds, sim, args.out + rd * 3 * args.stride,
                       args.stride, score, ei, ej, args.stats + rd, lane, !args.ops);
        lds_fence();
    }
}

// ---- host-side helpers ----

int stream_fill_lds_bytes(int R, bool pair_table, int wpb) {
    return stream_shared_bytes(R, pair_table) + wpb * stream_wave_bytes();
}
int stream_walk_lds_bytes(int La, int wpb) { return walk_shared_bytes(La) + wpb * walk_wave_bytes(); }
StreamRegion stream_region_for(int R, int band_slots, int Lb_max) { return stream_region(R, band_slots, Lb_max); }

template <int R, bool PT>
static const void* fill_fn() { return (const void*)nw_stream_fill<R, PT>; }

template <int R>
static const void* pick_fill(bool pair_table) {
    if constexpr (R <= 4) {
        if (pair_table) return fill_fn<R, true>();
    }
    return fill_fn<R, false>();
}

template <int R>
static hipError_t launch_stream_r(const KernelArgs& a, const LaunchCfg& fill, const LaunchCfg& walk, hipStream_t s,
                                  hipEvent_t after_fill) {
    if constexpr (R <= 4) {
        if (a.ptab)
            hipLaunchKernelGGL((nw_stream_fill<R, true>), dim3(fill.grid), dim3(64 * fill.wpb), fill.lds_bytes, s, a);
        else
            hipLaunchKernelGGL((nw_stream_fill<R, false>), dim3(fill.grid), dim3(64 * fill.wpb), fill.lds_bytes, s, a);
    } else {
        if (a.ptab) return hipErrorInvalidValue;
        hipLaunchKernelGGL((nw_stream_fill<R, false>), dim3(fill.grid), dim3(64 * fill.wpb), fill.lds_bytes, s, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (after_fill && (e = hipEventRecord(after_fill, s)) != hipSuccess) return e;
    hipLaunchKernelGGL((nw_stream_walk<R>), dim3(walk.grid), dim3(64 * walk.wpb), walk.lds_bytes, s, a);
    return hipGetLastError();
}

template <int R>
static hipError_t occupancy_r(bool pair_table, int fill_wpb, int walk_wpb, int fill_lds, int walk_lds, int* fill_blocks,
                              int* walk_blocks) {
    if (pair_table && R > 4) return hipErrorInvalidValue;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(fill_blocks, pick_fill<R>(pair_table), 64 * fill_wpb,
                                                               fill_lds);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(walk_blocks, nw_stream_walk<R>, 64 * walk_wpb, walk_lds);
}

#define NW_STREAM_DISPATCH(R_, CALL) \
    switch (R_) {                    \
        case 1: return CALL(1);      \
        case 2: return CALL(2);      \
        case 3: return CALL(3);      \
        case 4: return CALL(4);      \
        case 5: return CALL(5);      \
        case 6: return CALL(6);      \
        case 7: return CALL(7);      \
        case 8: return CALL(8);      \
        case 10: return CALL(10);    \
        case 12: return CALL(12);    \
        case 14: return CALL(14);    \
        case 16: return CALL(16);    \
        default: return hipErrorInvalidValue; \
    }

hipError_t launch_stream(const KernelArgs& a, const LaunchCfg& fill, const LaunchCfg& walk, hipStream_t s,
                         hipEvent_t after_fill) {
#define CALL_(r) launch_stream_r<r>(a, fill, walk, s, after_fill)
    NW_STREAM_DISPATCH(fill.R, CALL_)
#undef CALL_
}

hipError_t stream_occupancy(int R, bool pair_table, int fill_wpb, int walk_wpb, int fill_lds, int walk_lds,
                            int* fill_blocks, int* walk_blocks) {
#define CALL_(r) occupancy_r<r>(pair_table, fill_wpb, walk_wpb, fill_lds, walk_lds, fill_blocks, walk_blocks)
    NW_STREAM_DISPATCH(R, CALL_)
#undef CALL_
}

}  // namespace nw
