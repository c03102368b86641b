// nw_pair.hip -- two alignments per wavefront in packed int16 (v_pk_*_i16).
//
// Same recurrence, tie rules and output as nw_kernel.hip (the int32 kernel,
// which stays the exact fallback for reads whose traceback leaves the band and
// for parameter sets whose scores do not fit int16).  Differences:
//   * every VGPR holds read A in its low half and read B in its high half, so
//     each v_pk_add/sub/max_i16 advances two DP cells;
//   * the 4 traceback sign bits of both cells are gathered with two v_perm_b32
//     per row (sign-select bytes) and masked into byte-planes with v_and_or: one
//     dword per lane, column and 4-row group holds both reads' bits;
//   * the amplicon's rows are padded at the TOP with zero-score rows: such rows
//     reproduce the DP boundary (M = 0, H = 0, Y/X never chosen), so the last
//     amplicon row is always the bottom row of the last lane, and columns before
//     a lane's first column need no masking (they leave the lane in the
//     boundary state).
// The diagonal band is shared by the pair (union of both reads' bands).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_common.h"

namespace nw {

typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 as_v(unsigned u) { return __builtin_bit_cast(s16x2, u); }
__device__ __forceinline__ unsigned as_u(s16x2 v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ unsigned pk(int lo, int hi) { return ((unsigned)lo & 0xffffu) | ((unsigned)hi << 16); }
__device__ __forceinline__ int half(unsigned w, int h) { return (int)(short)(w >> (16 * h)); }

__device__ __forceinline__ unsigned dpp_shr1(unsigned old, unsigned v) {
    // lane l <- lane l-1; lane 0 keeps `old` (the boundary value it was initialised with)
    return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}

template <int R> struct PairGeo {
    static constexpr int R4 = (R + 3) & ~3;   // int16 profile rows per lane
    static constexpr int PB = 2 * R4;         // profile bytes per lane
    static constexpr int NG = R4 / 4;         // traceback dwords per (slot, lane)
};

struct PairLds {
    int coff, lastrow, runs, runs_cap, bits, total;
};

// Per-wave LDS: the traceback band, then a scratch region used by the fill
// (both reads' profile offsets + the last row) and afterwards by the run list.
__host__ __device__ inline PairLds pair_lds_layout(int R, int La, int Lb_max, int band_slots) {
    const int NG = ((R + 3) & ~3) / 4;
    PairLds w;
    int o = 0;
    w.bits = o;    o += align16(band_slots * 64 * 4 * NG);
    const int scratch = o;
    w.coff = o;    o += 2 * align16(2 * (Lb_max + 136));
    w.lastrow = o; o += align16(4 * (64 + Lb_max + 4));
    const int fill_end = o;
    const int runs_min = align16(4 * 256);
    w.runs = scratch;
    o = scratch + (fill_end - scratch > runs_min ? fill_end - scratch : runs_min);
    w.runs_cap = (o - scratch) / 4;
    w.total = align16(o);
    return w;
}

__host__ __device__ inline int pair_shared_bytes(int R, int La) {
    const int PB = 2 * ((R + 3) & ~3);
    return align16(NCODE * 64 * PB) + 256 + align16(La + 4);
}

template <class T, int N>
struct Arr { T v[N]; };

template <int R>
__device__ __forceinline__ void load_prof16(const unsigned char* p, Arr<unsigned, PairGeo<R>::R4 / 2>& out) {
    constexpr int R4 = PairGeo<R>::R4;
#pragma unroll
    for (int q = 0; q < R4 / 4; ++q) {
        const uint2 v = ((const uint2*)p)[q];
        out.v[2 * q] = v.x;
        out.v[2 * q + 1] = v.y;
    }
}

template <int R>
__global__ __launch_bounds__(kPairMaxThreads) void nw_pair_kernel(const KernelArgs args) {
    constexpr int R4 = PairGeo<R>::R4;
    constexpr int PB = PairGeo<R>::PB;
    constexpr int NG = PairGeo<R>::NG;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int La = args.La;
    const int O = args.gap_open, E = args.gap_extend;
    const unsigned O2 = pk(O, O), E2 = pk(E, E);
    const unsigned NEG2 = pk(-16384, -16384);
    const unsigned MO0 = pk(-O, -O);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    // ---- shared per-block state: int16 profile, ascii->code LUT, amplicon bytes ----
    unsigned char* prof_lds = smem;
    const int prof_bytes = NCODE * 64 * PB;
    unsigned char* lut_lds = smem + align16(prof_bytes);
    unsigned char* amp_lds = lut_lds + 256;
    for (int q = tid; q < prof_bytes / 16; q += blockDim.x)
        ((int4*)prof_lds)[q] = ((const int4*)args.prof)[q];
    for (int q = tid; q < 256; q += blockDim.x) lut_lds[q] = args.lut[q];
    for (int q = tid; q < La; q += blockDim.x) amp_lds[q] = args.amp[q];
    __syncthreads();

    const PairLds L = pair_lds_layout(R, La, args.Lb_max, args.band_slots);
    unsigned char* wbase = smem + pair_shared_bytes(R, La) + wave * L.total;
    const int coff_stride = align16(2 * (args.Lb_max + 136));   // bytes between read A's and B's offsets
    unsigned short* coff[2] = {(unsigned short*)(wbase + L.coff), (unsigned short*)(wbase + L.coff + coff_stride)};
    unsigned* lastrow = (unsigned*)(wbase + L.lastrow);
    unsigned* runs = (unsigned*)(wbase + L.runs);
    unsigned* bits = (unsigned*)(wbase + L.bits);
    const int slots = args.band_slots;

    const int nl = (La + R - 1) / R;       // lanes holding amplicon rows
    const int F = nl * R - La;             // zero-score rows padded on top of lane 0
    const int lr = nl - 1;                 // its bottom row is the last amplicon row
    const int prof_lane = lane * PB;
    const int pad_coff = NCODE_PAD * 64 * PB;
    const long long npairs = (args.n + 1) / 2;

    constexpr int CHUNK = 8;                  // pairs per dequeue
    const long long nchunks = (npairs + CHUNK - 1) / CHUNK;
    for (;;) {
    long long chunk = 0;
    if (lane == 0) chunk = atomicAdd(args.work_counter, 1);
    chunk = __shfl(chunk, 0, 64);
    if (chunk >= nchunks) break;
    const long long pend = min(npairs, (chunk + 1) * CHUNK);
    for (long long pw = chunk * CHUNK; pw < pend; ++pw) {
        long long rdv[2] = {2 * pw, 2 * pw + 1};
        int Lbv[2];
        long long offv[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (rdv[h] < args.n) {
                offv[h] = args.offsets[rdv[h]];
                Lbv[h] = (int)(args.offsets[rdv[h] + 1] - offv[h]);
                if (Lbv[h] <= 0) {
                    if (lane == 0) { Stat z = {}; z.flags = FLAG_EMPTY; args.stats[rdv[h]] = z; }
                    Lbv[h] = 0;
                }
            } else {
                offv[h] = 0;
                Lbv[h] = 0;
            }
        }
        const int Lmax = max(Lbv[0], Lbv[1]);
        if (Lmax == 0) continue;
        // band in padded-row coordinates (diagonal d = bj - g, g = ai + F)
        int lo0 = 0, hi0 = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (Lbv[h] > 0) { lo0 = min(lo0, Lbv[h] - La); hi0 = max(hi0, Lbv[h] - La); }
        const int m = (slots - (hi0 - lo0) - R) / 2;
        if (m < 0) {
            if (lane == 0) {
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (Lbv[h] > 0) args.fallback_list[atomicAdd(args.fallback_count, 1)] = rdv[h];
            }
            continue;
        }
        const int dlo = lo0 - m - F;

        // ---- stage both reads' profile row offsets, padded around [0, Lb) ----
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const unsigned char* rp = args.reads + offv[h];
            for (int q = lane - 64; q < Lmax + 72; q += 64) {
                const bool real = q >= 0 && q < Lbv[h];
                coff[h][64 + q] = (unsigned short)(real ? lut_lds[rp[q]] * 64 * PB : pad_coff);
            }
        }
        lds_fence();

        // ---- DP fill: both reads, packed ----
        unsigned Mol[R], Xl[R], Hold[R], capA[R], capB[R];
#pragma unroll
        for (int k = 0; k < R; ++k) { Mol[k] = MO0; Xl[k] = NEG2; Hold[k] = 0u; capA[k] = MO0; capB[k] = MO0; }
        unsigned sMo = MO0, sY = NEG2, sH = 0u;
        unsigned rMo = MO0, rY = NEG2, rH = 0u;   // lane 0 keeps these (the boundary above row 0)
        unsigned Htop = 0u;
        const int nsteps = Lmax + nl - 1;
        const int tA = Lbv[0] - 1 + lane, tB = Lbv[1] - 1 + lane;   // step of each read's last column
        // coff entry of column bj lives at index 64 + bj; lane l is at column t - l
        const unsigned short* cA = coff[0] + 64 - lane;
        const unsigned short* cB = coff[1] + 64 - lane;
        unsigned* bits_lane = bits + lane * NG;
        unsigned* lastrow_t = lastrow + 64 - lr;       // lane lr writes column t - lr
        const int slot0 = -lane - lane * R - dlo;      // slot at t = 0
        Arr<unsigned, R4 / 2> pa0, pb0, pa1, pb1;
        load_prof16<R>(prof_lds + cA[0] + prof_lane, pa0);
        load_prof16<R>(prof_lds + cB[0] + prof_lane, pb0);

        // One DP column per call: uses the scores in (pa, pb), prefetches the
        // next column's scores into (pn_a, pn_b).
        auto step = [&](int t, const Arr<unsigned, R4 / 2>& pa, const Arr<unsigned, R4 / 2>& pb,
                        Arr<unsigned, R4 / 2>& pn_a, Arr<unsigned, R4 / 2>& pn_b) {
            rMo = dpp_shr1(rMo, sMo);
            rY = dpp_shr1(rY, sY);
            rH = dpp_shr1(rH, sH);
            load_prof16<R>(prof_lds + cA[t + 1] + prof_lane, pn_a);
            load_prof16<R>(prof_lds + cB[t + 1] + prof_lane, pn_b);
            unsigned acc[NG];
#pragma unroll
            for (int g = 0; g < NG; ++g) acc[g] = 0u;
            s16x2 Hd = as_v(Htop), Mou = as_v(rMo), Yu = as_v(rY);
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const unsigned sel = (k & 1) ? 0x07060302u : 0x05040100u;
                const s16x2 sc = as_v(__builtin_amdgcn_perm(pb.v[k >> 1], pa.v[k >> 1], sel));
                const s16x2 M = Hd + sc;
                const s16x2 Xe = as_v(Xl[k]) - as_v(E2);
                const s16x2 X = __builtin_elementwise_max(as_v(Mol[k]), Xe);
                const s16x2 Ye = Yu - as_v(E2);
                const s16x2 Y = __builtin_elementwise_max(Mou, Ye);
                const s16x2 mxy = __builtin_elementwise_max(X, Y);
                const s16x2 H = __builtin_elementwise_max(M, mxy);
                const unsigned d1 = as_u(Ye - Mou);          // sign: Y opens (open > extend)
                const unsigned d2 = as_u(Xe - as_v(Mol[k])); // sign: X opens
                const unsigned d3 = as_u(Y - X);             // sign: X > Y
                const unsigned d4 = as_u(M - mxy);           // sign: M < max(X, Y)
                // v_perm selectors 8..11 give 0x00/0xff from bit 15/31 of a source: one byte
                // per (difference, read) -> [yA yB xA xB] and [bXA bXB bMA bMB]; row k of its
                // 4-row group lands in bit k (first word) and bit 4+k (second word) of each byte
                const unsigned tt = __builtin_amdgcn_perm(d2, d1, 0x0B0A0908u);
                const unsigned uu = __builtin_amdgcn_perm(d4, d3, 0x0B0A0908u);
                acc[k >> 2] = (tt & (0x01010101u << (k & 3))) | acc[k >> 2];
                acc[k >> 2] = (uu & (0x10101010u << (k & 3))) | acc[k >> 2];
                const s16x2 Mo = M - as_v(O2);
                Hd = as_v(Hold[k]);
                Hold[k] = as_u(H);
                Mol[k] = as_u(Mo);
                Xl[k] = as_u(X);
                Mou = Mo;
                Yu = Y;
            }
            sMo = as_u(Mou);
            sY = as_u(Yu);
            sH = Hold[R - 1];
            const int slot = slot0 + t;
            if ((unsigned)slot < (unsigned)slots) {
                unsigned* p = bits_lane + (size_t)slot * 64 * NG;
#pragma unroll
                for (int g = 0; g < NG; ++g) p[g] = acc[g];
            }
            if (lane == lr) lastrow_t[t] = sMo;     // Mo of the last amplicon row
            if (t == tA) {
#pragma unroll
                for (int k = 0; k < R; ++k) capA[k] = Mol[k];
            }
            if (t == tB) {
#pragma unroll
                for (int k = 0; k < R; ++k) capB[k] = Mol[k];
            }
            Htop = rH;
        };
        int t = 0;
        for (; t + 1 < nsteps; t += 2) {
            step(t, pa0, pb0, pa1, pb1);
            step(t + 1, pa1, pb1, pa0, pb0);
        }
        if (t < nsteps) step(t, pa0, pb0, pa1, pb1);
        lds_fence();

        // ---- start cells of both reads (before the run list overwrites the scratch) ----
        int score_v[2], ei_v[2], ej_v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int Lb = Lbv[h];
            score_v[h] = 0; ei_v[h] = 0; ej_v[h] = 0;
            if (Lb == 0) continue;
            long long key = -0x7fffffffffffffffll - 1;
            if (lane < nl) {
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const int ai = lane * R + k - F;
                    if (ai >= 0) {
                        const int v = half(h ? capB[k] : capA[k], h) + O;
                        const long long kk = (ai == La - 1) ? end_key(v, 3, 0) : end_key(v, 2, ai);
                        key = kk > key ? kk : key;
                    }
                }
            }
            for (int q = lane; q < Lb - 1; q += 64) {
                const long long kk = end_key(half(lastrow[64 + q], h) + O, 1, q);
                key = kk > key ? kk : key;
            }
            key = wave_max_i64(key);
            decode_end(key, La, Lb, &score_v[h], &ei_v[h], &ej_v[h]);
        }
        lds_fence();

        // ---- per read: walk, strings ----
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int Lb = Lbv[h];
            if (Lb == 0) continue;
            const long long rd = rdv[h];
            const int score = score_v[h], ei = ei_v[h], ej = ej_v[h];
            if (args.debug_mode == 1) {
                if (lane == 0) { Stat z = {}; z.score = score; z.end_i = ei; z.end_j = ej; args.stats[rd] = z; }
                continue;
            }
            auto nib = [&](int ai, int bjj, bool* oob) -> unsigned {
                const int g = ai + F;
                const int ln = g / R, k = g - ln * R;
                const int s = bjj - ln * R - dlo;
                if ((unsigned)s >= (unsigned)slots) { *oob = true; return 0u; }
                *oob = false;
                const int grp = k >> 2, kk = k & 3;
                const unsigned w = bits[((size_t)s * 64 + ln) * NG + grp];
                const int hb = 8 * h + kk, lb = 8 * h + 4 + kk;
                const unsigned yext = (w >> hb) & 1u, bX = (w >> lb) & 1u;
                const unsigned xext = (w >> (16 + hb)) & 1u, bM = (w >> (16 + lb)) & 1u;
                return bM | (bX << 1) | (xext << 2) | (yext << 3);
            };
            const int nruns = walk_runs(nib, La, Lb, ei, ej, runs, L.runs_cap, lane);
            if (nruns < 0) {
                if (lane == 0) args.fallback_list[atomicAdd(args.fallback_count, 1)] = rd;
                continue;
            }
            lds_fence();
            if (args.debug_mode == 2) {
                if (lane == 0) { Stat z = {}; z.score = score; z.aln_len = nruns; args.stats[rd] = z; }
                continue;
            }
            auto sim = [&](int ai, int code) {
                const int g = ai + F;
                return (int)*(const short*)(prof_lds + code * 64 * PB + (g / R) * PB + 2 * (g % R));
            };
            emit_alignment(runs, nruns, amp_lds, args.reads + offv[h], lut_lds, sim, args.out + rd * 3 * args.stride,
                           args.stride, score, ei, ej, args.stats + rd, lane);
            lds_fence();
        }
    }
    }
}

template <int R>
static hipError_t launch_pair_r(const KernelArgs& a, const LaunchCfg& c, hipStream_t s) {
    hipLaunchKernelGGL((nw_pair_kernel<R>), dim3(c.grid), dim3(64 * c.wpb), c.lds_bytes, s, a);
    return hipGetLastError();
}

int pair_lds_bytes_for(int R, int La, int Lb_max, int band_slots, int wpb) {
    return pair_shared_bytes(R, La) + wpb * pair_lds_layout(R, La, Lb_max, band_slots).total;
}

int pair_profile_bytes_per_lane(int R) { return 2 * ((R + 3) & ~3); }

hipError_t launch_pair(const KernelArgs& a, const LaunchCfg& c, hipStream_t s) {
    switch (c.R) {
        case 1: return launch_pair_r<1>(a, c, s);
        case 2: return launch_pair_r<2>(a, c, s);
        case 3: return launch_pair_r<3>(a, c, s);
        case 4: return launch_pair_r<4>(a, c, s);
        case 5: return launch_pair_r<5>(a, c, s);
        case 6: return launch_pair_r<6>(a, c, s);
        case 7: return launch_pair_r<7>(a, c, s);
        case 8: return launch_pair_r<8>(a, c, s);
        case 10: return launch_pair_r<10>(a, c, s);
        case 12: return launch_pair_r<12>(a, c, s);
        case 14: return launch_pair_r<14>(a, c, s);
        case 16: return launch_pair_r<16>(a, c, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace nw
