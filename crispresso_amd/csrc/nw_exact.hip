// nw_exact.hip -- exact int32 Gotoh/EDNAFULL aligner, one workgroup per read.
//
// Two uses:
//   * amplicons longer than the band and one-wave kernels take (1024 < La <=
//     8192 bp): every read of the batch goes through this kernel (configure_long in
//     nw_host.cpp).  EMBOSS needle has no amplicon length limit; CRISPResso users
//     with long amplicons (--needle_options_string) get the same
//     alignments, at a lower rate.
//   * optionally (CRISPR_NW_EXACT=multi) the reads no band certifies.  Measured on
//     the C2 batch it is not faster than the one-wave kernel (nw_kernel.hip) for those
//     ~15 reads: both are VALU-issue bound, and splitting the rows over more waves
//     adds the per-step hand-off and skew work to every wave.
//
// Layout (EMBOSS needle semantics; the oracle in oracle/ is the checker):
//   * W = ceil(rows / 64) waves, one row per lane up to 1024 bp, R = 2, 4, 8 rows per
//     lane beyond.  Lane g = 64 w + l owns rows [g R, g R + R) and at step t works on
//     column t - g - K w: a skewed wavefront down the lanes of a wave (DPP wave_shr:1
//     moves the bottom row's M - O, Y, H and the column's read code to the next lane).
//   * Between waves the hand-off goes through a 64-entry LDS ring per wave (lane 63
//     writes its values every step, lane 0 of the next wave reads them K + 1 steps
//     later).  The extra lag K per wave lets the waves synchronise once every B = 16
//     steps instead of every step; ring reads are prefetched P = 2 steps ahead (K = B +
//     P - 1 keeps every read behind a barrier).
//   * Substitution scores come from registers: each lane keeps its rows' 16 EDNAFULL
//     scores (scaled, int8) in four dwords and picks one with two v_perm_b32.
//   * Traceback: 4 bits per cell (nw_common.h walk_runs encoding), stored by step:
//     at step t the lanes of wave w write slot t - K w = column + g, so a slot holds
//     one nibble per row and a wave's stores are contiguous dwords (adjacent lanes'
//     nibbles merged by DPP, one lane in 8 / R stores).  Slot (bj + ai / R), nibble
//     ai is cell (ai, bj).  In LDS when it fits, else in a per-block HBM slab.
//   * Start cell (corner, last column bottom -> top, last row right -> left; the
//     same keys as nw_kernel.hip), then wave 0 walks the runs (walk_runs_wide) and
//     emits the record and the rows or the runs (emit_alignment / store_ops).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_common.h"

namespace nw {

constexpr int kExB = 16;                  // steps between barriers
constexpr int kExP = 2;                   // ring prefetch distance
constexpr int kExK = kExB + kExP - 1;     // extra lag per wave
constexpr int kExRing = 64;               // ring entries per wave (>= 1 + K - P + B)

struct ExactLds {
    int keys, ring, topc, lastrow, runs, tb, total;
};

// LDS layout of one block: keys [16] int64, rings [W - 1][64] int4, the read codes by
// column for wave 0's fill (the row above the amplicon) [steps + P], last row M [Lb_max],
// runs [La + Lb_max + 8], then the traceback slots when they live in LDS.
__host__ __device__ inline ExactLds exact_lds_layout(int La, int Lb_max, int R, int W, bool tb_lds) {
    ExactLds L;
    const int nl = (La + R - 1) / R;
    const int steps = Lb_max + nl + kExK * (W - 1) + kExB + kExP + 1;
    int o = 0;
    L.keys = o;    o += 16 * 8;
    L.ring = o;    o += (W > 1 ? W - 1 : 1) * kExRing * 16;
    L.topc = o;    o += align16(steps);
    L.lastrow = o; o += align16(4 * (Lb_max + 1));
    L.runs = o;    o += align16(4 * (La + Lb_max + 8));
    L.tb = o;
    const int64_t pitch = 32ll * W * R;      // bytes per slot: one nibble per padded row
    const int64_t tb_bytes = (int64_t)(Lb_max + nl + 1) * pitch;
    if (tb_lds) o += (int)align16((int)tb_bytes);
    L.total = align16(o);
    return L;
}

// Merges the nibbles of 8 / R adjacent lanes into the lowest lane's dword.
template <int R>
__device__ __forceinline__ unsigned pack_lanes(unsigned v) {
    if constexpr (R == 1) {
        v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xF5, 0xf, 0xf, false) << 4;    // quad_perm [1,1,3,3]
        v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xEE, 0xf, 0xf, false) << 8;    // quad_perm [2,3,2,3]
        v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xf, 0xf, false) << 16;  // row_shl:4
    } else if constexpr (R == 2) {
        v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xF5, 0xf, 0xf, false) << 8;
        v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xEE, 0xf, 0xf, false) << 16;
    } else if constexpr (R == 4) {
        v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xF5, 0xf, 0xf, false) << 16;
    }
    return v;
}

// TBL: traceback slots in LDS (else the block's HBM slab); a template parameter so that
// every access has a known address space (a generic pointer would make the compiler
// wait for all LDS traffic at every store, the ring prefetch included).
template <int R, bool TBL>
__global__ __launch_bounds__(1024) void nw_exact_kernel(const KernelArgs a, int64_t slab_bytes, int cap) {
    if (a.tail_prio && a.work_list) __builtin_amdgcn_s_setprio(3);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // work-list entries (null list: every read); cap: [0, min(count, grid)), one per
    // block, the one-wave kernel takes the rest
    long long count = exact_work_count(a);
    if (cap) count = min(count, (long long)gridDim.x);
    if ((long long)blockIdx.x >= count) return;   // most blocks: nothing to do
    const int La = a.La, O = a.gap_open, E = a.gap_extend;
    const int tid = threadIdx.x, lane = tid & 63, W = blockDim.x >> 6;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform
    const int g = tid;                       // lane index over the block
    const int nl = (La + R - 1) / R;         // lanes holding rows
    const bool has_rows = g < nl;
    const int glast = (La - 1) / R, klast = (La - 1) - glast * R;
    const ExactLds L = exact_lds_layout(La, a.Lb_max, R, W, TBL);
    long long* keys = (long long*)(smem + L.keys);
    int4* rings = (int4*)(smem + L.ring);
    unsigned char* topc = smem + L.topc;
    int* lastrow = (int*)(smem + L.lastrow);
    unsigned* runs = (unsigned*)(smem + L.runs);
    unsigned char* tb;
    if constexpr (TBL) tb = smem + L.tb;
    else tb = a.tb_global + (int64_t)blockIdx.x * slab_bytes;
    const int pitch = 32 * W * R;
    // this wave's fill: the row above the amplicon (wave 0: M - O = -O, Y = -inf, H = 0
    // and the column's read code) or the previous wave's ring
    const int4* src = rings + (w > 0 ? w - 1 : 0) * kExRing;
    // branch-free (both loads issued, the wave-uniform w selects): a branch per step splits
    // the unrolled block and keeps the compiler from interleaving the steps
    auto fill_at = [&](int t) -> int4 {
        const int4 r = src[(t - 1 - kExK) & (kExRing - 1)];
        const int h = end_lead(a, t + 1);   // top boundary at column t: H = leading end gap of t + 1 (0: free)
        const int c = (int)topc[t];
        const bool top = w == 0;
        return make_int4(top ? h - O : r.x, top ? NEG : r.y, top ? h : r.z, top ? c : r.w);
    };
    int4* ring_out = w + 1 < W ? rings + w * kExRing : nullptr;
    // the rows' scores: EDNAFULL(amplicon code, read code 0..15) as 16 int8 in 4 dwords
    // (a.sub16: [17 amplicon codes][4] dwords, code 16 all zero)
    unsigned sc[R][4];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int r = g * R + k;
        const int ca = r < La ? a.lut[a.amp[r]] : 16;
#pragma unroll
        for (int q = 0; q < 4; ++q) sc[k][q] = a.sub16[ca * 4 + q];
    }
    const int lag = g + kExK * w;            // bj = t - lag

    for (long long wi = blockIdx.x; wi < count; wi += gridDim.x) {
        const long long rd = exact_work_read(a, wi);
        const long long off = a.offsets[rd];
        const int Lb = (int)(a.offsets[rd + 1] - off);
        const unsigned char* rp = a.reads + off;
        Stat* st = a.stats + rd;
        if (Lb <= 0) {
            if (tid == 0) {
                Stat z = {};
                z.flags = FLAG_EMPTY;
                *st = z;
                if (a.ops) a.nops[rd] = 0;
            }
            continue;
        }
        const int steps = Lb + nl + kExK * (W - 1) - 1;
        const int nblk = (steps + kExB - 1) / kExB;
        // wave 0's fill: the row above the amplicon (M - O = -O, Y = -inf, H = 0) and the
        // code of column t
        for (int t = tid; t < nblk * kExB + kExP + 1; t += blockDim.x)
            topc[t] = (unsigned char)(t < Lb ? a.lut[rp[t]] : NCODE_PAD);
        __syncthreads();
        int Mol[R], Xl[R], Hold[R];   // column -1: H = M = leading end gap of the row (0: free)
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int h0 = end_lead(a, g * R + k + 1);
            Mol[k] = h0 - O; Xl[k] = NEG; Hold[k] = h0;
        }
        int sMo = Mol[R - 1], sY = NEG, sH = Hold[R - 1], sC = NCODE_PAD, Htop = end_lead(a, g * R);
        int4 f0 = fill_at(0), f1 = fill_at(1);
        for (int b = 0; b < nblk; ++b) {
            __syncthreads();   // ring entries of the earlier blocks are visible
#pragma unroll
            for (int i = 0; i < kExB; ++i) {
                const int t = b * kExB + i;
                const int4 f2 = fill_at(t + kExP);
                const int rMo = shr1(sMo, f0.x), rY = shr1(sY, f0.y), rH = shr1(sH, f0.z);
                const int cb = shr1(sC, f0.w);
                const int bj = t - lag;
                unsigned acc = 0;
                // every lane computes every step (no branch); lanes outside their rows' columns
                // keep their state and contribute no traceback bits
                const bool valid = has_rows && (unsigned)bj < (unsigned)Lb;
                {
                    // score byte: codes 0..7 from dwords 0-1, 8..15 from 2-3, 16 -> 0 (selector 12)
                    const unsigned sel = cb < 16 ? (unsigned)(cb & 7) : 12u;
                    const bool hi = (cb & 8) != 0 && cb < 16;
                    int Hd = Htop, Mou = rMo, Yu = rY, mlast = 0;
#pragma unroll
                    for (int k = 0; k < R; ++k) {
                        const unsigned lo8 = __builtin_amdgcn_perm(sc[k][1], sc[k][0], sel);
                        const unsigned hi8 = __builtin_amdgcn_perm(sc[k][3], sc[k][2], sel);
                        const int s = __builtin_amdgcn_sbfe((int)(hi ? hi8 : lo8), 0, 8);
                        const int M = Hd + s;
                        const int Xe = Xl[k] - E;
                        const int X = max(Mol[k], Xe);
                        const int Ye = Yu - E;
                        const int Y = max(Mou, Ye);
                        const int mxy = max(X, Y);
                        const int H = max(M, mxy);
                        unsigned nib = (unsigned)(Ye - Mou) >> 31;             // bit 3: Y opens
                        nib = __builtin_amdgcn_alignbit(nib, (unsigned)(Xe - Mol[k]), 31);   // bit 2: X opens
                        nib = __builtin_amdgcn_alignbit(nib, (unsigned)(X - Y), 31);         // bit 1: Y > X
                        nib = __builtin_amdgcn_alignbit(nib, (unsigned)(M - mxy), 31);       // bit 0: M < max
                        acc |= nib << (4 * k);
                        mlast = k == klast ? M : mlast;
                        Hd = Hold[k];
                        Hold[k] = valid ? H : Hold[k];
                        Mol[k] = valid ? M - O : Mol[k];
                        Xl[k] = valid ? X : Xl[k];
                        Mou = M - O;
                        Yu = Y;
                    }
                    acc = valid ? acc : 0u;
                    sMo = valid ? Mou : sMo;
                    sY = valid ? Yu : sY;
                    sH = Hold[R - 1];
                    if (valid && g == glast) lastrow[bj] = mlast;
                }
                sC = cb;
                Htop = rH;
                // traceback slot t - K w: this wave's lanes' nibbles, one dword per 8 / R lanes
                const unsigned word = pack_lanes<R>(acc);
                const int slot = t - kExK * w;   // wave-uniform
                if (slot >= 0 && slot < Lb + nl - 1 && (lane & (8 / R - 1)) == 0)
                    *(unsigned*)(tb + (int64_t)slot * pitch + g * R / 2) = word;
                if (ring_out && lane == 63) ring_out[t & (kExRing - 1)] = make_int4(sMo, sY, sH, sC);
                f0 = f1;
                f1 = f2;
            }
        }
        __syncthreads();   // last row, traceback slots and last-column values complete
        // ---- start cell: corner, then last column bottom -> top, then last row right -> left ----
        long long key = -0x7fffffffffffffffll - 1;
        if (has_rows) {
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int ai = g * R + k;
                if (ai < La) {   // -endweight: minus the trailing end gap of the rows below
                    const long long prio = (ai == La - 1) ? (3ll << 24) : ((2ll << 24) | ai);
                    const long long kk = ((long long)(Mol[k] + O - end_trail(a, La - 1 - ai)) << 32) | prio;
                    key = kk > key ? kk : key;
                }
            }
        }
        if (w == 0)
            for (int q = lane; q < Lb - 1; q += 64) {
                const long long kk = ((long long)(lastrow[q] - end_trail(a, Lb - 1 - q)) << 32) | ((1ll << 24) | q);
                key = kk > key ? kk : key;
            }
        key = wave_max_i64(key);
        if (lane == 0) keys[w] = key;
        __syncthreads();
        if (w == 0) {
            key = keys[0];
            for (int q = 1; q < W; ++q) key = keys[q] > key ? keys[q] : key;
            int score, ei, ej;
            decode_end(key, La, Lb, &score, &ei, &ej);
            auto nib = [&](int ai, int bj, bool* oob) {
                *oob = false;
                const int slot = bj + ai / R;
                return (unsigned)(tb[(int64_t)slot * pitch + (ai >> 1)] >> ((ai & 1) * 4)) & 0xFu;
            };
            const int nruns = walk_runs_wide<4>(nib, La, Lb, ei, ej, runs, La + Lb + 8, lane);
            lds_fence();
            if (nruns < 0) {   // not reached: every cell is stored
                if (lane == 0) { Stat z = {}; z.flags = FLAG_EMPTY; z.score = score; *st = z; }
            } else {
                auto sim = [&](int ai, int code) { return (int)((a.rowpos[ai] >> code) & 1u); };
                if (a.ops) store_ops(a, rd, runs, nruns, lane);
                emit_alignment(runs, nruns, a.amp, rp, a.lut, sim, a.out ? a.out + rd * 3 * a.stride : nullptr,
                               a.stride, score, ei, ej, st, lane, !a.ops);
            }
        }
        __syncthreads();   // LDS reused by the next read
    }
}

int exact_rows_per_lane(int La) {
    for (int R : {1, 2, 4, 8})
        if ((La + R - 1) / R <= 1024) return R;
    return -1;
}

int exact_waves(int La) {
    const int R = exact_rows_per_lane(La);
    if (R < 0) return -1;
    return ((La + R - 1) / R + 63) / 64;
}

int exact_lds_bytes(int La, int Lb_max, bool tb_lds) {
    const int R = exact_rows_per_lane(La);
    if (R < 0) return -1;
    return exact_lds_layout(La, Lb_max, R, exact_waves(La), tb_lds).total;
}

int64_t exact_slab_bytes(int La, int Lb_max) {
    const int R = exact_rows_per_lane(La);
    if (R < 0) return -1;
    const int W = exact_waves(La);
    const int nl = (La + R - 1) / R;
    return (int64_t)(Lb_max + nl + 1) * 32 * W * R;
}

hipError_t launch_exact(const KernelArgs& a, int grid, int lds_bytes, bool tb_lds, int64_t slab_bytes, bool cap,
                        hipStream_t s) {
    const int R = exact_rows_per_lane(a.La);
    const dim3 block(64 * exact_waves(a.La)), g(grid);
#define NW_EXACT_CASE(RR)                                                                                  \
    case RR:                                                                                             \
        if (tb_lds) hipLaunchKernelGGL((nw_exact_kernel<RR, true>), g, block, lds_bytes, s, a, slab_bytes, (int)cap); \
        else hipLaunchKernelGGL((nw_exact_kernel<RR, false>), g, block, lds_bytes, s, a, slab_bytes, (int)cap);       \
        break;
    switch (R) {
        NW_EXACT_CASE(1)
        NW_EXACT_CASE(2)
        NW_EXACT_CASE(4)
        NW_EXACT_CASE(8)
        default: return hipErrorInvalidValue;
    }
#undef NW_EXACT_CASE
    return hipGetLastError();
}

}  // namespace nw
