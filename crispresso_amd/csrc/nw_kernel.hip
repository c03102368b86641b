// nw_kernel.hip -- batched EMBOSS-needle-compatible global alignment for gfx950.
//
// Replaces the per-read DP inside the `needle` process that CRISPResso spawns
// (CRISPResso/CRISPRessoCORE.py:1791-1806 forward, 1812-1828 HDR, 1910-1936 RC).
// Semantics are the ones DESIGN.md "EMBOSS semantics" states (affine Gotoh,
// EDNAFULL, free end gaps, EMBOSS tie rules); the CPU restatement in oracle/ is
// the parity checker.
//
// Mapping (one alignment per 64-lane wavefront):
//   * rows = amplicon (a), columns = read (b).  Lane l owns rows [l*R, l*R+R).
//   * the wave walks columns; at step t lane l works on column t-l (a skewed
//     anti-diagonal wavefront).  The bottom row of lane l (Mo, Y, H) moves to
//     lane l+1 with one DPP wave_shr:1 per value per step -- no LDS round trip.
//   * substitution scores come from a per-amplicon profile in LDS laid out
//     [code][lane][RP] int8, so one ds_read_b32/b64 yields a lane's R scores.
//   * traceback: 4 bits per cell (best-state >M, Y>X, X-extend, Y-extend), every
//     cell stored: in LDS (TB_LDS_FULL) or a per-wave HBM slab (TB_GLOBAL_FULL).
//     This is the exact fallback of the certified band path (nw_band.hip): the
//     reads no band level certifies, rare codes, -endweight, and every read when
//     the band does not apply (penalties outside its int16 range).
//   * the walk is done by the whole wave in runs: 64 lanes test 64 cells of the
//     current diagonal/row/column at once and a ballot finds where the run ends.
//   * the three alignment strings are written straight to HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_common.h"

namespace nw {

template <int R> struct Geo {
    static constexpr int RP = R <= 4 ? 4 : (R <= 8 ? 8 : 16);      // profile bytes per lane
    static constexpr int ES = R <= 2 ? 1 : (R <= 4 ? 2 : (R <= 8 ? 4 : 8));  // tb bytes per (column, lane)
    static constexpr int NW = (R + 7) / 8;                         // 32-bit bit-accumulators
};


__device__ __forceinline__ unsigned push_sign(unsigned acc, int d) {
    // (acc << 1) | (d < 0)
    return __builtin_amdgcn_alignbit(acc, (unsigned)d, 31);
}


// Orders this wave's traceback stores before other lanes' loads of them.
template <int MODE>
__device__ __forceinline__ void tb_fence() {
    if constexpr (MODE != TB_GLOBAL_FULL) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    }
    __builtin_amdgcn_wave_barrier();
}


// Per-wave LDS layout (offsets in bytes from the wave's base), all 16-aligned.
struct WaveLds {
    int raw, coff, lastrow, runs, bits, total;
};


__host__ __device__ inline int es_of(int R) { return R <= 2 ? 1 : (R <= 4 ? 2 : (R <= 8 ? 4 : 8)); }

__host__ __device__ inline WaveLds wave_lds_layout(int R, int La, int Lb_max, int mode) {
    WaveLds w;
    int o = 0;
    w.raw = o;     o += align16(Lb_max + 4);
    w.coff = o;    o += align16(2 * (Lb_max + 4));
    w.lastrow = o; o += align16(4 * (Lb_max + 1 + 64));   // + a dummy slot per lane (branch-free store)
    w.runs = o;    o += align16(4 * (La + Lb_max + 8));
    w.bits = o;
    if (mode == TB_LDS_FULL) o += align16(Lb_max * 64 * es_of(R));
    w.total = align16(o);
    return w;
}

__host__ __device__ inline int shared_lds_bytes(int R, int La) {
    int RP = R <= 4 ? 4 : (R <= 8 ? 8 : 16);
    return align16(NCODE * 64 * RP) + 256 + align16(La + 4);
}

// Where the traceback bits of cell (ai, bj) live: column bj's slot, lane ai / R.
template <int R>
struct TbStore {
    unsigned char* base;
    __device__ __forceinline__ unsigned char* at(int s, int lane) const {
        return base + ((size_t)s * 64 + lane) * Geo<R>::ES;
    }
    // nibble of cell (ai, bj) (every cell is stored: *oob is always false)
    __device__ __forceinline__ unsigned nibble(int ai, int bj, bool* oob) const {
        constexpr int ES = Geo<R>::ES;
        const int lane = ai / R, k = ai - lane * R;
        *oob = false;
        const unsigned char* p = at(bj, lane);
        unsigned w;
        int nr, kk;
        if constexpr (ES == 1) { w = *p; nr = R; kk = k; }
        else if constexpr (ES == 2) { w = *(const unsigned short*)p; nr = R; kk = k; }
        else if constexpr (ES == 4) { w = *(const unsigned*)p; nr = R; kk = k; }
        else {
            const int wi = k >> 3;
            w = ((const unsigned*)p)[wi];
            nr = (R - 8 * wi) < 8 ? (R - 8 * wi) : 8;
            kk = k & 7;
        }
        return (w >> (4 * (nr - 1 - kk))) & 0xFu;
    }
};

template <int R>
__device__ __forceinline__ void store_bits(unsigned char* p, const unsigned (&acc)[Geo<R>::NW]) {
    constexpr int ES = Geo<R>::ES;
    if constexpr (ES == 1) *p = (unsigned char)acc[0];
    else if constexpr (ES == 2) *(unsigned short*)p = (unsigned short)acc[0];
    else if constexpr (ES == 4) *(unsigned*)p = acc[0];
    else { ((unsigned*)p)[0] = acc[0]; ((unsigned*)p)[1] = acc[1]; }
}

template <int R>
__device__ __forceinline__ void load_prof(const unsigned char* prof_lds, int off, int (&sc)[Geo<R>::RP / 4]) {
    constexpr int RP = Geo<R>::RP;
    if constexpr (RP == 4) {
        sc[0] = *(const int*)(prof_lds + off);
    } else if constexpr (RP == 8) {
        int2 v = *(const int2*)(prof_lds + off);
        sc[0] = v.x; sc[1] = v.y;
    } else {
        int4 v = *(const int4*)(prof_lds + off);
        sc[0] = v.x; sc[1] = v.y; sc[2] = v.z; sc[3] = v.w;
    }
}




template <int R, int MODE>
__global__ __launch_bounds__(256) void nw_align_kernel(const KernelArgs args) {
    constexpr int RP = Geo<R>::RP;
    constexpr int NWD = Geo<R>::NW;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int La = args.La;
    const int O = args.gap_open, E = args.gap_extend;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wpb = blockDim.x >> 6;
    if (args.tail_prio && args.work_list) __builtin_amdgcn_s_setprio(3);
    const long long nwork = exact_work_count(args);
    // a work list (or batch) shorter than the grid: blocks past its end leave before any set-up
    if (args.work_lo + (long long)blockIdx.x * wpb >= nwork) return;

    // ---- shared per-block state: profile, ascii->code LUT, amplicon bytes ----
    unsigned char* prof_lds = smem;
    const int prof_bytes = NCODE * 64 * RP;
    unsigned char* lut_lds = smem + align16(prof_bytes);
    unsigned char* amp_lds = lut_lds + 256;
    for (int q = tid; q < prof_bytes / 16; q += blockDim.x)
        ((int4*)prof_lds)[q] = ((const int4*)args.prof)[q];
    for (int q = tid; q < 256; q += blockDim.x) lut_lds[q] = args.lut[q];
    for (int q = tid; q < La; q += blockDim.x) amp_lds[q] = args.amp[q];
    __syncthreads();

    const WaveLds L = wave_lds_layout(R, La, args.Lb_max, MODE);
    unsigned char* wbase = smem + shared_lds_bytes(R, La) + wave * L.total;
    unsigned char* raw = wbase + L.raw;
    unsigned short* coff = (unsigned short*)(wbase + L.coff);
    int* lastrow = (int*)(wbase + L.lastrow);
    unsigned* runs = (unsigned*)(wbase + L.runs);
    const long long gw = (long long)blockIdx.x * wpb + wave;
    const long long nwaves = (long long)gridDim.x * wpb;
    TbStore<R> tb;
    if constexpr (MODE == TB_GLOBAL_FULL) tb.base = args.tb_global + gw * args.tb_wave_bytes;
    else tb.base = wbase + L.bits;

    const int nl = (La + R - 1) / R;        // lanes holding real rows
    const int ai0 = lane * R;
    const int lr = (La - 1) / R;            // lane holding the last row
    const int klast = (La - 1) - lr * R;
    const int prof_lane = lane * RP;
    const int pad_coff = NCODE_PAD * 64 * RP;   // offset of the all-zero pad code

    for (long long wi = args.work_lo + gw; wi < nwork; wi += nwaves) {
        const long long rd = exact_work_read(args, wi);
        const long long off = args.offsets[rd];
        const int Lb = (int)(args.offsets[rd + 1] - off);
        Stat* st = args.stats + rd;
        if (Lb <= 0) {
            if (lane == 0) {
                Stat z = {};
                z.flags = FLAG_EMPTY;
                *st = z;
                if (args.ops) args.nops[rd] = 0;
            }
            continue;
        }
        // ---- stage the read: raw bytes + profile offsets of each column ----
        const unsigned char* rp = args.reads + off;
        for (int q = lane; q < Lb + 4; q += 64) {
            unsigned char c = q < Lb ? rp[q] : (unsigned char)'N';
            raw[q] = c;
            coff[q] = (unsigned short)(q < Lb ? lut_lds[c] * 64 * RP : pad_coff);
        }
        lds_fence();

        // ---- DP fill ----
        // column -1 (left boundary): H = M = 0 with free end gaps, the leading end-gap
        // value of row ai + 1 with -endweight; X = -inf
        int Mol[R], Xl[R], Hold[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int h0 = end_lead(args, ai0 + k + 1);
            Mol[k] = h0 - O; Xl[k] = NEG; Hold[k] = h0;
        }
        int sMo = Mol[R - 1], sY = NEG, sH = Hold[R - 1];   // what this lane's bottom row sends down
        int Htop = end_lead(args, ai0);                      // H[row above][column-1]
        const int nsteps = Lb + nl - 1;
        // prefetch pipeline: coff for bj+1 loaded one step ahead, scores for bj loaded one step ahead
        int bj0 = -lane;
        int c_next = coff[min(max(bj0 + 1, 0), Lb + 3)];
        int sc[RP / 4];
        load_prof<R>(prof_lds, coff[min(max(bj0, 0), Lb + 3)] + prof_lane, sc);
        for (int t = 0; t < nsteps; ++t) {
            const int bj = t - lane;
            // lane 0's row above is the top boundary at column t (leading end gap of t + 1)
            const int top = end_lead(args, t + 1);
            const int rMo = shr1(sMo, top - O);
            const int rY = shr1(sY, NEG);
            const int rH = shr1(sH, top);
            // issue next loads before the compute that hides their latency
            int sc_n[RP / 4];
            load_prof<R>(prof_lds, c_next + prof_lane, sc_n);
            const int c_nn = coff[min(max(bj + 2, 0), Lb + 3)];
            if (bj >= 0 && bj < Lb && lane < nl) {
                unsigned acc[NWD];
                unsigned nib[R];   // each cell's 4 traceback bits, built independently (no serial chain
                                   // through the whole step: one wave per SIMD runs this kernel, so its
                                   // dependency depth is its latency)
                int Hd = Htop, Mou = rMo, Yu = rY;
                int mlast = 0;
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const int s = __builtin_amdgcn_sbfe(sc[k >> 2], 8 * (k & 3), 8);
                    const int M = Hd + s;
                    const int Xe = Xl[k] - E;
                    const int X = max(Mol[k], Xe);
                    const int Ye = Yu - E;
                    const int Y = max(Mou, Ye);
                    const int mxy = max(X, Y);
                    const int H = max(M, mxy);
                    unsigned a = (unsigned)(Ye - Mou) >> 31;   // Y opens (open > extend)
                    a = push_sign(a, Xe - Mol[k]);            // X opens
                    a = push_sign(a, X - Y);                  // Y > X (X wins an X == Y tie)
                    a = push_sign(a, M - mxy);                // M < max(X, Y)
                    nib[k] = a;
                    mlast = (k == klast) ? M : mlast;
                    Hd = Hold[k];
                    Hold[k] = H;
                    Mol[k] = M - O;
                    Xl[k] = X;
                    Mou = M - O;
                    Yu = Y;
                }
                sMo = Mou; sY = Yu; sH = Hold[R - 1];
                // word w: cells 8w .. 8w + nr - 1, the first cell in the top nibble; pairs of cells
                // first (a chain over pairs, not over cells)
#pragma unroll
                for (int w = 0; w < NWD; ++w) {
                    constexpr int kNr8 = 8;
                    const int k0 = kNr8 * w, nr = (R - k0) < kNr8 ? (R - k0) : kNr8;
                    unsigned v = 0;
#pragma unroll
                    for (int k = 0; k < kNr8; k += 2) {
                        if (k >= nr) break;
                        if (k + 1 < nr) v = (v << 8) | (nib[k0 + k] << 4) | nib[k0 + k + 1];
                        else v = (v << 4) | nib[k0 + k];
                    }
                    acc[w] = v;
                }
                store_bits<R>(tb.at(bj, lane), acc);
                lastrow[lane == lr ? bj : args.Lb_max + 1 + lane] = mlast;   // the last row's M (other lanes: a dummy slot)
            }
            Htop = rH;
#pragma unroll
            for (int w = 0; w < RP / 4; ++w) sc[w] = sc_n[w];
            c_next = c_nn;
        }
        // Mol[k] + O is M of the last column for this lane's rows.
        // ---- start cell: corner, then last column bottom->top, then last row right->left ----
        long long key = -0x7fffffffffffffffll - 1;
        if (lane < nl) {
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int ai = ai0 + k;
                if (ai < La) {   // -endweight: minus the trailing end gap of the rows below
                    const long long prio = (ai == La - 1) ? (3ll << 24) : ((2ll << 24) | ai);
                    const long long kk = ((long long)(Mol[k] + O - end_trail(args, La - 1 - ai)) << 32) | prio;
                    key = kk > key ? kk : key;
                }
            }
        }
        tb_fence<MODE>();
        for (int q = lane; q < Lb - 1; q += 64) {
            const long long kk = ((long long)(lastrow[q] - end_trail(args, Lb - 1 - q)) << 32) | ((1ll << 24) | q);
            key = kk > key ? kk : key;
        }
        key = wave_max_i64(key);
        int score, ei, ej;   // 1-based start cell
        decode_end(key, La, Lb, &score, &ei, &ej);

        // ---- traceback in runs ----
        auto nib = [&](int ai, int bj, bool* oob) { return tb.nibble(ai, bj, oob); };
        const int nruns = walk_runs(nib, La, Lb, ei, ej, runs, La + Lb + 8, lane);
        if (nruns < 0) {
            if (lane == 0) args.fallback_list[atomicAdd(args.fallback_count, 1)] = rd;
            continue;
        }
        lds_fence();
        // ---- emit strings, forward order ----
        auto sim = [&](int ai, int code) {
            return (int)(signed char)prof_lds[code * 64 * RP + (ai / R) * RP + (ai % R)];
        };
        if (args.ops) store_ops(args, rd, runs, nruns, lane);
        emit_alignment(runs, nruns, amp_lds, raw, lut_lds, sim, args.out + rd * 3 * args.stride, args.stride,
                       score, ei, ej, st, lane, !args.ops);
        lds_fence();
    }
}

}  // namespace nw

// ---------------------------------------------------------------- launcher

namespace nw {

template <int R>
static hipError_t launch_r(const KernelArgs& a, const LaunchCfg& c, hipStream_t s) {
    const dim3 grid(c.grid), block(64 * c.wpb);
    switch (c.tb_mode) {
        case TB_LDS_FULL: hipLaunchKernelGGL((nw_align_kernel<R, TB_LDS_FULL>), grid, block, c.lds_bytes, s, a); break;
        case TB_GLOBAL_FULL: hipLaunchKernelGGL((nw_align_kernel<R, TB_GLOBAL_FULL>), grid, block, c.lds_bytes, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int lds_bytes_for(int R, int La, int Lb_max, int tb_mode, int wpb) {
    if (rows_per_lane_for(R * 64) != R) return -1;
    return shared_lds_bytes(R, La) + wpb * wave_lds_layout(R, La, Lb_max, tb_mode).total;
}

int rows_per_lane_for(int La) {
    int r = (La + 63) / 64;
    if (r <= 8) return r;
    if (r <= 10) return 10;
    if (r <= 12) return 12;
    if (r <= 14) return 14;
    if (r <= 16) return 16;
    return -1;
}

int tb_bytes_per_wave(int R, int Lb_max) { return align16(Lb_max * 64 * es_of(R)); }

int profile_rp(int R) { return R <= 4 ? 4 : (R <= 8 ? 8 : 16); }

hipError_t launch(const KernelArgs& a, const LaunchCfg& c, hipStream_t s) {
    switch (c.R) {
        case 1: return launch_r<1>(a, c, s);
        case 2: return launch_r<2>(a, c, s);
        case 3: return launch_r<3>(a, c, s);
        case 4: return launch_r<4>(a, c, s);
        case 5: return launch_r<5>(a, c, s);
        case 6: return launch_r<6>(a, c, s);
        case 7: return launch_r<7>(a, c, s);
        case 8: return launch_r<8>(a, c, s);
        case 10: return launch_r<10>(a, c, s);
        case 12: return launch_r<12>(a, c, s);
        case 14: return launch_r<14>(a, c, s);
        case 16: return launch_r<16>(a, c, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace nw
