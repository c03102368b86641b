// nw_common.h -- device helpers shared by the aligner kernels: lane moves,
// fences, the run-based traceback walk and the string emitter.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_device.h"

namespace nw {

constexpr int NEG = -(1 << 28);

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

__device__ __forceinline__ int shr1(int v, int fill) {
    // DPP wave_shr:1 -- lane l receives lane l-1's value, lane 0 keeps `fill`.
    return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xf, 0xf, false);
}

__device__ __forceinline__ void lds_fence() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ unsigned char upcase(unsigned char c) {
    return (c >= 'a' && c <= 'z') ? (unsigned char)(c - 32) : c;
}

__device__ __forceinline__ long long wave_max_i64(long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        long long u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}

// Wave reductions on DPP (row_shr within 16-lane rows, then row_bcast:15/31):
// six VALU ops with no LDS round trip; the result is read from lane 63.
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp_max_step(unsigned v) {
    const unsigned o = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
    return v > o ? v : o;
}
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp_add_step(unsigned v) {
    return v + (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
    v = dpp_max_step<0x111, 0xf>(v);
    v = dpp_max_step<0x112, 0xf>(v);
    v = dpp_max_step<0x114, 0xf>(v);
    v = dpp_max_step<0x118, 0xf>(v);
    v = dpp_max_step<0x142, 0xa>(v);
    v = dpp_max_step<0x143, 0xc>(v);
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ unsigned wave_sum_u32(unsigned v) {
    v = dpp_add_step<0x111, 0xf>(v);
    v = dpp_add_step<0x112, 0xf>(v);
    v = dpp_add_step<0x114, 0xf>(v);
    v = dpp_add_step<0x118, 0xf>(v);
    v = dpp_add_step<0x142, 0xa>(v);
    v = dpp_add_step<0x143, 0xc>(v);
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ int wave_sum(int v) { return (int)wave_sum_u32((unsigned)v); }

// ---- single-pass block prefix (decoupled look-back) --------------------------------
// One launch instead of block sums + one scan block + scatter.  Block b publishes an
// 8-byte status {epoch, flag, value} per block: first its own aggregate (AGG), then its
// inclusive prefix (INC) once it has it; it finds its exclusive prefix by reading back
// over its predecessors, 64 at a time (one per lane), summing aggregates down to the
// nearest inclusive prefix.  The status words are written and read with agent-scope
// 8-byte atomics (sc1: at the memory side, coherent across the XCDs' L2s, no L2
// write-back fence -- MI355X_MICROARCH.md, inter-workgroup visibility); nothing else is
// handed between blocks inside the launch.  `epoch` (30 bits, new per launch) replaces
// zeroing the array between launches.  Relies on workgroups being dispatched in index
// order (a predecessor is resident or done when a block waits for it); a wait that never
// ends is cut off after ~10^7 polls and reported through *bad (the caller's error flag)
// instead of hanging the device.
constexpr unsigned kLbAgg = 1u, kLbInc = 2u;
__device__ __forceinline__ unsigned long long lb_word(unsigned epoch, unsigned flag, unsigned value) {
    return ((unsigned long long)((epoch << 2) | flag) << 32) | value;
}
// Called by every lane of ONE wave of block b (uniform control flow); returns the
// exclusive prefix of block b's `agg` (the same value in every lane).
__device__ inline unsigned lookback_excl(unsigned long long* st, long long b, unsigned epoch, unsigned agg,
                                         int* bad) {
    const int lane = threadIdx.x & 63;
    epoch &= 0x3fffffffu;
    if (b == 0) {
        if (lane == 0) __hip_atomic_store(st, lb_word(epoch, kLbInc, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0u;
    }
    if (lane == 0) __hip_atomic_store(st + b, lb_word(epoch, kLbAgg, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned excl = 0u;
    long long j = b - 1;   // the newest predecessor not yet summed
    int polls = 0;
    for (;;) {
        const long long idx = j - lane;
        unsigned long long v = lb_word(epoch, kLbInc, 0u);   // before block 0: an inclusive 0
        if (idx >= 0) v = __hip_atomic_load(st + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned tag = (unsigned)(v >> 32);
        const bool ready = (tag >> 2) == epoch && (tag & 3u) != 0u;
        const unsigned long long inc = __ballot(ready && (tag & 3u) == kLbInc);
        const unsigned long long notr = __ballot(!ready);
        const int first = inc ? (int)__builtin_ctzll(inc) : 64;      // nearest inclusive prefix
        const unsigned long long need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
        if (notr & need) {   // a predecessor before it has not published yet: poll again
            if (++polls > (1 << 23)) {
                if (lane == 0) *bad = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += wave_sum_u32(lane <= first ? (unsigned)v : 0u);
        if (first < 64) break;
        j -= 64;
    }
    if (lane == 0)
        __hip_atomic_store(st + b, lb_word(epoch, kLbInc, excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// Candidate key for the traceback start cell.  Scan order of the reference
// walk start (corner, then last column bottom->top, then last row right->left,
// first strict maximum) becomes "largest (score, priority)".
__device__ __forceinline__ long long end_key(int score, int cls, int pos) {
    return ((long long)score << 32) | (((long long)cls << 24) | pos);
}
// The same order in 32 bits when |score| < 2^15 and pos < 2^14 (int16 kernels).
__device__ __forceinline__ unsigned end_key32(int score, int cls, int pos) {
    return ((unsigned)(score + 32768) << 16) | ((unsigned)cls << 14) | (unsigned)pos;
}
__device__ __forceinline__ long long end_key_widen(unsigned k) {
    return end_key((int)(k >> 16) - 32768, (int)((k >> 14) & 3), (int)(k & 0x3fff));
}
__device__ __forceinline__ void decode_end(long long key, int La, int Lb, int* score, int* ei, int* ej) {
    *score = (int)(key >> 32);
    const int prio = (int)(key & 0xffffffff);
    if ((prio >> 24) == 3) { *ei = La; *ej = Lb; }
    else if ((prio >> 24) == 2) { *ei = (prio & 0xffffff) + 1; *ej = Lb; }
    else { *ei = La; *ej = (prio & 0xffffff) + 1; }
}

// Run codes stored in LDS: type << 28 | length.
enum { RUN_M = 0, RUN_X = 1, RUN_Y = 2 };

// Traceback walk in runs.  `nib(ai, bj, &oob)` returns the 4-bit cell code
// (bit0: M < max(X,Y), bit1: Y > X, bit2: X opens, bit3: Y opens) of the
// 0-based cell, setting oob when the cell is not stored.  Writes runs in
// end->start order to `runs` (lane 0, at most `cap`), returns the count, or -1
// when the walk needs a cell outside the stored band or more than `cap` runs.
template <class Nib>
__device__ int walk_runs(const Nib& nib, int La, int Lb, int ei, int ej, unsigned* runs, int cap, int lane) {
    int nruns = 0, last_type = -1;
    bool full = false;
    auto push = [&](int type, int n) {
        if (n <= 0) return;
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
    if (ei == La && ej < Lb) push(RUN_X, Lb - ej);
    else if (ej == Lb && ei < La) push(RUN_Y, La - ei);
    int i = ei, j = ej, state = RUN_M;
    while (i > 0 && j > 0) {
        bool oob = false;
        unsigned long long m;
        int nb = RUN_M;
        if (state == RUN_M) {
            const int ci = i - 1 - lane, cj = j - 1 - lane;
            const bool valid = ci >= 1 && cj >= 1;
            const unsigned c = valid ? nib(ci - 1, cj - 1, &oob) : 0u;
            oob = valid && oob;
            // EMBOSS tie rules (pinned by the reference's e2e values):
            // M when M >= max(X, Y), else X when X >= Y; a gap run ends only where open > extend
            const int best = (c & 1u) ? ((c & 2u) ? RUN_Y : RUN_X) : RUN_M;
            m = __ballot(!valid || oob || best != RUN_M);
            if (m == 0) { push(RUN_M, 64); i -= 64; j -= 64; continue; }
            nb = __builtin_amdgcn_readlane(best, (int)__builtin_ctzll(m));
        } else if (state == RUN_X) {
            const int cj = j - lane;
            const bool valid = cj >= 1;
            const unsigned c = valid ? nib(i - 1, cj - 1, &oob) : 0u;
            oob = valid && oob;
            m = __ballot(!valid || oob || (c & 4u));
            if (m == 0) { push(RUN_X, 64); j -= 64; continue; }
        } else {
            const int ci = i - lane;
            const bool valid = ci >= 1;
            const unsigned c = valid ? nib(ci - 1, j - 1, &oob) : 0u;
            oob = valid && oob;
            m = __ballot(!valid || oob || (c & 8u));
            if (m == 0) { push(RUN_Y, 64); i -= 64; continue; }
        }
        const int k0 = (int)__builtin_ctzll(m);
        if ((__ballot(oob) & (1ull << k0)) || full) return -1;
        push(state, k0 + 1);
        if (state != RUN_Y) j -= k0 + 1;
        if (state != RUN_X) i -= k0 + 1;
        state = (state == RUN_M) ? nb : RUN_M;
    }
    if (i > 0) push(RUN_Y, i);
    if (j > 0) push(RUN_X, j);
    return full ? -1 : nruns;
}

// walk_runs with CPL consecutive run cells per lane: one ballot tests 64*CPL
// cells (lane k holds run offsets k*CPL .. k*CPL+CPL-1), so a 250-cell match run
// costs one round trip to the band instead of four.  Same results as walk_runs.
template <int CPL, class Nib>
__device__ int walk_runs_wide(const Nib& nib, int La, int Lb, int ei, int ej, unsigned* runs, int cap, int lane) {
    int nruns = 0, last_type = -1;
    bool full = false;
    auto push = [&](int type, int n) {
        if (n <= 0) return;
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
    if (ei == La && ej < Lb) push(RUN_X, Lb - ej);
    else if (ej == Lb && ei < La) push(RUN_Y, La - ei);
    constexpr int W = 64 * CPL;
    int i = ei, j = ej, state = RUN_M;
    while (i > 0 && j > 0) {
        int first = CPL, first_best = RUN_M;
        bool first_oob = false;
        unsigned c[CPL];
        bool valid[CPL], oob[CPL];
        // all CPL lookups first (independent loads in flight together), then the tests
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const int kk = lane * CPL + u;
            oob[u] = false;
            if (state == RUN_M) {
                const int ci = i - 1 - kk, cj = j - 1 - kk;
                valid[u] = ci >= 1 && cj >= 1;
                c[u] = valid[u] ? nib(ci - 1, cj - 1, &oob[u]) : 0u;
            } else if (state == RUN_X) {
                const int cj = j - kk;
                valid[u] = cj >= 1;
                c[u] = valid[u] ? nib(i - 1, cj - 1, &oob[u]) : 0u;
            } else {
                const int ci = i - kk;
                valid[u] = ci >= 1;
                c[u] = valid[u] ? nib(ci - 1, j - 1, &oob[u]) : 0u;
            }
        }
#pragma unroll
        for (int u = CPL - 1; u >= 0; --u) {
            const int best = (c[u] & 1u) ? ((c[u] & 2u) ? RUN_Y : RUN_X) : RUN_M;
            const bool go = state == RUN_M ? best == RUN_M : (c[u] & (state == RUN_X ? 4u : 8u)) == 0;
            if (!valid[u] || oob[u] || !go) {
                first = u;
                first_oob = valid[u] && oob[u];
                first_best = best;
            }
        }
        const unsigned long long m = __ballot(first < CPL);
        if (m == 0) {
            push(state, W);
            if (state != RUN_Y) j -= W;
            if (state != RUN_X) i -= W;
            continue;
        }
        const int L = (int)__builtin_ctzll(m);
        const int k0 = L * CPL + __builtin_amdgcn_readlane(first, L);
        const int nb = __builtin_amdgcn_readlane(first_best, L);
        if (__builtin_amdgcn_readlane((int)first_oob, L) || full) return -1;
        push(state, k0 + 1);
        if (state != RUN_Y) j -= k0 + 1;
        if (state != RUN_X) i -= k0 + 1;
        state = (state == RUN_M) ? nb : RUN_M;
    }
    if (i > 0) push(RUN_Y, i);
    if (j > 0) push(RUN_X, j);
    return full ? -1 : nruns;
}

// Writes the aligned amplicon / markup / aligned read for the runs (forward
// order) and the per-read record.  `sim_score(ai, code)` is the substitution
// score of amplicon row ai against residue code (only its sign matters).
// Ops output (KernelArgs::ops): the runs (LDS, end -> start order) of read rd, start
// -> end, into its slot, or -- more runs than a slot holds -- into the spill area
// (bump-allocated, the position in slot[0]).  A full spill area sets ops_ctl[1]
// (the host reports it).  Rows are not written in this mode.
__device__ inline void store_ops(const KernelArgs& a, long long rd, const unsigned* runs, int nruns, int lane) {
    // the walk / exact kernels: one read per wave, its runs contiguous in the row-major area
    // (one line per read); its slot's first column-major word holds the spill position
    uint32_t* slot = a.ops + rd;
    uint32_t* dst = a.ops + a.ops_stride * a.ops_slot + rd * a.ops_slot;
    int32_t flag = kNopsRows;
    if (nruns > a.ops_slot) {
        flag = 0;
        int pos = 0;
        if (lane == 0) pos = atomicAdd(a.ops_ctl, nruns);
        pos = __builtin_amdgcn_readfirstlane(pos);
        if ((long long)pos + nruns > a.spill_cap) {
            if (lane == 0) {
                atomicOr(a.ops_ctl + 1, 1);
                a.nops[rd] = 0;
            }
            return;
        }
        if (lane == 0) slot[0] = (uint32_t)pos;
        dst = a.spill + pos;
    }
    if (lane == 0) a.nops[rd] = nruns | flag;
    for (int q = lane; q < nruns; q += 64) dst[q] = runs[nruns - 1 - q];
}

template <class Score>
__device__ void emit_alignment(const unsigned* runs, int nruns, const unsigned char* amp, const unsigned char* raw,
                               const unsigned char* lut, const Score& sim_score, unsigned char* o_ref,
                               int64_t stride, int score, int ei, int ej, Stat* st, int lane, bool rows = true) {
    unsigned char* o_mk = o_ref + stride;
    unsigned char* o_rd = o_mk + stride;
    int col = 0, ia = 0, jb = 0;
    int n_id = 0, n_sim = 0, n_gap = 0;
    for (int q = nruns - 1; q >= 0; --q) {
        const unsigned rc = (unsigned)__builtin_amdgcn_readfirstlane((int)runs[q]);   // uniform: scalar branches
        const int type = (int)(rc >> 28);
        const int n = (int)(rc & 0x0fffffffu);
        for (int p = lane; p < n; p += 64) {
            unsigned char ca = '-', cb = '-', mk = ' ';
            if (type != RUN_X) ca = amp[ia + p];
            if (type != RUN_Y) cb = raw[jb + p];
            // a '-' already in the input (RC-pass reads, CRISPRessoCORE.py:1846) prints
            // like a gap, so it counts as one, as for an alignment gap
            const bool gapcol = ca == '-' || cb == '-';
            n_gap += gapcol;
            if (type == RUN_M && !gapcol) {
                const bool id = upcase(ca) == upcase(cb);
                const bool sim = id || sim_score(ia + p, (int)lut[cb]) > 0;
                mk = id ? '|' : (sim ? ':' : '.');
                n_id += id;
                n_sim += sim;
            }
            if (rows) {
                o_ref[col + p] = ca;
                o_mk[col + p] = mk;
                o_rd[col + p] = cb;
            }
        }
        col += n;
        if (type != RUN_X) ia += n;
        if (type != RUN_Y) jb += n;
    }
    if (col < 1024) {   // uniform: the three per-lane counts fit 10 bits each -> one reduction
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

}  // namespace nw
