// nw_ops.hip -- ops output compaction.
//
// In ops mode (KernelArgs::ops, include/crispr_nw.h nw_align_ops) every aligner
// kernel leaves a read's traceback runs in its fixed slot (or the spill area) and
// the run count in nops[r].  What crosses PCIe is one contiguous run array plus
// the per-read start offsets, made by ONE launch per chunk of reads: block b sums
// the runs of its kOpsBlockReads reads, finds the runs of the blocks before it by
// look-back (nw_common.h lookback_excl: no second scan launch), writes the reads'
// offsets (the call's running base + local offset) and copies their runs into the
// staging array.  The last block writes the chunk's ctl (base, total, path counts)
// and its pinned host mirror (no copy launch in the chunk's chain).  The running base
// alternates between two words (ctl[kOpsCtl + parity]): chunk k reads one and writes the
// other, so no block of a launch can see its own chunk's update.
// The host copies staging[0, ctl[2]) to ops_out + ctl[1].
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "nw_common.h"

namespace nw {

namespace {

constexpr int kOpsThreads = 256;
constexpr int kOpsPerThread = kOpsBlockReads / kOpsThreads;   // 4

// exclusive scan over the block of one int64 per thread (LDS, Hillis-Steele over waves)
__device__ long long block_excl_scan(long long v, long long* total) {
    __shared__ long long wsum[kOpsThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    long long incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    long long before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kOpsThreads / 64; ++w) {
        before += w < wave ? wsum[w] : 0;
        all += wsum[w];
    }
    __syncthreads();
    *total = all;
    return before + incl - v;
}

__global__ __launch_bounds__(kOpsThreads) void nw_ops_compact(const int32_t* nops, const uint32_t* slots, int slot,
                                                              int64_t stride, const uint32_t* spill, int64_t n,
                                                              unsigned long long* status, unsigned epoch, int parity,
                                                              int64_t* ctl, int64_t* ops_off, uint32_t* staging,
                                                              int64_t staging_cap, const int32_t* opsctl,
                                                              OpsCounts cnt, int64_t* hctl, int prio, OpsHostOut ho,
                                                              Stat* stats, OpsKnown kn) {
    __shared__ int sh_bad;
    __shared__ unsigned sh_excl;
    if (prio) __builtin_amdgcn_s_setprio(3);
    const long long r0 = (long long)blockIdx.x * kOpsBlockReads + threadIdx.x * kOpsPerThread;
    int c4[kOpsPerThread];
    bool rows4[kOpsPerThread], known4[kOpsPerThread];
    // the known alignment (a copy of the known sequence takes its record and runs)
    const int kraw = kn.stat ? *kn.nops : 0;
    const int kc = kraw & (kNopsKnown - 1);
    long long s = 0;
#pragma unroll
    for (int k = 0; k < kOpsPerThread; ++k) {
        const int raw = r0 + k < n ? nops[r0 + k] : 0;
        known4[k] = kn.stat && (raw & kNopsKnown);
        c4[k] = known4[k] ? kc : raw & (kNopsKnown - 1);
        rows4[k] = (raw & kNopsRows) != 0;
        s += c4[k];
    }
    if (kn.stat) {   // the known copies' records, before the host copy below reads them
        const Stat ks = *kn.stat;
#pragma unroll
        for (int k = 0; k < kOpsPerThread; ++k)
            if (known4[k]) stats[r0 + k] = ks;
    }
    if (threadIdx.x == 0) sh_bad = 0;
    long long total;
    const long long local = block_excl_scan(s, &total);   // (its barriers order sh_bad's reset)
    if (threadIdx.x < 64) {
        const unsigned e = lookback_excl(status, blockIdx.x, epoch, (unsigned)total, &sh_bad);
        if (threadIdx.x == 0) sh_excl = e;
    }
    __syncthreads();
    const long long base = ctl[kOpsCtl + parity];
    long long off = (long long)sh_excl + local;
    bool over = false;
    if (ho.dstats) {   // the call's last chunk: records and offsets straight to the caller (coalesced rows)
        long long o = off;
#pragma unroll
        for (int k = 0; k < kOpsPerThread; ++k) {
            const long long r = r0 + k;
            if (r >= n) break;
            ho.hstats[2 * r] = ho.dstats[2 * r];
            ho.hstats[2 * r + 1] = ho.dstats[2 * r + 1];
            ho.hoff[r] = base + o;
            o += c4[k];
        }
    }
#pragma unroll
    for (int k = 0; k < kOpsPerThread; ++k) {
        const long long r = r0 + k;
        if (r >= n) break;
        ops_off[r] = base + off;
        const int c = c4[k];
        // column-major: run q of read r at slots[q * stride + r] (consecutive reads' first runs
        // share lines); row-major (rows4): contiguous at slots[stride * slot + r * slot]
        const uint32_t* src = slots + r;
        long long step = stride;
        if (known4[k]) {   // the known alignment's 1-read layout (ops_stride 1)
            step = 1;
            src = c > kn.slot ? kn.spill + kn.slots[0] : ((kraw & kNopsRows) ? kn.slots + kn.slot : kn.slots);
        } else if (c > slot) {
            src = spill + src[0];
            step = 1;
        } else if (rows4[k]) {
            src = slots + stride * slot + r * slot;
            step = 1;
        }
        if (off + c > staging_cap) {
            over = true;
        } else if (ho.hops) {
            uint32_t* h = ho.hops + base + off;
            const bool fits = base + off + c <= ho.hcap;   // (short: the host reports NW_E_CAPACITY)
            for (int q = 0; q < c; ++q) {
                const uint32_t v = src[q * step];
                staging[off + q] = v;
                if (fits) h[q] = v;
            }
        } else {
            for (int q = 0; q < c; ++q) staging[off + q] = src[q * step];
        }
        off += c;
    }
    if (over) {
        atomicOr((unsigned long long*)(ctl + 3), 1ull);
        if (hctl) hctl[3] |= 1;   // every writer sets the same bit over the value the last block left
    }
    if (threadIdx.x == 0 && sh_bad) {
        atomicOr((unsigned long long*)(ctl + 3), 4ull);
        if (hctl) hctl[3] |= 4;
    }
    if (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1) {
        const long long chunk_total = (long long)sh_excl + total;
        ctl[1] = base;
        ctl[2] = chunk_total;
        ops_off[n] = base + chunk_total;   // the end of the chunk's last read (the next chunk's first offset)
        ctl[0] = base + chunk_total;
        ctl[kOpsCtl + (parity ^ 1)] = base + chunk_total;
        if (opsctl[1]) ctl[3] |= 2;   // a kernel found the spill area full
        if (cnt.fallback && cnt.fallback[3]) ctl[3] |= 4;   // an aligner kernel's look-back was cut off
        // the call's reads by path, summed over chunks (nw_batch_path_counts after nw_align_ops)
        long long fb = 0;
        if (cnt.fallback) fb += cnt.fallback[0];
        // a chunk that skipped its second level (KernelArgs::redo_direct) sent the redo
        // list to the exact kernel
        const bool direct = cnt.direct > 0 && cnt.redo && *cnt.redo <= cnt.direct;
        if (direct) fb += *cnt.redo;
        // seeded: DP reads the wide level takes first, but the 32-diagonal level's; a padding entry
        // repeats its segment's last read, so it sits in whichever share that read's pair went to
        const long long ns = cnt.seeded ? (long long)*cnt.seeded : 0ll;
        const long long pad = cnt.seed_pad ? (long long)*cnt.seed_pad : 0ll;
        long long n2 = cnt.seeded_l2 ? ns - (long long)*cnt.seeded_l2 : 0ll;
        long long nw = ns - n2;
        const long long pw = nw < pad ? nw : pad;
        nw -= pw;
        n2 -= pad - pw;
        ctl[4] += fb + nw;
        ctl[8] += cnt.exact ? (long long)*cnt.exact : fb;
        if (cnt.redo && !direct) ctl[5] += *cnt.redo;
        ctl[5] += n2;
        const long long dp = (cnt.band ? *cnt.band : 0) + ns - pad;
        ctl[6] += dp;
        if (cnt.one_level) ctl[7] += dp;
        if (hctl)
            for (int q = 0; q < kOpsCtl; ++q) hctl[q] = ctl[q];
    }
}

}  // namespace

hipError_t launch_ops_compact(const int32_t* nops, const uint32_t* slots, int slot, int64_t stride, const uint32_t* spill, int64_t n,
                              unsigned long long* status, unsigned epoch, int parity, int64_t* ctl, int64_t* ops_off,
                              uint32_t* staging, int64_t staging_cap, int32_t* opsctl, const OpsCounts& cnt,
                              hipStream_t s, int64_t* hctl, const OpsHostOut* host, Stat* stats, const OpsKnown* known) {
    const OpsHostOut ho = host ? *host : OpsHostOut{};
    const OpsKnown kn = known && stats ? *known : OpsKnown{};
    const int nblk = (int)std::max<int64_t>(1, (n + kOpsBlockReads - 1) / kOpsBlockReads);
    hipLaunchKernelGGL(nw_ops_compact, dim3(nblk), dim3(kOpsThreads), 0, s, nops, slots, slot, stride, spill, n, status, epoch,
                       parity, ctl, ops_off, staging, staging_cap, opsctl, cnt, hctl, cnt.prio, ho, stats, kn);
    return hipGetLastError();
}

}  // namespace nw
