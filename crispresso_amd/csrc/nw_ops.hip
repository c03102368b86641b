// nw_ops.hip -- ops output compaction.
//
// In ops mode (KernelArgs::ops, include/crispr_nw.h nw_align_ops) every aligner
// kernel leaves a read's traceback runs in its fixed slot (or the spill area) and
// the run count in nops[r].  What crosses PCIe is one contiguous run array plus
// the per-read start offsets: three launches per chunk of reads --
//   blocksum: runs per block of kOpsBlockReads reads,
//   scan:     exclusive scan of the block sums (one block); the chunk's base is
//             the running total of the call's earlier chunks (ctl[0], in-stream);
//             the chunk's ctl also goes straight to the caller's pinned host mirror
//             (no copy launch in the chunk's chain),
//   compact:  per-read offsets (ops_off = chunk base + local offset) and the
//             copy of every read's runs into the staging array at its local offset.
// The host copies staging[0, ctl[2]) to ops_out + ctl[1].
#include <hip/hip_runtime.h>
#include <stdint.h>

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

__global__ __launch_bounds__(kOpsThreads) void nw_ops_blocksum(const int32_t* nops, int64_t n, int64_t* blk) {
    const long long r0 = (long long)blockIdx.x * kOpsBlockReads + threadIdx.x * kOpsPerThread;
    long long s = 0;
#pragma unroll
    for (int k = 0; k < kOpsPerThread; ++k) s += r0 + k < n ? nops[r0 + k] : 0;
    long long total;
    block_excl_scan(s, &total);
    if (threadIdx.x == 0) blk[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void nw_ops_scan(int64_t* blk, int nblk, int64_t* ctl, const int32_t* opsctl,
                                                    OpsCounts cnt, int64_t* hctl) {
    __shared__ long long part[1024];
    long long carry = 0;
    for (int t0 = 0; t0 < nblk; t0 += 1024) {
        const int t = t0 + (int)threadIdx.x;
        const long long v = t < nblk ? blk[t] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const long long u = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += u;
            __syncthreads();
        }
        if (t < nblk) blk[t] = carry + part[threadIdx.x] - v;
        carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        ctl[1] = ctl[0];
        ctl[2] = carry;
        ctl[0] += carry;
        if (opsctl[1]) ctl[3] |= 2;   // a kernel found the spill area full
        // the call's reads by path, summed over chunks (nw_batch_path_counts after nw_align_ops)
        long long fb = 0;
        if (cnt.fallback) fb += cnt.fallback[0];
        // a chunk that skipped its second level (KernelArgs::redo_direct) sent the redo
        // list to the exact kernel
        const bool direct = cnt.direct > 0 && cnt.redo && *cnt.redo <= cnt.direct;
        if (direct) fb += *cnt.redo;
        ctl[4] += fb;
        if (cnt.redo && !direct) ctl[5] += *cnt.redo;
        if (cnt.band) ctl[6] += *cnt.band;
        if (cnt.band && cnt.one_level) ctl[7] += *cnt.band;
        if (hctl)
            for (int q = 0; q < kOpsCtl; ++q) hctl[q] = ctl[q];
    }
}

__global__ __launch_bounds__(kOpsThreads) void nw_ops_compact(const int32_t* nops, const uint32_t* slots, int slot,
                                                              const uint32_t* spill, int64_t n, const int64_t* blk,
                                                              int64_t* ctl, int64_t* ops_off, uint32_t* staging,
                                                              int64_t staging_cap, int64_t* hctl) {
    const long long r0 = (long long)blockIdx.x * kOpsBlockReads + threadIdx.x * kOpsPerThread;
    int cnt[kOpsPerThread];
    long long s = 0;
#pragma unroll
    for (int k = 0; k < kOpsPerThread; ++k) {
        cnt[k] = r0 + k < n ? nops[r0 + k] : 0;
        s += cnt[k];
    }
    long long total;
    long long off = blk[blockIdx.x] + block_excl_scan(s, &total);
    const long long base = ctl[1];
    bool over = false;
#pragma unroll
    for (int k = 0; k < kOpsPerThread; ++k) {
        const long long r = r0 + k;
        if (r >= n) break;
        ops_off[r] = base + off;
        const int c = cnt[k];
        const uint32_t* src = slots + r * slot;
        if (c > slot) src = spill + src[0];
        if (off + c > staging_cap) {
            over = true;
        } else {
            for (int q = 0; q < c; ++q) staging[off + q] = src[q];
        }
        off += c;
    }
    if (over) {
        atomicOr((unsigned long long*)(ctl + 3), 1ull);
        if (hctl) hctl[3] |= 1;   // every writer sets the same bit over the value the scan left
    }
}

}  // namespace

hipError_t launch_ops_compact(const int32_t* nops, const uint32_t* slots, int slot, const uint32_t* spill, int64_t n,
                              int64_t* blk, int64_t* ctl, int64_t* ops_off, uint32_t* staging, int64_t staging_cap,
                              int32_t* opsctl, const OpsCounts& cnt, hipStream_t s, int64_t* hctl) {
    const int nblk = (int)((n + kOpsBlockReads - 1) / kOpsBlockReads);
    if (nblk <= 0) {
        hipLaunchKernelGGL(nw_ops_scan, dim3(1), dim3(1024), 0, s, blk, 0, ctl, opsctl, cnt, hctl);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(nw_ops_blocksum, dim3(nblk), dim3(kOpsThreads), 0, s, nops, n, blk);
    hipLaunchKernelGGL(nw_ops_scan, dim3(1), dim3(1024), 0, s, blk, nblk, ctl, opsctl, cnt, hctl);
    hipLaunchKernelGGL(nw_ops_compact, dim3(nblk), dim3(kOpsThreads), 0, s, nops, slots, slot, spill, n, blk, ctl,
                       ops_off, staging, staging_cap, hctl);
    return hipGetLastError();
}

}  // namespace nw
