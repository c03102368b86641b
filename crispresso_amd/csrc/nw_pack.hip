// nw_pack.hip -- 2-bit packed read input (nw_align_ops_packed).
//
// The call-level path is PCIe-bound when reads cross as one byte per base: 250 MB
// per 1M C2 reads at ~54 GB/s is 4.8 ms, over three times the kernels' 1.4 ms.  The
// kernels need no more than the base codes: every comparison they make is
// case-insensitive (the rows are rebuilt on the host from the caller's text,
// nw_expand_ops).  So the batch crosses as 2 bits per base (A C T G = 0 1 2 3:
// (byte >> 1) & 3 of A C G T a c g t) plus an exception list for every other byte
// (N, IUPAC codes, '-', ...: position and the byte itself), and is unpacked here
// into the byte layout the aligner kernels read.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_device.h"

namespace nw {

namespace {

// Bases [b0, b1) (batch positions) from the packed stream (device copy starting at
// stream byte pbyte0, a multiple of 4) into dst[pos - bias] (bias a multiple of 16).
// Thread: 16 bases = one packed dword -> one 16-byte store (byte stores at the edges).
// Blocks from `nub` on rebuild the chunk's offsets instead (one block per group of
// kLenGroup reads: the group's base offset + an exclusive scan of its uint16 lengths).
__global__ __launch_bounds__(256) void nw_unpack_kernel(const uint32_t* packed, int64_t pbyte0, int64_t b0, int64_t b1,
                                                        uint8_t* dst, int64_t bias, unsigned nub, const LenSeg ls) {
    if (blockIdx.x >= nub) {
        __shared__ int64_t wsum[4];
        const int64_t g = ls.g0 + (blockIdx.x - nub);
        const int64_t r0 = g * kLenGroup + 4 * threadIdx.x;   // this thread's 4 reads
        const uint16_t* len = ls.len + r0;
        // lengths of the reads below r_hi only (the chunk's own and the group's earlier ones)
        uint32_t l[4];
        if (r0 + 4 <= ls.r_hi) {
            const uint2 w = *(const uint2*)len;
            l[0] = w.x & 0xffffu; l[1] = w.x >> 16; l[2] = w.y & 0xffffu; l[3] = w.y >> 16;
        } else {
#pragma unroll
            for (int m = 0; m < 4; ++m) l[m] = r0 + m < ls.r_hi ? len[m] : 0u;
        }
        const int64_t t4 = (int64_t)l[0] + l[1] + l[2] + l[3];
        // wave inclusive scan of the 4-read sums, then the waves' totals
        int64_t inc = t4;
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_up(inc, d, 64);
            if (lane >= d) inc += o;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        int64_t base = ls.gbase[g] + inc - t4;
        for (int w = 0; w < wave; ++w) base += wsum[w];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int64_t r = r0 + m;
            if (r >= ls.r_lo && r <= ls.r_hi) ls.d_off[r] = base;
            base += l[m];
        }
        return;
    }
    const int64_t first = b0 & ~(int64_t)15;
    const int64_t i0 = first + 16 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (i0 >= b1) return;
    const uint32_t w = packed[(i0 / 4 - pbyte0) / 4];
    uint32_t out[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t code = (w >> (2 * (4 * q + k))) & 3u;
            // A C T G
            const uint32_t ch = 0x47544341u >> (8 * code) & 0xffu;
            v |= ch << (8 * k);
        }
        out[q] = v;
    }
    uint8_t* d = dst + (i0 - bias);
    if (i0 >= b0 && i0 + 16 <= b1) {
        *(uint4*)d = make_uint4(out[0], out[1], out[2], out[3]);
    } else {
        for (int k = 0; k < 16; ++k)
            if (i0 + k >= b0 && i0 + k < b1) d[k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
    }
}

// The exception bytes [e0, e1) of the list (positions ascending) over the unpacked codes.
__global__ __launch_bounds__(256) void nw_exceptions_kernel(const int64_t* pos, const uint8_t* byte, int64_t e0,
                                                            int64_t e1, uint8_t* dst, int64_t bias) {
    const int64_t e = e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < e1) dst[pos[e] - bias] = byte[e];
}

}  // namespace

hipError_t launch_unpack(const uint32_t* packed, int64_t pbyte0, int64_t b0, int64_t b1, const int64_t* exc_pos,
                         const uint8_t* exc_byte, int64_t e0, int64_t e1, uint8_t* dst, int64_t bias, hipStream_t s,
                         const LenSeg* lens) {
    const int64_t words = b1 > b0 ? (b1 - (b0 & ~(int64_t)15) + 15) / 16 : 0;
    const unsigned nub = (unsigned)((words + 255) / 256);
    const unsigned nlb = lens ? (unsigned)lens->ngroups : 0u;
    if (nub + nlb > 0)
        hipLaunchKernelGGL(nw_unpack_kernel, dim3(nub + nlb), dim3(256), 0, s, packed, pbyte0, b0, b1, dst, bias, nub,
                           lens ? *lens : LenSeg{});
    if (e1 > e0)
        hipLaunchKernelGGL(nw_exceptions_kernel, dim3((unsigned)((e1 - e0 + 255) / 256)), dim3(256), 0, s, exc_pos,
                           exc_byte, e0, e1, dst, bias);
    return hipGetLastError();
}

}  // namespace nw
