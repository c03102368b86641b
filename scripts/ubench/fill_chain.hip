// fill_chain.hip -- microbenchmark: issue rate of nw_band_fill<16>'s per-step
// instruction chain on gfx950 (measure before claiming a floor).
//
// The loop body is the fill's step (nw_band.hip, step lambda) with the same
// dependencies -- DPP row_shr:2 / row_shl:2 of the previous step's values, packed
// u16 max / add / sub, v_perm + v_and_or for the traceback bits -- but scores come
// from registers (MODE 0: no LDS), from an LDS table with the fill's random
// per-lane addresses (MODE 1), or from a conflict-free LDS layout where every lane
// reads its own bank (MODE 2).  Reported: wave-instructions issued per SIMD per
// cycle, against the guide's 0.5 (one wave64 VALU instruction per 2 cycles).
//
// Build/run: hipcc --offload-arch=gfx950 -O3 fill_chain.hip -o fill_chain && ./fill_chain  (scripts/ubench/run.sh)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned max2(unsigned a, unsigned b) {
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ unsigned add2(unsigned a, unsigned b) {
    return __builtin_bit_cast(unsigned, __builtin_bit_cast(s16x2, a) + __builtin_bit_cast(s16x2, b));
}
__device__ __forceinline__ unsigned sub2(unsigned a, unsigned b) {
    return __builtin_bit_cast(unsigned, __builtin_bit_cast(s16x2, a) - __builtin_bit_cast(s16x2, b));
}
template <int S> __device__ __forceinline__ unsigned row_shr(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x110 + S, 0xf, 0xf, true);
}
template <int S> __device__ __forceinline__ unsigned row_shl(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x100 + S, 0xf, 0xf, true);
}
__device__ __forceinline__ unsigned and_or(unsigned a, unsigned m, unsigned c) {
    unsigned d;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(m), "v"(c));
    return d;
}

template <int MODE>
__global__ __launch_bounds__(512) void chain(unsigned* out, int steps, unsigned seed) {
    __shared__ unsigned tab[1024];
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) tab[k] = 0x00050005u * (k % 7) + k;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    unsigned mT0, mT1, mU0, mU1;
    asm volatile("s_mov_b32 %0, 0x01010101" : "=s"(mT0));
    asm volatile("s_mov_b32 %0, 0x02020202" : "=s"(mT1));
    asm volatile("s_mov_b32 %0, 0x10101010" : "=s"(mU0));
    asm volatile("s_mov_b32 %0, 0x20202020" : "=s"(mU1));
    unsigned Hp0 = seed ^ lane, Hp1 = Hp0 * 3, MoP = Hp0 + 7, XP = Hp1 + 9, YP = Hp0 ^ 0x55;
    unsigned acc = 0, sc0 = lane * 0x00010001u, sc1 = sc0 + 0x00030003u;
    unsigned addr = (lane * 37 + seed) & 1023;   // MODE 1: random per-lane addresses, as the fill's table reads
    const unsigned OE2 = 0x00130013u;
    for (int t = 0; t < steps; t += 2) {
        if constexpr (MODE == 1) {
            sc0 = tab[addr & 255];
            sc1 = tab[(addr >> 8) & 255];
            addr = addr * 1103515245u + 12345u;
        } else if constexpr (MODE == 2) {
            sc0 = tab[(lane & 31) + 32 * (t & 7)];
            sc1 = tab[(lane & 31) + 32 * ((t + 1) & 7)];
        }
        // step with parity 0
        {
            const unsigned Ml = row_shr<2>(MoP), Xl = row_shr<2>(XP);
            const unsigned X = max2(Ml, Xl), d2 = sub2(Xl, Ml);
            const unsigned Y = max2(MoP, YP), d1 = sub2(YP, MoP);
            const unsigned M = add2(Hp0, sc0);
            const unsigned mxy = max2(X, Y);
            const unsigned H = max2(M, mxy);
            const unsigned d3 = sub2(Y, X), d4 = sub2(M, mxy);
            Hp0 = H;
            MoP = sub2(M, OE2);
            XP = X;
            YP = Y;
            acc = and_or(__builtin_amdgcn_perm(d2, d1, 0x0B0A0908u), mT0, acc);
            acc = and_or(__builtin_amdgcn_perm(d4, d3, 0x0B0A0908u), mU0, acc);
        }
        // step with parity 1
        {
            const unsigned Mu = row_shl<2>(MoP), Yu = row_shl<2>(YP);
            const unsigned Y = max2(Mu, Yu), d1 = sub2(Yu, Mu);
            const unsigned X = max2(MoP, XP), d2 = sub2(XP, MoP);
            const unsigned M = add2(Hp1, sc1);
            const unsigned mxy = max2(X, Y);
            const unsigned H = max2(M, mxy);
            const unsigned d3 = sub2(Y, X), d4 = sub2(M, mxy);
            Hp1 = H;
            MoP = sub2(M, OE2);
            XP = X;
            YP = Y;
            acc = and_or(__builtin_amdgcn_perm(d2, d1, 0x0B0A0908u), mT1, acc);
            acc = and_or(__builtin_amdgcn_perm(d4, d3, 0x0B0A0908u), mU1, acc);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ Hp0 ^ Hp1 ^ MoP ^ XP ^ YP;
}

int main() {
    int cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
    const int steps = 1 << 14;
    unsigned* out;
    hipMalloc(&out, sizeof(unsigned) * 512 * cus * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // VALU wave-instructions per step in the loop body (ISA count of the step: 2 DPP, 9 max/add/sub,
    // 2 perm, 2 and_or) -- measured from the kernel's ISA by the caller; here per two steps
    const double valu_per_2steps = 32.0;   // MODE 0 ISA: 8 pk_sub_i16, 8 pk_max, 4 dpp, 4 perm, 4 and_or, 2 pk_sub_u16, 2 pk_add (MODE 1/2 add the LDS reads)
    std::printf("mode waves_per_simd ms  wave_instr_per_simd_per_cycle(at 2.4 GHz)\n");
    for (int mode = 0; mode < 3; ++mode) {
        for (int wps : {1, 2, 4, 6, 8}) {
            const int blocks = cus * wps / 2;   // 512-thread blocks = 8 waves = 2 per SIMD
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(chain<0>, dim3(blocks), dim3(512), 0, 0, out, steps, 7u);
                if (mode == 1) hipLaunchKernelGGL(chain<1>, dim3(blocks), dim3(512), 0, 0, out, steps, 7u);
                if (mode == 2) hipLaunchKernelGGL(chain<2>, dim3(blocks), dim3(512), 0, 0, out, steps, 7u);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep == 1) {
                    const double instr = (double)blocks * 8 * (steps / 2) * valu_per_2steps;   // wave-instructions
                    const double per_simd_cycle = instr / (cus * 4.0) / (ms * 1e-3 * 2.4e9);
                    std::printf("%d %d %.3f %.3f\n", mode, wps, ms, per_simd_cycle);
                }
            }
        }
    }
    return 0;
}
