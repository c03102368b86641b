// issue_rate.hip -- microbenchmark: throughput of the VALU instruction classes the
// band fill uses, 8 independent chains per wave (no dependency stalls), 8 waves per
// SIMD.  Reported: wave-instructions per SIMD per cycle at 2.4 GHz (guide: 0.5 for
// a wave64 VALU instruction).  Run by scripts/ubench/run.sh.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHAINS 8

template <int OP>
__global__ __launch_bounds__(512) void rate(unsigned* out, int iters, unsigned seed, unsigned long long* clk) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    unsigned v[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) v[k] = seed * (k + 1) + threadIdx.x;
    const unsigned m = seed | 0x01010101u;
    for (int t = 0; t < iters; ++t) {
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) {
            if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[k]) : "v"(m));
            if constexpr (OP == 1) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v[k]) : "v"(m));
            if constexpr (OP == 2) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(v[k]) : "v"(m));
            if constexpr (OP == 3) asm volatile("v_mov_b32_dpp %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v[k]));
            if constexpr (OP == 4) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(v[k]) : "v"(m));
            if constexpr (OP == 5) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(v[k]) : "v"(m));
            if constexpr (OP == 6) asm volatile("v_pk_sub_i16 %0, %0, %1" : "+v"(v[k]) : "v"(m));
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) r ^= v[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0 && threadIdx.x == 0) *clk = c1 - c0;   // shader clocks of one wave's loop
}

static unsigned long long* g_clk;
static unsigned long long clk_of_last() {
    unsigned long long c = 0;
    (void)hipMemcpy(&c, g_clk, sizeof c, hipMemcpyDeviceToHost);
    return c;
}

template <int OP>
static float run(unsigned* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(rate<OP>, dim3(blocks), dim3(512), 0, 0, out, iters, 3u, g_clk);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    return ms;
}

int main() {
    int cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
    const int iters = 1 << 18, blocks = cus * 4;   // 8 waves per SIMD; >= 10 ms per launch (the DVFS clock settles)
    unsigned* out;
    (void)hipMalloc(&out, sizeof(unsigned) * 512 * blocks);
    (void)hipMalloc(&g_clk, sizeof(unsigned long long));
    const char* names[] = {"v_add_u32", "v_pk_add_u16", "v_pk_max_u16", "v_mov_b32_dpp row_shr", "v_perm_b32",
                           "v_and_or_b32", "v_pk_sub_i16"};
    float ms[7];
    unsigned long long clk[7];
    ms[0] = run<0>(out, blocks, iters); clk[0] = clk_of_last();
    ms[1] = run<1>(out, blocks, iters); clk[1] = clk_of_last();
    ms[2] = run<2>(out, blocks, iters); clk[2] = clk_of_last();
    ms[3] = run<3>(out, blocks, iters); clk[3] = clk_of_last();
    ms[4] = run<4>(out, blocks, iters); clk[4] = clk_of_last();
    ms[5] = run<5>(out, blocks, iters); clk[5] = clk_of_last();
    ms[6] = run<6>(out, blocks, iters); clk[6] = clk_of_last();
    std::printf("instruction  ms  per_simd_per_cycle(2.4GHz)  shader_clocks_of_one_wave  per_simd_per_shader_clock"
                "  implied_clock_GHz\n");
    for (int k = 0; k < 7; ++k) {
        const double instr = (double)blocks * 8 * iters * CHAINS;
        const double per_wave = (double)iters * CHAINS;
        // 8 waves share the SIMD for the whole loop: per-SIMD rate = 8 * per-wave instructions / wave clocks
        std::printf("%-24s %.3f %.3f %llu %.3f %.2f\n", names[k], ms[k], instr / (cus * 4.0) / (ms[k] * 1e-3 * 2.4e9),
                    clk[k], 8.0 * per_wave / (double)clk[k], (double)clk[k] / (ms[k] * 1e-3) / 1e9);
    }
    return 0;
}
