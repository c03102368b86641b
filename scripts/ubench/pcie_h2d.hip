// pcie_h2d.hip -- host -> device bandwidth of the call's upload (64.5 MB of 2-bit reads +
// lengths per 1M C2 reads) by transfer form: one copy engine stream (one copy / the call's 7
// chunk copies), two streams in parallel (chunks alternated), kernels reading the pinned
// host buffer themselves (zero-copy), and a copy stream plus reading kernels together.
// Run by scripts/ubench/run.sh; one line per form: ms, GB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void pull16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static float time_it(hipStream_t s0, const std::vector<hipStream_t>& extra, void (*body)(void*), void* ctx) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<hipEvent_t> done(extra.size());
    for (auto& e : done) (void)hipEventCreate(&e);
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a, s0);
        for (auto s : extra) (void)hipStreamWaitEvent(s, a, 0);
        body(ctx);
        for (size_t k = 0; k < extra.size(); ++k) {
            (void)hipEventRecord(done[k], extra[k]);
            (void)hipStreamWaitEvent(s0, done[k], 0);
        }
        (void)hipEventRecord(b, s0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

struct Ctx {
    char* h;
    char* d;
    size_t bytes;
    hipStream_t s[3];
    int grid;
    int parts;
    double kernel_frac;
};

int main() {
    Ctx c{};
    c.bytes = 64500000ull & ~(size_t)15;
    if (hipHostMalloc((void**)&c.h, c.bytes, hipHostMallocDefault) != hipSuccess || hipMalloc(&c.d, c.bytes) != hipSuccess)
        return 1;
    for (size_t i = 0; i < c.bytes; ++i) c.h[i] = (char)(i * 131);
    for (auto& s : c.s) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    auto report = [&](const char* what, float ms, size_t bytes) {
        std::printf("%-58s %.3f ms  %.1f GB/s\n", what, ms, bytes / (ms * 1e-3) / 1e9);
    };
    // one stream: one copy, and the call's chunking (1/8, 1/4, 1, 1, 1, 1/4, 1/8 of ~4.6 chunks)
    for (int parts : {1, 7, 28}) {
        c.parts = parts;
        float ms = time_it(c.s[0], {}, [](void* p) {
            Ctx& x = *(Ctx*)p;
            const size_t per = (x.bytes / x.parts) & ~(size_t)15;
            for (int k = 0; k < x.parts; ++k) {
                const size_t lo = k * per, n = k == x.parts - 1 ? x.bytes - lo : per;
                (void)hipMemcpyAsync(x.d + lo, x.h + lo, n, hipMemcpyHostToDevice, x.s[0]);
            }
        }, &c);
        char name[64];
        std::snprintf(name, sizeof name, "hipMemcpyAsync, 1 stream, %d copies", parts);
        report(name, ms, c.bytes);
    }
    // two streams, chunks alternated
    for (int parts : {2, 8}) {
        c.parts = parts;
        float ms = time_it(c.s[0], {c.s[1]}, [](void* p) {
            Ctx& x = *(Ctx*)p;
            const size_t per = (x.bytes / x.parts) & ~(size_t)15;
            for (int k = 0; k < x.parts; ++k) {
                const size_t lo = k * per, n = k == x.parts - 1 ? x.bytes - lo : per;
                (void)hipMemcpyAsync(x.d + lo, x.h + lo, n, hipMemcpyHostToDevice, x.s[k & 1]);
            }
        }, &c);
        char name[64];
        std::snprintf(name, sizeof name, "hipMemcpyAsync, 2 streams, %d copies", parts);
        report(name, ms, c.bytes);
    }
    // zero-copy: kernels read the pinned host buffer
    for (int grid : {256, 1024, 2048, 4096}) {
        c.grid = grid;
        float ms = time_it(c.s[0], {}, [](void* p) {
            Ctx& x = *(Ctx*)p;
            hipLaunchKernelGGL(pull16, dim3(x.grid), dim3(256), 0, x.s[0], (const uint4*)x.h, (uint4*)x.d, x.bytes / 16);
        }, &c);
        char name[64];
        std::snprintf(name, sizeof name, "kernel reads pinned host memory, grid %d", grid);
        report(name, ms, c.bytes);
    }
    // a copy stream and reading kernels on another stream, splitting the bytes
    for (double f : {0.25, 0.4, 0.5}) {
        c.kernel_frac = f;
        c.grid = 1024;
        float ms = time_it(c.s[0], {c.s[1]}, [](void* p) {
            Ctx& x = *(Ctx*)p;
            const size_t kb = (size_t)(x.bytes * x.kernel_frac) & ~(size_t)15;
            (void)hipMemcpyAsync(x.d + kb, x.h + kb, x.bytes - kb, hipMemcpyHostToDevice, x.s[0]);
            hipLaunchKernelGGL(pull16, dim3(x.grid), dim3(256), 0, x.s[1], (const uint4*)x.h, (uint4*)x.d, kb / 16);
        }, &c);
        char name[64];
        std::snprintf(name, sizeof name, "copy stream + reading kernel (%.0f %% by kernel)", f * 100);
        report(name, ms, c.bytes);
    }
    // D2H for reference: 45 MB of records + runs
    {
        const size_t db = 45000000ull;
        c.parts = 1;
        float ms = time_it(c.s[0], {}, [](void* p) {
            Ctx& x = *(Ctx*)p;
            (void)hipMemcpyAsync(x.h, x.d, 45000000ull, hipMemcpyDeviceToHost, x.s[0]);
        }, &c);
        report("hipMemcpyAsync D2H 45 MB, 1 stream", ms, db);
        ms = time_it(c.s[0], {c.s[1]}, [](void* p) {
            Ctx& x = *(Ctx*)p;
            (void)hipMemcpyAsync(x.d + 32000000ull, x.h + 32000000ull, 32000000ull, hipMemcpyHostToDevice, x.s[1]);
            (void)hipMemcpyAsync(x.h, x.d, 32000000ull, hipMemcpyDeviceToHost, x.s[0]);
        }, &c);
        report("H2D 32 MB + D2H 32 MB concurrently (2 streams)", ms, 64000000ull);
    }
    return 0;
}
