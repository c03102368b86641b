// GPU kernel stores into pinned host memory vs hipMemcpyAsync D2H: bandwidth of each for
// the call's download sizes (records + offsets + runs, ~45 MB per 1M reads).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main() {
    const size_t bytes = 45ull << 20, n = bytes / 16;
    uint4 *d = nullptr, *h = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess || hipHostMalloc((void**)&h, bytes, hipHostMallocDefault) != hipSuccess) return 1;
    (void)hipMemset(d, 1, bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int grid : {256, 1024, 4096}) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a, 0);
            hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, 0, d, h, n);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("kernel stores grid %d: %.3f ms, %.1f GB/s\n", grid, ms, bytes / ms / 1e6);
        }
    }
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a, 0);
        (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep == 2) printf("hipMemcpyAsync D2H: %.3f ms, %.1f GB/s\n", ms, bytes / ms / 1e6);
    }
    // scattered 4-byte stores (one per thread, stride 1): the per-read run copy pattern
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(copy16, dim3(1024), dim3(64), 0, 0, d, h, n / 4);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep == 2) printf("kernel stores, 64-thread blocks, quarter size: %.3f ms, %.1f GB/s\n", ms, bytes / 4 / ms / 1e6);
    }
    // kernel loads from pinned host memory (H2D by the GPU) vs hipMemcpyAsync H2D
    for (int grid : {1024, 4096}) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a, 0);
            hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, 0, h, d, n);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("kernel loads from host grid %d: %.3f ms, %.1f GB/s\n", grid, ms, bytes / ms / 1e6);
        }
    }
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a, 0);
        (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, 0);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep == 2) printf("hipMemcpyAsync H2D: %.3f ms, %.1f GB/s\n", ms, bytes / ms / 1e6);
    }
    // a D2H copy on a second stream next to an H2D one: full duplex?
    hipStream_t s1, s2;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    uint4* h2 = nullptr;
    uint4* d2 = nullptr;
    (void)hipHostMalloc((void**)&h2, bytes, hipHostMallocDefault);
    (void)hipMalloc(&d2, bytes);
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a, s1);
        (void)hipStreamWaitEvent(s2, a, 0);
        (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1);
        hipLaunchKernelGGL(copy16, dim3(1024), dim3(256), 0, s2, d2, h2, n);
        (void)hipEventRecord(b, s2);
        (void)hipStreamSynchronize(s1);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep == 2) printf("H2D copy + D2H kernel stores together: kernel side done after %.3f ms\n", ms);
    }
    printf("check %u\n", h[n - 1].x);
    return 0;
}
