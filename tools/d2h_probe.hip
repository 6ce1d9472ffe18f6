// Device -> host text bandwidth probe (the aligned_pairs.txt path is bound by moving ~55 GB of text
// to the host at N = 5 000): (a) one hipMemcpyAsync into pinned memory, (b) the same bytes split over
// 4 streams, (c) a kernel storing straight into pinned host memory (device-visible through its
// pointer), 16 bytes per lane.
//   hipcc --offload-arch=gfx950 -O3 -o tools/d2h_probe tools/d2h_probe.hip && tools/d2h_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double ms_since(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const size_t bytes = (size_t)4 << 30;
    void *d = nullptr, *h = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess || hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(d, 7, bytes);
    hipStream_t s[4];
    for (auto& x : s) hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0, s[0]);
        hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s[0]);
        hipEventRecord(e1, s[0]);
        hipEventSynchronize(e1);
        printf("one memcpy      : %.1f GB/s\n", bytes / ms_since(e0, e1) / 1e6);
    }
    for (int rep = 0; rep < 2; ++rep) {
        hipDeviceSynchronize();
        hipEventRecord(e0, 0);
        for (int k = 0; k < 4; ++k) hipStreamWaitEvent(s[k], e0, 0);
        for (int k = 0; k < 4; ++k)
            hipMemcpyAsync((char*)h + k * (bytes / 4), (char*)d + k * (bytes / 4), bytes / 4, hipMemcpyDeviceToHost, s[k]);
        hipDeviceSynchronize();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        printf("4 streams       : %.1f GB/s\n", bytes / ms_since(e0, e1) / 1e6);
    }
    for (int grid : {8, 16, 32, 64, 128, 256, 1024, 4096}) {
        hipEventRecord(e0, s[0]);
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, s[0], (const uint4*)d, (uint4*)h, bytes / 16);
        hipEventRecord(e1, s[0]);
        hipEventSynchronize(e1);
        printf("kernel stores %4d blocks: %.1f GB/s\n", grid, bytes / ms_since(e0, e1) / 1e6);
    }
    std::vector<unsigned char> chk(16);
    std::memcpy(chk.data(), h, 16);
    printf("check byte %d\n", chk[0]);
    hipHostFree(h);
    hipFree(d);
    return 0;
}
