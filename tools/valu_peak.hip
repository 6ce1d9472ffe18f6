// Measured int32 VALU roofline on gfx950 (the aligner's bound; SURVEY.md §8(d) asks for a
// microbenchmark).  Each thread runs 8 independent chains of the instruction mix the DP cell
// uses (add, max, compare + cndmask); we time it at 1..8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o /tmp/valu_peak && /tmp/valu_peak
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(256) k_valu(int* out, int iters, int seed) {
    int a0 = threadIdx.x + seed, a1 = a0 * 3, a2 = a0 ^ 5, a3 = a0 + 7;
    int a4 = a0 * 5, a5 = a0 ^ 9, a6 = a0 + 11, a7 = a0 * 13;
    const int c = seed | 1;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            if (MODE == 0) {  // plain adds
                a0 += c; a1 += a0; a2 += c; a3 += a2; a4 += c; a5 += a4; a6 += c; a7 += a6;
            } else if (MODE == 1) {  // max + add
                a0 = max(a0 + c, a1); a1 = max(a1 - c, a2); a2 = max(a2 + c, a3); a3 = max(a3 - c, a4);
                a4 = max(a4 + c, a5); a5 = max(a5 - c, a6); a6 = max(a6 + c, a7); a7 = max(a7 - c, a0);
            } else {  // compare + select (the counter-selection pattern)
                a0 = (a1 == a2) ? a3 : a0 + 1; a1 = (a2 == a3) ? a4 : a1 + 1;
                a2 = (a3 == a4) ? a5 : a2 + 1; a3 = (a4 == a5) ? a6 : a3 + 1;
                a4 = (a5 == a6) ? a7 : a4 + 1; a5 = (a6 == a7) ? a0 : a5 + 1;
                a6 = (a7 == a0) ? a1 : a6 + 1; a7 = (a0 == a1) ? a2 : a7 + 1;
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int MODE>
double run(int waves_per_simd, int ops_per_iter) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = 1 per SIMD
    const int iters = 4096;
    int* out;
    hipMalloc(&out, (size_t)blocks * 256 * sizeof(int));
    hipLaunchKernelGGL(k_valu<MODE>, dim3(blocks), dim3(256), 0, 0, out, 16, 1);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_valu<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, 1);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipFree(out);
    const double lane_ops = (double)blocks * 256 * iters * 16 * ops_per_iter;
    return lane_ops / (ms * 1e-3) / 1e12;
}

int main() {
    const char* names[3] = {"add", "max+add", "cmp+cndmask+add"};
    for (int w : {1, 2, 3, 4, 8}) {
        printf("waves/SIMD %d:  %-16s %7.2f Tlane-op/s   %-16s %7.2f   %-16s %7.2f\n", w, names[0],
               run<0>(w, 8), names[1], run<1>(w, 16), names[2], run<2>(w, 24));
    }
    return 0;
}
