// Phase timing of the one-wave-per-stream compressed-length kernel (zlen_wave.hpp, built with
// -DZLW_PROF): window load, key sort, parse, final flush, in s_memtime ticks summed over waves.
// Synthetic 1 000 bp DNA pairs (x + y concatenations).  Build: see tools/profile_zlw.sh.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../taxi2_amd/csrc/ncd_kernels.hpp"

int main() {
    const int L = 1000, nseq = 2000, nst = 200000;
    std::vector<uint8_t> seqs((size_t)nseq * L);
    uint32_t r = 12345;
    std::vector<uint8_t> anc(L);
    for (auto& c : anc) { r = r * 1664525u + 1013904223u; c = "ACGT"[(r >> 28) & 3]; }
    for (int s = 0; s < nseq; ++s)
        for (int i = 0; i < L; ++i) {
            r = r * 1664525u + 1013904223u;
            seqs[(size_t)s * L + i] = ((r >> 24) % 10 == 0) ? "ACGT"[(r >> 20) & 3] : anc[i];
        }
    uint8_t* d_seq;
    hipMalloc(&d_seq, seqs.size());
    hipMemcpy(d_seq, seqs.data(), seqs.size(), hipMemcpyHostToDevice);
    std::vector<taxi2::ZStream> st(nst);
    for (int k = 0; k < nst; ++k) {
        r = r * 1664525u + 1013904223u;
        const int a = r % nseq;
        r = r * 1664525u + 1013904223u;
        const int b = r % nseq;
        st[k] = taxi2::ZStream{d_seq + (size_t)a * L, d_seq + (size_t)b * L, L, L};
    }
    taxi2::ZStream* d_st;
    int32_t* d_out;
    hipMalloc(&d_st, st.size() * sizeof(taxi2::ZStream));
    hipMalloc(&d_out, (size_t)nst * 4);
    hipMemcpy(d_st, st.data(), st.size() * sizeof(taxi2::ZStream), hipMemcpyHostToDevice);
    const int nmax = 2 * L;
    const size_t lds = taxi2::zlw::lds_bytes(nmax);
    int per_cu = 0, dev = 0, cus = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)taxi2::k_zlen_wave, 64, lds);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = cus * per_cu;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(taxi2::k_zlen_wave, dim3(grid), dim3(64), lds, 0, d_st, (int64_t)nst, nmax, d_out);
    hipDeviceSynchronize();
    unsigned long long z[8] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(taxi2::zlw::zlw_prof), z, sizeof z);
    hipEventRecord(e0);
    hipLaunchKernelGGL(taxi2::k_zlen_wave, dim3(grid), dim3(64), lds, 0, d_st, (int64_t)nst, nmax, d_out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpyFromSymbol(z, HIP_SYMBOL(taxi2::zlw::zlw_prof), sizeof z);
    const double tot = (double)(z[0] + z[1] + z[2] + z[3]);
    printf("streams %d grid %d (per CU %d, LDS %zu B): %.2f ms, %.3g streams/s\n", nst, grid, per_cu, lds, ms,
           nst / (ms * 1e-3));
    const char* names[4] = {"window", "sort", "parse", "flush"};
    for (int k = 0; k < 4; ++k) printf("  %-7s %5.1f %%\n", names[k], 100.0 * z[k] / tot);
    return 0;
}
