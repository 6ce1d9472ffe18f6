// VALU issue ceiling on gfx950 for the instructions the packed aligner (k_alignt2) issues.
//
// Each thread runs NCH independent register chains of ONE instruction (inline asm, so the
// compiler can neither fold nor re-schedule the chain), at 1..8 waves per SIMD.  Reported per
// instruction and occupancy:
//   cyc/instr/SIMD = (s_memtime cycles of the slowest wave) / (wave-instructions issued per SIMD)
//   lane-op/s      = wave-instructions x 64 / wall time (HIP events)
//   clock          = s_memtime / s_memrealtime x 100 MHz (the clock the chip held)
// MI355X_MICROARCH.md (Wave scheduling, constants table) states a wave64 VALU instruction issues
// over 2 cycles on a SIMD-32 (4 cycles for one wave alone); this measures it for the packed 16-bit
// integer ops, v_perm / v_bfi, 32-bit integer ops and v_add_f32 as the calibration.
//
//   hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o tools/valu_peak && tools/valu_peak
//   (ISA: add -save-temps; the committed listing is profiles/r2/valu_peak_isa.txt)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int NCH = 8;     // independent chains per thread
constexpr int UNROLL = 32;  // asm blocks per loop iteration (256 measured instructions per loop branch)

#define CH8(INS)                                                                                                 \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS      \
                     " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"               \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
                 : "v"(c))
#define CH8_3(INS)                                                                                               \
    asm volatile(INS " %0, %0, %8, %9\n\t" INS " %1, %1, %8, %9\n\t" INS " %2, %2, %8, %9\n\t" INS                \
                     " %3, %3, %8, %9\n\t" INS " %4, %4, %8, %9\n\t" INS " %5, %5, %8, %9\n\t" INS                \
                     " %6, %6, %8, %9\n\t" INS " %7, %7, %8, %9"                                                  \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
                 : "v"(c), "v"(d))
// one-source forms (v_mov_b32) and 64-bit-register forms (v_pk_*_f32 on register pairs)
#define CH8_1(INS)                                                                                               \
    asm volatile(INS " %0, %8\n\t" INS " %1, %8\n\t" INS " %2, %8\n\t" INS " %3, %8\n\t" INS " %4, %8\n\t" INS   \
                     " %5, %8\n\t" INS " %6, %8\n\t" INS " %7, %8"                                                   \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
                 : "v"(c))
#define CH8_V(INS)                                                                                               \
    asm volatile(INS " %0, %0, %8, vcc\n\t" INS " %1, %1, %8, vcc\n\t" INS " %2, %2, %8, vcc\n\t" INS             \
                     " %3, %3, %8, vcc\n\t" INS " %4, %4, %8, vcc\n\t" INS " %5, %5, %8, vcc\n\t" INS             \
                     " %6, %6, %8, vcc\n\t" INS " %7, %7, %8, vcc"                                                \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
                 : "v"(c))
#define CH4_64(INS)                                                                                              \
    asm volatile(INS " %0, %0, %4\n\t" INS " %1, %1, %4\n\t" INS " %2, %2, %4\n\t" INS " %3, %3, %4"                \
                 : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3])                                                \
                 : "v"(cq))

// SDWA form (the packed aligner's substitution add: one 16-bit word added into the high half)
#define CH8_S(INS)                                                                                               \
    asm volatile(INS " %0, %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
                 INS " %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
                 INS " %2, %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
                 INS " %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
                 INS " %4, %4, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t" \
                 INS " %5, %5, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t" \
                 INS " %6, %6, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t" \
                 INS " %7, %7, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1"      \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
                 : "v"(c))

// three-source bit operation with its truth table (the pre-aligned tile kernel's v_bitop3 0x48)
#define CH8_B(INS)                                                                                               \
    asm volatile(INS " %0, %0, %8, %9 bitop3:0x48\n\t" INS " %1, %1, %8, %9 bitop3:0x48\n\t" INS             \
                     " %2, %2, %8, %9 bitop3:0x48\n\t" INS " %3, %3, %8, %9 bitop3:0x48\n\t" INS              \
                     " %4, %4, %8, %9 bitop3:0x48\n\t" INS " %5, %5, %8, %9 bitop3:0x48\n\t" INS              \
                     " %6, %6, %8, %9 bitop3:0x48\n\t" INS " %7, %7, %8, %9 bitop3:0x48"                        \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
                 : "v"(c), "v"(d))

// instruction table: name, form (2 = dst,src0,src1; 3 = three sources; 1 = mov; v = with vcc; 6 = 64-bit pair;
// b = bitop3 with a truth table)
#define VALU_LIST(X)                                                                                             \
    X(0, "v_add_f32", 2) X(1, "v_add_u32", 2) X(2, "v_sub_u32", 2) X(3, "v_max_i32", 2) X(4, "v_min_u32", 2)     \
    X(5, "v_max_f32", 2) X(6, "v_min_f32", 2) X(7, "v_and_b32", 2) X(8, "v_or_b32", 2) X(9, "v_xor_b32", 2)      \
    X(10, "v_lshlrev_b32", 2) X(11, "v_mul_u32_u24", 2) X(12, "v_max_i16", 2) X(13, "v_pk_add_u16", 2)         \
    X(14, "v_pk_max_i16", 2) X(15, "v_pk_sub_i16", 2) X(16, "v_pk_add_f16", 2) X(17, "v_pk_max_f16", 2)         \
    X(18, "v_sub_f32", 2) X(19, "v_cndmask_b32", v) X(20, "v_mov_b32", 1) X(21, "v_fma_f32", 3)                 \
    X(22, "v_max3_f32", 3) X(23, "v_med3_f32", 3) X(24, "v_max3_i32", 3) X(25, "v_med3_i32", 3)                 \
    X(26, "v_add3_u32", 3) X(27, "v_perm_b32", 3) X(28, "v_bfi_b32", 3) X(29, "v_alignbit_b32", 3)              \
    X(30, "v_bfe_u32", 3) X(31, "v_lshl_add_u32", 3) X(32, "v_and_or_b32", 3) X(33, "v_pk_mad_u16", 3)          \
    X(34, "v_pk_fma_f16", 3) X(35, "v_mad_u32_u24", 3) X(36, "v_pk_add_f32", 6) X(37, "v_pk_mul_f32", 6)       \
    X(38, "v_max_u16", 2) X(39, "v_add_u16", 2) X(40, "v_max_f16", 2) X(41, "v_cvt_f32_i32", 1)               \
    X(42, "v_add_u32_sdwa", s) X(43, "v_pk_maximum3_f16", 3) X(44, "v_pk_max_u16", 2)                        \
    X(45, "v_bcnt_u32_b32", 2) X(46, "v_bitop3_b32", b) X(47, "v_add_f64", 6) X(48, "v_mul_f64", 6)
#define FORM_2(INS) CH8(INS)
#define FORM_3(INS) CH8_3(INS)
#define FORM_1(INS) CH8_1(INS)
#define FORM_v(INS) CH8_V(INS)
#define FORM_6(INS) CH4_64(INS)
#define FORM_s(INS) CH8_S(INS)
#define FORM_b(INS) CH8_B(INS)

template <int MODE>
__global__ void __launch_bounds__(256) k_valu(unsigned* out, unsigned long long* cyc, int iters, unsigned seed) {
    unsigned a[NCH];
    unsigned long long q[4];
#pragma unroll
    for (int k = 0; k < NCH; ++k) a[k] = threadIdx.x * (k + 3) + seed;
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = ((unsigned long long)a[2 * k] << 32) | a[2 * k + 1];
    const unsigned c = seed | 1u, d = seed ^ 0x05040100u;
    const unsigned long long cq = ((unsigned long long)c << 32) | d;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
#define CASE(M, NAME, F) \
    if constexpr (MODE == M) FORM_##F(NAME);
            VALU_LIST(CASE)
#undef CASE
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = 0;
#pragma unroll
    for (int k = 0; k < NCH; ++k) s ^= a[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) s ^= (unsigned)(q[k] ^ (q[k] >> 32));
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        const int wv = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        cyc[2 * wv] = t1 - t0;
        cyc[2 * wv + 1] = r1 - r0;
    }
}

struct Res {
    double tlops, cyc_per_instr, ghz;
};

template <int MODE>
Res run(int waves_per_simd, bool is64) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
    const int waves = blocks * 4;
    const int iters = 2048;
    unsigned* out;
    unsigned long long* cyc;
    hipMalloc(&out, (size_t)blocks * 256 * sizeof(unsigned));
    hipMalloc(&cyc, (size_t)waves * 2 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k_valu<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, 64, 1u);  // warm
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_valu<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1u);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h((size_t)waves * 2);
    hipMemcpy(h.data(), cyc, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    unsigned long long cmax = 0, rmax = 0;
    for (int w = 0; w < waves; ++w) {
        if (h[2 * w] > cmax) cmax = h[2 * w];
        if (h[2 * w + 1] > rmax) rmax = h[2 * w + 1];
    }
    hipFree(out);
    hipFree(cyc);
    const double instr_per_wave = (double)iters * UNROLL * (is64 ? 4 : NCH);
    Res r;
    r.tlops = (double)waves * 64 * instr_per_wave / (ms * 1e-3) / 1e12;
    r.cyc_per_instr = (double)cmax / (instr_per_wave * waves_per_simd);
    r.ghz = rmax ? (double)cmax / (double)rmax * 0.1 : 0.0;
    return r;
}

template <int MODE>
void row(const char* name, bool is64) {
    printf("%-16s", name);
    for (int w : {1, 2, 4, 8}) {
        const Res r = run<MODE>(w, is64);
        printf("  w%d: %5.2f cyc %6.1f T %4.2f GHz", w, r.cyc_per_instr, r.tlops, r.ghz);
    }
    printf("\n");
    fflush(stdout);
}

int main() {
    printf("cyc = SIMD cycles per wave64 instruction (all waves of the SIMD together); T = lane-op/s x 1e12;\n"
           "%d independent chains per thread (4 register pairs for the 64-bit forms), 256-thread blocks (one wave "
           "per SIMD each), CUs x w blocks\n", NCH);
#define ROW(M, NAME, F) row<M>(NAME, #F[0] == '6');
    VALU_LIST(ROW)
#undef ROW
    return 0;
}
