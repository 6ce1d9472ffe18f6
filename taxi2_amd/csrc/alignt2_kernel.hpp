// Packed trace-and-walk aligner: alignt_kernel.hpp with TWO pairs per lane, one in each 16-bit
// half of every register (v_pk_max_i16 / v_pk_add_u16 / v_pk_sub_i16 / v_pk_mad_u16).
//
// The fill of alignt_kernel.hpp is VALU-issue bound (0.25 instructions per SIMD-clock) at ~25
// ops per cell, all of them 32-bit max / add / sub / med3 / alignbit on scores that never
// exceed a few thousand.  In 16-bit halves one instruction serves two DP cells, so the score
// and sign arithmetic halves; the trace packing becomes arithmetic on both halves at once
// (balanced base-4 digits) and one v_perm per two columns gathers the four bytes.
//
// Streams.  A chain's pairs (same column sequence) alternate between stream 0 (low halves) and
// stream 1 (high halves); each stream feeds its pairs' rows back to back, so at step s lane l
// works on row s - l of BOTH streams.  Everything per row (row info ring, first / last-row
// resets, end-gap row scores, column-0 boundary, substitution words) exists once per stream.
//
// Per cell and pair the byte is (int8) (16 sc + 4 sb + sa) << 2 | tagF << 1 | tagG with the
// signs sa = sign(G - X), sb = sign(cg - cx), sc = sign(cf - cy) of alignt_kernel.hpp (default
// scores: no tagF, it follows from sa and tagG because opens <= extends, and the byte is
// (128 tagG + 16 sc + 4 sb + sa) mod 256, three multiply-adds from Gn: at_dec_def).  Bytes
// are stored per lane and step as [k][stream] (2K bytes, one 16-byte store for K = 8).
//
// Substitution scores come from an LDS table eqt[base][thread][K/2] of 16-bit fields (the
// doubled match / mismatch score of each column against a row byte "ACGT"[base]); per step each
// stream reads its row's K/2 words (one ds_read_b128), per cell one v_perm builds the packed
// pair of scores.  Rows with any other byte build their words by byte compares (rare path,
// column bytes read from global memory).  LDS is what bounds residency here (walker state for
// 16 walks only, 16-bit column constants broadcast to both halves with op_sel_hi).
//
// 16-bit range: values stay within [-(2 P (nA + nB) + 2 |eo| + 2 |io|), 2 ma min(nA, nB) + 1]
// (P = largest per-column penalty) and the -inf boundary is -16384; the host admits a launch
// only when every difference fits int16 (at_fits16), else it uses the 32-bit kernel.
#pragma once
#include "alignt_kernel.hpp"

namespace taxi2 {

typedef short at_s2 __attribute__((ext_vector_type(2)));

// Debug build only (-DTAXI2_GUARD, `make guard`): every global access and risky LDS index of
// k_alignt2 is range-checked; a violation is recorded in at_guard_err (a code per site) and the
// access skipped, so an out-of-bounds bug is located without faulting the GPU.  The guard build
// also POISONS what a launch must never read before writing it, so a read of stale state shows up
// on the first launch of a process instead of depending on what earlier kernels left behind:
// every LDS array at kernel start and the row ring / wave ring at every chain start (0xA5 bytes;
// a row record, ring entry or walk state still holding the pattern when read sets a code), and
// the chain's trace buffer before its fill (0x64 bytes: outside the valid trace-byte ranges --
// [-88, 87] for the tagF layout, [-22, 21] or that + 128 for the default-score layout -- so the
// walker flags any byte the fill of ITS chain did not store).
#ifdef TAXI2_GUARD
__device__ unsigned int at_guard_err;
#define AT_OK(cond, code) ((cond) ? true : (atomicOr(&at_guard_err, (unsigned)(code)), false))
// event counters of one launch: chains, pairs, thread-0 trace stores, fin writes, finished walks,
// thread-0 first rows, steps, column counts
__device__ unsigned int at_diag[8];
#define AT_DIAG(k, v) atomicAdd(&at_diag[k], (unsigned)(v))
#else
#define AT_OK(cond, code) true
#define AT_DIAG(k, v) ((void)0)
#endif
constexpr uint32_t AT_POISON_LDS = 0xA5A5A5A5u;
// guard codes (bit per site)
enum : unsigned {
    AG_STORE = 1, AG_LOAD = 2, AG_ROWSEQ = 4, AG_COLSEQ = 8, AG_ROWBYTE = 16, AG_FIN = 32, AG_PI = 64, AG_OUT = 128,
    AG_CHUNK = 256, AG_TRACE_POISON = 512, AG_ROW_POISON = 1024, AG_RING_POISON = 2048, AG_WALK_POISON = 4096,
};
// fill `bytes` bytes of LDS at p with the poison pattern (all threads of the workgroup)
__device__ __forceinline__ void at_poison_lds(void* p, size_t bytes) {
    uint32_t* w = (uint32_t*)p;
    for (size_t k = threadIdx.x; k < bytes / 4; k += blockDim.x) w[k] = AT_POISON_LDS;
}

// Measured and settled (the experiment knobs are gone from the tree):
// * the raw-difference trace always forms its bytes (a wave-uniform skip of out-of-band steps
//   spilled at 80 VGPRs: 3.57e6 vs 3.92e6 pairs/s); the sign-digit trace (non-default scores, the
//   4-fill-wave shapes, the queued pass) keeps round 2's skip (A2_SKIP_SIGN: 2.73e6 vs 2.47e6);
// * Iy opens from the left column's best state B (Biopython's F = max(M, Ix): 4.02e6 vs 4.26e6);
// * the Ix column updates stay in the cell loop (at the top of the step: 4.16e6 vs 4.29e6), with the
//   per-column open constants from LDS (one uniform constant + column nB's: 4.11e6 vs 4.28e6);
// * column k+1's M is formed before column k's new B (3 instead of 9 back-edge moves) and vector
//   memory is drained before the last fill wave's step loop (4.47e6 -> 4.55e6);
// * the best state is one v_pk_maximum3_f16 (BIAS16 below: 4.53e6 -> 4.74e6).
#ifndef A2_SKIP_SIGN
#define A2_SKIP_SIGN 1
#endif
// Raw-difference trace (default scores) up to this many fill waves.  The 4-fill-wave shapes (1 025 -
// 2 048 columns) keep the 2-byte sign-digit trace: on them the 4-byte raw trace measured 8 % slower
// (1 200 / 1 500 / 2 000 bp: 8.1e5 / 6.5e5 / 4.7e5 vs 8.8e5 / 7.1e5 / 5.05e5 pairs/s,
// profiles/r3/long_*.json)
constexpr int A2_RAW_MAX_W = 2;
template <int W, bool DEF>
constexpr bool a2_raw() { return DEF && W <= A2_RAW_MAX_W; }
#ifndef TAXI2_AT2_CHUNK
#define TAXI2_AT2_CHUNK 8
#endif
constexpr int AT2_CHUNK = TAXI2_AT2_CHUNK;  // pairs per cursor step (both streams): 2 AT2_CHUNK walks per walker wave
constexpr int NEG16 = -16384;
// Cells are stored BIASED: each 16-bit half holds v + 32768 (unsigned, never wrapping under
// at_fits16).  Maxima are then unsigned (v_pk_max_u16), differences of two cells are the signed
// differences (the bias cancels), and adding a constant pair (c_hi, c_lo) to both halves at once is
// ONE 32-bit v_add_u32 of the integer c_hi * 65536 + c_lo: no half leaves [0, 65535], so no carry
// crosses between the halves.  v_add_u32 issues in 2.28 SIMD cycles, v_pk_add_u16 in 4.09
// (profiles/r2/valu_peak.txt).
// The default-score best-open fill uses a bias of 20480 instead, so that every value the fill
// can hold there -- the -16384 sentinel less a few opens up to the 1 024-column maximum, [4 000,
// 24 000] biased -- is a positive NORMAL f16 bit pattern ([0x0400, 0x7BFF]), whose order as a float is
// its order as an unsigned integer: the cell's best state is then ONE v_pk_maximum3_f16 (gfx950) of
// (M, Ix, Iy) instead of two v_pk_max_u16.  Every other packed form keeps the same bias (the
// range at_fits16 admits, [-16384 - small, 16383], still maps into [0, 65535]).
constexpr int BIAS16 = 20480;
constexpr int AT_ESC = AT_DONE + 1;  // walk state: stepped outside the stored trace band
constexpr uint32_t NEG16X2 = (uint32_t)(NEG16 + BIAS16) * 0x00010001u;  // -16384 biased, both halves

__device__ __forceinline__ at_s2 as_s2(uint32_t v) { return __builtin_bit_cast(at_s2, v); }
__device__ __forceinline__ uint32_t as_u32(at_s2 v) { return __builtin_bit_cast(uint32_t, v); }
typedef unsigned short at_u2 __attribute__((ext_vector_type(2)));
// maximum of biased cells: unsigned per half
__device__ __forceinline__ at_s2 pmax(at_s2 a, at_s2 b) {
    return __builtin_bit_cast(at_s2, __builtin_elementwise_max(__builtin_bit_cast(at_u2, a), __builtin_bit_cast(at_u2, b)));
}
__device__ __forceinline__ uint32_t pk2(int lo, int hi) { return ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16); }
// a biased cell pair from two unbiased values
__device__ __forceinline__ uint32_t pk2b(int lo, int hi) { return pk2(lo + BIAS16, hi + BIAS16); }
// the integer c_hi * 65536 + c_lo of a packed pair of signed 16-bit constants (what a v_add_u32 adds)
__host__ __device__ __forceinline__ uint32_t pk_int(uint32_t packed) { return packed - ((packed & 0x8000u) << 1); }
// biased cells + a constant pair given as pk_int: both halves in one 32-bit add
__device__ __forceinline__ at_s2 padd32(at_s2 a, uint32_t c) { return __builtin_bit_cast(at_s2, __builtin_bit_cast(uint32_t, a) + c); }
// per half clamp to [-1, 1] (the compiler would expand it into compares and selects)
__device__ __forceinline__ at_s2 psign(at_s2 d) {
    uint32_t r;
    asm("v_pk_max_i16 %0, %1, -1 op_sel_hi:[1,0]\n\tv_pk_min_i16 %0, %0, 1 op_sel_hi:[1,0]" : "=&v"(r) : "v"(as_u32(d)));
    return as_s2(r);
}
// per half clamp to [-2, 1]
__device__ __forceinline__ at_s2 pclamp21(at_s2 d) {
    uint32_t r;
    asm("v_pk_max_i16 %0, %1, -2 op_sel_hi:[1,0]\n\tv_pk_min_i16 %0, %0, 1 op_sel_hi:[1,0]" : "=&v"(r) : "v"(as_u32(d)));
    return as_s2(r);
}
// per half a * 4 + b
__device__ __forceinline__ at_s2 pmad4(at_s2 a, at_s2 b) {
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, 4, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(as_u32(a)), "v"(as_u32(b)));
    return as_s2(r);
}
// per half a * 8 + b
__device__ __forceinline__ at_s2 pmad8(at_s2 a, at_s2 b) {
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, 8, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(as_u32(a)), "v"(as_u32(b)));
    return as_s2(r);
}
// Default-score trace byte: (128 tagG + 16 sc + 4 sb + sa) mod 256, digits in [-2, 1] (sc, sb in
// [-1, 1]), built by three multiply-adds from Gn (whose bit 0 is tagG: 128 Gn mod 256 = 128 tagG).
// Code t = 16 sc + 4 sb + sa lies in [-22, 21], so tag 0 bytes are t (as int8) and tag 1 bytes are
// t + 128: an int8 outside [-22, 21] means tag 1 and t = (int8)(byte ^ 0x80).
__device__ __forceinline__ int at_dec_def(uint32_t b, bool& tag) {
    const int x = (int)(int8_t)(uint8_t)b;
    tag = x < -22 || x > 21;
    return tag ? (int)(int8_t)(uint8_t)(b ^ 0x80u) : x;
}
// per half a * 16 + b
__device__ __forceinline__ uint32_t pmad16(at_s2 a, uint32_t b) {
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, 16, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(as_u32(a)), "v"(b));
    return r;
}

// Host: do all differences of the packed fill fit int16?
__host__ __device__ inline bool at_fits16(const KScores& k, int max_len) {
    auto ab = [](int v) { return v < 0 ? -v : v; };
    const long long P = std::max({ab(k.ma), ab(k.mi), ab(k.ie), ab(k.ee)});
    const long long O = std::max(ab(k.io), ab(k.eo));
    const long long lo = 2 * (P * 2 * (long long)max_len + 2 * O + 2);
    // + the drift of the default-score fill: stored values exceed the true ones by (i + j) |2 ie|
    const long long hi = 2 * (long long)ab(k.ma) * max_len + 2 + 2 * (long long)ab(k.ie) * 2 * max_len;
    return lo + 2 * O + 2 * P - NEG16 + 8 < 32767 && hi + 2 * O + 2 * P - NEG16 + 8 < 32767;
}

// Walker loads through global-address-space pointers (global_load, not flat_load: the pointers
// come from LDS structs, so the compiler cannot infer their space).  Trace bytes bypass the
// vector L1 (the buffer was rewritten two chains ago).
typedef const __attribute__((address_space(1))) uint8_t a2_gbyte;
typedef const __attribute__((address_space(1))) uint32_t a2_gword;
__device__ __forceinline__ uint32_t a2_load_byte(const uint8_t* p) { return *(a2_gbyte*)p; }
__device__ __forceinline__ uint32_t a2_load_trace(const uint8_t* p) { return *(const volatile a2_gbyte*)p; }
__device__ __forceinline__ uint32_t a2_load_trace32(const uint8_t* p) { return *(const volatile a2_gword*)p; }

// Raw-difference trace (default scores, the band pass).  Instead of forming sign digits per cell
// (3 subtracts, 3 clamps and 3 multiply-adds per column pair: ~45 % of the fill's issue cycles),
// the fill stores two exact differences of the cell's own states per pair.  Since round 3 the fill
// is the best-open form (alignt2_body, cells): plain scores, states M, Ix, Iy and their maximum B,
// and the bytes are
//   D1 = M - Ix   and   D2 = M - Iy
// as int8: one 32-bit subtract each over both halves and one v_perm per column gather the four
// bytes (D1 lo, D1 hi, D2 lo, D2 hi).  Between the states of one cell these differences are bounded
// by the scores (default scores: both in [-9, 17] over every cell of the CPU model,
// tools/proto_bopen.c), so the int8 is exact.  The high half's bytes carry the low half's borrow
// (the subtract is 32-bit): the walker adds back (lo byte < 0).
// From (D1, D2) of a cell the walker has all three state values relative to each other, so it
// decides the first path's ties exactly (walk_run).  The walker also sums the score of its moves; a
// walk whose sum differs from the fill's optimum (impossible while the differences fit int8: any
// wrong decision leaves the optimal path strictly) queues its pair for the sign-digit full-trace
// pass, like a walk that leaves the band.
__device__ __forceinline__ void a2_raw_de(uint32_t w, int sm, int& d, int& e) {
    if (sm == 0) {
        d = (int)(int8_t)(uint8_t)w;
        e = (int)(int8_t)(uint8_t)(w >> 16);
    } else {
        d = (int)(int8_t)(uint8_t)((w >> 8) + ((w >> 7) & 1u));
        e = (int)(int8_t)(uint8_t)((w >> 24) + ((w >> 23) & 1u));
    }
}

// Walker base code without a branch tree: A 0, C 1, T 2, G 3 (bits 1-2 of the byte, either case),
// 4 for any other byte.  Transitions (A<->G, C<->T) differ in both bits, transversions in one.
__device__ __forceinline__ uint32_t a2_wcode(uint32_t c) {
    const uint32_t d = (c & 0xDFu) - 0x41u;  // 'A' -> 0, 'C' -> 2, 'G' -> 6, 'T' -> 19
    const bool ok = d < 20u && ((0x80045u >> d) & 1u);
    return ok ? ((c >> 1) & 3u) : 4u;
}

// Row records.  One 8-byte LDS entry per step row g holds both streams: .x = two 16-bit row
// words (stream 0 low, stream 1 high), .y = the trace band of the row (below).  Row word bits:
// 0-7 the row byte, 8 first row of its pair, 9 last row, 10 no row, 11-12 "ACGT" code of an
// exact A/C/G/T byte, 13 any other byte (byte-compare substitution path).  The chain pairs of
// stream `st` are tab[st], tab[st + 2], ...
constexpr uint32_t A2_FIRST = 1u << 8, A2_LAST = 1u << 9, A2_NONE = 1u << 10, A2_OTHER = 1u << 13;

__device__ __forceinline__ uint32_t a2_row_word(const ChainPair* __restrict__ tab, int n, int st, int rows, int g,
                                                int& irow, int& nA) {
    irow = 0;
    nA = 0;
    if (g >= rows) return A2_NONE;
    int k = st;
    for (int t = st + 2; t < n; t += 2)
        if (tab[t].r0 <= g) k = t;
    const ChainPair& cp = tab[k];
    const int i = g - cp.r0;
    const uint32_t c = AT_OK(i >= 0 && i < cp.nA, AG_ROWBYTE) ? cp.rseq[i] : 'A';
    const uint32_t ec = c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
    uint32_t v = c | (ec < 4u ? ec << 11 : A2_OTHER);
    if (i == 0) v |= A2_FIRST;
    if (i == cp.nA - 1) v |= A2_LAST;
    irow = i + 1;
    nA = cp.nA;
    return v;
}

// Trace band.  The fill stores the trace bytes of row i (1-based) of a pair only for the column
// blocks (K columns, one lane) that meet the diagonal strip
//   j - i  in  [min(0, nB - nA) - band, max(0, nB - nA) + band]
// (band <= 0: every block).  The strip holds both corners, so a first path that stays inside it
// is walked from stored bytes alone; a walk that would step outside stops and its pair is queued
// for a second launch with the full trace (k_alignt2's esc_* arguments), so results never depend
// on the band.  Blocks [lo, hi] of row i; lo > hi: none.
__host__ __device__ __forceinline__ void a2_band_blocks(int i, int nA, int nB, int band, int K, int& lo, int& hi) {
    if (band <= 0) {
        lo = 0;
        hi = (nB - 1) / K;
        return;
    }
    const int dl = min(0, nB - nA) - band, dh = max(0, nB - nA) + band;
    lo = (max(1, i + dl) - 1) / K;
    hi = (min(nB, i + dh) - 1) / K;
}
// .y of a row record: the union of both streams' block ranges as lo | (hi - lo) << 16, tested by a
// fill lane with ONE 16-bit subtract and compare ((u16)(t - lo) <= hi - lo); no row: lo = 0x8000
__device__ __forceinline__ uint2 a2_row_record(const ChainPair* __restrict__ tab, int n, int rows0, int rows1, int g,
                                               int nB, int band, int K) {
    int i0, i1, a0, a1;
    const uint32_t w0 = a2_row_word(tab, n, 0, rows0, g, i0, a0);
    const uint32_t w1 = a2_row_word(tab, n, 1, rows1, g, i1, a1);
    int lo = 0x7FFF, hi = -1;
    if (i0 > 0) {
        int l, h;
        a2_band_blocks(i0, a0, nB, band, K, l, h);
        lo = min(lo, l);
        hi = max(hi, h);
    }
    if (i1 > 0) {
        int l, h;
        a2_band_blocks(i1, a1, nB, band, K, l, h);
        lo = min(lo, l);
        hi = max(hi, h);
    }
    const uint32_t y = hi < lo ? 0x8000u : (uint32_t)lo | ((uint32_t)(hi - lo) << 16);
    return make_uint2(w0 | (w1 << 16), y);
}

// Optional aligned strings (round 3): every walk also writes its alignment, right-aligned in the
// slot of its ordered pair -- bytes [nA + nB - len, nA + nB) of sx / sy + slot * cap, len in
// slen[slot], slot = p * nslot + o (o = 0 the (a, b) alignment, 1 the (b, a) one; nslot = 1 for
// single-orientation launches) -- in (a, b) column order: sx holds a's side, sy b's, whichever
// sequence the chain put on the rows.  One fill then serves the metrics AND aligned_pairs.txt
// (versus_all.py:746-750 feeds the same aligned pair to both).
struct StrOut {
    uint8_t* sx;
    uint8_t* sy;
    int32_t* slen;
    int cap, nslot;
};

// RAW: the raw-difference trace (default scores; 4 K bytes per lane and step, [step][lane][k] words),
// else the sign-digit code (2 K bytes per lane and step, [step][lane][k][stream] bytes)
template <int K, int W, bool DEF, bool RAW>
__device__ __forceinline__ void
alignt2_body(SetView XS, SetView YS, PairSrc ps, KScores scin, MetricSpec ms, int chunk_req, int out_mode,
             double* __restrict__ out, int32_t* __restrict__ sout, uint8_t* __restrict__ trace, int64_t buf_bytes,
             int cap_rows, int hops, unsigned long long* __restrict__ next, int band, int64_t* __restrict__ esc_list,
             unsigned long long* __restrict__ esc_n, StrOut so) {
    static_assert(K % 2 == 0 && K <= 16, "16-bit score fields: K / 2 words per stream and base");
    constexpr int TB = RAW ? 4 * K : 2 * K;  // trace bytes per lane and step
    constexpr int NT = 64 * W;
    constexpr int XR = a1c_xr(W);
    constexpr int KW = K / 2;
    const KScores sc0 = DEF ? KScores{1, -1, -8, -1, -1, -1} : scin;  // align.py:20-27 defaults
    // RAW (best-open fill, below): plain scores; otherwise doubled scores with tie tags in bit 0
    const KScores sc = RAW ? sc0 : doubled(sc0);
    constexpr uint32_t ODD = RAW ? 0u : 0x00010001u;  // Ix / F kept odd (tagged forms only)
    // Drift (default scores, where every gap extend is ie): cells store V(i, j) - (i + j) dz, so
    // Ix(i, j) = max(G(i-1, j) + o, Ix(i-1, j) + e) becomes max(G + (o - dz), Ix) and likewise for
    // Iy: both extend additions vanish; M absorbs -2 dz in its substitution table.
    // (the best-open form of other scores needs one extend for internal and end gaps, pick_variantt2,
    // so it drifts too: its state differences are then bounded by the scores)
    const int dz = (DEF || RAW) ? sc.ie : 0;
    __shared__ uint2 xinfo[XR];  // row records (a2_row_record)
    __shared__ ChainPair tab[2][AT2_CHUNK];
    __shared__ int fin[2][AT2_CHUNK];
    __shared__ uint32_t fin_n[2];
    __shared__ AtChain chs[2];
    __shared__ uint2 ring[(W > 1 ? W - 1 : 1) * RING];
    __shared__ uint32_t colc[K][NT];            // Ix open (end-gap score on column nB), as pk_int
    __shared__ uint32_t colx[DEF ? 1 : K][NT];  // Ix extend (non-default scores), as pk_int
    __shared__ uint32_t eqt[4][NT][KW];         // 16-bit substitution score fields by row base
    __shared__ int64_t s_qc, s_qend;
    __shared__ int s_n, s_rows[2];
    __shared__ int s_fill;  // fill waves done with the current interval (cumulative per chain)
    __shared__ AtWalk wks[2 * AT2_CHUNK];
    __shared__ int escf[2][AT2_CHUNK];  // pair already queued for the full-trace pass

#ifdef TAXI2_GUARD
    at_poison_lds(xinfo, sizeof xinfo);
    at_poison_lds(tab, sizeof tab);
    at_poison_lds(fin, sizeof fin);
    at_poison_lds(fin_n, sizeof fin_n);
    at_poison_lds(chs, sizeof chs);
    at_poison_lds(ring, sizeof ring);
    at_poison_lds(colc, sizeof colc);
    at_poison_lds(colx, sizeof colx);
    at_poison_lds(eqt, sizeof eqt);
    at_poison_lds(wks, sizeof wks);
    at_poison_lds(escf, sizeof escf);
    if (threadIdx.x == 0) s_n = s_rows[0] = s_rows[1] = s_fill = (int)AT_POISON_LDS;
    __syncthreads();
#endif
    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: ring pointers etc. in SGPRs
    const bool walker = w == W;
    const int nm = ms.n;
    // second pass (ps.sel set): the pairs the band pass queued; *ps.dcount of them, pair p = sel[q]
    const int64_t total = ps.dcount ? (int64_t)min((unsigned long long)ps.count, *ps.dcount) : ps.count;
    const int64_t chunk = chunk_req >= 1 ? min((int64_t)chunk_req, (int64_t)AT2_CHUNK)
                                         : max((int64_t)1, min((int64_t)AT2_CHUNK, total / ((int64_t)gridDim.x * 8)));
    uint8_t* const bufs = trace + (size_t)blockIdx.x * 2 * (size_t)buf_bytes;

    if (tid == 0) {
        s_qc = 0;
        s_qend = 0;
    }
    int cur = 0;
    int prev_n = 0;

    auto walk_init = [&](int pb, int n) {
        const int nw = out_mode == OUT_BOTH ? 2 * n : n;
        if (lane >= 2 * AT2_CHUNK) return;
        // every field of every walk slot is written, idle slots included (an idle slot's pi
        // indexes tab[] in walk_run; it must not be whatever an earlier kernel left in LDS)
        AtWalk& W_ = wks[lane];
        W_ = AtWalk{0, 0, AT_DONE, 0, 0, 0, 0u, 0u, 0u, 0, 0, 0, 0};
        if (lane < AT2_CHUNK) escf[pb][lane] = 0;
        if (lane < nw) {
            const int pi = lane < n ? lane : lane - n;
            const ChainPair& cp = tab[pb][pi];
            W_.pi = pi;
            W_.prio = out_mode == OUT_BOTH ? (lane >= n) : cp.swp;
            W_.i = cp.nA + 1;
            W_.j = chs[pb].nB + 1;
            W_.st = AT_M;
            W_.first = 1;
        }
    };
    // hop until `budget` hops (< 0: unbounded) or, with target > 0, until the fill waves have
    // signalled `target` interval completions: the walker uses exactly the time the fill waves
    // spend on their interval and delays the barrier by at most one hop
    auto walk_run = [&](int pb, int budget, int target) {
        AtWalk& W_ = wks[lane < 2 * AT2_CHUNK ? lane : 0];
        int st = lane < 2 * AT2_CHUNK ? W_.st : AT_DONE;
        if (!AT_OK(st != (int)AT_POISON_LDS && W_.pi != (int)AT_POISON_LDS, AG_WALK_POISON)) st = AT_DONE;
        if (!__any(st != AT_DONE)) return;
        const int pi = W_.pi;
        const ChainPair& cp = tab[pb][AT_OK(st == AT_DONE || (pi >= 0 && pi < chs[pb].n), AG_PI) ? pi : 0];
        const AtChain& ch = chs[pb];
        const int fx = cp.fx, lx = cp.lx, fy = ch.fy, ly = ch.ly, r0 = cp.r0, sm = cp.pad;
        const int prio = W_.prio;
        // the stored strip (a2_band_blocks) holds every cell with nj - ni in [bdl, bdl + bwd]; a walk
        // stepping onto any other cell stops (AT_ESC) and its pair is queued after the hop loop
        const int bdl = min(0, ch.nB - cp.nA) - band;
        const uint32_t bwd = (uint32_t)(abs(ch.nB - cp.nA) + 2 * band);
        const uint8_t* rs = cp.rseq;
        const uint8_t* cs = ch.cseq;
        const uint8_t* tr = bufs + (size_t)pb * (size_t)buf_bytes + sm;
        int i = W_.i, j = W_.j, first = W_.first;
        uint32_t cb = W_.cb, xa = W_.xa, yb = W_.yb;
        int valid = W_.valid, ts = W_.ts, tv = W_.tv, gap = W_.gap;
        int sc2 = W_.sc2, ncol = W_.ncol;
        const int nA_ = cp.nA, nB_ = ch.nB;
        for (int h = 0; budget < 0 || h < budget; ++h) {
            if (!__any(st < AT_DONE)) break;
            if (target > 0 && __hip_atomic_load(&s_fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
            if (st >= AT_DONE) continue;
            int ni, nj;
            if (st == AT_M) {
                if (!first) {
                    const int bx = base_code(xa), by = base_code(yb);
                    if (bx < 4 && by < 4) {
                        ++valid;
                        const int dd = bx ^ by;
                        ts += dd == 2;
                        tv += (dd != 0) & (dd != 2);
                    }
                    if constexpr (RAW) sc2 += xa == yb ? sc.ma : sc.mi;
                }
                ni = i - 1;
                nj = j - 1;
            } else if (st == AT_IX) {
                if (base_code(xa) < 4 && j - 1 >= fy && j <= ly) ++gap;
                ni = i - 1;
                nj = j;
            } else {
                if (base_code(yb) < 4 && i - 1 >= fx && i <= lx) ++gap;
                ni = i;
                nj = j - 1;
            }
            if (so.sx && !first) {  // this column of the alignment, right to left, in (a, b) order
                const uint32_t rc = st == AT_IY ? (uint32_t)'-' : xa, cc = st == AT_IX ? (uint32_t)'-' : yb;
                const size_t o = ((size_t)cp.p * so.nslot + ((prio ^ cp.swp) & (so.nslot - 1))) * (size_t)so.cap +
                                 (size_t)(nA_ + nB_ - 1 - ncol);
                so.sx[o] = (uint8_t)(cp.swp ? cc : rc);
                so.sy[o] = (uint8_t)(cp.swp ? rc : cc);
                ++ncol;
            }
            first = 0;
            if constexpr (RAW) {
                if (ni == 0 && nj == 0) {  // the gap run (if any) opened at the start: end-gap open
                    if (st != AT_M) sc2 += sc.eo;
                    // the walked score must be the fill's optimum, else a decision was wrong
                    if (sc2 != fin[pb][pi] + (nA_ + nB_) * dz) {  // best-open form: plain scores
                        st = AT_ESC;
                        continue;
                    }
                }
            }
            if (ni == 0 && nj == 0) {
                const int64_t p = cp.p;
                double* o;
                if (out_mode == OUT_BOTH) o = out + (p * 2 + ((prio ^ cp.swp) ? 1 : 0)) * nm;
                else o = out + p * nm;
                AT_DIAG(4, 1);
                if (AT_OK(p >= 0 && p < ps.count, AG_OUT))
                for (int m = 0; m < nm; ++m)
                    o[m] = metric_value(ms.code[m], (uint32_t)valid, (uint32_t)ts, (uint32_t)tv, (uint32_t)gap);
                if (sout && (out_mode != OUT_BOTH || !prio) && AT_OK(pi >= 0 && pi < AT2_CHUNK && fin[pb][pi] != (int)AT_POISON_LDS, AG_FIN))  // undo the drift of cell (nA, nB)
                    sout[p] = RAW ? fin[pb][pi] + (cp.nA + chs[pb].nB) * dz : (fin[pb][pi] + (cp.nA + chs[pb].nB) * dz) >> 1;
                if (so.slen) so.slen[p * so.nslot + ((prio ^ cp.swp) & (so.nslot - 1))] = ncol;
                st = AT_DONE;
                continue;
            }
            uint32_t nb = 0;
            // stepping outside the stored strip: the byte read below is stale and the walk stops
            // (no branch here: a divergent exit in the hop loop doubled its code)
            bool esc = false;
            if (ni >= 1 && nj >= 1) {
                esc = band > 0 && (uint32_t)(nj - ni - bdl) > bwd;
                const int t = (nj - 1) / K;
                const int k = nj - 1 - t * K;
                const int s = r0 + ni - 1 + (t & 63);
                if constexpr (RAW) {
                    const size_t off = ((size_t)s * NT + t) * TB + 4 * k;
                    if (AT_OK(off + 4 <= (size_t)buf_bytes, AG_LOAD)) nb = a2_load_trace32(tr - sm + off);
                    int dv_, ev_;
                    a2_raw_de(nb, sm, dv_, ev_);
                    // guard build: the poison (0x64 = 100) lies far outside the differences' range
                    (void)AT_OK(esc || (dv_ >= -64 && dv_ <= 63 && ev_ >= -64 && ev_ <= 63), AG_TRACE_POISON);
                } else {
                    const size_t off = ((size_t)s * NT + t) * TB + 2 * k + sm;
                    if (AT_OK(off < (size_t)buf_bytes, AG_LOAD)) nb = a2_load_trace(tr - sm + off);
                    // guard build: the fill of this chain stored every byte the walk reads
                    (void)AT_OK(esc || (DEF ? ((int)(int8_t)(uint8_t)nb >= -22 && (int)(int8_t)(uint8_t)nb <= 21) ||
                                                  ((int)(int8_t)(uint8_t)(nb ^ 0x80u) >= -22 && (int)(int8_t)(uint8_t)(nb ^ 0x80u) <= 21)
                                            : ((int)(int8_t)(uint8_t)nb >= -88 && (int)(int8_t)(uint8_t)nb <= 87)),
                                AG_TRACE_POISON);
                }
            }
            xa = (ni >= 1 && AT_OK(ni - 1 < cp.nA, AG_ROWSEQ)) ? a2_load_byte(rs + ni - 1) : 0u;
            yb = (nj >= 1 && AT_OK(nj - 1 < ch.nB, AG_COLSEQ)) ? a2_load_byte(cs + nj - 1) : 0u;
            if constexpr (RAW) {
                // best-open trace: D1 = M - X and D2 = M - Y of (ni, nj) give the three state values
                // relative to each other; the candidates of the move into (i, j) are taken at (ni, nj)
                // relative to the one that extends, and the first in priority order (A: M, Ix, Iy;
                // B: M, Iy, Ix) among those at the maximum is the next state
                int d1v, d2v;
                a2_raw_de(nb, sm, d1v, d2v);
                int vM, vX, vY;
                if (st == AT_M) {  // best state of (ni, nj), relative to Ix
                    vM = d1v;
                    vX = 0;
                    vY = d1v - d2v;
                } else if (st == AT_IX) {  // Ix(i, j) from (i-1, j): M + co, Ix (extend), Iy + co
                    const int co = (j == nB_ ? sc.eo : sc.io) - dz;
                    vM = d1v + co;
                    vX = 0;
                    vY = d1v - d2v + co;
                } else {  // Iy(i, j) from (i, j-1): M + oy, Ix + oy, Iy (extend)
                    const int oy = (i == nA_ ? sc.eo : sc.io) - dz;
                    vM = d2v + oy;
                    vX = d2v - d1v + oy;
                    vY = 0;
                }
                const int vm = max(vM, max(vX, vY));
                int nst = vM == vm ? AT_M : prio ? (vY == vm ? AT_IY : AT_IX) : (vX == vm ? AT_IX : AT_IY);
                if (ni == 0) nst = AT_IY;
                else if (nj == 0) nst = AT_IX;
                if (st == AT_IX) {  // gap moves: extend when the run continues, end scores on the edges
                    const bool en = j == nB_ || j == 0;
                    sc2 += nst == AT_IX ? (en ? sc.ee : sc.ie) : (en ? sc.eo : sc.io);
                } else if (st == AT_IY) {
                    const bool en = i == nA_ || i == 0;
                    sc2 += nst == AT_IY ? (en ? sc.ee : sc.ie) : (en ? sc.eo : sc.io);
                }
                i = ni;
                j = nj;
                st = esc ? AT_ESC : nst;
                continue;
            }
            // byte: (int8) code << 2 | tags, code = 16 sc + 4 sb + sa, digits sa in [-2, 1],
            // sb, sc in [-1, 1] (balanced base 4: u = code + 22 has digits sa + 2, sb + 1, sc + 1)
            // (default scores: the byte is the code itself with tagG as its 128 bit, at_dec_def)
            bool tagG, ctag;
            const int nu = (DEF ? at_dec_def(nb, tagG) : ((int)(int8_t)(uint8_t)nb >> 2)) + 22;
            const int cu = (DEF ? at_dec_def(cb, ctag) : ((int)(int8_t)(uint8_t)cb >> 2)) + 22;
            (void)ctag;
            if (!DEF) tagG = nb & 1u;
            // class of (ni, nj) from sa = clamp(G - X1, -2, 1) and tagG (X1 = 2 Ix + 1, G tagged):
            // 1 -> M if tagG else Iy; 0 -> M (M = Ix); -1 -> Ix = Iy tie; -2 -> Ix
            const int sa = (nu & 3) - 2;
            const bool clsM = sa == 0 || (sa == 1 && tagG);
            int nst;
            if (ni == 0) {
                nst = AT_IY;
            } else if (nj == 0) {
                nst = AT_IX;
            } else if (st == AT_M) {  // best state of (ni, nj)
                nst = clsM ? AT_M : sa == 1 ? AT_IY : sa == -1 ? (prio ? AT_IY : AT_IX) : AT_IX;
            } else if (st == AT_IX) {  // how Ix(i, j) was formed: sign of real (G + o) - (Ix + e)
                const int sb = ((cu >> 2) & 3) - 1;
                // a tie goes to G when G is M (both priorities) or, G = Iy, under B (Iy > Ix)
                const bool gp = sb > 0 || (sb == 0 && (tagG || prio));
                nst = gp ? (tagG ? AT_M : AT_IY) : AT_IX;
            } else {  // how Iy(i, j) was formed: sign of real (F + o) - (Iy + e)
                const int sc_ = (cu >> 4) - 1;
                // tagF of (ni, nj).  Default scores (open <= extend) store none: an F path needs
                // F + oy >= Y + ey, impossible when Iy is the strict maximum (oy <= ey), so M >= Ix
                // exactly when the cell's class is M; the Ix and Ix = Iy classes have Ix > M.
                const bool tagF = DEF ? clsM : (nb & 2u);
                // a tie goes to F under A (M, Ix > Iy) and, under B, only when F is M
                const bool fp = sc_ > 0 || (sc_ == 0 && (tagF || !prio));
                nst = fp ? (tagF ? AT_M : AT_IX) : AT_IY;
            }
            cb = nb;
            i = ni;
            j = nj;
            st = esc ? AT_ESC : nst;
        }
        if (st == AT_ESC) {  // queue the pair (once, whichever orientation stopped) for the full-trace pass
            if (atomicOr(&escf[pb][pi], 1) == 0 && AT_OK(esc_list != nullptr, AG_OUT)) esc_list[atomicAdd(esc_n, 1ull)] = cp.p;
            st = AT_DONE;
        }
        if (lane >= 2 * AT2_CHUNK) return;
        W_.i = i;
        W_.j = j;
        W_.st = st;
        W_.first = first;
        W_.cb = cb;
        W_.xa = xa;
        W_.yb = yb;
        W_.valid = valid;
        W_.ts = ts;
        W_.tv = tv;
        W_.gap = gap;
        W_.sc2 = sc2;
        W_.ncol = ncol;
    };

    // Best-open walker (RAW), written branch-free: the three state cases of the move out of (i, j)
    // are selects over one straight-line hop instead of three divergent branches (the walker wave
    // shares its SIMD with the fill waves, so its VALU count is the cost).  Same decisions, counters,
    // strings, score check and escapes as walk_run.  The candidates of the move into (i, j) are taken
    // at (ni, nj) relative to Ix there plus a per-case offset:
    //   diagonal arrival: (M, Ix, Iy) - Ix           = (D1,      0, D1 - D2)
    //   Ix arrival:       (M + co, Ix, Iy + co) - Ix = (D1 + co, 0, D1 - D2 + co)
    //   Iy arrival:       (M + oy, Ix + oy, Iy) - (Ix + oy) = (D1, 0, D1 - D2 - oy)
    auto walk_run_raw = [&](int pb, int budget, int target) {
        AtWalk& W_ = wks[lane < 2 * AT2_CHUNK ? lane : 0];
        int st = lane < 2 * AT2_CHUNK ? W_.st : AT_DONE;
        if (!AT_OK(st != (int)AT_POISON_LDS && W_.pi != (int)AT_POISON_LDS, AG_WALK_POISON)) st = AT_DONE;
        if (!__any(st != AT_DONE)) return;
        const int pi = W_.pi;
        const ChainPair& cp = tab[pb][AT_OK(st == AT_DONE || (pi >= 0 && pi < chs[pb].n), AG_PI) ? pi : 0];
        const AtChain& ch = chs[pb];
        const int fx = cp.fx, lx = cp.lx, fy = ch.fy, ly = ch.ly, r0 = cp.r0, sm = cp.pad;
        const int prio = W_.prio;
        const int bdl = min(0, ch.nB - cp.nA) - band;
        const uint32_t bwd = (uint32_t)(abs(ch.nB - cp.nA) + 2 * band);
        const uint8_t* rs = cp.rseq;
        const uint8_t* cs = ch.cseq;
        const uint8_t* trb = bufs + (size_t)pb * (size_t)buf_bytes;
        int i = W_.i, j = W_.j, first = W_.first;
        uint32_t xa = W_.xa, yb = W_.yb;
        int valid = W_.valid, ts = W_.ts, tv = W_.tv, gap = W_.gap;
        int sc2 = W_.sc2, ncol = W_.ncol;
        const int nA_ = cp.nA, nB_ = ch.nB;
        const int co_i = sc.io - sc.ie, co_e = sc.eo - sc.ee;  // opens relative to their extends
        const int bsh = sm ? 8 : 0;                       // this stream's byte of each 16-bit half
        for (int h = 0; budget < 0 || h < budget; ++h) {
            if (!__any(st < AT_DONE)) break;
            if (target > 0 && __hip_atomic_load(&s_fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
            if (st < AT_DONE) {
                const bool isM = st == AT_M, isX = st == AT_IX, isY = st == AT_IY;
                // counters and score of the move out of (i, j) (xa, yb: its row / column bytes)
                const uint32_t bx = a2_wcode(xa), by = a2_wcode(yb);
                const uint32_t dd = bx ^ by;
                const bool cnt = isM && !first && (bx | by) < 4u;
                valid += cnt;
                ts += cnt && dd == 3u;                 // a2_wcode: A<->G, C<->T differ in both bits
                tv += cnt && (dd == 1u || dd == 2u);
                gap += (isX && bx < 4 && j - 1 >= fy && j <= ly) || (isY && by < 4 && i - 1 >= fx && i <= lx);
                sc2 += (isM && !first) ? (xa == yb ? sc.ma : sc.mi) : 0;
                const int ni = isY ? i : i - 1, nj = isX ? j : j - 1;
                if (so.sx && !first) {  // this column of the alignment, right to left, in (a, b) order
                    const uint32_t rc = isY ? (uint32_t)'-' : xa, cc = isX ? (uint32_t)'-' : yb;
                    const size_t o = ((size_t)cp.p * so.nslot + ((prio ^ cp.swp) & (so.nslot - 1))) * (size_t)so.cap +
                                     (size_t)(nA_ + nB_ - 1 - ncol);
                    so.sx[o] = (uint8_t)(cp.swp ? cc : rc);
                    so.sy[o] = (uint8_t)(cp.swp ? rc : cc);
                    ++ncol;
                }
                first = 0;
                if (ni == 0 && nj == 0) {  // the walk is complete (once per walk)
                    if (!isM) sc2 += sc.eo;  // the gap run (if any) opened at the start: end-gap open
                    if (sc2 != fin[pb][pi] + (nA_ + nB_) * dz) {  // a wrong decision: queue the pair
                        st = AT_ESC;
                    } else {
                        const int64_t p = cp.p;
                        double* o = out_mode == OUT_BOTH ? out + (p * 2 + ((prio ^ cp.swp) ? 1 : 0)) * nm : out + p * nm;
                        AT_DIAG(4, 1);
                        if (AT_OK(p >= 0 && p < ps.count, AG_OUT))
                            for (int m = 0; m < nm; ++m)
                                o[m] = metric_value(ms.code[m], (uint32_t)valid, (uint32_t)ts, (uint32_t)tv, (uint32_t)gap);
                        if (sout && (out_mode != OUT_BOTH || !prio) && AT_OK(pi >= 0 && pi < AT2_CHUNK && fin[pb][pi] != (int)AT_POISON_LDS, AG_FIN))
                            sout[p] = fin[pb][pi] + (nA_ + nB_) * dz;
                        if (so.slen) so.slen[p * so.nslot + ((prio ^ cp.swp) & (so.nslot - 1))] = ncol;
                        st = AT_DONE;
                    }
                } else {
                    const bool in = ni >= 1 && nj >= 1;
                    const bool esc = in && band > 0 && (uint32_t)(nj - ni - bdl) > bwd;
                    // trace word and bytes of (ni, nj) (row / column 0: clamped, the value unused)
                    const int cj = max(nj, 1) - 1, ci = max(ni, 1) - 1;
                    const uint32_t t = (uint32_t)cj / K, k = (uint32_t)cj - t * K;
                    const uint32_t off = (((uint32_t)(r0 + ci) + (t & 63u)) * (uint32_t)NT + t) * (uint32_t)TB + 4u * k;
                    const uint32_t xa_ = a2_load_byte(rs + ci), yb_ = a2_load_byte(cs + cj);
                    uint32_t nb = 0u;
                    if (AT_OK(off + 4 <= (size_t)buf_bytes, AG_LOAD)) nb = a2_load_trace32(trb + off);
                    xa = ni >= 1 ? xa_ : 0u;
                    yb = nj >= 1 ? yb_ : 0u;
                    // D1, D2 of this stream: bytes 0 / 2 (stream 0) or 1 / 3 plus the low half's borrow
                    const int d1v = (int)(int8_t)(uint8_t)((nb >> bsh) + (sm ? ((nb >> 7) & 1u) : 0u));
                    const int d2v = (int)(int8_t)(uint8_t)((nb >> (16 + bsh)) + (sm ? ((nb >> 23) & 1u) : 0u));
                    (void)AT_OK(esc || !in || (d1v >= -64 && d1v <= 63 && d2v >= -64 && d2v <= 63), AG_TRACE_POISON);
                    const int co = j == nB_ ? co_e : co_i, oy = i == nA_ ? co_e : co_i;
                    const int vM = d1v + (isX ? co : 0);
                    const int vY = d1v - d2v + (isX ? co : isY ? -oy : 0);
                    const int vm = max(max(vM, vY), 0);
                    int nst = vM == vm ? AT_M : prio ? (vY == vm ? AT_IY : AT_IX) : (vm == 0 ? AT_IX : AT_IY);
                    nst = ni == 0 ? AT_IY : nj == 0 ? AT_IX : nst;
                    // gap moves: extend when the run continues, end scores on the edges
                    const bool ext = isX ? nst == AT_IX : nst == AT_IY;
                    const bool en = isX ? (j == nB_ || j == 0) : (i == nA_ || i == 0);
                    sc2 += isM ? 0 : ext ? (en ? sc.ee : sc.ie) : (en ? sc.eo : sc.io);
                    i = ni;
                    j = nj;
                    st = esc ? AT_ESC : nst;
                }
            }
        }
        if (st == AT_ESC) {  // queue the pair (once, whichever orientation stopped) for the full-trace pass
            if (atomicOr(&escf[pb][pi], 1) == 0 && AT_OK(esc_list != nullptr, AG_OUT)) esc_list[atomicAdd(esc_n, 1ull)] = cp.p;
            st = AT_DONE;
        }
        if (lane >= 2 * AT2_CHUNK) return;
        W_.i = i;
        W_.j = j;
        W_.st = st;
        W_.first = first;
        W_.xa = xa;
        W_.yb = yb;
        W_.valid = valid;
        W_.ts = ts;
        W_.tv = tv;
        W_.gap = gap;
        W_.sc2 = sc2;
        W_.ncol = ncol;
    };
    auto walk = [&](int pb, int budget, int target) {
        if constexpr (RAW) walk_run_raw(pb, budget, target);
        else walk_run(pb, budget, target);
    };

    // The fill waves and the walker wave run separate copies of the chain loop (same barrier
    // sequence): the fill state (columns, carries) is then not live across the walker code,
    // which kept it in registers for the whole loop and spilled both to scratch.
    auto chain_loop = [&](auto WK) {
        constexpr bool IS_W = decltype(WK)::value;
        for (;;) {
            // ---- cut the next chain (thread 0); its pairs alternate between the two streams
            __syncthreads();
            if (!IS_W && tid == 0) {
                int n = 0, rows[2] = {0, 0};
                const uint8_t* ccol = nullptr;
                while (n == 0) {
                    if (s_qc >= s_qend) {
                        const int64_t q0 = (int64_t)atomicAdd(next, (unsigned long long)chunk);
                        if (q0 >= total) break;
                        s_qc = q0;
                        s_qend = min(q0 + chunk, total);
                    }
                    int64_t q = s_qc;
                    for (; q < s_qend; ++q) {
                        const int64_t p = ps.sel ? ps.sel[q] : q;
                        int64_t a, b;
                        decode_pair(ps, p, a, b);
                        const int4 ma = XS.meta[a];
                        const int4 mb = YS.meta[b];
                        if (ma.x == 0 || mb.x == 0) {
                            if (n > 0) break;
                            for (int m = 0; m < nm; ++m) {
                                if (out_mode == OUT_BOTH) {
                                    out[(p * 2 + 0) * nm + m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                                    out[(p * 2 + 1) * nm + m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                                } else {
                                    out[p * nm + m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                                }
                            }
                            if (sout) {
                                const int ne = ma.x + mb.x;
                                sout[p] = ne == 0 ? 0 : sc0.eo + sc0.ee * (ne - 1);
                            }
                            if (so.sx) {  // the other sequence against gaps, every slot alike
                                const int L = ma.x + mb.x;
                                const uint8_t* xs_ = XS.bytes + XS.offs[a];
                                const uint8_t* ys_ = YS.bytes + YS.offs[b];
                                for (int o = 0; o < so.nslot; ++o) {
                                    uint8_t* ox = so.sx + ((size_t)p * so.nslot + o) * (size_t)so.cap;
                                    uint8_t* oy = so.sy + ((size_t)p * so.nslot + o) * (size_t)so.cap;
                                    for (int t = 0; t < L; ++t) {
                                        ox[t] = ma.x ? xs_[t] : (uint8_t)'-';
                                        oy[t] = mb.x ? ys_[t] : (uint8_t)'-';
                                    }
                                    so.slen[p * so.nslot + o] = L;
                                }
                            }
                            continue;
                        }
                        const uint8_t* xa_ = XS.bytes + XS.offs[a];
                        const uint8_t* yb_ = YS.bytes + YS.offs[b];
                        const bool swp = at_swap(xa_, yb_, ma.x, mb.x, ccol, n);
                        const uint8_t* cseq = swp ? xa_ : yb_;
                        const int4 rm = swp ? mb : ma;
                        const int sm = n & 1;
                        if (n > 0 && (cseq != ccol || rows[sm] + rm.x > cap_rows)) break;
                        if (n == 0) {
                            const int4 cm = swp ? ma : mb;
                            ccol = cseq;
                            chs[cur] = AtChain{cseq, 0, cm.x, cm.y, cm.z};
                        }
                        if (!AT_OK(n < AT2_CHUNK, AG_CHUNK)) break;
                        tab[cur][n] = ChainPair{swp ? yb_ : xa_, p, rm.x, rm.y,
                                                rm.z, rows[sm], swp ? 1 : 0, sm};
                        rows[sm] += rm.x;
                        ++n;
                    }
                    s_qc = q;
                }
                if (n > 0) chs[cur].n = n;
                if (n > 0) {
                    AT_DIAG(0, 1);
                    AT_DIAG(1, n);
                    AT_DIAG(6, max(rows[0], rows[1]) + 63);
                    AT_DIAG(7, chs[cur].nB);
                }
                s_n = n;
                s_rows[0] = rows[0];
                s_rows[1] = rows[1];
                fin_n[0] = fin_n[1] = 0u;
                s_fill = 0;
            }
            __syncthreads();
            const int n = s_n;
            const int rows0 = s_rows[0], rows1 = s_rows[1];
            const int pb = cur ^ 1;
            if constexpr (IS_W) walk_init(pb, prev_n);
            if (n == 0) {
                if constexpr (IS_W) walk(pb, -1, 0);
                break;
            }
            const int nB = chs[cur].nB;
#ifdef TAXI2_GUARD
            {  // poison the row ring, the wave ring and this chain's trace buffer (see AT_OK)
                at_poison_lds(xinfo, sizeof xinfo);
                at_poison_lds(ring, sizeof ring);
                if constexpr (!IS_W) {
                    uint4* tb = (uint4*)(bufs + (size_t)cur * (size_t)buf_bytes);
                    const size_t nv = ((size_t)(max(rows0, rows1) + 63) * NT * TB + 15) / 16;
                    const uint4 pz = make_uint4(0x64646464u, 0x64646464u, 0x64646464u, 0x64646464u);
                    for (size_t v = tid; v < nv && AT_OK(v * 16 + 16 <= (size_t)buf_bytes, AG_STORE); v += NT) tb[v] = pz;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
#endif

            // ---- fill-lane column constants (once per chain)
            const int j0 = (w * 64 + lane) * K + 1;
            if constexpr (!IS_W) {
                const uint8_t* cseq = chs[cur].cseq;
                uint32_t ew[4][KW];
    #pragma unroll
                for (int r = 0; r < 4; ++r)
    #pragma unroll
                    for (int q = 0; q < KW; ++q) ew[r][q] = 0u;
    #pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int j = j0 + k;
                    uint32_t c = 0u;
                    if (j <= nB) c = cseq[j - 1];
    #pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int s = ((j <= nB && c == (uint32_t)"ACGT"[r]) ? sc.ma : sc.mi) - 2 * dz;
                        ew[r][k / 2] |= ((uint32_t)s & 0xFFFFu) << (16 * (k & 1));
                    }
                    const int oc = ((j == nB) ? sc.eo : sc.io) - dz, ec = (j == nB) ? sc.ee : sc.ie;
                    colc[k][tid] = pk_int(pk2(oc, oc));
                    if (!DEF) colx[DEF ? 0 : k][tid] = pk_int(pk2(ec, ec));
                }
    #pragma unroll
                for (int r = 0; r < 4; ++r)
    #pragma unroll
                    for (int q = 0; q < KW; ++q) eqt[r][tid][q] = ew[r][q];
            }
            // rows 0..63, and "no row" for the ring slots read as rows -63..-1 by the lanes the
            // wavefront has not reached yet (overwritten only when row XR-64 is prefetched)
            if (tid < 64) xinfo[tid] = a2_row_record(tab[cur], n, rows0, rows1, tid, nB, band, K);
            else if (tid < 128) xinfo[XR - 128 + tid] = make_uint2(A2_NONE | (A2_NONE << 16), 0x8000u);
            uint32_t stG[K], stX[K];
    #pragma unroll
            for (int k = 0; k < K; ++k) {
                const int g0 = sc.eo + sc.ee * (j0 + k - 1) - (j0 + k) * dz;
                stG[k] = pk2b(g0, g0);
                stX[k] = NEG16X2 | ODD;  // Ix kept odd (tagged forms)
            }
            uint32_t payF = NEG16X2 | ODD, payY = NEG16X2;
            // column-0 boundary of wave 0's lane 0 (row g = s): odd F = 2 Ix(i, 0) + 1 - i dz with
            // Ix(i, 0) = eo + ee (i - 1); default scores (ee = dz) make it one constant
            // (best-open form: B(i, 0) = Ix(i, 0), plain)
            const uint32_t bnd1 = pk2b(sc.eo - dz + (RAW ? 0 : 1), sc.eo - dz + (RAW ? 0 : 1));
            uint32_t bnd = bnd1;
            uint32_t carry = 0u;
            const uint2* ring_in = (w > 0 && !IS_W) ? ring + (size_t)(w - 1) * RING : nullptr;
            uint2* ring_out = (w < W - 1) ? ring + (size_t)w * RING : nullptr;
            uint8_t* trb = bufs + (size_t)cur * (size_t)buf_bytes;
            __syncthreads();  // xinfo block 0, column tables

            // One systolic step of a fill wave, specialised on the wave's role: FW = wave 0 (column-0
            // boundary from the row record, no ring read), HO = writes the ring to the next wave.  Per-step
            // uniform branches on w cost spilled SGPR masks (v_readlane) on every step.
            auto step = [&](auto FW, auto HO, const int s) {
                            // lane id recomputed (two v_mbcnt) rather than kept live across the chain
                            // loop: at 80 VGPRs it was spilled and reloaded from scratch every step
                            // (still so after the next-column M ordering: kept live, the step loop
                            // reloads three dwords from scratch per step in the ISA)
                            int ln;
                            asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
                            const int g = s - ln;
                            // this lane's column block, from the lane id: threadIdx is not kept live
                            // across the loop (it was spilled and reloaded in the first-row path)
                            const int tq = w * 64 + ln;
                            const uint2 rec = xinfo[g & (XR - 1)];
                            uint2 o_ring = make_uint2(0u, 0u);
                            if constexpr (!decltype(FW)::value) o_ring = ring_in[(s + 1) & (RING - 1)];
                            // trace band (a2_row_record): store iff (u16)(block - lo) <= hi - lo (covers
                            // j0 <= nB).  The lane mask is formed here, a whole cell block ahead of the
                            // store, so the exec-mask update there never waits on the compare.
                            const bool in_band = (uint16_t)((uint16_t)tq - (uint16_t)rec.y) <= (uint16_t)(rec.y >> 16);
                            const uint64_t bmask = __builtin_amdgcn_ballot_w64(in_band);
                            asm volatile("" ::"s"(bmask));
                            const uint32_t rw = rec.x;
                            (void)AT_OK(rw != AT_POISON_LDS, AG_ROW_POISON);
                            uint32_t inF, inY;
                            if constexpr (decltype(FW)::value) {  // column 0: Ix(i, 0) = eo + ee (i - 1), Iy = -inf
                                if constexpr (!DEF && !RAW) {  // one row on per step; a first row restarts its half
                                    const uint32_t mf = ((rw & A2_FIRST) ? 0xFFFFu : 0u) | ((rw & (A2_FIRST << 16)) ? 0xFFFF0000u : 0u);
                                    bnd = (bnd1 & mf) | (as_u32(as_s2(bnd) + (at_s2){(short)sc.ee, (short)sc.ee}) & ~mf);
                                }
                                inF = shr_old(payF, bnd);
                                inY = shr_old(payY, NEG16X2);
                            } else {
                                const uint2 o = o_ring;
                                // lane 0 reads row s; rows past the chain's last are never read back
                                (void)AT_OK(s >= max(rows0, rows1) || o.x != AT_POISON_LDS, AG_RING_POISON);
                                inF = shr_old(payF, o.x);
                                inY = shr_old(payY, o.y);
                            }
                            // Rows without a pair ("no row": before a lane's first row, after a stream's
                            // last) are computed anyway: their halves are garbage that is never read and
                            // is reset by the next first row, and a skip branch cost phi copies of the
                            // whole column state on every step.
                            {
                                if (tq == 0 && (rw & (A2_FIRST | (A2_FIRST << 16)))) AT_DIAG(5, 1);
                                if (rw & (A2_FIRST | (A2_FIRST << 16))) {  // a new pair starts in a stream
                                    uint32_t m = ((rw & A2_FIRST) ? 0xFFFFu : 0u) | ((rw & (A2_FIRST << 16)) ? 0xFFFF0000u : 0u);
                                    int jb = tq * K;
                                    asm volatile("" : "+v"(jb), "+v"(m));
    #pragma unroll
                                    for (int k = 0; k < K; ++k) {
                                        const int g0 = sc.eo + sc.ee * (jb + k) - (jb + k + 1) * dz;
                                        stG[k] = (pk2b(g0, g0) & m) | (stG[k] & ~m);
                                        stX[k] = ((NEG16X2 | ODD) & m) | (stX[k] & ~m);
                                    }
                                    // diagonal of column j0 at row 1 = best of (0, j0 - 1), | 1
                                    // (best-open form: B(0, jb), plain)
                                    const int c0 = RAW ? (jb == 0 ? 0 : sc.eo + sc.ee * (jb - 1) - jb * dz)
                                                       : jb == 0 ? 1 : (sc.eo + sc.ee * (jb - 1) - jb * dz) | 1;
                                    carry = (pk2b(c0, c0) & m) | (carry & ~m);
                                }
                                // substitution words of both rows
                                uint32_t eq0[KW], eq1[KW];
                                {
                                    // the per-thread table address is recomputed here (one op) rather
                                    // than kept live across the chain loop (it was spilled to scratch)
                                    const uint32_t* t0 = eqt[(rw >> 11) & 3u][tq];
                                    const uint32_t* t1 = eqt[(rw >> 27) & 3u][tq];
    #pragma unroll
                                    for (int q = 0; q < KW; ++q) {
                                        eq0[q] = t0[q];
                                        eq1[q] = t1[q];
                                    }
                                }
                                if (rw & (A2_OTHER | (A2_OTHER << 16))) {  // a row byte other than A/C/G/T
                                    const uint8_t* cseq = chs[cur].cseq;
                                    const uint32_t b0 = rw & 0xFFu, b1 = (rw >> 16) & 0xFFu;
    #pragma unroll
                                    for (int q = 0; q < KW; ++q) {
                                        uint32_t v0 = 0u, v1 = 0u;
    #pragma unroll
                                        for (int h = 0; h < 2; ++h) {
                                            const int jc = j0 + 2 * q + h;
                                            const uint32_t cb_ = jc <= nB ? (uint32_t)cseq[jc - 1] : 0u;
                                            const int s0_ = ((cb_ != 0u && cb_ == b0) ? sc.ma : sc.mi) - 2 * dz;
                                            const int s1_ = ((cb_ != 0u && cb_ == b1) ? sc.ma : sc.mi) - 2 * dz;
                                            v0 |= ((uint32_t)s0_ & 0xFFFFu) << (16 * h);
                                            v1 |= ((uint32_t)s1_ & 0xFFFFu) << (16 * h);
                                        }
                                        if (rw & A2_OTHER) eq0[q] = v0;
                                        if (rw & (A2_OTHER << 16)) eq1[q] = v1;
                                    }
                                }
                                // end-gap Iy scores on each stream's last row: io + last * (eo - io) per half,
                                // minus 1 because the F payload is kept odd (below; not in the best-open form)
                                // Formed directly as pk_int words: with l = 1 in each half of a last row,
                                // pk_int(l * d + c per half) = l * d + c * 0x10001 (mod 2^32) -- one 24-bit
                                // multiply-add (d sign-extended from 16 bits) instead of a packed
                                // multiply-add and the three-op pk_int borrow fix-up
                                const uint32_t lastw = (rw >> 9) & 0x00010001u;
                                const uint32_t oy1i = (uint32_t)((int)lastw * (int)(short)(sc.eo - sc.io)) +
                                                      (uint32_t)(sc.io - dz - (RAW ? 0 : 1)) * 0x00010001u;
                                const uint32_t eyi = DEF ? pk_int(pk2(sc.ie, sc.ie))
                                                         : (uint32_t)((int)lastw * (int)(short)(sc.ee - sc.ie)) +
                                                               (uint32_t)sc.ie * 0x00010001u;
                                // Representation (doubled scores): G = max(M, Iy) tagged (M odd, Iy even);
                                // Ix and F = max(M, Ix) kept ODD (2v + 1, no tag): then the diagonal
                                // max(G, Ix) | 1 = max(G | 1, X1) needs no fix-up, Ix candidates built on G | 1
                                // and X1 stay odd and F + (oy - 1) stays even, so no "& ~1" either.  Ties the
                                // tags used to break inside cg - cx and cf - cy now show as 0 signs, and the
                                // walker breaks them with the neighbour's tag (it reads that byte anyway).
                                at_s2 d1 = as_s2(carry);
                                at_s2 F1 = as_s2(inF), Y = as_s2(inY);
                                uint32_t acc[RAW ? K : KW];
                                // TR = false: no lane of the wave stores this step's trace (every block is
                                // outside both streams' bands), so the trace codes are not formed at all --
                                // the same cells, ~13 fewer VALU instructions per cell pair
                                auto cells = [&](auto TR) {
                                if constexpr (RAW) {
                                    // Best-open form (default scores, raw-difference trace).  Opens are no
                                    // cheaper than extends (co, oy <= 0 in drift units), so Ix may open from
                                    // B = max(M, Ix, Iy) instead of max(M, Iy) (Ix + o <= Ix + e), Iy likewise,
                                    // and the diagonal input of the next column is B itself: per cell
                                    //   M = B(i-1, j-1) + s,  X = max(B_up + co_j, X_up),  F = max(M, X),
                                    //   Y = max(F_left + oy_i, Y_left),  B = max(F, Y)
                                    // -- four maxima and no tag fix-ups (Iy keeps Biopython's open from
                                    // M and Ix, F: the left-to-right chain is one maximum per column).  The values of M, Ix and Iy are
                                    // Biopython's, so the walker decides every tie of the first path from
                                    // D1 = M - X and D2 = M - Y (stored as int8; [-9, 17] over every cell of
                                    // the CPU model, tools/proto_bopen.c).  Registers: stG = B, stX = X of
                                    // the previous row, F1 = F and Y of the left column, d1 = diagonal B.
                                    // M of column k from the diagonal B and the substitution halves of column k
                                    // (other scores: a per-half add, the drifted substitution may be negative)
                                    auto mcell = [&](at_s2 diag, int k) {
                                        const uint32_t sel = (k & 1) ? 0x07060302u : 0x05040100u;
                                        const at_s2 sM = as_s2(__builtin_amdgcn_perm(eq1[k / 2], eq0[k / 2], sel));
                                        return DEF ? padd32(diag, as_u32(sM)) : diag + sM;
                                    };
                                    at_s2 Mk = mcell(d1, 0);
    #pragma unroll
                                    for (int k = 0; k < K; ++k) {
                                        const at_s2 Bu = as_s2(stG[k]), Xu = as_s2(stX[k]);
                                        // the next column's M first: B(i-1, k) dies here, so column k's new B
                                        // can take its register
                                        const at_s2 M = Mk;
                                        if (k + 1 < K) Mk = mcell(Bu, k + 1);
                                        // Ix open of column j from LDS (the end-gap score on column nB)
                                        const at_s2 Xn = pmax(padd32(Bu, colc[k][tq]), Xu);
                                        const at_s2 Yn = pmax(padd32(F1, oy1i), Y);  // Iy opens from B
                                        at_s2 Bn;
                                        if constexpr (DEF) {
                                            // max of three normal positive f16 patterns = their unsigned max
                                            uint32_t b3;
                                            asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(b3) : "v"(as_u32(M)), "v"(as_u32(Xn)), "v"(as_u32(Yn)));
                                            Bn = as_s2(b3);
                                        } else {
                                            Bn = pmax(pmax(M, Xn), Yn);
                                        }
                                        if constexpr (decltype(TR)::value) {
                                            // D1 = M - X, D2 = M - Y over both halves with 32-bit subtracts
                                            // (the high half carries the low half's borrow: a2_raw_de)
                                            const uint32_t dD = as_u32(M) - as_u32(Xn);
                                            const uint32_t dE = as_u32(M) - as_u32(Yn);
                                            acc[k] = __builtin_amdgcn_perm(dE, dD, 0x06040200u);
                                        }
                                        d1 = Bu;
                                        stG[k] = as_u32(Bn);
                                        stX[k] = as_u32(Xn);
                                        F1 = Bn;
                                        Y = Yn;
                                    }
                                } else {
    #pragma unroll
                                for (int k = 0; k < K; ++k) {
                                    const at_s2 G = as_s2(stG[k]), X1 = as_s2(stX[k]);
                                    const at_s2 G1 = as_s2(as_u32(G) | 0x00010001u);
                                    const at_s2 nd1 = pmax(G1, X1);
                                    const uint32_t sel = (k & 1) ? 0x07060302u : 0x05040100u;
                                    const at_s2 sM = as_s2(__builtin_amdgcn_perm(eq1[k / 2], eq0[k / 2], sel));
                                    // default scores: both substitution halves are >= 0 (drift), so M is one
                                    // 32-bit add too; other scores may subtract: per-half add
                                    const at_s2 M = DEF ? padd32(d1, as_u32(sM)) : d1 + sM;
                                    const at_s2 cg = padd32(G1, colc[k][tq]);
                                    const at_s2 cx = DEF ? X1 : padd32(X1, colx[DEF ? 0 : k][tq]);  // drift: + ie - dz = 0
                                    const at_s2 Xn1 = pmax(cg, cx);
                                    const at_s2 cf = padd32(F1, oy1i), cy = DEF ? Y : padd32(Y, eyi);
                                    const at_s2 Yn = pmax(cf, cy);
                                    const at_s2 Gn = pmax(M, Yn), Fn1 = pmax(M, Xn1);
                                    if constexpr (decltype(TR)::value && RAW) {
                                        // D = Gn - Xn1, E = Fn1 - Yn over both halves with 32-bit subtracts
                                        // (2.28 cycles, vs 4.09 for v_pk_sub); bytes D lo, D hi, E lo, E hi
                                        const uint32_t dD = as_u32(Gn) - as_u32(Xn1);
                                        const uint32_t dE = as_u32(Fn1) - as_u32(Yn);
                                        acc[k] = __builtin_amdgcn_perm(dE, dD, 0x06040200u);
                                    } else if constexpr (decltype(TR)::value) {
                                    uint32_t code;
                                    if constexpr (DEF) {
                                        // tagF is implied (see the walker); byte = 128 tagG + 16 sc + 4 sb + sa:
                                        // three multiply-adds starting from Gn (at_dec_def)
                                        code = as_u32(pmad4(pmad4(pmad8(Gn, psign(cf - cy)), psign(cg - cx)), pclamp21(Gn - Xn1)));
                                    } else {  // byte = 4 (16 sc + 4 sb + sa) + tags; tagF = M >= Ix  <=>  M - X1 >= 0 (both odd)
                                        const at_s2 t2 = pmad4(pmad4(psign(cf - cy), psign(cg - cx)), pclamp21(Gn - Xn1));
                                        const uint32_t t4 = as_u32(t2 << (at_s2){2, 2});
                                        const uint32_t ge = ~as_u32(M - Xn1) >> 14;  // bit 15 / 31 -> bit 1 / 17
                                        code = t4 | (as_u32(Gn) & 0x00010001u) | (ge & 0x00020002u);
                                    }
                                    if (k % 2 == 0) acc[k / 2] = code;
                                    else acc[k / 2] = __builtin_amdgcn_perm(code, acc[k / 2], 0x06040200u);
                                    }
                                    stG[k] = as_u32(Gn);
                                    stX[k] = as_u32(Xn1);
                                    F1 = Fn1;
                                    Y = Yn;
                                    d1 = nd1;
                                }
                                }
                                };
                                if (!RAW && A2_SKIP_SIGN && !bmask) {
                                    cells(std::false_type{});
                                } else {
                                cells(std::true_type{});
                                if (in_band &&
                                    AT_OK(((size_t)s * NT + tq + 1) * TB <= (size_t)buf_bytes, AG_STORE)) {
                                    // 32-bit offset from the uniform buffer base (one VGPR, saddr store; a
                                    // buffer is at most a few tens of MB)
                                    uint32_t* dst = (uint32_t*)(trb + (((uint32_t)s * NT + (uint32_t)tq) * (uint32_t)TB));
                                    if (tq == 0) AT_DIAG(2, 1);
                                    if constexpr (RAW && K % 4 == 0) {
    #pragma unroll
                                        for (int q = 0; q < K / 4; ++q)
                                            ((uint4*)dst)[q] = make_uint4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                                    } else if constexpr (RAW) {
    #pragma unroll
                                        for (int q = 0; q < K / 2; ++q) ((uint2*)dst)[q] = make_uint2(acc[2 * q], acc[2 * q + 1]);
                                    } else if constexpr (K == 16) {
                                        ((uint4*)dst)[0] = make_uint4(acc[0], acc[1], acc[2], acc[3]);
                                        ((uint4*)dst)[1] = make_uint4(acc[4], acc[5], acc[6], acc[7]);
                                    } else if constexpr (K == 8) {
                                        *(uint4*)dst = make_uint4(acc[0], acc[1], acc[2], acc[3]);
                                    } else {
    #pragma unroll
                                        for (int q = 0; q < KW; ++q) dst[q] = acc[q];
                                    }
                                }
                                }
                                const at_s2 F = F1;
                                payF = as_u32(F);
                                payY = as_u32(Y);
                                if constexpr (decltype(HO)::value)
                                    if (ln == 63) ring_out[(g + 1) & (RING - 1)] = make_uint2(payF, payY);
                                if ((rw & (A2_LAST | (A2_LAST << 16))) && tq == (nB - 1) / K) {  // owner of column nB
                                    const int out_k = (nB - 1) % K;
                                    uint32_t eG = stG[0], eX = stX[0];
    #pragma unroll
                                    for (int k = 1; k < K; ++k) {
                                        uint32_t m = (k == out_k) ? ~0u : 0u;
                                        asm volatile("" : "+v"(m));
                                        eG = (stG[k] & m) | (eG & ~m);
                                        eX = (stX[k] & m) | (eX & ~m);
                                    }
                                    const at_s2 e = RAW ? as_s2(eG) : pmax(as_s2(eG), as_s2(eX));  // best of (nA, nB)
                                    if (rw & (A2_LAST | (A2_LAST << 16))) AT_DIAG(3, 1);
                                    const uint32_t eu = as_u32(e);  // unbias the final cells
                                    if ((rw & A2_LAST) && AT_OK(2 * fin_n[0] < AT2_CHUNK, AG_FIN))
                                        fin[cur][2 * fin_n[0]++] = (int)(eu & 0xFFFFu) - BIAS16;
                                    if ((rw & (A2_LAST << 16)) && AT_OK(2 * fin_n[1] + 1 < AT2_CHUNK, AG_FIN))
                                        fin[cur][2 * fin_n[1]++ + 1] = (int)(eu >> 16) - BIAS16;
                                }
                            }
                            // best of (i, j0 - 1) (| 1 in the tagged forms): the next row's diagonal
                            if constexpr (RAW) carry = inF;
                            else carry = as_u32(pmax(as_s2(inF), as_s2(inY))) | 0x00010001u;
            };

            const int rmax = max(rows0, rows1);
            const int nsteps = rmax + 63;
            const int nblk = (nsteps + INTERVAL - 1) / INTERVAL;
            const int nint = nblk + WAVE_LAG * (W - 1);
            for (int it = 0; it < nint; ++it) {
                if constexpr (IS_W) {
                    walk(pb, hops, W * (it + 1));
                } else {
                    const int blk = it - WAVE_LAG * w;
                    if (blk >= 0 && blk < nblk) {
                        const int s0 = blk * INTERVAL;
                        const int s1 = min(s0 + INTERVAL, nsteps);
                        if (w == 0) {
                            for (int s = s0; s < s1; ++s) step(std::true_type{}, std::integral_constant<bool, (W > 1)>{}, s);
                        } else if (w == W - 1) {
                            // no vector memory in flight into the last wave's step loop (a scratch reload
                            // of a register it writes would cost a vmcnt(0) inside every step; gfx9
                            // encoding: vmcnt 0, expcnt 7, lgkmcnt 15).  Only there: the same wait before
                            // every role's loop changes the register assignment and brings it back.
                            __builtin_amdgcn_s_waitcnt(0x0F70);
                            for (int s = s0; s < s1; ++s) step(std::false_type{}, std::false_type{}, s);
                        } else {
                            for (int s = s0; s < s1; ++s) step(std::false_type{}, std::true_type{}, s);
                        }
                    }
                }
                const int gpre = (it + 1) * INTERVAL + tid;
                if (tid < INTERVAL && it + 1 < nblk) xinfo[gpre & (XR - 1)] = a2_row_record(tab[cur], n, rows0, rows1, gpre, nB, band, K);
                if (it + 1 == nint) __builtin_amdgcn_s_waitcnt(0);
                if (!IS_W && lane == 0) atomicAdd(&s_fill, 1);  // this fill wave is done with interval it
                __syncthreads();
            }
            if constexpr (IS_W) walk(pb, -1, 0);
            prev_n = n;
            cur ^= 1;
        }
    };
    if (walker) chain_loop(std::true_type{});
    else chain_loop(std::false_type{});
}

// The band pass (every pair of the launch, trace strip of half-width `band`; 0 = full trace) ...
// RAWT: the best-open fill with the raw-difference trace (default scores on W <= 2; other scores whose
// opens are no better than their extends, capi.hip pick_variantt2), else the tagged fill with sign digits
template <int K, int W, bool DEF, int OCC, bool RAWT = a2_raw<W, DEF>()>
__global__ void __launch_bounds__(64 * (W + 1), OCC)
k_alignt2(SetView XS, SetView YS, PairSrc ps, KScores scin, MetricSpec ms, int chunk_req, int out_mode,
          double* __restrict__ out, int32_t* __restrict__ sout, uint8_t* __restrict__ trace, int64_t buf_bytes,
          int cap_rows, int hops, unsigned long long* __restrict__ next, int band, int64_t* __restrict__ esc_list,
          unsigned long long* __restrict__ esc_n, StrOut so) {
    alignt2_body<K, W, DEF, RAWT>(XS, YS, ps, scin, ms, chunk_req, out_mode, out, sout, trace, buf_bytes, cap_rows,
                                 hops, next, band, esc_list, esc_n, so);
}
// ... and the full-trace pass over the pairs it queued (ps.sel / ps.dcount): a kernel of its own
// name, so a profile shows the second pass (normally empty) apart from the first.  It stores the
// sign-digit code, which is exact for any scores, so a pair queued by a raw walk's score check
// cannot fail again.
template <int K, int W, bool DEF, int OCC>
__global__ void __launch_bounds__(64 * (W + 1), OCC)
k_alignt2_queued(SetView XS, SetView YS, PairSrc ps, KScores scin, MetricSpec ms, int chunk_req, int out_mode,
                 double* __restrict__ out, int32_t* __restrict__ sout, uint8_t* __restrict__ trace, int64_t buf_bytes,
                 int cap_rows, int hops, unsigned long long* __restrict__ next, StrOut so) {
    // nothing queued (the usual case): leave before any set-up -- the full body's prologue over the
    // resident grid cost ~1 ms per launch (1 % of the config-3 step) with an empty queue
    if (ps.dcount && *ps.dcount == 0) return;
    alignt2_body<K, W, DEF, false>(XS, YS, ps, scin, ms, chunk_req, out_mode, out, sout, trace, buf_bytes, cap_rows,
                                   hops, next, 0, nullptr, nullptr, so);
}

}  // namespace taxi2
