// Row-shared packed aligner (default scores): the packed trace-and-walk fill of alignt2_kernel.hpp
// with the two 16-bit halves of every register holding two pairs that share their ROW sequence
// instead of their column sequence.
//
// Why.  In k_alignt2 a lane's two halves are two different row sequences against the same column
// sequence, so the substitution score of a cell pair needs a v_perm per column (the two halves'
// fields come from two different table rows) -- one of the ten VALU instructions per column pair,
// and a 4.09-cycle one.  Here the halves are two column sequences x0, x1 against one row sequence
// y: the table word eqt[base(y_i)][lane][k] already holds (s(x0_k, y_i), s(x1_k, y_i)), so M is one
// 32-bit add of an LDS word, and everything per row (the record, first / last row, the row byte,
// the end-gap Iy open) is ONE value for both halves.
//
// Column shift.  Half h's columns are shifted right by off_h = (K - nB_h % K) % K virtual
// columns, so that its last column nB_h sits in the last slot of its lane.  Then the Ix open
// constant is the internal one on every slot but the last (an inline constant: no per-column LDS
// constants), and column nB's readout is slot K - 1 (no dynamic select).  The off_h leading
// "pre-columns" reproduce the column-0 boundary exactly: with default scores in drift coordinates
// (cells hold V(i, j) - (i + j) ie) the boundary is B(i, 0) = 0, Iy(i, 0) = -inf, and a pre-column
// with substitution 0 and the internal open keeps B = 0 on every row (M = B(i-1, c-1) + 0 = 0,
// Ix <= -7, Iy = the row's Iy open <= 0), while its Iy = oy reaches the first real column as the
// same Iy(i, 1) = max(B(i, 0) + oy, Iy(i, 0)) = oy the boundary gives.
//
// Work.  The host cuts the launch's pairs into segments of (x0, x1, consecutive y) with both pairs
// (x_h, y) in the launch (x1 = -1: one pair per unit, the other half idle); a unit = one y and its
// one or two pairs.  A chain = up to AR_UNITS consecutive units of one segment: the units' rows
// stream back to back through the systolic layout of alignt2_kernel.hpp (two fill waves, one
// walker wave, raw-difference trace, best-open fill, the f16 maximum3 best state).  Walks, trace
// band, escape queue and the walkers' score check are alignt2_kernel.hpp's; queued pairs are redone
// by k_alignt2_queued over the launch's PairSrc (the pair indices are the same).
#pragma once
#include "alignt2_kernel.hpp"

namespace taxi2 {

// steps between the fill waves' progress checks / publications (a divisor of INTERVAL). Config-3
// launch time, one box: 8 -> 96.7 ms, 16 -> 93.8, 32 -> 92.5; another box: 16 -> 95.3, 32 -> 94.5,
// 64 -> 95.2 (ring 256, profiles/r5/ar_blk/); with the 512-row ring, 32 -> 91.7 and 64 -> 91.2 ms, same-box
// A/B x3 (profiles/r5/ar_blk/ring512_*)
#ifndef TAXI2_AR_BLK
#define TAXI2_AR_BLK 64
#endif
constexpr int AR_BLK = TAXI2_AR_BLK;
// Rows buffered between the fill waves (the ring) and how far wave 0 may run ahead of wave 1: wave 0
// rewrites a ring slot AR_RING - 63 steps after wave 1 read it, and the row record of row r
// (XR = 512 slots, written up to 64 rows ahead) AR_XR - 64 - 63 rows after wave 1's oldest use.
// Ring 256 -> 512 (4 KB of LDS per workgroup, AR_AHEAD 193 -> 353): 92.9 -> 92.3 ms per config-3
// launch, same-box A/B x3 (profiles/r5/ar_ring/).
#ifndef TAXI2_AR_RING
#define TAXI2_AR_RING 512
#endif
constexpr int AR_RING = TAXI2_AR_RING;
constexpr int AR_AHEAD = (AR_RING - 63) < (512 - 64 - 63 - AR_BLK) ? (AR_RING - 63) : (512 - 64 - 63 - AR_BLK);
// Liveness of the two fill waves' pacing (the step loop's waits): wave 1 finishing block k needs
// wave 0 through step (k + 1) AR_BLK + 63, published at the block end after it; wave 0 may start that
// block only while it is at most AR_AHEAD steps ahead of wave 1's published k AR_BLK.  A ring of 128
// (AR_AHEAD 65 < 96 at AR_BLK 32) deadlocks on the GPU.
static_assert(AR_AHEAD >= AR_BLK * (1 + (63 + AR_BLK - 1) / AR_BLK), "fill waves would deadlock");
#ifndef TAXI2_AR_UNITS
#define TAXI2_AR_UNITS 8
#endif
constexpr int AR_UNITS = TAXI2_AR_UNITS;  // units (row sequences, up to two pairs each) per chain
// Trace layout.  AR_TS = 0 (default): [step][lane][4K bytes], a lane's K columns contiguous.
// AR_TS >= 1: the columns are cut into pieces of ar_pw(K) columns (16 bytes for K % 4 == 0), and
// piece q of all lanes over AR_TS consecutive steps is one run, [step / AR_TS][piece][lane][step %
// AR_TS][piece bytes], so that the walker's diagonal hops (one step back per hop within a lane) share
// a line for AR_TS hops.  Measured at config 3, band 64: AR_TS = 2 cuts the walker's
// fetch from 110 to 74 KB per pair but the fill is 1 % slower; AR_TS = 1 is 11 % and AR_TS = 4
// (42 KB per pair) 17 % slower -- the fill's stores, not the walker's reads, set the cost.
#ifndef TAXI2_AR_TS
#define TAXI2_AR_TS 0
#endif
constexpr int AR_TS = TAXI2_AR_TS;
// wave-uniform skip of the trace VALU on steps with no lane in the band (see the step's cells)
#ifndef TAXI2_AR_SKIP
#define TAXI2_AR_SKIP 0
#endif
constexpr bool AR_SKIP = TAXI2_AR_SKIP != 0;
// prefetch of the next step's table offset (see the fill's step loop): off -- the extra live register
// takes the kernel to 130 VGPRs, i.e. 3 waves per SIMD instead of 4 (tools/isa_alignr.hip)
#ifndef TAXI2_AR_PREC
#define TAXI2_AR_PREC 0
#endif
constexpr bool AR_PREC = TAXI2_AR_PREC != 0;
__host__ __device__ constexpr int ar_pw(int K) { return K % 4 == 0 ? 4 : 2; }
// byte offset of (step, lane, column k) in a chain's trace buffer (NT lanes)
// (AR_TS = 0: the plain [step][lane][4K bytes] layout, for comparison)
template <int K, int NT>
__device__ __forceinline__ uint32_t ar_trace_step_off(uint32_t step) {  // of (step, lane 0, column 0)
    constexpr uint32_t PW = ar_pw(K), PB = 4 * PW, NP = K / PW;
    if constexpr (AR_TS == 0) return step * (NT * 4 * K);
    else return (step / AR_TS) * (NP * NT * AR_TS * PB) + (step % AR_TS) * PB;
}
template <int K> constexpr uint32_t ar_lane_bytes() { return AR_TS == 0 ? 4 * K : AR_TS * 4 * ar_pw(K); }
template <int K, int NT> constexpr uint32_t ar_piece_stride() { return AR_TS == 0 ? 4 * ar_pw(K) : NT * AR_TS * 4 * ar_pw(K); }
template <int K, int NT>
__device__ __forceinline__ uint32_t ar_trace_off(uint32_t step, uint32_t lane, uint32_t k) {
    constexpr uint32_t PW = ar_pw(K);
    return ar_trace_step_off<K, NT>(step) + lane * ar_lane_bytes<K>() + (k / PW) * ar_piece_stride<K, NT>() + (k % PW) * 4;
}
// trace buffer rows for a chain of `rows` rows: steps up to rows + 62, rounded up to whole blocks
__host__ __device__ constexpr int ar_trace_rows(int rows) { return rows + 64 + AR_TS; }

// Profiling build only (-DAR_PROF, `make variant VNAME=arprof VFLAGS=-DAR_PROF`): per-wave s_memtime
// totals of the launch -- [0] fill step loops, [1] fill chain-end barrier, [2] chain set-up (cut,
// tables, first barrier), [3] walker walking, [4] fill waits for the other fill wave, [5] walker
// chain-end barrier, [6] chains
#ifdef AR_PROF
__device__ unsigned long long ar_prof[8];
#define AR_NOW() __builtin_amdgcn_s_memtime()
#endif

// Host-built segment: units u0 .. u0 + nb - 1 are (x0, x1, y = b0 + (u - u0)); pair (x_h, y) has
// launch index p_h + (u - u0) (x1 = -1, p1 = -1: one pair per unit).
// Swapped segment (sw = number of pairs > 0): the pairs (x0, y) of ONE row, y = b0 .. b0 + sw - 1 at
// launch indices p0 .. p0 + sw - 1, which no second row shares (a launch with an odd number of rows
// over these columns).  Unit du is the row sequence x0 against the two column sequences y = b0 +
// 2 du and b0 + 2 du + 1 -- both halves busy, where a (x0, -1, y) unit idles one -- and is a chain of
// its own (a chain keeps its column sequences).
struct ArSeg {
    int64_t x0, x1, b0, nb, p0, p1, u0, sw;
};

struct ArRow {  // one unit of a chain: its row sequence and pairs
    const uint8_t* rseq;
    int64_t p[2];  // launch index of pair (x_h, y); -1: idle half
    int nA, fx, lx, r0;
};
struct ArChain {
    const uint8_t* cseq[2];
    int nB[2], fy[2], ly[2], off[2];
    int n;
    int swp;  // 1: the rows are the pairs' FIRST sequence (a swapped segment's unit)
};
struct ArWalk {
    int i, j, st, first, t, h, prio;
    uint32_t xa, yb;
    int valid, ts, tv, gap, sc2, ncol;
};

// Row record (LDS, one per chain row): .x = byte offset of the row base's table (eqt) for an
// A/C/G/T byte, .y = band lo (byte 0) and width (byte 1) in lanes, the row byte (byte 2) and flags,
// .z = the row's Iy open as a pk_int addend (the "open-shifted" cells below), .w = the column-0
// boundary B(i, 0) = 0 in that form.
constexpr uint32_t AR_PRE = 1u << 31;    // first or last row of a unit, or a byte other than A/C/G/T
constexpr uint32_t AR_LAST = 1u << 30;   // last row of a unit
constexpr uint32_t AR_FIRST = 1u << 29;  // first row of a unit
constexpr uint32_t AR_OTHER = 1u << 28;  // byte other than A/C/G/T (byte-compare substitution)
constexpr uint32_t AR_NOBAND = 0x0080u;  // lo 128, width 0: no lane stores

// Default scores in drift coordinates (dz = ie = -1): substitution ma - 2 dz / mi - 2 dz, opens
// relative to the extend, the column-0 / row-0 boundary 0.
//
// Open-shifted cells.  The state kept per cell is G = B + o_i (the best score plus the row's Iy
// open) instead of B: then Ix(i, j) = max(G(i-1, j), Ix(i-1, j)) and Iy(i, j) = max(G(i, j-1),
// Iy(i, j-1)) need no add, and M(i, j) = G(i-1, j-1) + (s - co_i) takes the open into the table
// word -- one add per cell (G = B + o_i) instead of two (B + co for Ix and for Iy).  o_i is the
// internal open except on a unit's last row (the end-gap open), whose G feeds nothing but its own
// row's Iy (the next row is a unit's first, whose states are reset).  The end column's Ix open
// (slot K - 1 of its owner lane) adds cend - co_i once per step.  M, Ix, Iy and the trace are the
// same values as before; only the stored best is shifted.
constexpr int AR_EQ_MATCH = 3, AR_EQ_MISMATCH = 1, AR_CO_I = -7, AR_CO_E = 0;

__device__ __forceinline__ uint32_t ar_pk_int(int lo, int hi) { return pk_int(pk2(lo, hi)); }

// 8 bytes at any byte address (one unaligned global store)
__device__ __forceinline__ void ar_store8(uint8_t* p, uint64_t v) { __builtin_memcpy(p, &v, 8); }

// band lanes [lo, hi] of row i (1-based) of a pair with nA rows and nB columns, shifted by off;
// lo > hi: none (a2_band_blocks in virtual columns)
__device__ __forceinline__ void ar_band_lanes(int i, int nA, int nB, int off, int band, int K, int& lo, int& hi) {
    int jl, jh;
    if (band <= 0) {
        jl = 1;
        jh = nB;
    } else {
        jl = max(1, i + min(0, nB - nA) - band);
        jh = min(nB, i + max(0, nB - nA) + band);
    }
    lo = (jl + off - 1) / K;
    hi = (jh + off - 1) / K;
}

// the .z / .w words of a record: the row's open (pk_int) and B = 0 shifted by it (a biased pattern)
__device__ __forceinline__ uint4 ar_record(uint32_t x, uint32_t y, bool last) {
    const uint32_t o = last ? ar_pk_int(AR_CO_E, AR_CO_E) : ar_pk_int(AR_CO_I, AR_CO_I);
    return make_uint4(x, y, o, pk2b(0, 0) + o);
}

template <int K, int W>
__device__ __forceinline__ uint4 ar_row_record(const ArRow* __restrict__ tab, const ArChain& ch, int n, int rows, int g,
                                               int band) {
    constexpr int NT = 64 * W;
    if (g < 0 || g >= rows) return ar_record(0u, AR_NOBAND, false);
    int t = 0;
    for (int q = 1; q < n; ++q)
        if (tab[q].r0 <= g) t = q;
    const ArRow& r = tab[t];
    const int i = g - r.r0;  // 0-based row of the unit
    const uint32_t c = r.rseq[i];
    const uint32_t ec = c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
    uint32_t y = c << 16;
    uint32_t x = 0u;
    if (ec < 4u) x = ec * (uint32_t)(NT * K * 4);
    else y |= AR_OTHER | AR_PRE;
    if (i == 0) y |= AR_FIRST | AR_PRE;
    if (i == r.nA - 1) y |= AR_LAST | AR_PRE;
    int lo = 0x7FFF, hi = -1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (r.p[h] < 0) continue;
        int l, u;
        ar_band_lanes(i + 1, r.nA, ch.nB[h], ch.off[h], band, K, l, u);
        lo = min(lo, l);
        hi = max(hi, u);
    }
    y |= hi < lo ? AR_NOBAND : ((uint32_t)lo | ((uint32_t)(hi - lo) << 8));
    return ar_record(x, y, i == r.nA - 1);
}

// <= 128 VGPRs: 4 waves per SIMD, so that the 5 workgroups of 3 waves the LDS allows fit a CU (the
// launch bound alone lets the allocator take more and lose a workgroup per CU)
template <int K, int W, int OCC>
__global__ void __launch_bounds__(64 * (W + 1), OCC) __attribute__((amdgpu_num_vgpr(128)))
k_alignr(SetView XS, SetView YS, const ArSeg* __restrict__ segs, int nseg, int64_t total, int64_t npairs,
         MetricSpec ms, int chunk_req, int out_mode, double* __restrict__ out, int32_t* __restrict__ sout,
         uint8_t* __restrict__ trace, int64_t buf_bytes, int cap_rows, unsigned long long* __restrict__ next,
         int band, int64_t* __restrict__ esc_list, unsigned long long* __restrict__ esc_n, StrOut so) {
    static_assert(K % 2 == 0 && K <= 8 && W <= 2, "row-shared shapes: K <= 8 columns per lane, one or two fill waves");
    constexpr int NT = 64 * W;
    constexpr int XR = a1c_xr(W);
    constexpr int dz = -1;                          // default scores: ie
    const KScores sc{1, -1, -8, -1, -1, -1};        // align.py:20-27 defaults
    constexpr int NW = 4 * AR_UNITS;                // walks per chain (both orientations of 2 pairs per unit)
    __shared__ uint4 xinfo[XR];
    __shared__ ArRow tab[2][AR_UNITS];
    __shared__ ArChain chs[2];
    __shared__ int fin[2][AR_UNITS][2];
    __shared__ uint2 ring[(W > 1 ? W - 1 : 1) * AR_RING];
    // (s(x0_k, base), s(x1_k, base)) - co_i as pk_int, per lane and slot, in pieces of EP slots:
    // eqt[base][k / EP][lane][k % EP], so that the step's vector reads (EP words per lane) are
    // lane-contiguous -- a lane-major [lane][K] row (32 bytes per lane at K = 8) made every 16-byte
    // read a 2-way bank conflict (1.64 conflict cycles per LDS instruction)
    constexpr int EP = ar_pw(K);
    __shared__ uint32_t eqt[4][K / EP][NT][EP];
    __shared__ int64_t s_qc, s_qend;
    __shared__ int s_n, s_rows, s_seg;
    __shared__ int s_prog[2];  // steps completed by each fill wave in the current chain
    __shared__ ArWalk wks[NW];
    __shared__ int escf[2][AR_UNITS][2];

    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool walker = w == W;
    const int nm = ms.n;
    const int64_t chunk = chunk_req >= 1 ? min((int64_t)chunk_req, (int64_t)AR_UNITS)
                                         : max((int64_t)1, min((int64_t)AR_UNITS, total / ((int64_t)gridDim.x * 8)));
    uint8_t* const bufs = trace + (size_t)blockIdx.x * 2 * (size_t)buf_bytes;
    if (tid == 0) {
        s_qc = 0;
        s_qend = 0;
        s_seg = 0;
    }
    int cur = 0, prev_n = 0;

    // outputs of a pair with an empty side (no fill): metrics of no columns, the end-gap score,
    // the other sequence against gaps as its alignment (both orientation slots alike)
    auto empty_pair = [&](int64_t p, const uint8_t* xs_, int lx_, const uint8_t* ys_, int ly_) {
        for (int m = 0; m < nm; ++m) {
            const double v = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
            if (out_mode == OUT_BOTH) {
                out[(p * 2 + 0) * nm + m] = v;
                out[(p * 2 + 1) * nm + m] = v;
            } else {
                out[p * nm + m] = v;
            }
        }
        const int ne = lx_ + ly_;
        if (sout) sout[p] = ne == 0 ? 0 : sc.eo + sc.ee * (ne - 1);
        if (so.sx) {
            for (int o = 0; o < so.nslot; ++o) {
                uint8_t* ox = so.sx + ((size_t)p * so.nslot + o) * (size_t)so.cap;
                uint8_t* oy = so.sy + ((size_t)p * so.nslot + o) * (size_t)so.cap;
                for (int t = 0; t < ne; ++t) {
                    ox[t] = lx_ ? xs_[t] : (uint8_t)'-';
                    oy[t] = ly_ ? ys_[t] : (uint8_t)'-';
                }
                so.slen[p * so.nslot + o] = ne;
            }
        }
    };

    // walk slot q of the chain in buffer pb: unit q % n, half (q / n) & 1, orientation q / 2n (both)
    auto walk_init = [&](int pb, int n) {
        if (lane >= NW) return;
        ArWalk& W_ = wks[lane];
        W_ = ArWalk{0, 0, AT_DONE, 0, 0, 0, 0, 0u, 0u, 0, 0, 0, 0, 0, 0};
        if (lane < AR_UNITS * 2) escf[pb][lane >> 1][lane & 1] = 0;
        const int nw = (out_mode == OUT_BOTH ? 4 : 2) * n;
        if (lane < nw) {
            const int t = lane % n, h = (lane / n) & 1, o = lane / (2 * n);
            const ArRow& r = tab[pb][t];
            if (r.p[h] >= 0) {
                W_.t = t;
                W_.h = h;
                // rows = y, the pair's second sequence: orientation A (prio 0) is (y, x) = slot 1; in a
                // swapped chain the rows are x and the pair's own orientation (x, y) is prio 0
                W_.prio = out_mode == OUT_BOTH ? o : (chs[pb].swp ? 0 : 1);
                W_.i = r.nA + 1;
                W_.j = chs[pb].nB[h] + 1;
                W_.st = AT_M;
                W_.first = 1;
            }
        }
    };

    // branch-free best-open walker (alignt2_kernel.hpp walk_run_raw), per-half column sequence and
    // shift; walks the chain in buffer pb to the end.  Aligned strings (so.sx): each walk keeps the
    // last 8 columns it produced in a 64-bit window per string and stores the window (8 bytes,
    // unaligned) every 8 columns and at the walk's end -- not a byte store per column and string
    auto walk = [&](int pb) {
        ArWalk& W_ = wks[lane < NW ? lane : 0];
        int st = lane < NW ? W_.st : AT_DONE;
        if (!__any(st != AT_DONE)) return;
        const int t = W_.t, h = W_.h, prio = W_.prio;
        const ArRow& r = tab[pb][t];
        const ArChain& ch = chs[pb];
        const int nA_ = r.nA, nB_ = ch.nB[h], off = ch.off[h];
        const int fx = r.fx, lx = r.lx, fy = ch.fy[h], ly = ch.ly[h], r0 = r.r0;
        const int64_t p = r.p[h];
        const int bdl = min(0, nB_ - nA_) - band;
        const uint32_t bwd = (uint32_t)(abs(nB_ - nA_) + 2 * band);
        const uint8_t* rs = r.rseq;
        const uint8_t* cs = ch.cseq[h];
        const uint8_t* trb = bufs + (size_t)pb * (size_t)buf_bytes;
        int i = W_.i, j = W_.j, first = W_.first;
        uint32_t xa = W_.xa, yb = W_.yb;
        int valid = W_.valid, ts = W_.ts, tv = W_.tv, gap = W_.gap, sc2 = W_.sc2, ncol = W_.ncol;
        uint64_t wx = 0, wy = 0;  // string windows (column, row sequence): bits 0-7 = the last column produced
        const int co_i = sc.io - sc.ie, co_e = sc.eo - sc.ee;
        const int bsh = h ? 8 : 0;
        // rows are the pair's second sequence (orientation A = (y, x), prio 0, is slot 1), or its
        // first in a swapped chain (prio 0 is then slot 0)
        const int oslot = ch.swp ? prio : prio ^ 1;
        const size_t sbase = so.sx ? ((size_t)p * so.nslot + (oslot & (so.nslot - 1))) * (size_t)so.cap : 0;
        // the string of the column sequence and of the row sequence: x = the pair's first
        uint8_t* const dcol = ch.swp ? so.sy : so.sx;
        uint8_t* const drow = ch.swp ? so.sx : so.sy;
        for (;;) {
            if (!__any(st < AT_DONE)) break;
            if (st < AT_DONE) {
                const bool isM = st == AT_M, isX = st == AT_IX, isY = st == AT_IY;
                const uint32_t bx = a2_wcode(xa), by = a2_wcode(yb);
                const uint32_t dd = bx ^ by;
                const bool cnt = isM && !first && (bx | by) < 4u;
                valid += cnt;
                ts += cnt && dd == 3u;
                tv += cnt && (dd == 1u || dd == 2u);
                gap += (isX && bx < 4 && j - 1 >= fy && j <= ly) || (isY && by < 4 && i - 1 >= fx && i <= lx);
                sc2 += (isM && !first) ? (xa == yb ? sc.ma : sc.mi) : 0;
                const int ni = isY ? i : i - 1, nj = isX ? j : j - 1;
                if (so.sx && !first) {  // this column of the alignment, right to left
                    const uint32_t rc = isY ? (uint32_t)'-' : xa, cc = isX ? (uint32_t)'-' : yb;
                    wx = (wx << 8) | cc;
                    wy = (wy << 8) | rc;
                    ++ncol;
                    if ((ncol & 7) == 0) {  // columns [E - ncol, E - ncol + 8) of the slot (E = nA + nB)
                        const size_t o = sbase + (size_t)(nA_ + nB_ - ncol);
                        ar_store8(dcol + o, wx);
                        ar_store8(drow + o, wy);
                    }
                }
                first = 0;
                if (ni == 0 && nj == 0) {
                    if (!isM) sc2 += sc.eo;
                    if (sc2 != fin[pb][t][h] + (nA_ + nB_) * dz) {
                        st = AT_ESC;
                    } else {
                        double* o = out_mode == OUT_BOTH ? out + (p * 2 + oslot) * nm : out + p * nm;
                        for (int m = 0; m < nm; ++m)
                            o[m] = metric_value(ms.code[m], (uint32_t)valid, (uint32_t)ts, (uint32_t)tv, (uint32_t)gap);
                        if (sout && (out_mode != OUT_BOTH || oslot == 0)) sout[p] = fin[pb][t][h] + (nA_ + nB_) * dz;
                        if (so.slen) so.slen[p * so.nslot + (oslot & (so.nslot - 1))] = ncol;
                        if (so.sx && (ncol & 7)) {  // the columns since the last window store
                            const size_t o = sbase + (size_t)(nA_ + nB_ - ncol);
                            if (ncol >= 8) {  // the window's older bytes are already in place
                                ar_store8(dcol + o, wx);
                                ar_store8(drow + o, wy);
                            } else {
                                for (int q = 0; q < ncol; ++q) {
                                    dcol[o + q] = (uint8_t)(wx >> (8 * q));
                                    drow[o + q] = (uint8_t)(wy >> (8 * q));
                                }
                            }
                        }
                        st = AT_DONE;
                    }
                } else {
                    const bool in = ni >= 1 && nj >= 1;
                    const bool esc = in && band > 0 && (uint32_t)(nj - ni - bdl) > bwd;
                    const int cj = max(nj, 1) - 1 + off, ci = max(ni, 1) - 1;  // virtual column of (ni, nj) - 1
                    const uint32_t tl = (uint32_t)cj / K, k = (uint32_t)cj - tl * K;
                    const uint32_t toff = ar_trace_off<K, NT>((uint32_t)(r0 + ci) + (tl & 63u), tl, k);
                    const uint32_t xa_ = a2_load_byte(rs + ci), yb_ = a2_load_byte(cs + max(nj, 1) - 1);
                    const uint32_t nb = a2_load_trace32(trb + toff);
                    xa = ni >= 1 ? xa_ : 0u;
                    yb = nj >= 1 ? yb_ : 0u;
                    const int d1v = (int)(int8_t)(uint8_t)((nb >> bsh) + (h ? ((nb >> 7) & 1u) : 0u));
                    const int d2v = (int)(int8_t)(uint8_t)((nb >> (16 + bsh)) + (h ? ((nb >> 23) & 1u) : 0u));
                    const int co = j == nB_ ? co_e : co_i, oy = i == nA_ ? co_e : co_i;
                    const int vM = d1v + (isX ? co : 0);
                    const int vY = d1v - d2v + (isX ? co : isY ? -oy : 0);
                    const int vm = max(max(vM, vY), 0);
                    int nst = vM == vm ? AT_M : prio ? (vY == vm ? AT_IY : AT_IX) : (vm == 0 ? AT_IX : AT_IY);
                    nst = ni == 0 ? AT_IY : nj == 0 ? AT_IX : nst;
                    const bool ext = isX ? nst == AT_IX : nst == AT_IY;
                    const bool en = isX ? (j == nB_ || j == 0) : (i == nA_ || i == 0);
                    sc2 += isM ? 0 : ext ? (en ? sc.ee : sc.ie) : (en ? sc.eo : sc.io);
                    i = ni;
                    j = nj;
                    st = esc ? AT_ESC : nst;
                }
            }
        }
        if (st == AT_ESC) {  // queue the pair (once) for the full-trace pass (k_alignt2_queued)
            if (atomicOr(&escf[pb][t][h], 1) == 0 && esc_list) esc_list[atomicAdd(esc_n, 1ull)] = p;
            st = AT_DONE;
        }
        if (lane >= NW) return;
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

    auto chain_loop = [&](auto WK) {
        constexpr bool IS_W = decltype(WK)::value;
#ifdef AR_PROF
        unsigned long long pf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        unsigned long long tA = AR_NOW();
#endif
        for (;;) {
            // ---- cut the next chain (thread 0): up to AR_UNITS units of one segment
            __syncthreads();
            if (!IS_W && tid == 0) {
                int n = 0, rows = 0;
                while (n == 0) {
                    if (s_qc >= s_qend) {
                        // guided: shorter chains once fewer than two rounds of full ones are left, so
                        // that the workgroups finish closer together (the launch's tail)
                        int64_t c = chunk;
                        const int64_t left =
                            total - (int64_t)__hip_atomic_load(next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (left < (int64_t)gridDim.x * chunk * 2) c = max((int64_t)1, chunk / 2);
                        if (left < (int64_t)gridDim.x * chunk) c = max((int64_t)1, chunk / 4);
                        const int64_t q0 = (int64_t)atomicAdd(next, (unsigned long long)c);
                        if (q0 >= total) break;
                        s_qc = q0;
                        s_qend = min(q0 + c, total);
                        // segment of unit q0 (binary search; units run in segment order)
                        int lo = 0, hi = nseg - 1;
                        while (lo < hi) {
                            const int mid = (lo + hi + 1) >> 1;
                            if (segs[mid].u0 <= q0) lo = mid;
                            else hi = mid - 1;
                        }
                        s_seg = lo;
                    }
                    int64_t q = s_qc;
                    for (; q < s_qend; ++q) {
                        int sg = s_seg;
                        while (sg + 1 < nseg && segs[sg + 1].u0 <= q) ++sg;
                        if (n > 0 && sg != s_seg) break;  // a chain keeps one segment's columns
                        s_seg = sg;
                        const ArSeg S = segs[sg];
                        if (S.sw > 0) {  // swapped: row x0 against columns b0 + 2 du (+ 1), a chain of its own
                            if (n > 0) break;
                            const int64_t du = q - S.u0;
                            const int4 mr = XS.meta[S.x0];
                            const uint8_t* xr_ = XS.bytes + XS.offs[S.x0];
                            int64_t ph[2];
                            int4 mc[2];
                            const uint8_t* cs_[2];
                            bool live[2];
#pragma unroll
                            for (int hh = 0; hh < 2; ++hh) {
                                const int64_t k = 2 * du + hh;
                                ph[hh] = k < S.sw ? S.p0 + k : -1;
                                live[hh] = ph[hh] >= 0;
                                mc[hh] = live[hh] ? YS.meta[S.b0 + k] : make_int4(0, 0, 0, 0);
                                cs_[hh] = live[hh] ? YS.bytes + YS.offs[S.b0 + k] : YS.bytes;
                                if (live[hh] && (mc[hh].x == 0 || mr.x == 0)) {  // an empty side: no fill
                                    empty_pair(ph[hh], xr_, mr.x, cs_[hh], mc[hh].x);
                                    live[hh] = false;
                                }
                            }
                            if (!live[0] && !live[1]) continue;
                            ArChain& c = chs[cur];
#pragma unroll
                            for (int hh = 0; hh < 2; ++hh) {
                                const int nb_ = live[hh] ? mc[hh].x : 0;
                                c.cseq[hh] = cs_[hh];
                                c.nB[hh] = nb_;
                                c.fy[hh] = live[hh] ? mc[hh].y : 0;
                                c.ly[hh] = live[hh] ? mc[hh].z : 0;
                                c.off[hh] = nb_ > 0 ? (K - nb_ % K) % K : 0;
                            }
                            c.swp = 1;
                            tab[cur][0] = ArRow{xr_, {live[0] ? ph[0] : -1, live[1] ? ph[1] : -1}, mr.x, mr.y, mr.z, 0};
                            rows = mr.x;
                            n = 1;
                            ++q;
                            break;
                        }
                        const int64_t du = q - S.u0;
                        const int64_t b = S.b0 + du;
                        const int4 mb = YS.meta[b];
                        const uint8_t* yb_ = YS.bytes + YS.offs[b];
                        const int64_t xh[2] = {S.x0, S.x1};
                        const int64_t ph[2] = {S.p0 + du, S.x1 >= 0 ? S.p1 + du : -1};
                        int4 mx[2];
                        const uint8_t* xs_[2];
                        bool live[2];
#pragma unroll
                        for (int hh = 0; hh < 2; ++hh) {
                            live[hh] = xh[hh] >= 0;
                            if (live[hh]) {
                                mx[hh] = XS.meta[xh[hh]];
                                xs_[hh] = XS.bytes + XS.offs[xh[hh]];
                                if (mx[hh].x == 0 || mb.x == 0) {  // an empty side: outputs now, no fill
                                    empty_pair(ph[hh], xs_[hh], mx[hh].x, yb_, mb.x);
                                    live[hh] = false;
                                }
                            }
                        }
                        if (!live[0] && !live[1]) continue;
                        if (n > 0 && rows + mb.x > cap_rows) break;
                        if (n == 0) {
                            ArChain& c = chs[cur];
#pragma unroll
                            for (int hh = 0; hh < 2; ++hh) {
                                const bool on = xh[hh] >= 0;
                                const int4 m = on ? XS.meta[xh[hh]] : make_int4(0, 0, 0, 0);
                                c.cseq[hh] = on ? XS.bytes + XS.offs[xh[hh]] : XS.bytes;
                                c.nB[hh] = m.x;
                                c.fy[hh] = m.y;
                                c.ly[hh] = m.z;
                                c.off[hh] = m.x > 0 ? (K - m.x % K) % K : 0;
                            }
                            c.swp = 0;
                        }
                        tab[cur][n] = ArRow{yb_, {live[0] ? ph[0] : -1, live[1] ? ph[1] : -1}, mb.x, mb.y, mb.z, rows};
                        rows += mb.x;
                        ++n;
                        if (n == (int)chunk || n == AR_UNITS) {
                            ++q;
                            break;
                        }
                    }
                    s_qc = q;
                }
                chs[cur].n = n;
                s_n = n;
                s_rows = rows;
                s_prog[0] = s_prog[1] = 0;
            }
            __syncthreads();
            const int n = s_n;
            const int rows = s_rows;
            const int pb = cur ^ 1;
            if constexpr (IS_W) walk_init(pb, prev_n);
            if (n == 0) {
                if constexpr (IS_W) walk(pb);
                break;
            }
            const ArChain& ch = chs[cur];
            // ---- fill-lane substitution table (once per chain): virtual column v of half h is real
            // column v - off_h; pre-columns (v <= off_h) score 0, columns past nB_h anything
            if constexpr (!IS_W) {
                const int v0 = tid * K + 1;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    int jr[2];
                    uint32_t cb[2];
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                        jr[hh] = v0 + k - ch.off[hh];
                        cb[hh] = (jr[hh] >= 1 && jr[hh] <= ch.nB[hh]) ? (uint32_t)ch.cseq[hh][jr[hh] - 1] : 0u;
                    }
#pragma unroll
                    for (int rb = 0; rb < 4; ++rb) {
                        int s2[2];
#pragma unroll
                        for (int hh = 0; hh < 2; ++hh)
                            s2[hh] = (jr[hh] < 1 ? 0 : (cb[hh] == (uint32_t)"ACGT"[rb] ? AR_EQ_MATCH : AR_EQ_MISMATCH)) - AR_CO_I;
                        eqt[rb][k / EP][tid][k % EP] = ar_pk_int(s2[0], s2[1]);
                    }
                }
            }
            if (tid < 64) xinfo[tid] = ar_row_record<K, W>(tab[cur], ch, n, rows, tid, band);
            else if (tid < 128) xinfo[XR - 128 + tid] = ar_record(0u, AR_NOBAND, false);
            // lane's end-column Ix open (slot K - 1): the end-gap open in the half whose column nB_h
            // is this lane's last slot, the internal open elsewhere
            const int tq0 = w * 64 + lane;
            const int nbv0 = ch.nB[0] + ch.off[0], nbv1 = ch.nB[1] + ch.off[1];
            const uint32_t cend = ar_pk_int((ch.nB[0] > 0 && tq0 == nbv0 / K - 1) ? AR_CO_E : AR_CO_I,
                                            (ch.nB[1] > 0 && tq0 == nbv1 / K - 1) ? AR_CO_E : AR_CO_I);
            const int own0 = ch.nB[0] > 0 ? nbv0 / K - 1 : -1, own1 = ch.nB[1] > 0 ? nbv1 / K - 1 : -1;
            const uint32_t COI = ar_pk_int(AR_CO_I, AR_CO_I);
            const uint32_t GZ = pk2b(0, 0) + COI;  // B = 0 shifted by the internal open
            const uint32_t cadj = cend - COI;      // the end column's Ix open over the internal one
            uint32_t stG[K], stX[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                stG[k] = GZ;
                stX[k] = NEG16X2;
            }
            uint32_t payF = NEG16X2, payY = NEG16X2, carry = GZ;
            uint8_t* trb = bufs + (size_t)cur * (size_t)buf_bytes;
            const int ln = __lane_id();
            const uint32_t ln16 = (uint32_t)ln << 4;
            __syncthreads();  // xinfo block 0, tables
#ifdef AR_PROF
            pf[2] += AR_NOW() - tA;
            pf[6] += 1;
#endif

            // one systolic step of fill wave WI (a compile-time index: the ring slots, the lane's
            // column block and its table row are immediate offsets).  Wave 0 takes the column-0
            // boundary; every wave but the last hands its last lane's row on through the ring.
            auto rec_addr = [&](const int s) -> const char* {  // this lane's row record at step s
                return (const char*)xinfo + ((((uint32_t)s << 4) - ln16) & ((XR - 1) << 4));
            };
            // recx: the record's table offset (.x), read ahead of the step when AR_PREC
            auto step = [&](auto WIC, const int s, const uint32_t recx) {
                constexpr int WI = decltype(WIC)::value;
                constexpr bool FW = WI == 0, HO = WI < W - 1;
                const int g = s - ln;
                const int tq = WI * 64 + ln;
                const uint4 rec = *(const uint4*)rec_addr(s);
                uint2 o_ring = make_uint2(0u, 0u);
                if constexpr (!FW) o_ring = ring[(WI - 1) * AR_RING + ((s + 1) & (AR_RING - 1))];
                const bool in_band = (uint8_t)((uint32_t)tq - rec.y) <= (uint8_t)(rec.y >> 8);
                const uint64_t bmask = __builtin_amdgcn_ballot_w64(in_band);
                asm volatile("" ::"s"(bmask));
                const bool pre = (int)rec.y < 0;  // AR_PRE
                const uint32_t orow = rec.z;      // the row's Iy open (pk_int)
                uint32_t inF, inY;
                if constexpr (FW) {  // column 0: B(i, 0) = 0 (shifted: rec.w), Iy(i, 0) = -inf (drift)
                    inF = shr_old(payF, rec.w);
                    inY = shr_old(payY, NEG16X2);
                } else {
                    inF = shr_old(payF, o_ring.x);
                    inY = shr_old(payY, o_ring.y);
                }
                uint32_t eq[K];
                {
                    // the row base's table, this lane's EP words of each piece (lane-contiguous reads)
                    // (lane-first base: the other address forms cost the allocator a 129th VGPR, i.e.
                    // one wave per SIMD at the 128-register budget)
                    const char* tb = (const char*)&eqt[0][0][tq][0] + recx;
#pragma unroll
                    for (int q = 0; q < K / EP; ++q) {
                        const char* pq = tb + (size_t)(q * NT) * (EP * 4);
                        if constexpr (EP == 4) {
                            const uint4 v = *(const uint4*)__builtin_assume_aligned(pq, 16);
                            eq[4 * q] = v.x;
                            eq[4 * q + 1] = v.y;
                            eq[4 * q + 2] = v.z;
                            eq[4 * q + 3] = v.w;
                        } else {
                            const uint2 v = *(const uint2*)__builtin_assume_aligned(pq, 8);
                            eq[2 * q] = v.x;
                            eq[2 * q + 1] = v.y;
                        }
                    }
                }
                if (pre) {  // a unit's first or last row, or a byte other than A/C/G/T
                    if (rec.y & AR_FIRST) {  // row 0 of the new pair: B = 0, Ix = -inf, diagonal B(0, j0 - 1) = 0
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            stG[k] = GZ;
                            stX[k] = NEG16X2;
                        }
                        carry = GZ;
                    }
                    if (rec.y & AR_OTHER) {  // byte compares against both halves' columns
                        const uint32_t rb = (rec.y >> 16) & 0xFFu;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            int s2[2];
#pragma unroll
                            for (int hh = 0; hh < 2; ++hh) {
                                const int jr = tq * K + k + 1 - ch.off[hh];
                                const uint32_t cb = (jr >= 1 && jr <= ch.nB[hh]) ? (uint32_t)ch.cseq[hh][jr - 1] : 0u;
                                s2[hh] = (jr < 1 ? 0 : (cb == rb ? AR_EQ_MATCH : AR_EQ_MISMATCH)) - AR_CO_I;
                            }
                            eq[k] = ar_pk_int(s2[0], s2[1]);
                        }
                    }
                }
                at_s2 F1 = as_s2(inF), Y = as_s2(inY);
                uint32_t acc[K];
                // Best-open fill on open-shifted cells (alignt2_kernel.hpp cells, RAW): M = G(i-1, j-1) +
                // (s - co_i), X = max(G_up, X_up), Y = max(G_left, Y_left), B = maximum3(M, X, Y), G = B + o_i.
                // TR: also the trace words (D1 = M - Ix, D2 = M - Iy of both halves, one v_perm)
                auto cells = [&](auto TRC) {
                    constexpr bool TR = decltype(TRC)::value;
                    at_s2 Mk = padd32(as_s2(carry), eq[0]);
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const at_s2 Gu = as_s2(stG[k]), Xu = as_s2(stX[k]);
                        const at_s2 M = Mk;
                        if (k + 1 < K) Mk = padd32(Gu, eq[k + 1]);
                        const at_s2 Xn = pmax(k == K - 1 ? padd32(Gu, cadj) : Gu, Xu);
                        const at_s2 Yn = pmax(F1, Y);
                        uint32_t b3;
                        asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(b3) : "v"(as_u32(M)), "v"(as_u32(Xn)), "v"(as_u32(Yn)));
                        if constexpr (TR) {
                            const uint32_t dD = as_u32(M) - as_u32(Xn);
                            const uint32_t dE = as_u32(M) - as_u32(Yn);
                            acc[k] = __builtin_amdgcn_perm(dE, dD, 0x06040200u);
                        }
                        const at_s2 Gn = padd32(as_s2(b3), orow);
                        stG[k] = as_u32(Gn);
                        stX[k] = as_u32(Xn);
                        F1 = Gn;
                        Y = Yn;
                    }
                };
                // AR_SKIP: a wave with no lane in the trace band this step (~36 % of (fill wave, step)
                // pairs at config 3) runs the cells without the trace's 3 VALU per cell pair; the
                // branch is wave-uniform (the band ballot in an SGPR)
                if (AR_SKIP && bmask == 0) cells(std::false_type{});
                else cells(std::true_type{});
                if (in_band) {
                    constexpr uint32_t PSTRIDE = ar_piece_stride<K, NT>();  // bytes between pieces
                    // uniform step offset (SGPR) + the lane's constant: one VALU add, saddr stores per piece
                    const uint32_t o0 = (uint32_t)__builtin_amdgcn_readfirstlane(ar_trace_step_off<K, NT>((uint32_t)s)) +
                                        (uint32_t)tq * ar_lane_bytes<K>();
                    if constexpr (K % 4 == 0) {
#pragma unroll
                        for (int q = 0; q < K / 4; ++q)
                            *(uint4*)((trb + q * PSTRIDE) + o0) = make_uint4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                    } else {
#pragma unroll
                        for (int q = 0; q < K / 2; ++q) *(uint2*)((trb + q * PSTRIDE) + o0) = make_uint2(acc[2 * q], acc[2 * q + 1]);
                    }
                }
                payF = as_u32(F1);
                payY = as_u32(Y);
                if constexpr (HO)
                    if (ln == 63) ring[WI * AR_RING + ((g + 1) & (AR_RING - 1))] = make_uint2(payF, payY);
                if (pre && (rec.y & AR_LAST) && (tq == own0 || tq == own1)) {  // owner of a half's column nB_h
                    int t = 0;
                    for (int q = 1; q < n; ++q)
                        if (tab[cur][q].r0 <= g) t = q;
                    const uint32_t e = stG[K - 1] - orow;  // B = G - o_i
                    if (tq == own0) fin[cur][t][0] = (int)(e & 0xFFFFu) - BIAS16;
                    if (tq == own1) fin[cur][t][1] = (int)(e >> 16) - BIAS16;
                }
                carry = inF;  // G(i, j0 - 1): the next row's diagonal
            };

            const int nsteps = rows + 63;
            // No interval barriers: the fill waves pace each other through two LDS progress counters
            // (steps completed, published every AR_BLK steps), so a wave whose steps store no trace
            // runs ahead instead of waiting at a barrier for the in-band wave (the band covers wave 0
            // early in a unit and wave 1 late: ~60 % of barrier intervals were unbalanced).  Wave 1 at
            // step s reads ring slot s + 1, written by wave 0 at step s + 63; wave 0 at step s
            // rewrites the slot wave 1 read at step s - 255 - 63.  The row records of the next 64 rows
            // are written by wave 0 itself before it needs them, and wave 1 (>= 79 steps behind,
            // <= 303 ahead is what wave 0 may run) reads them long before they are rewritten.  The
            // walker walks the previous chain to its end; the chain's last barrier joins everyone.
            if constexpr (IS_W) {
#ifdef AR_PROF
                const unsigned long long t1 = AR_NOW();
#endif
                walk(pb);
#ifdef AR_PROF
                pf[3] += AR_NOW() - t1;
#endif
            } else {
                const int mine = w, other = w ^ 1;
                for (int s0 = 0; s0 < nsteps; s0 += AR_BLK) {
                    const int s1 = min(s0 + AR_BLK, nsteps);
#ifdef AR_PROF
                    const unsigned long long t0 = AR_NOW();
#endif
                    if (W > 1) {  // wait for the other fill wave
                        const int need = w == 0 ? s1 - AR_AHEAD : s1 + 63;
                        while (__hip_atomic_load(&s_prog[other], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
                            __builtin_amdgcn_s_sleep(1);
                    }
#ifdef AR_PROF
                    const unsigned long long t1 = AR_NOW();
                    pf[4] += t1 - t0;
#endif
                    // AR_PREC: step s + 1's table offset (record word .x) is read during step s, so its
                    // eqt reads issue at the top of the step instead of behind a dependent LDS read.  Within
                    // the block only: wave 0 writes the next 64 rows' records after a block whose end
                    // is a multiple of 64, so a record past s1 may not be written yet.
                    auto recx_at = [&](const int s) { return *(const uint32_t*)rec_addr(s); };
                    auto run = [&](auto WIC) {
                        if constexpr (AR_PREC) {
                            uint32_t rx = recx_at(s0);
                            for (int s = s0; s < s1; ++s) {
                                const uint32_t nxt = recx_at(s + 1 < s1 ? s + 1 : s);
                                step(WIC, s, rx);
                                rx = nxt;
                            }
                        } else {
                            for (int s = s0; s < s1; ++s) step(WIC, s, recx_at(s));
                        }
                    };
                    if (w == 0) {
                        run(std::integral_constant<int, 0>{});
                    } else if constexpr (W > 1) {
                        run(std::integral_constant<int, 1>{});
                    }
#ifdef AR_PROF
                    pf[0] += AR_NOW() - t1;
#endif
                    if (w == 0 && (s1 & (INTERVAL - 1)) == 0) {  // the next 64 rows' records
                        const int gpre = s1 + lane;
                        xinfo[gpre & (XR - 1)] = ar_row_record<K, W>(tab[cur], ch, n, rows, gpre, band);
                    }
                    // publish (the ring / record writes above complete first: release)
                    if (lane == 0)
                        __hip_atomic_store(&s_prog[mine], s1 >= nsteps ? 0x3FFFFFFF : s1, __ATOMIC_RELEASE,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                __builtin_amdgcn_s_waitcnt(0);  // this chain's trace stores are done before the walker reads them
            }
#ifdef AR_PROF
            const unsigned long long t2 = AR_NOW();
#endif
            __syncthreads();  // the chain is filled and the previous one walked
#ifdef AR_PROF
            pf[IS_W ? 5 : 1] += AR_NOW() - t2;
            tA = AR_NOW();
#endif
            prev_n = n;
            cur ^= 1;
        }
#ifdef AR_PROF
        if (lane == 0)
            for (int q = 0; q < 8; ++q) atomicAdd(&ar_prof[q], pf[q]);
#endif
    };
    if (walker) chain_loop(std::true_type{});
    else chain_loop(std::false_type{});
}

}  // namespace taxi2
