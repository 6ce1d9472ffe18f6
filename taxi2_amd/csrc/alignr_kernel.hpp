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
// Wave 0 writes the next INTERVAL rows' records after a block whose end is a multiple of INTERVAL:
// every block end must be able to be one, and no block may outrun the rows written
static_assert(AR_BLK <= INTERVAL && INTERVAL % AR_BLK == 0, "AR_BLK must divide INTERVAL (row records)");
#ifndef TAXI2_AR_UNITS
#define TAXI2_AR_UNITS 8
#endif
constexpr int AR_UNITS = TAXI2_AR_UNITS;
// Bound of one pacing wait (polls of s_sleep 1, ~64 clocks each: ~0.5 s at 2.4 GHz, against ~1e3
// polls for the longest wait measured).  Pacing is deadlock-free by the static_assert above; the
// bound turns a pacing or launch-shape error into a failed launch (pace_err -> taxi2_last_error)
// instead of a hung device.
#ifndef TAXI2_AR_SPIN_CAP
#define TAXI2_AR_SPIN_CAP (1 << 24)
#endif
constexpr int AR_SPIN_CAP = TAXI2_AR_SPIN_CAP;
// wave priorities (s_setprio 0-3) of the walker and of fill waves 0 / 1.  Config-3 launch, same box,
// two runs each (profiles/r6/prio/): 0,0,0 87.9 ms; 0,1,1 86.6; 0,2,1 86.4; 0,1,2 90.4 -- the walker
// fills idle issue slots, and the leading fill wave (which the other waits on) goes first
#ifndef TAXI2_AR_PRIO
#define TAXI2_AR_PRIO 0, 2, 1
#endif
constexpr int AR_PRIOS[3] = {TAXI2_AR_PRIO};
constexpr int AR_PRIO_WALK = AR_PRIOS[0], AR_PRIO_W0 = AR_PRIOS[1], AR_PRIO_W1 = AR_PRIOS[2];  // units (row sequences, up to two pairs each) per chain
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
__device__ unsigned long long ar_prof[12];  // + [7] fill-wave polls, [8] walker loop iterations, [9] fill steps
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

// The fill's constants for Gotoh scores with ONE extend for internal and end gaps (ie == ee; the
// host admits such sets through ar_scores_ok): drift dz = ie, substitution s - 2 ie, opens relative
// to the extend co_i = io - ie, co_e = eo - ee.  Under such scores the column-0 and row-0 boundaries
// are B(i, 0) = B(0, j) = co_e (i, j >= 1) and B(0, 0) = 0 in drift coordinates; the default scores
// (co_e = 0) make them one flat 0.  DEF kernels use the constant default set (folded by the compiler).
struct ArSc {
    int eqm, eqx, coi, coe;  // match / mismatch substitution in drift coordinates, the two opens
    int ma, mi, io, ie, eo, ee;
};
__host__ __device__ constexpr ArSc ar_sc(int ma, int mi, int io, int ie, int eo, int ee) {
    return ArSc{ma - 2 * ie, mi - 2 * ie, io - ie, eo - ee, ma, mi, io, ie, eo, ee};
}
constexpr ArSc AR_DEFAULT = ar_sc(1, -1, -8, -1, -1, -1);  // align.py:20-27
static_assert(AR_DEFAULT.eqm == AR_EQ_MATCH && AR_DEFAULT.eqx == AR_EQ_MISMATCH && AR_DEFAULT.coi == AR_CO_I &&
                  AR_DEFAULT.coe == AR_CO_E,
              "default constants");
// Scores k_alignr takes besides the defaults: one extend (the drift), every open no better than its
// extend (the best-open recurrences), scores within +-12 (the int8 raw trace, alignt2_kernel.hpp),
// an internal open no better than the end open relative to their extend (co_i <= co_e: the
// pre-columns then reproduce the column-0 boundary, see the first-row reset), and every stored value
// of an L-column fill inside the normal f16 range the best state's v_pk_maximum3_f16 needs (BIAS16:
// drift-coordinate values in [-19 456, 11 263]; the -16 384 sentinel sits below every real value).
__host__ __device__ inline bool ar_scores_ok(int ma, int mi, int io, int ie, int eo, int ee, int L) {
    bool small = true;
    for (const int v : {ma, mi, io, ie, eo, ee}) small = small && v >= -12 && v <= 12;
    const ArSc S = ar_sc(ma, mi, io, ie, eo, ee);
    return ie == ee && io <= ie && eo <= ee && small && S.coi <= S.coe &&
           (long long)L * (S.eqm > 0 ? S.eqm : 0) + 64 <= 11000;
}

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
__device__ __forceinline__ uint4 ar_record(const ArSc& S, uint32_t x, uint32_t y, bool last) {
    const uint32_t o = last ? ar_pk_int(S.coe, S.coe) : ar_pk_int(S.coi, S.coi);
    return make_uint4(x, y, o, pk2b(S.coe, S.coe) + o);  // column 0: B(i, 0) = co_e (i >= 1)
}

template <int K, int W>
__device__ __forceinline__ uint4 ar_row_record(const ArSc& S, const ArRow* __restrict__ tab, const ArChain& ch, int n, int rows, int g,
                                               int band) {
    constexpr int NT = 64 * W;
    if (g < 0 || g >= rows) return ar_record(S, 0u, AR_NOBAND, false);
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
    return ar_record(S, x, y, i == r.nA - 1);
}

// <= 128 VGPRs: 4 waves per SIMD, so that the 5 workgroups of 3 waves the LDS allows fit a CU (the
// launch bound alone lets the allocator take more and lose a workgroup per CU)
template <int K, int W, int OCC, bool DEF>
__global__ void __launch_bounds__(64 * (W + 1), OCC) __attribute__((amdgpu_num_vgpr(128)))
k_alignr(SetView XS, SetView YS, KScores ksc, const ArSeg* __restrict__ segs, int nseg, int64_t total, int64_t npairs,
         MetricSpec ms, int chunk_req, int out_mode, double* __restrict__ out, int32_t* __restrict__ sout,
         uint8_t* __restrict__ trace, int64_t buf_bytes, int cap_rows, unsigned long long* __restrict__ next,
         int band, int64_t* __restrict__ esc_list, unsigned long long* __restrict__ esc_n, StrOut so,
         unsigned int* __restrict__ pace_err) {
    static_assert(K % 2 == 0 && K <= 8 && W <= 2, "row-shared shapes: K <= 8 columns per lane, one or two fill waves");
    constexpr int NT = 64 * W;
    constexpr int XR = a1c_xr(W);
    // the scores' fill constants: the defaults folded in (DEF), else the launch's one-extend set
    const ArSc S = DEF ? AR_DEFAULT : ar_sc(ksc.ma, ksc.mi, ksc.io, ksc.ie, ksc.eo, ksc.ee);
    const int dz = S.ie;  // the drift
    const KScores sc{S.ma, S.mi, S.io, S.ie, S.eo, S.ee};
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
    __shared__ uint8_t wct[256];  // the walker's base codes: a2_wcode of every byte

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
    for (int c = tid; c < 256; c += 64 * (W + 1)) wct[c] = (uint8_t)a2_wcode((uint32_t)c);  // (first barrier below)
    // set when a fill wave's wait for its partner exceeds AR_SPIN_CAP polls: the wave stops waiting
    // for the rest of the launch and the host reports the launch as failed (pace_err)
    bool stalled = false;

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

    // The walker (one lane per walk, up to NW = 4 AR_UNITS walks of the previous chain): the best-open
    // traceback of alignt2_kernel.hpp walk_run_raw, specialised to the default scores and written for
    // few VALU per step -- its instructions take issue slots from the fill waves on the same SIMD
    // (round 6: the walker was 11.6 % of the kernel's VALU, 137 per step; with no walker at all the
    // launch ran 9.7 % faster, profiles/r6/).  Per step of every walk:
    //  * the cell (i, j) in state st is accounted from its bytes' codes (an LDS table of a2_wcode);
    //  * the path score is checked through its decomposition under the default scores: a path with
    //    nm M columns of which nmatch match and nio internal gap opens scores 2 nmatch + nm - 7 nio
    //    - (nA + nB) (M: +1 / -1; every gap column -1; an internal open -7 more, an end open nothing),
    //    which must equal the fill's optimum (fin - nA - nB in drift coordinates);
    //  * the predecessor's sequence bytes and trace word are loaded through 32-bit offsets from the
    //    uniform sequence-set and trace bases (the row bytes are never masked: a walk on row 0 or
    //    column 0 moves in Iy / Ix, whose accounting reads only the other byte);
    //  * a walk reaching (0, 0) parks in AT_FIN with its counters; every parked walk is checked and
    //    written after the loop in one pass (the f64 metric epilogue once per wave, not once per
    //    finishing lane).
    // Aligned strings (so.sx): each walk keeps the last 8 columns it produced in a 64-bit window per
    // string and stores the window (8 bytes, unaligned) every 8 columns and at the walk's end.
    static_assert(AR_TS == 0, "the walker addresses the plain [step][lane][4K] trace layout");
    constexpr int AT_FIN = AT_ESC + 1;
#ifdef AR_PROF
    unsigned long long wit = 0;  // walker loop iterations
#endif
    auto walk = [&](int pb) {
#ifdef AR_NOWALK
        return;
#endif
        ArWalk& W_ = wks[lane < NW ? lane : 0];
        int st = lane < NW ? W_.st : AT_DONE;
        if (!__any(st != AT_DONE)) return;
        const int t = W_.t, h = W_.h, prio = W_.prio;
        const ArRow& r = tab[pb][t];
        const ArChain& ch = chs[pb];
        // rows are the pair's second sequence (orientation A = (y, x), prio 0, is slot 1), or its
        // first in a swapped chain (prio 0 is then slot 0)
        const bool swp = __builtin_amdgcn_readfirstlane(ch.swp) != 0;
        const uint8_t* const rbase = swp ? XS.bytes : YS.bytes;  // the row / column sequence sets
        const uint8_t* const cbase = swp ? YS.bytes : XS.bytes;
        const int nA_ = r.nA, nB_ = ch.nB[h], off = ch.off[h], r0 = r.r0;
        const uint32_t roff = (uint32_t)(r.rseq - rbase), coff = (uint32_t)(ch.cseq[h] - cbase);
        // internal-gap column ranges of the p-gaps count: fx + 1 <= i <= lx, fy + 1 <= j <= ly
        const int fx1 = r.fx + 1, fy1 = ch.fy[h] + 1;
        const uint32_t giw = (uint32_t)max(r.lx - r.fx, 0), gjw = (uint32_t)max(ch.ly[h] - ch.fy[h], 0);
        const int64_t p = r.p[h];
        const int bdl = min(0, nB_ - nA_) - band;
        const uint32_t bwd = (uint32_t)(abs(nB_ - nA_) + 2 * band);
        const uint8_t* const trb = bufs + (size_t)pb * (size_t)buf_bytes;
        // the high half's trace bytes carry the low half's borrow (a2_raw_de): added back per 16 bits
        const uint32_t hmask = h ? 0x00800080u : 0u;
        const uint32_t bsh = h ? 8u : 0u;
        const int oslot = swp ? prio : prio ^ 1;
        const size_t sbase = so.sx ? ((size_t)p * so.nslot + (oslot & (so.nslot - 1))) * (size_t)so.cap : 0;
        uint8_t* const dcol = swp ? so.sy : so.sx;  // the string of the column sequence and of the row one
        uint8_t* const drow = swp ? so.sx : so.sy;
        int i = nA_ + 1, j = nB_ + 1;  // the virtual end cell, in M: its first move picks the end state
        uint32_t xa = 0u, yb = 0u;
        int valid = 0, ts = 0, tv = 0, gap = 0, nmc = 0, nmatch = 0, nio = 0, ncol = 0;
        int nioe = 0;  // end-gap opens (generic scores only: the default end open scores 0)
        // the Ix open of the end column and the Iy open of the last row (end gaps), the internal one
        // elsewhere (uniform: scalar selects)
        const int coe = S.coe, coi = S.coi;
        // linear gaps (io = ie, eo = ee: both opens 0 over the extend) take the reference's
        // Needleman-Wunsch traceback (align.py:151-157 through Biopython's linear-gap algorithm;
        // oracle/restatement.py _nw): at each cell the first of H, V, D (swapped: V, H, D) at the
        // cell's maximum.  With zero opens the fill's Ix(i, j) = B(i - 1, j) and Iy(i, j) = B(i, j - 1)
        // (B >= Ix, Iy), i.e. the NW candidates v and h, and D1 / D2 are d - v and d - h.
        const bool lin = !DEF && coi == 0 && coe == 0;
        uint64_t wx = 0, wy = 0;  // string windows (column, row sequence): bits 0-7 = the last column produced
        bool first = true;        // the virtual end cell (uniform: every walk starts together)
        // Every lane runs the body every step (no per-lane region: its merge copies cost ~20 VALU a
        // step); a walk that ends parks its outcome in its LDS record and keeps stepping harmlessly
        // (clamped loads, no stores) until the wave's last walk ends.
        bool alive = lane < NW && st < AT_DONE;
        for (;;) {
            if (!__any(alive)) break;
#ifdef AR_PROF
            ++wit;
#endif
            const bool isM = st == AT_M, isX = st == AT_IX, isY = st == AT_IY;
            // ---- account the cell (i, j) in state st
            const uint32_t bx = wct[xa], by = wct[yb];
            const bool mcol = isM && !first;
            const bool cnt = mcol && (bx | by) < 4u;
            const uint32_t dd = bx ^ by;
            valid += cnt;
            ts += cnt && dd == 3u;
            tv += cnt && dd - 1u < 2u;
            gap += (isX && bx < 4u && (uint32_t)(j - fy1) < gjw) || (isY && by < 4u && (uint32_t)(i - fx1) < giw);
            nmc += mcol;
            nmatch += mcol && xa == yb;
            const int ni = i - (isY ? 0 : 1), nj = j - (isX ? 0 : 1);
            if (so.sx && !first) {  // this column of the alignment, right to left
                const uint32_t rc = isY ? (uint32_t)'-' : xa, cc = isX ? (uint32_t)'-' : yb;
                wx = (wx << 8) | cc;
                wy = (wy << 8) | rc;
                ++ncol;
                if ((ncol & 7) == 0 && alive) {  // columns [E - ncol, E - ncol + 8) of the slot (E = nA + nB)
                    const size_t o = sbase + (size_t)(nA_ + nB_ - ncol);
                    ar_store8(dcol + o, wx);
                    ar_store8(drow + o, wy);
                }
            }
            // ---- the predecessor (ni, nj): its bytes and trace word (clamped into the matrix on row /
            // column 0, where the move is forced and the word unused)
            const int ci = max(ni, 1) - 1, cjr = max(nj, 1) - 1;
            const uint32_t cj = (uint32_t)(cjr + off);  // virtual column
            const uint32_t tstep = (uint32_t)(r0 + ci) + ((cj / K) & 63u);
            const uint32_t toff = tstep * (uint32_t)(NT * 4 * K) + cj * 4u;
            const uint32_t xn = a2_load_byte(rbase + (roff + (uint32_t)ci));
            const uint32_t yn = a2_load_byte(cbase + (coff + (uint32_t)cjr));
            uint32_t nb = a2_load_trace32(trb + toff);
            nb = as_u32(as_s2(nb) + as_s2((nb & hmask) << 1));  // v_pk_add_u16: no carry between halves
            const int d1v = (int)(int8_t)(uint8_t)(nb >> bsh);          // M - Ix of (ni, nj)
            const int d2v = (int)(int8_t)(uint8_t)(nb >> (bsh + 16u));  // M - Iy
            // ---- the predecessor's state (first-path tie order), relative to its Ix
            const int co = j == nB_ ? coe : coi;  // Ix open of column j (end gap: eo - ee)
            const int oy = i == nA_ ? coe : coi;  // Iy open of row i
            const int aX = isX ? co : 0;
            const int aY = isX ? co : isY ? -oy : 0;
            const int vM = d1v + aX, vY = d1v - d2v + aY;
            const int vm = max(max(vM, vY), 0);
            const int alt = prio ? AT_IX + (vY == vm) : AT_IY - (vm == 0);  // Ix = 1, Iy = 2
            int nst = vM == vm ? AT_M : alt;
            if (!DEF && lin) {  // linear gaps: the single-matrix move of (ni, nj), gaps before the diagonal
                const int vv = -d1v, vh = -d2v, vb = max(max(vv, vh), 0);  // v - d, h - d, best - d
                nst = prio ? (vv == vb ? AT_IX : vh == vb ? AT_IY : AT_M) : (vh == vb ? AT_IY : vv == vb ? AT_IX : AT_M);
            }
            nst = ni == 0 ? AT_IY : nj == 0 ? AT_IX : nst;
            // a gap run's open (its last move, walked backward): internal unless on an edge
            const bool en = isX ? (j == nB_ || j == 0) : (i == nA_ || i == 0);
            nio += !isM && nst != st && !en;
            // (an end gap run reaching the origin is opened there: row 0 / column 0 of the fill)
            if constexpr (!DEF) nioe += !isM && en && (nst != st || (ni | nj) == 0);
            const bool fin_now = alive && (ni | nj) == 0;
            const bool esc_now = alive && !fin_now && ni >= 1 && nj >= 1 && band > 0 && (uint32_t)(nj - ni - bdl) > bwd;
            if (fin_now || esc_now) {  // park the walk's outcome (no values leave this region)
                ArWalk& R = wks[lane];
                R.st = fin_now ? AT_FIN : AT_ESC;
                R.valid = valid;
                R.ts = ts;
                R.tv = tv;
                R.gap = gap;
                // the path's score in drift coordinates: s - 2 ie per M column, one open per gap run
                R.sc2 = DEF ? 2 * nmatch + nmc - 7 * nio
                            : S.eqm * nmatch + S.eqx * (nmc - nmatch) + coi * nio + coe * nioe;
                R.ncol = ncol;
                if (fin_now && so.sx && (ncol & 7)) {  // the columns since the last window store
                    const size_t o8 = sbase + (size_t)(nA_ + nB_ - ncol);
                    if (ncol >= 8) {  // the window's older bytes are already in place
                        ar_store8(dcol + o8, wx);
                        ar_store8(drow + o8, wy);
                    } else {
                        for (int q = 0; q < ncol; ++q) {
                            dcol[o8 + q] = (uint8_t)(wx >> (8 * q));
                            drow[o8 + q] = (uint8_t)(wy >> (8 * q));
                        }
                    }
                }
            }
            alive = alive && !fin_now && !esc_now;
            st = nst;
            i = ni;
            j = nj;
            xa = xn;
            yb = yn;
            first = false;
        }
        // ---- every parked walk: its score check (the path's score against the fill's optimum) and
        // outputs, in one pass of the wave
        if (lane < NW) {
            const ArWalk& R = wks[lane];
            int fst = R.st;
            if (fst == AT_FIN) {
                if (R.sc2 != fin[pb][t][h]) {
                    fst = AT_ESC;
                } else {
                    double* o = out_mode == OUT_BOTH ? out + (p * 2 + oslot) * nm : out + p * nm;
                    for (int m = 0; m < nm; ++m)
                        o[m] = metric_value(ms.code[m], (uint32_t)R.valid, (uint32_t)R.ts, (uint32_t)R.tv, (uint32_t)R.gap);
                    if (sout && (out_mode != OUT_BOTH || oslot == 0)) sout[p] = fin[pb][t][h] + (nA_ + nB_) * dz;
                    if (so.slen) so.slen[p * so.nslot + (oslot & (so.nslot - 1))] = R.ncol;
                }
            }
            if (fst == AT_ESC) {  // queue the pair (once) for the full-trace pass (k_alignt2_queued)
                if (atomicOr(&escf[pb][t][h], 1) == 0 && esc_list) esc_list[atomicAdd(esc_n, 1ull)] = p;
                // a launch without that pass (esc_list null: band 0, so only a failed score check
                // gets here) reports its results invalid through the host-mapped flag
                if (!esc_list) __hip_atomic_fetch_or(pace_err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        if (lane < NW) W_.st = AT_DONE;
    };

    auto chain_loop = [&](auto WK) {
        constexpr bool IS_W = decltype(WK)::value;
        // issue priority (s_setprio): the walker has slack (it ends its walks well before the fill
        // ends the next chain), so its instructions should take the SIMD's idle issue slots only
        if constexpr (IS_W) {
            __builtin_amdgcn_s_setprio(AR_PRIO_WALK);
        } else {
            if (w == 0) __builtin_amdgcn_s_setprio(AR_PRIO_W0);
            else __builtin_amdgcn_s_setprio(AR_PRIO_W1);
        }
#ifdef AR_PROF
        unsigned long long pf[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
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
                            s2[hh] = (jr[hh] < 1 ? 0 : (cb[hh] == (uint32_t)"ACGT"[rb] ? S.eqm : S.eqx)) - S.coi;
                        eqt[rb][k / EP][tid][k % EP] = ar_pk_int(s2[0], s2[1]);
                    }
                }
            }
            if (tid < 64) xinfo[tid] = ar_row_record<K, W>(S, tab[cur], ch, n, rows, tid, band);
            else if (tid < 128) xinfo[XR - 128 + tid] = ar_record(S, 0u, AR_NOBAND, false);
            // lane's end-column Ix open (slot K - 1): the end-gap open in the half whose column nB_h
            // is this lane's last slot, the internal open elsewhere
            const int tq0 = w * 64 + lane;
            const int nbv0 = ch.nB[0] + ch.off[0], nbv1 = ch.nB[1] + ch.off[1];
            const uint32_t cend = ar_pk_int((ch.nB[0] > 0 && tq0 == nbv0 / K - 1) ? S.coe : S.coi,
                                            (ch.nB[1] > 0 && tq0 == nbv1 / K - 1) ? S.coe : S.coi);
            const int own0 = ch.nB[0] > 0 ? nbv0 / K - 1 : -1, own1 = ch.nB[1] > 0 ? nbv1 / K - 1 : -1;
            const uint32_t COI = ar_pk_int(S.coi, S.coi);
            // row 0 of a unit, shifted by the internal open (G = B + o_i): B(0, j) = co_e on every
            // column but real column 0 (virtual column off_h), where B(0, 0) = 0; the pre-columns
            // left of it hold co_e too, so that every pre-column keeps B(i, v) = co_e on the rows
            // below (M = B(i - 1, v - 1) + 0, Ix and Iy lower as long as co_i <= co_e) and real
            // column 0 carries the boundary B(i, 0) = co_e.  The default scores make it one flat 0.
            const uint32_t GZ = pk2b(S.coe, S.coe) + COI;
            const uint32_t cadj = cend - COI;  // the end column's Ix open over the internal one
            // (lane 0 only) the slot holding real column 0 of each half (-1: off_h = 0, the
            // boundary input itself) and the diagonal input of row 1 (B(0, virtual column 0))
            const int z0 = ch.off[0] - 1, z1 = ch.off[1] - 1;
            const uint32_t GZ0 = tq0 == 0 ? pk2b(ch.off[0] > 0 ? S.coe : 0, ch.off[1] > 0 ? S.coe : 0) + COI : GZ;
            uint32_t stG[K], stX[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                stG[k] = GZ;
                stX[k] = NEG16X2;
            }
            uint32_t payF = NEG16X2, payY = NEG16X2, carry = GZ;
            uint8_t* trb = bufs + (size_t)cur * (size_t)buf_bytes;
            const int ln = __lane_id();
            // (opaque: the compiler would otherwise fold (s << 4) - (ln << 4) into (s - ln) << 4, one
            // more VALU in every step's record address)
            uint32_t ln16 = (uint32_t)ln << 4;
            asm volatile("" : "+v"(ln16));
            uint32_t eq_lane = (uint32_t)ln * (EP * 4);  // the lane's byte offset in a table piece
            asm volatile("" : "+v"(eq_lane));
            // the lane's column bytes of both halves (bytes k of colb[h]) and its pre-columns (bit
            // 8 h + k): a row byte other than A/C/G/T compares against these (rare rows; kept in
            // registers so that this path does not set the step loop's register pressure)
            constexpr int CW = (K + 3) / 4;
            uint32_t colb[2][CW];
            uint32_t premask = 0;
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
                for (int q = 0; q < CW; ++q) colb[hh][q] = 0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int jr = tq0 * K + k + 1 - ch.off[hh];
                    const uint32_t cb = (jr >= 1 && jr <= ch.nB[hh]) ? (uint32_t)ch.cseq[hh][jr - 1] : 0u;
                    colb[hh][k / 4] |= cb << (8 * (k % 4));
                    if (jr < 1) premask |= 1u << (8 * hh + k);
                }
            }
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
            // A step's LDS operands -- the lane's row record, its row base's table words and (waves
            // after the first) the ring entry of its first lane -- are read one step AHEAD, during the
            // previous step: the record at the step's top, the table words (which need the record)
            // half way through its cells.  Without it every step began with two dependent LDS round
            // trips.  Prefetches stay inside the progress block: wave 0 writes the next 64 rows'
            // records only after a block whose end is a multiple of 64 (the last step prefetches
            // itself again).
            struct StepIn {
                uint4 rec;
                uint32_t eq[K];
                uint2 ring;
            };
            auto load_rec = [&](auto WIC, const int s, StepIn& o) {
                constexpr int WI = decltype(WIC)::value;
                o.rec = *(const uint4*)rec_addr(s);
                if constexpr (WI > 0) o.ring = ring[(WI - 1) * AR_RING + ((s + 1) & (AR_RING - 1))];
                else o.ring = make_uint2(0u, 0u);
            };
            auto load_eq = [&](auto WIC, StepIn& o) {
                constexpr int WI = decltype(WIC)::value;
                constexpr int tq = WI * 64;
                // the row base's table, this lane's EP words of each piece (lane-contiguous reads)
                const char* tb = (const char*)&eqt[0][0][tq][0] + eq_lane + o.rec.x;
#pragma unroll
                for (int q = 0; q < K / EP; ++q) {
                    const char* pq = tb + (size_t)(q * NT) * (EP * 4);
                    if constexpr (EP == 4) {
                        const uint4 v = *(const uint4*)__builtin_assume_aligned(pq, 16);
                        o.eq[4 * q] = v.x;
                        o.eq[4 * q + 1] = v.y;
                        o.eq[4 * q + 2] = v.z;
                        o.eq[4 * q + 3] = v.w;
                    } else {
                        const uint2 v = *(const uint2*)__builtin_assume_aligned(pq, 8);
                        o.eq[2 * q] = v.x;
                        o.eq[2 * q + 1] = v.y;
                    }
                }
            };
            auto step = [&](auto WIC, const int s, StepIn& I, const int sn, StepIn& N) {
                constexpr int WI = decltype(WIC)::value;
                constexpr bool FW = WI == 0, HO = WI < W - 1;
                const int g = s - ln;
                const int tq = WI * 64 + ln;
                const uint4 rec = I.rec;
                load_rec(WIC, sn, N);  // the next step's record (and ring entry)
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
                    inF = shr_old(payF, I.ring.x);
                    inY = shr_old(payY, I.ring.y);
                }
                uint32_t* const eq = I.eq;
                if (pre) {  // a unit's first or last row, or a byte other than A/C/G/T
                    if (rec.y & AR_FIRST) {  // row 0 of the new pair: B = co_e (0 at column 0), Ix = -inf
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            stG[k] = GZ;
                            stX[k] = NEG16X2;
                        }
                        carry = GZ0;  // the diagonal B(0, j0 - 1)
                        if constexpr (!DEF) {
                            if (tq == 0 && S.coe != 0) {  // the lane holding real column 0 (rare)
                                const uint32_t g0 = pk2b(0, 0) + COI;
#pragma unroll
                                for (int k = 0; k < K; ++k) {
                                    if (k == z0) stG[k] = (stG[k] & 0xFFFF0000u) | (g0 & 0xFFFFu);
                                    if (k == z1) stG[k] = (stG[k] & 0xFFFFu) | (g0 & 0xFFFF0000u);
                                }
                            }
                        }
                    }
                    if (rec.y & AR_OTHER) {  // byte compares against both halves' columns
                        const uint32_t rb = (rec.y >> 16) & 0xFFu;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            int s2[2];
#pragma unroll
                            for (int hh = 0; hh < 2; ++hh) {
                                const uint32_t cb = (colb[hh][k / 4] >> (8 * (k % 4))) & 0xFFu;
                                s2[hh] = (((premask >> (8 * hh + k)) & 1u) ? 0 : (cb == rb ? S.eqm : S.eqx)) - S.coi;
                            }
                            eq[k] = ar_pk_int(s2[0], s2[1]);
                            __builtin_amdgcn_sched_barrier(0);  // one column at a time: few live values
                        }
                    }
                }
                at_s2 F1 = as_s2(inF), Y = as_s2(inY);
                uint32_t acc[K];
                constexpr uint32_t PSTRIDE = ar_piece_stride<K, NT>();  // bytes between pieces
                // uniform step offset (SGPR) + the lane's constant: one VALU add, saddr stores per piece
                const uint32_t o0 = (uint32_t)__builtin_amdgcn_readfirstlane(ar_trace_step_off<K, NT>((uint32_t)s)) +
                                    (uint32_t)tq * ar_lane_bytes<K>();
                // the trace words of columns 4 q .. 4 q + 3, as soon as they are computed (K % 4 == 0)
                auto store_piece = [&](const int q) {
                    if (in_band) *(uint4*)((trb + q * PSTRIDE) + o0) = make_uint4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                };
                // Best-open fill on open-shifted cells (alignt2_kernel.hpp cells, RAW): M = G(i-1, j-1) +
                // (s - co_i), X = max(G_up, X_up), Y = max(G_left, Y_left), B = maximum3(M, X, Y), G = B + o_i.
                // TR: also the trace words (D1 = M - Ix, D2 = M - Iy of both halves, one v_perm)
                auto cells = [&](auto TRC) {
                    constexpr bool TR = decltype(TRC)::value;
                    at_s2 Mk = padd32(as_s2(carry), eq[0]);
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        if (k == K / 2) {  // the next step's table words (its record has arrived by now)
                            __builtin_amdgcn_sched_barrier(0);
                            load_eq(WIC, N);
                        }
                        if constexpr (TR && K % 4 == 0)
                            if (k % 4 == 0 && k > 0) store_piece(k / 4 - 1);
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
                if constexpr (K % 4 == 0) {
                    store_piece(K / 4 - 1);
                } else if (in_band) {
#pragma unroll
                    for (int q = 0; q < K / 2; ++q) *(uint2*)((trb + q * PSTRIDE) + o0) = make_uint2(acc[2 * q], acc[2 * q + 1]);
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
                    if (W > 1 && !stalled) {  // wait for the other fill wave (a bounded wait, see AR_SPIN_CAP)
                        const int need = w == 0 ? s1 - AR_AHEAD : s1 + 63;
                        int polls = 0;
                        while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_prog[other], __ATOMIC_ACQUIRE,
                                                                                __HIP_MEMORY_SCOPE_WORKGROUP)) < need) {
                            __builtin_amdgcn_s_sleep(1);
#ifdef AR_PROF
                            pf[7] += 1;
#endif
                            if (++polls >= AR_SPIN_CAP) {
                                stalled = true;
                                break;
                            }
                        }
                        if (stalled && lane == 0) __hip_atomic_fetch_or(pace_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
#ifdef AR_PROF
                    const unsigned long long t1 = AR_NOW();
                    pf[4] += t1 - t0;
#endif
                    // two step states used alternately (a loop unrolled by two: no copies between steps)
                    auto run = [&](auto WIC) {
                        StepIn A, B;
                        load_rec(WIC, s0, A);
                        load_eq(WIC, A);
                        int s = s0;
                        for (; s + 1 < s1; s += 2) {
                            step(WIC, s, A, s + 1, B);
                            step(WIC, s + 1, B, s + 2 < s1 ? s + 2 : s + 1, A);
                        }
                        if (s < s1) step(WIC, s, A, s, B);
                    };
                    if (w == 0) {
                        run(std::integral_constant<int, 0>{});
                    } else if constexpr (W > 1) {
                        run(std::integral_constant<int, 1>{});
                    }
#ifdef AR_PROF
                    pf[0] += AR_NOW() - t1;
                    pf[9] += s1 - s0;
#endif
                    if (w == 0 && (s1 & (INTERVAL - 1)) == 0) {  // the next 64 rows' records
                        const int gpre = s1 + lane;
                        xinfo[gpre & (XR - 1)] = ar_row_record<K, W>(S, tab[cur], ch, n, rows, gpre, band);
                    }
                    // publish (the ring / record writes above complete first: release)
                    // (a stalled wave publishes "done": its partner never waits on it again)
                    if (lane == 0)
                        __hip_atomic_store(&s_prog[mine], (stalled || s1 >= nsteps) ? 0x3FFFFFFF : s1, __ATOMIC_RELEASE,
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
        {
            pf[8] = wit;
            for (int q = 0; q < 12; ++q) atomicAdd(&ar_prof[q], pf[q]);
        }
#endif
    };
    if (walker) chain_loop(std::true_type{});
    else chain_loop(std::false_type{});
}

}  // namespace taxi2
