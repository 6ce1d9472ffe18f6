// Global alignment + distance counters, one pair per workgroup, systolic over 64-lane waves.
//
// Replaces Biopython PairwiseAligner(**Scores).align(x, y)[0] (align.py:151-157) followed by
// calc.seq_distances_* on the aligned strings (distances.py:319-348), for BOTH ordered pairs
// (x, y) and (y, x) in one dynamic-programming fill.
//
// Algorithm (restated in oracle/taxi2_oracle.c, pinned by tests/golden/align_tests.json):
//   Gotoh global fill with states M (diagonal), Ix (consume x, gap in y), Iy (consume y, gap
//   in x); end-gap scores on the last row / column; NW single matrix when every open ==
//   extend.  The first Biopython alignment follows the first tied predecessor in priority
//   M>Ix>Iy (NW: H>V>D).  Because that traceback is a deterministic function of the cell it
//   starts from, the alignment's column counters (valid, transitions, transversions, gaps)
//   are carried FORWARD through the fill: C(cell) = C(first tied predecessor) + column
//   contribution.  No traceback matrix is ever stored.  The (y, x) alignment is the same
//   fill with the Ix/Iy priority exchanged (NW: V>H>D), so each cell carries two counter
//   sets ("A" = (x, y), "B" = (y, x)).
//
// Mapping to gfx950:
//   * a workgroup of W waves owns one pair; lane l of wave w owns columns
//     j0 = (w*64 + l)*K + 1 .. j0+K-1 of the column sequence and keeps their previous-row
//     state in VGPRs (15 x K); rows stream through the lanes as a systolic wavefront: at local
//     step s lane l works on row i = s - l + 1.
//   * lane l-1 -> lane l hand-off of the last column state is one DPP `wave_shr:1` per
//     32-bit word (counters use bound_ctrl zero-fill for wave 0's left boundary); wave w-1
//     lane 63 -> wave w lane 0 goes through an LDS ring, wave w running two 64-step
//     intervals behind (one s_barrier per interval).
//   * a cell only needs its diagonal neighbour's best state (score + the two priority-selected
//     counter pairs, 5 VGPRs), so that summary is taken before the column is overwritten in
//     place: no register copies between cells or steps.
//   * counters are packed two fields per VGPR: w0 = valid | ts << 16, w1 = gap | tv << 20
//     (lengths <= 4095); the M contribution is a 32-bit per-column LUT shifted by the row's
//     base code (bits 0-3 valid, 8-15 the column byte, 16-19 transition, 20-23 transversion),
//     so every counter increment is one VALU op.
//   * the default TaxI2 scores (align.py:20-27) are a compile-time specialization so every
//     score and gap penalty is an inline constant.
//   * pure integer VALU work: no MFMA (nothing here is a dense contraction).
#pragma once
#include "common.hpp"

namespace taxi2 {

struct C2 {
    uint32_t w0, w1;  // w0 = valid | ts<<16, w1 = gap | tv<<20
};

__device__ __forceinline__ C2 csel(bool c, C2 a, C2 b) { return C2{c ? a.w0 : b.w0, c ? a.w1 : b.w1}; }
__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }

// wave_shr:1 -- lane l receives lane l-1's value; lane 0 keeps `old`.
__device__ __forceinline__ uint32_t shr_old(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}
// wave_shr:1 with bound_ctrl: lane 0 receives 0.
__device__ __forceinline__ uint32_t shr_zero(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
}

// ---------------------------------------------------------------- Gotoh state per column
struct GState {
    int M, X, Y;
    C2 m0, m1, x0, x1, y0, y1;  // counters of the traceback path from this cell/state;
                                // suffix 0 = orientation A (x, y), 1 = orientation B (y, x)
};

// Best state of a cell under both priorities (what the diagonal successor reads).
struct GBest {
    int h;
    C2 a, b;
};

__device__ __forceinline__ GBest g_best(const GState& e) {
    const int h = imax3(e.M, e.X, e.Y);
    const bool tm = e.M == h, tx = e.X == h, ty = e.Y == h;
    return GBest{h, csel(tm, e.m0, csel(tx, e.x0, e.y0)), csel(tm, e.m1, csel(ty, e.y1, e.x1))};
}

__device__ __forceinline__ GState g_row0(int j, const KScores& sc) {
    GState s;
    s.M = (j == 0) ? 0 : NEG_INF;
    s.X = NEG_INF;
    s.Y = (j == 0) ? NEG_INF : sc.eo + sc.ee * (j - 1);
    s.m0 = s.m1 = s.x0 = s.x1 = s.y0 = s.y1 = C2{0u, 0u};
    return s;
}

// Column-0 boundary at row i (only the Ix score is finite; all counters are zero).
__device__ __forceinline__ GState g_shr_first(const GState& v, int i, const KScores& sc) {
    GState r;
    r.M = (int)shr_old((uint32_t)v.M, (uint32_t)NEG_INF);
    r.X = (int)shr_old((uint32_t)v.X, (uint32_t)(sc.eo + sc.ee * (i - 1)));
    r.Y = (int)shr_old((uint32_t)v.Y, (uint32_t)NEG_INF);
#define T2_SZ(f) r.f.w0 = shr_zero(v.f.w0); r.f.w1 = shr_zero(v.f.w1);
    T2_SZ(m0) T2_SZ(m1) T2_SZ(x0) T2_SZ(x1) T2_SZ(y0) T2_SZ(y1)
#undef T2_SZ
    return r;
}

__device__ __forceinline__ GState g_shr_old(const GState& v, const GState& o) {
    GState r;
    r.M = (int)shr_old((uint32_t)v.M, (uint32_t)o.M);
    r.X = (int)shr_old((uint32_t)v.X, (uint32_t)o.X);
    r.Y = (int)shr_old((uint32_t)v.Y, (uint32_t)o.Y);
#define T2_SO(f) r.f.w0 = shr_old(v.f.w0, o.f.w0); r.f.w1 = shr_old(v.f.w1, o.f.w1);
    T2_SO(m0) T2_SO(m1) T2_SO(x0) T2_SO(x1) T2_SO(y0) T2_SO(y1)
#undef T2_SO
    return r;
}

// One Gotoh cell, in place.  d = best of (i-1, j-1); u = (i-1, j) on entry, (i, j) on exit;
// l = (i, j-1).  Returns the best of the old u for the next column's diagonal.
__device__ __forceinline__ GBest g_cell(const GBest& d, GState& u, const GState& l, int s,
                                        uint32_t inc0, uint32_t inc1, uint32_t gx, uint32_t gy,
                                        int ox, int ex, int oy, int ey) {
    const GBest nd = g_best(u);
    GState r;
    // M: diagonal move from the best state of (i-1, j-1)
    r.M = d.h + s;
    r.m0 = C2{d.a.w0 + inc0, d.a.w1 + inc1};
    r.m1 = C2{d.b.w0 + inc0, d.b.w1 + inc1};
    // Ix: consume x[i-1] against a gap (from above); A: M>Ix>Iy, B: M>Iy>Ix
    {
        const int ca = u.M + ox, cb = u.X + ex, cc = u.Y + ox;
        const int X = imax3(ca, cb, cc);
        r.X = X;
        const bool xa = ca == X, xb = cb == X, xc = cc == X;
        const C2 a = csel(xa, u.m0, csel(xb, u.x0, u.y0));
        const C2 b = csel(xa, u.m1, csel(xc, u.y1, u.x1));
        r.x0 = C2{a.w0, a.w1 + gx};
        r.x1 = C2{b.w0, b.w1 + gx};
    }
    // Iy: consume y[j-1] against a gap (from the left)
    {
        const int ca = l.M + oy, cb = l.X + oy, cc = l.Y + ey;
        const int Y = imax3(ca, cb, cc);
        r.Y = Y;
        const bool ya = ca == Y, yb = cb == Y, yc = cc == Y;
        const C2 a = csel(ya, l.m0, csel(yb, l.x0, l.y0));
        const C2 b = csel(ya, l.m1, csel(yc, l.y1, l.x1));
        r.y0 = C2{a.w0, a.w1 + gy};
        r.y1 = C2{b.w0, b.w1 + gy};
    }
    u = r;
    return nd;
}

// ---------------------------------------------------------------- NW (linear gaps)
struct NState {
    int S;
    C2 a, b;
};
using NBest = NState;

__device__ __forceinline__ NState n_row0(int j, const KScores& sc) {
    return NState{j * sc.ee, C2{0u, 0u}, C2{0u, 0u}};
}
__device__ __forceinline__ NState n_shr_first(const NState& v, int i, const KScores& sc) {
    NState r;
    r.S = (int)shr_old((uint32_t)v.S, (uint32_t)(i * sc.ee));
    r.a.w0 = shr_zero(v.a.w0);
    r.a.w1 = shr_zero(v.a.w1);
    r.b.w0 = shr_zero(v.b.w0);
    r.b.w1 = shr_zero(v.b.w1);
    return r;
}
__device__ __forceinline__ NState n_shr_old(const NState& v, const NState& o) {
    NState r;
    r.S = (int)shr_old((uint32_t)v.S, (uint32_t)o.S);
    r.a.w0 = shr_old(v.a.w0, o.a.w0);
    r.a.w1 = shr_old(v.a.w1, o.a.w1);
    r.b.w0 = shr_old(v.b.w0, o.b.w0);
    r.b.w1 = shr_old(v.b.w1, o.b.w1);
    return r;
}

// NW cell in place: D = diagonal, V = from above (consumes x), H = from the left (consumes y).
// Traceback priority A: H>V>D, B: V>H>D.  vg / hg = vertical / horizontal gap score.
__device__ __forceinline__ NBest n_cell(const NBest& d, NState& u, const NState& l, int s,
                                        uint32_t inc0, uint32_t inc1, uint32_t gx, uint32_t gy,
                                        int vg, int hg) {
    const NBest nd = u;
    const int cd = d.S + s, cv = u.S + vg, ch = l.S + hg;
    const int S = imax3(cd, cv, ch);
    const bool tv = cv == S, th = ch == S;
    const C2 dA{d.a.w0 + inc0, d.a.w1 + inc1}, dB{d.b.w0 + inc0, d.b.w1 + inc1};
    const C2 vA{u.a.w0, u.a.w1 + gx}, vB{u.b.w0, u.b.w1 + gx};
    const C2 hA{l.a.w0, l.a.w1 + gy}, hB{l.b.w0, l.b.w1 + gy};
    u.S = S;
    u.a = csel(th, hA, csel(tv, vA, dA));
    u.b = csel(tv, vB, csel(th, hB, dB));
    return nd;
}

// ---------------------------------------------------------------- LDS ring entry
struct RingEntry {
    uint4 q[4];  // 16 words; Gotoh uses 15, NW 5
};

__device__ __forceinline__ void ring_put(RingEntry* e, const GState& s) {
    e->q[0] = make_uint4((uint32_t)s.M, (uint32_t)s.X, (uint32_t)s.Y, s.m0.w0);
    e->q[1] = make_uint4(s.m0.w1, s.m1.w0, s.m1.w1, s.x0.w0);
    e->q[2] = make_uint4(s.x0.w1, s.x1.w0, s.x1.w1, s.y0.w0);
    e->q[3] = make_uint4(s.y0.w1, s.y1.w0, s.y1.w1, 0u);
}
__device__ __forceinline__ void ring_get(const RingEntry* e, GState& s) {
    const uint4 a = e->q[0], b = e->q[1], c = e->q[2], d = e->q[3];
    s.M = (int)a.x; s.X = (int)a.y; s.Y = (int)a.z; s.m0.w0 = a.w;
    s.m0.w1 = b.x; s.m1.w0 = b.y; s.m1.w1 = b.z; s.x0.w0 = b.w;
    s.x0.w1 = c.x; s.x1.w0 = c.y; s.x1.w1 = c.z; s.y0.w0 = c.w;
    s.y0.w1 = d.x; s.y1.w0 = d.y; s.y1.w1 = d.z;
}
__device__ __forceinline__ void ring_put(RingEntry* e, const NState& s) {
    e->q[0] = make_uint4((uint32_t)s.S, s.a.w0, s.a.w1, s.b.w0);
    e->q[1] = make_uint4(s.b.w1, 0u, 0u, 0u);
}
__device__ __forceinline__ void ring_get(const RingEntry* e, NState& s) {
    const uint4 a = e->q[0], b = e->q[1];
    s.S = (int)a.x; s.a.w0 = a.y; s.a.w1 = a.z; s.b.w0 = a.w; s.b.w1 = b.x;
}

constexpr int RING = 256;      // rows buffered between consecutive waves (power of 2)
constexpr int INTERVAL = 64;   // steps between workgroup barriers (W > 1)
constexpr int WAVE_LAG = 2;    // intervals wave w runs behind wave w-1

// Output layout selector.
enum OutMode : int { OUT_BOTH = 0, OUT_AB = 1 };

template <bool LINEAR>
struct StateOf {
    using T = GState;
    using B = GBest;
};
template <>
struct StateOf<true> {
    using T = NState;
    using B = NBest;
};

template <bool LINEAR>
__device__ __forceinline__ typename StateOf<LINEAR>::B best_of(const typename StateOf<LINEAR>::T& s) {
    if constexpr (LINEAR) return s;
    else return g_best(s);
}

// Per-lane, per-pair column constants.
template <int K>
struct LaneCols {
    uint32_t lut[K];   // bits 0-3 valid / 16-19 ts / 20-23 tv by row base; 8-15 column byte
    uint32_t ixbits;   // column j: x-gap column lies in the common range (j-1 >= fy, j <= ly)
    uint32_t ynbits;   // column j: y[j-1] is ACGT
    uint32_t lastbits; // column j == nB (end-gap scores for Ix / vertical)
};

// One systolic step for this lane: receive the left column state, then update K cells of
// row i = s - lane + 1.  `carry` is the best-state summary of the left input of the
// previous step (the diagonal of this step's first cell) and is replaced by this step's.
template <int K, int W, bool LINEAR, bool FIRST>
__device__ __forceinline__ void dp_step(int s, int lane, int nA, typename StateOf<LINEAR>::T (&st)[K],
                                        typename StateOf<LINEAR>::B& carry, const LaneCols<K>& lc,
                                        const uint32_t* __restrict__ xinfo,
                                        const RingEntry* __restrict__ ring_in, RingEntry* __restrict__ ring_out,
                                        const KScores& sc) {
    using S = typename StateOf<LINEAR>::T;
    using B = typename StateOf<LINEAR>::B;
    S in;
    if constexpr (FIRST) {
        if constexpr (LINEAR) in = n_shr_first(st[K - 1], s + 1, sc);
        else in = g_shr_first(st[K - 1], s + 1, sc);
    } else {
        S old;
        ring_get(ring_in + ((s + 1) & (RING - 1)), old);
        if constexpr (LINEAR) in = n_shr_old(st[K - 1], old);
        else in = g_shr_old(st[K - 1], old);
    }
    const int i = s - lane + 1;
    if (i >= 1 && i <= nA) {
        const uint32_t xi = xinfo[i - 1];
        const uint32_t xb = xi & 0xFFu;
        const uint32_t xsh = (xi >> 8) & 31u;
        const uint32_t gxm = ((xi >> 14) & 1u) ? lc.ixbits : 0u;
        const uint32_t gym = ((xi >> 13) & 1u) ? lc.ynbits : 0u;
        const bool lastrow = (i == nA);
        const int oy = lastrow ? sc.eo : sc.io;
        const int ey = lastrow ? sc.ee : sc.ie;
        B d = carry;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t lut = lc.lut[k];
            const int sv = (((lut >> 8) & 0xFFu) == xb) ? sc.ma : sc.mi;
            const uint32_t t = lut >> xsh;
            const uint32_t inc0 = t & 0x00010001u;  // valid, ts
            const uint32_t inc1 = t & 0x00100000u;  // tv
            const uint32_t gx = (gxm >> k) & 1u;    // gap (Ix move)
            const uint32_t gy = (gym >> k) & 1u;    // gap (Iy move)
            const bool lastcol = (lc.lastbits >> k) & 1u;
            if constexpr (LINEAR) {
                d = n_cell(d, st[k], k == 0 ? in : st[k - 1], sv, inc0, inc1, gx, gy,
                           lastcol ? sc.ee : sc.ie, ey);
            } else {
                d = g_cell(d, st[k], k == 0 ? in : st[k - 1], sv, inc0, inc1, gx, gy,
                           lastcol ? sc.eo : sc.io, lastcol ? sc.ee : sc.ie, oy, ey);
            }
        }
        if (W > 1 && ring_out != nullptr && lane == 63) ring_put(ring_out + (i & (RING - 1)), st[K - 1]);
    }
    carry = best_of<LINEAR>(in);
}

// Dynamic LDS: [uint32 xinfo[xcap]] [RingEntry ring[W-1][RING]]
// xinfo[i-1] = byte | lut shift << 8 (base 0..3, 24 = not ACGT) |
//              (row i contributes Iy gaps: i-1 >= fx && i <= lx) << 13 | (byte is ACGT) << 14
template <int K, int W, bool LINEAR, bool DEF, int OCC>
__global__ void __launch_bounds__(64 * W, OCC)
k_align(SetView XS, SetView YS, PairSrc ps, KScores scin, MetricSpec ms, int xcap, int out_mode,
        double* __restrict__ out, int32_t* __restrict__ sout) {
    using S = typename StateOf<LINEAR>::T;
    using B = typename StateOf<LINEAR>::B;
    const KScores sc = DEF ? KScores{1, -1, -8, -1, -1, -1} : scin;  // align.py:20-27 defaults
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* xinfo = reinterpret_cast<uint32_t*>(smem);
    RingEntry* rings = reinterpret_cast<RingEntry*>(smem + ((size_t)xcap * 4 + 15) / 16 * 16);

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int nm = ms.n;

    for (int64_t p = blockIdx.x; p < ps.count; p += gridDim.x) {
        int64_t a, b;
        decode_pair(ps, p, a, b);
        const int4 ma = XS.meta[a];
        const int4 mb = YS.meta[b];
        // Rows = the shorter sequence, columns = the longer one (cost ~ (rows + 63) x capacity).
        const bool swp = ma.x > mb.x;
        const uint8_t* rseq = swp ? YS.bytes + YS.offs[b] : XS.bytes + XS.offs[a];
        const uint8_t* cseq = swp ? XS.bytes + XS.offs[a] : YS.bytes + YS.offs[b];
        const int4 rm = swp ? mb : ma;
        const int4 cm = swp ? ma : mb;
        const int nA = rm.x, nB = cm.x;
        const int fx = rm.y, lx = rm.z, fy = cm.y, ly = cm.z;

        double* o_ab;
        double* o_ba = nullptr;
        if (out_mode == OUT_BOTH) {
            o_ab = out + (p * 2 + 0) * nm;
            o_ba = out + (p * 2 + 1) * nm;
        } else {
            o_ab = out + p * nm;
        }

        if (nA == 0 || nB == 0) {  // one side empty: no ACGT column can exist
            if (threadIdx.x == 0) {
                for (int m = 0; m < nm; ++m) {
                    o_ab[m] = __builtin_nan("");
                    if (o_ba) o_ba[m] = __builtin_nan("");
                }
                if (sout) {
                    const int n = nA + nB;
                    sout[p] = n == 0 ? 0 : (LINEAR ? n * sc.ee : sc.eo + sc.ee * (n - 1));
                }
            }
            continue;
        }

        __syncthreads();  // previous pair is done with xinfo / rings
        for (int i = threadIdx.x; i < nA; i += 64 * W) {
            const uint32_t c = rseq[i];
            const uint32_t bc = (uint32_t)base_code(c);
            const uint32_t riy = (i >= fx && i + 1 <= lx) ? 1u : 0u;
            xinfo[i] = c | ((bc < 4u ? bc : 24u) << 8) | (riy << 13) | ((bc < 4u ? 1u : 0u) << 14);
        }
        __syncthreads();

        // ---- per-lane column constants
        const int j0 = (w * 64 + lane) * K + 1;
        LaneCols<K> lc;
        lc.ixbits = lc.ynbits = lc.lastbits = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = j0 + k;
            uint32_t l = 0;
            if (j <= nB) {
                const uint32_t c = cseq[j - 1];
                const int yb = base_code(c);
                if (yb < 4) {
#pragma unroll
                    for (int xb = 0; xb < 4; ++xb) {
                        const int dd = xb ^ yb;
                        l |= 1u << xb;                             // valid
                        if (dd == 2) l |= 1u << (16 + xb);         // transition
                        else if (dd) l |= 1u << (20 + xb);         // transversion
                    }
                    lc.ynbits |= 1u << k;
                }
                l |= c << 8;
                if (j - 1 >= fy && j <= ly) lc.ixbits |= 1u << k;
                if (j == nB) lc.lastbits |= 1u << k;
            }
            lc.lut[k] = l;
        }

        S st[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if constexpr (LINEAR) st[k] = n_row0(j0 + k, sc);
            else st[k] = g_row0(j0 + k, sc);
        }
        B carry;
        if constexpr (LINEAR) carry = n_row0(j0 - 1, sc);
        else carry = g_best(g_row0(j0 - 1, sc));

        const RingEntry* ring_in = (w > 0) ? rings + (size_t)(w - 1) * RING : nullptr;
        RingEntry* ring_out = (w < W - 1) ? rings + (size_t)w * RING : nullptr;

        const int nsteps = nA + 63;  // local steps 0 .. nA+62
        const int nblk = (nsteps + INTERVAL - 1) / INTERVAL;
        const int nint = (W > 1) ? nblk + WAVE_LAG * (W - 1) : 1;

        for (int it = 0; it < nint; ++it) {
            const int blk = (W > 1) ? it - WAVE_LAG * w : 0;
            const int s0 = (W > 1) ? blk * INTERVAL : 0;
            const int s1 = (W > 1) ? min(s0 + INTERVAL, nsteps) : nsteps;
            if (W == 1 || (blk >= 0 && blk < nblk)) {
                if (w == 0) {
                    for (int s = s0; s < s1; ++s)
                        dp_step<K, W, LINEAR, true>(s, lane, nA, st, carry, lc, xinfo, ring_in, ring_out, sc);
                } else {
                    for (int s = s0; s < s1; ++s)
                        dp_step<K, W, LINEAR, false>(s, lane, nA, st, carry, lc, xinfo, ring_in, ring_out, sc);
                }
            }
            if (W > 1) __syncthreads();
        }

        // ---- epilogue: the lane owning column nB holds row nA
        const int jl = nB - 1;
        const int ow = jl / (64 * K);
        const int ol = (jl / K) & 63;
        if (w == ow && lane == ol) {
            const int kk = jl % K;
            S e = st[0];
#pragma unroll
            for (int k = 1; k < K; ++k)
                if (k == kk) e = st[k];
            const B fin = best_of<LINEAR>(e);
            C2 ca, cb;
            int score;
            if constexpr (LINEAR) {
                ca = fin.a;
                cb = fin.b;
                score = fin.S;
            } else {
                ca = fin.a;
                cb = fin.b;
                score = fin.h;
            }
            // orientation A is (rows, cols); map back to (a, b)
            const C2 ab = swp ? cb : ca;
            const C2 ba = swp ? ca : cb;
            for (int m = 0; m < nm; ++m) {
                o_ab[m] = metric_value(ms.code[m], ab.w0 & 0xFFFFu, ab.w0 >> 16, ab.w1 >> 20,
                                       ab.w1 & 0xFFFFFu);
                if (o_ba)
                    o_ba[m] = metric_value(ms.code[m], ba.w0 & 0xFFFFu, ba.w0 >> 16, ba.w1 >> 20,
                                           ba.w1 & 0xFFFFFu);
            }
            if (sout) sout[p] = score;
        }
    }
}

}  // namespace taxi2
