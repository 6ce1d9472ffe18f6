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
//     state in VGPRs (11 x K); rows stream through the lanes as a systolic wavefront: at local
//     step s lane l works on row i = s - l + 1.
//   * lane l-1 -> lane l hand-off of the last column state is one DPP `wave_shr:1` per
//     32-bit word (counters use bound_ctrl zero-fill for wave 0's left boundary); wave w-1
//     lane 63 -> wave w lane 0 goes through an LDS ring, wave w running two 64-step
//     intervals behind (one s_barrier per interval).
//   * per column only G = max(M, Iy) and Ix are kept (with both orientations' counters); the
//     3-way Biopython priorities reduce to 2-way selects on (G, Ix) and (F = max(M, Ix), Iy)
//     (see GCol below), and a cell's diagonal summary is derived from the column state before
//     the column is overwritten in place: no register copies between cells or steps.
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
// A column keeps, for the cell of the previous row: G = max(M, Iy) (+ whether M won, `gsrc`)
// and Ix, each with the counters of both orientations.  That is all the next row needs:
//   * Ix(i,j) = max(M + o, Ix + e, Iy + o) over (i-1, j) = max(G + o, Ix + e), and the 3-way
//     priorities reduce to 2-way rules on (G, Ix):
//       A (M>Ix>Iy): take G iff G+o > Ix+e, or equal and G came from M;
//       B (M>Iy>Ix): take G iff G+o >= Ix+e;
//   * the diagonal successor's best state = max(G, Ix) with the same two rules (offsets 0).
// A cell hands its right neighbour F = max(M, Ix) (+ `fsrc` = M won) and Iy:
//   * Iy(i,j+1) = max(F + o, Iy + e): A takes F iff F+o >= Iy+e (M and Ix beat Iy);
//     B takes F iff F+o > Iy+e, or equal and F came from M (Iy beats Ix in B);
//   * the best state of the cell = max(F, Iy) with the same rules (offsets 0).
// Tie-tagged scores: every score is stored doubled and bit 0 of G / F is the "M won" flag
// (M is formed odd, Ix / Iy are kept even), so max(M, Iy) sets the flag by itself and each
// rule above is ONE compare: "G+o > Ix+e, or equal and gsrc" == (2G+gsrc+2o > 2Ix+2e) and
// "G+o >= Ix+e" == (2G+gsrc+2o >= 2Ix+2e).  No boolean state crosses cells, rows or the
// divergent active-row branch.  The Gotoh path runs on doubled scores (KScores2).
// (Derivation checked exhaustively against the 3-way rules by the GPU parity tests.)
struct GCol {
    int G;      // 2 * max(M, Iy) + (M won)
    C2 ga, gb;  // counters of G's state; a = orientation A (x, y), b = orientation B (y, x)
    int X;      // 2 * Ix
    C2 xa, xb;
};

struct GLeft {
    int F;      // 2 * max(M, Ix) + (M won)
    C2 fa, fb;
    int Y;      // 2 * Iy
    C2 ya, yb;
};

// Best state of a cell under both priorities (what the diagonal successor reads); h is the
// doubled score with an arbitrary bit 0.
struct GBest {
    int h;
    C2 a, b;
};

__device__ __forceinline__ KScores doubled(const KScores& k) {
    return KScores{2 * k.ma, 2 * k.mi, 2 * k.io, 2 * k.ie, 2 * k.eo, 2 * k.ee};
}

__device__ __forceinline__ GBest g_best_col(const GCol& u) {
    const bool pa = u.G > u.X;
    const bool pb = u.G >= u.X;
    return GBest{max(u.G, u.X), csel(pa, u.ga, u.xa), csel(pb, u.gb, u.xb)};
}

__device__ __forceinline__ GBest g_best_left(const GLeft& l) {
    const bool pa = l.F >= l.Y;
    const bool pb = l.F > l.Y;
    return GBest{max(l.F, l.Y), csel(pa, l.fa, l.ya), csel(pb, l.fb, l.yb)};
}

// Row 0 (doubled scores d): M(0,0) = 0, Iy(0,j) = eo + ee*(j-1), everything else -inf,
// counters 0.
__device__ __forceinline__ GCol g_col_row0(int j, const KScores& d) {
    GCol c;
    c.G = (j == 0) ? 1 : d.eo + d.ee * (j - 1);
    c.X = NEG_INF;
    c.ga = c.gb = c.xa = c.xb = C2{0u, 0u};
    return c;
}
__device__ __forceinline__ GLeft g_left_row0(int j, const KScores& d) {
    GLeft l;
    l.F = (j == 0) ? 1 : NEG_INF;
    l.Y = (j == 0) ? NEG_INF : d.eo + d.ee * (j - 1);
    l.fa = l.fb = l.ya = l.yb = C2{0u, 0u};
    return l;
}

// Lane 0 of wave 0 receives column 0 at row i: Ix = eo + ee*(i-1) (so F = Ix, untagged),
// M = Iy = -inf, counters 0 (bound_ctrl zero-fill).
__device__ __forceinline__ GLeft g_shr_first(const GLeft& v, int i, const KScores& d) {
    GLeft r;
    r.F = (int)shr_old((uint32_t)v.F, (uint32_t)(d.eo + d.ee * (i - 1)));
    r.Y = (int)shr_old((uint32_t)v.Y, (uint32_t)NEG_INF);
#define T2_SZ(f) r.f.w0 = shr_zero(v.f.w0); r.f.w1 = shr_zero(v.f.w1);
    T2_SZ(fa) T2_SZ(fb) T2_SZ(ya) T2_SZ(yb)
#undef T2_SZ
    return r;
}

__device__ __forceinline__ GLeft g_shr_old(const GLeft& v, const GLeft& o) {
    GLeft r;
    r.F = (int)shr_old((uint32_t)v.F, (uint32_t)o.F);
    r.Y = (int)shr_old((uint32_t)v.Y, (uint32_t)o.Y);
#define T2_SO(f) r.f.w0 = shr_old(v.f.w0, o.f.w0); r.f.w1 = shr_old(v.f.w1, o.f.w1);
    T2_SO(fa) T2_SO(fb) T2_SO(ya) T2_SO(yb)
#undef T2_SO
    return r;
}

// One Gotoh cell, in place, on doubled scores.  d = best of (i-1, j-1); u = column state of
// (i-1, j) on entry, (i, j) on exit; l = left payload of (i, j-1) on entry, (i, j) on exit.
// Returns the best of (i-1, j) for the next column's diagonal.
__device__ __forceinline__ GBest g_cell(const GBest& d, GCol& u, GLeft& l, int s, uint32_t inc0,
                                        uint32_t inc1, uint32_t gx, uint32_t gy, int ox, int ex, int oy,
                                        int ey) {
    const GBest nd = g_best_col(u);
    // M: diagonal move from the best state of (i-1, j-1); odd = tagged "M"
    const int M = (d.h | 1) + s;
    const C2 ma{d.a.w0 + inc0, d.a.w1 + inc1};
    const C2 mb{d.b.w0 + inc0, d.b.w1 + inc1};
    // Ix: consume x[i-1] against a gap (from above)
    const int cg = u.G + ox, cx = u.X + ex;
    const int X = max(cg, cx) & ~1;
    C2 xa = csel(cg > cx, u.ga, u.xa);
    C2 xb = csel(cg >= cx, u.gb, u.xb);
    xa.w1 += gx;
    xb.w1 += gx;
    // Iy: consume y[j-1] against a gap (from the left)
    const int cf = l.F + oy, cy = l.Y + ey;
    const int Y = max(cf, cy) & ~1;
    C2 ya = csel(cf >= cy, l.fa, l.ya);
    C2 yb = csel(cf > cy, l.fb, l.yb);
    ya.w1 += gy;
    yb.w1 += gy;
    // column state of (i, j) for the next row: M wins ties (M odd, Y even)
    const bool gs = M > Y;
    u.G = max(M, Y);
    u.ga = csel(gs, ma, ya);
    u.gb = csel(gs, mb, yb);
    u.X = X;
    u.xa = xa;
    u.xb = xb;
    // left payload of (i, j) for the next column
    const bool fs = M > X;
    l.F = max(M, X);
    l.fa = csel(fs, ma, xa);
    l.fb = csel(fs, mb, xb);
    l.Y = Y;
    l.ya = ya;
    l.yb = yb;
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
    uint4 q[4];  // 16 words; Gotoh uses 10, NW 5
};

__device__ __forceinline__ void ring_put(RingEntry* e, const GLeft& s) {
    e->q[0] = make_uint4((uint32_t)s.F, s.fa.w0, s.fa.w1, s.fb.w0);
    e->q[1] = make_uint4(s.fb.w1, (uint32_t)s.Y, s.ya.w0, s.ya.w1);
    e->q[2] = make_uint4(s.yb.w0, s.yb.w1, 0u, 0u);
}
__device__ __forceinline__ void ring_get(const RingEntry* e, GLeft& s) {
    const uint4 a = e->q[0], b = e->q[1], c = e->q[2];
    s.F = (int)a.x; s.fa.w0 = a.y; s.fa.w1 = a.z; s.fb.w0 = a.w;
    s.fb.w1 = b.x; s.Y = (int)b.y; s.ya.w0 = b.z; s.ya.w1 = b.w;
    s.yb.w0 = c.x; s.yb.w1 = c.y;
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

// Per-variant state types: T = per-column state, P = lane-to-lane payload, B = diagonal summary.
template <bool LINEAR>
struct StateOf {
    using T = GCol;
    using P = GLeft;
    using B = GBest;
};
template <>
struct StateOf<true> {
    using T = NState;
    using P = NState;
    using B = NBest;
};

// Per-lane, per-pair column constants.
template <int K>
struct LaneCols {
    uint32_t lut[K];   // bits 0-3 valid / 16-19 ts / 20-23 tv by row base; 8-15 column byte
    uint32_t ixbits;   // column j: x-gap column lies in the common range (j-1 >= fy, j <= ly)
    uint32_t ynbits;   // column j: y[j-1] is ACGT
    uint32_t lastbits; // column j == nB (end-gap scores for Ix / vertical)
};

// One systolic step for this lane: receive the left payload, then update K cells of row
// i = s - lane + 1.  `pay` is this lane's outgoing payload (its last column, previous row on
// entry, this row on exit); `carry` is the best-state summary of the left input of the
// previous step (the diagonal of this step's first cell) and is replaced by this step's.
template <int K, int W, bool LINEAR, bool FIRST>
__device__ __forceinline__ void dp_step(int s, int lane, int nA, typename StateOf<LINEAR>::T (&st)[K],
                                        typename StateOf<LINEAR>::P& pay, typename StateOf<LINEAR>::B& carry,
                                        const LaneCols<K>& lc, const uint32_t* __restrict__ xinfo,
                                        const RingEntry* __restrict__ ring_in, RingEntry* __restrict__ ring_out,
                                        const KScores& sc) {
    using P = typename StateOf<LINEAR>::P;
    using B = typename StateOf<LINEAR>::B;
    P in;
    if constexpr (FIRST) {
        if constexpr (LINEAR) in = n_shr_first(pay, s + 1, sc);
        else in = g_shr_first(pay, s + 1, sc);
    } else {
        P old;
        ring_get(ring_in + ((s + 1) & (RING - 1)), old);
        if constexpr (LINEAR) in = n_shr_old(pay, old);
        else in = g_shr_old(pay, old);
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
        P l = in;
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
                d = n_cell(d, st[k], k == 0 ? l : st[k - 1], sv, inc0, inc1, gx, gy,
                           lastcol ? sc.ee : sc.ie, ey);
            } else {
                d = g_cell(d, st[k], l, sv, inc0, inc1, gx, gy, lastcol ? sc.eo : sc.io,
                           lastcol ? sc.ee : sc.ie, oy, ey);
            }
        }
        if constexpr (LINEAR) pay = st[K - 1];
        else pay = l;
        if (W > 1 && ring_out != nullptr && lane == 63) ring_put(ring_out + (i & (RING - 1)), pay);
    }
    if constexpr (LINEAR) carry = in;
    else carry = g_best_left(in);
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
    const KScores sc0 = DEF ? KScores{1, -1, -8, -1, -1, -1} : scin;  // align.py:20-27 defaults
    const KScores sc = LINEAR ? sc0 : doubled(sc0);  // DP scores (Gotoh: tie-tagged, doubled)
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
                    o_ab[m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                    if (o_ba) o_ba[m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                }
                if (sout) {
                    const int n = nA + nB;
                    sout[p] = n == 0 ? 0 : (LINEAR ? n * sc0.ee : sc0.eo + sc0.ee * (n - 1));
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
            else st[k] = g_col_row0(j0 + k, sc);
        }
        typename StateOf<LINEAR>::P pay;
        B carry;
        if constexpr (LINEAR) {
            pay = st[K - 1];
            carry = n_row0(j0 - 1, sc);
        } else {
            pay = g_left_row0(j0 + K - 1, sc);
            carry = g_best_col(g_col_row0(j0 - 1, sc));
        }

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
                        dp_step<K, W, LINEAR, true>(s, lane, nA, st, pay, carry, lc, xinfo, ring_in, ring_out, sc);
                } else {
                    for (int s = s0; s < s1; ++s)
                        dp_step<K, W, LINEAR, false>(s, lane, nA, st, pay, carry, lc, xinfo, ring_in, ring_out, sc);
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
            C2 ca, cb;
            int score;
            if constexpr (LINEAR) {
                ca = e.a;
                cb = e.b;
                score = e.S;
            } else {
                const GBest fin = g_best_col(e);
                ca = fin.a;
                cb = fin.b;
                score = fin.h >> 1;
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
