// Single-orientation aligner with a divergence flag (Gotoh scores, sequences <= 4095).
//
// Same fill as align_kernel.hpp (Biopython first-path Gotoh, forward-carried counters,
// systolic lanes, tie-tagged doubled scores) but each state carries the counters of ONE
// traceback orientation.  Why that is enough: the (x, y) alignment (priority A = M>Ix>Iy) and
// the (y, x) alignment (priority B = M>Iy>Ix) trace the same DP values and differ only where a
// predecessor choice ties between Ix and Iy.  In tie-tagged form such a "divergent" tie is an
// exact equality of two tagged scores (cg == cx, cf == cy, G == X, F == Y; ties that involve M
// differ by the tag bit and both priorities resolve them to M).  So pass 1 runs orientation A
// and counts, along A's path, the divergent ties it passes (a counter field like any other).
// If the count is 0, B's traceback makes A's choice at every cell of A's path, so B's
// alignment IS A's alignment and both ordered pairs get the same counters.  Pairs with a
// count > 0 go to a device worklist and pass 2 re-runs them in orientation B.  Both results
// are bit-exact; pass 2 typically sees a few percent of the pairs (0 % on the reference's
// sample files, ~10 % on highly similar synthetic families).
//
// Per cell this halves the counter work of the two-orientation kernel (5 selects x NW words,
// one add per move), and the divergent-tie count rides the gap add as the carry-in of one
// v_addc.  Counter words, NW = 2 (lengths <= 1023):  w0 = valid | ts << 10 | tv << 20,
// w1 = divergent ties | gap << 14 (both <= nA + nB + 1 <= 2047).  NW = 3 (lengths <= 4095):
// w0 = valid | ts << 16, w1 = ties | gap << 14 (<= 8191 each), w2 = tv << 20 (so the row-base LUT
// bit for tv is already in place: one AND, no shift).
//
// The M score uses an equality field instead of a byte compare: per lane, eqp[r] holds for
// each of its K columns a 3-bit field = 4 where the column byte is "ACGT"[r], so for the usual
// exact A/C/G/T row byte the doubled substitution score is mismatch + field (default scores:
// -2 + {0, 4}); rows with any other byte take a (rare, wave-uniformly skipped) compare path.
#pragma once
#include "align_kernel.hpp"

namespace taxi2 {

constexpr uint32_t A1_GAP = 1u << 14;          // gap unit in w1 (= the x-gap flag bit of the LUT)
constexpr int A1_MAX_LEN = 1023;               // NW = 2 counters
constexpr int A1_MAX_LEN_LONG = 4095;          // NW = 3 counters
constexpr int A1_MAX_K = 10;                   // 3-bit equality fields in one word

// Counter words of one orientation; layout per NW above.
template <int NW>
struct Cnt {
    uint32_t w[NW];
};
template <int NW>
__device__ __forceinline__ Cnt<NW> cselw(bool c, const Cnt<NW>& a, const Cnt<NW>& b) {
    Cnt<NW> r;
#pragma unroll
    for (int k = 0; k < NW; ++k) r.w[k] = c ? a.w[k] : b.w[k];
    return r;
}
template <int NW>
__device__ __forceinline__ Cnt<NW> cnt_zero() {
    Cnt<NW> r;
#pragma unroll
    for (int k = 0; k < NW; ++k) r.w[k] = 0u;
    return r;
}
// w0 units of a diagonal nucleotide column, shifted into place by the row base (LUT bits r, +ts, +tv)
template <int NW> constexpr uint32_t a1_inc0_mask() { return NW == 2 ? 0x00100401u : 0x00010001u; }
template <int NW> constexpr int a1_ts_bit() { return NW == 2 ? 10 : 16; }

template <int NW>
struct S1Col {
    int G;  // 2 * max(M, Iy) + (M won)
    Cnt<NW> g;
    int X;  // 2 * Ix
    Cnt<NW> x;
};
template <int NW>
struct S1Left {
    int F;  // 2 * max(M, Ix) + (M won)
    Cnt<NW> f;
    int Y;  // 2 * Iy
    Cnt<NW> y;
};
template <int NW>
struct S1Best {
    int h;
    Cnt<NW> c;
};

// Best of a column state (the diagonal successor's source / the final cell).
// A: G wins iff G > X (tagged);  B: G wins iff G >= X.  Divergent iff G == X.
template <bool B, bool TRACK, int NW>
__device__ __forceinline__ S1Best<NW> s1_best_col(const S1Col<NW>& u) {
    const bool take = B ? (u.G >= u.X) : (u.G > u.X);
    S1Best<NW> r{max(u.G, u.X), cselw(take, u.g, u.x)};
    if (TRACK) r.c.w[1] += (u.G == u.X) ? 1u : 0u;
    return r;
}
// Best of a left payload.  A: F wins iff F >= Y;  B: iff F > Y.  Divergent iff F == Y.
template <bool B, bool TRACK, int NW>
__device__ __forceinline__ S1Best<NW> s1_best_left(const S1Left<NW>& l) {
    const bool take = B ? (l.F > l.Y) : (l.F >= l.Y);
    S1Best<NW> r{max(l.F, l.Y), cselw(take, l.f, l.y)};
    if (TRACK) r.c.w[1] += (l.F == l.Y) ? 1u : 0u;
    return r;
}

// Row 0 / column 0 boundaries on doubled scores d (see g_col_row0 / g_left_row0).
template <int NW>
__device__ __forceinline__ S1Col<NW> s1_col_row0(int j, const KScores& d) {
    S1Col<NW> c;
    c.G = (j == 0) ? 1 : d.eo + d.ee * (j - 1);
    c.X = NEG_INF;
    c.g = c.x = cnt_zero<NW>();
    return c;
}
template <int NW>
__device__ __forceinline__ S1Left<NW> s1_left_row0(int j, const KScores& d) {
    S1Left<NW> l;
    l.F = (j == 0) ? 1 : NEG_INF;
    l.Y = (j == 0) ? NEG_INF : d.eo + d.ee * (j - 1);
    l.f = l.y = cnt_zero<NW>();
    return l;
}
template <int NW>
__device__ __forceinline__ S1Left<NW> s1_shr_first(const S1Left<NW>& v, int i, const KScores& d) {
    S1Left<NW> r;
    r.F = (int)shr_old((uint32_t)v.F, (uint32_t)(d.eo + d.ee * (i - 1)));
    r.Y = (int)shr_old((uint32_t)v.Y, (uint32_t)NEG_INF);
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        r.f.w[k] = shr_zero(v.f.w[k]);
        r.y.w[k] = shr_zero(v.y.w[k]);
    }
    return r;
}
template <int NW>
__device__ __forceinline__ S1Left<NW> s1_shr_old(const S1Left<NW>& v, const S1Left<NW>& o) {
    S1Left<NW> r;
    r.F = (int)shr_old((uint32_t)v.F, (uint32_t)o.F);
    r.Y = (int)shr_old((uint32_t)v.Y, (uint32_t)o.Y);
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        r.f.w[k] = shr_old(v.f.w[k], o.f.w[k]);
        r.y.w[k] = shr_old(v.y.w[k], o.y.w[k]);
    }
    return r;
}

// One cell in place (see g_cell for the state algebra); inc0 / inc2 = valid/ts(/tv) units of the
// M move in w0 / w2 (NW = 3), gx / gy = gap units of the Ix / Iy moves, sM = doubled substitution.
template <bool B, bool TRACK, int NW>
__device__ __forceinline__ S1Best<NW> s1_cell(const S1Best<NW>& d, S1Col<NW>& u, S1Left<NW>& l, int sM,
                                              uint32_t inc0, uint32_t inc2, uint32_t gx, uint32_t gy, int ox,
                                              int ex, int oy, int ey) {
    const S1Best<NW> nd = s1_best_col<B, TRACK>(u);
    const int M = (d.h | 1) + sM;
    Cnt<NW> m = d.c;
    m.w[0] += inc0;
    if constexpr (NW == 3) m.w[2] += inc2;
    // Ix from above. A: G-path iff cg > cx;  B: iff cg >= cx.
    const int cg = u.G + ox, cx = u.X + ex;
    const int X = max(cg, cx) & ~1;
    Cnt<NW> x = cselw(B ? (cg >= cx) : (cg > cx), u.g, u.x);
    asm volatile("" : "+v"(gx));  // opaque: keeps "w1 + gap unit + tie" one v_addc
    x.w[1] += gx;
    if (TRACK) x.w[1] += (cg == cx) ? 1u : 0u;
    // Iy from the left. A: F-path iff cf >= cy;  B: iff cf > cy.
    const int cf = l.F + oy, cy = l.Y + ey;
    const int Y = max(cf, cy) & ~1;
    Cnt<NW> y = cselw(B ? (cf > cy) : (cf >= cy), l.f, l.y);
    asm volatile("" : "+v"(gy));
    y.w[1] += gy;
    if (TRACK) y.w[1] += (cf == cy) ? 1u : 0u;
    // M wins ties against Iy and Ix under both priorities (M odd, X / Y even)
    const bool gs = M > Y;
    u.G = max(M, Y);
    u.g = cselw(gs, m, y);
    u.X = X;
    u.x = x;
    const bool fs = M > X;
    l.F = max(M, X);
    l.f = cselw(fs, m, x);
    l.Y = Y;
    l.y = y;
    return nd;
}

struct RingEntry1 {
    uint4 q[2];
};
template <int NW>
__device__ __forceinline__ void ring_put(RingEntry1* e, const S1Left<NW>& s) {
    if constexpr (NW == 2) {
        e->q[0] = make_uint4((uint32_t)s.F, s.f.w[0], s.f.w[1], (uint32_t)s.Y);
        e->q[1] = make_uint4(s.y.w[0], s.y.w[1], 0u, 0u);
    } else {
        e->q[0] = make_uint4((uint32_t)s.F, s.f.w[0], s.f.w[1], s.f.w[2]);
        e->q[1] = make_uint4((uint32_t)s.Y, s.y.w[0], s.y.w[1], s.y.w[2]);
    }
}
template <int NW>
__device__ __forceinline__ void ring_get(const RingEntry1* e, S1Left<NW>& s) {
    const uint4 a = e->q[0], b = e->q[1];
    if constexpr (NW == 2) {
        s.F = (int)a.x;
        s.f.w[0] = a.y;
        s.f.w[1] = a.z;
        s.Y = (int)a.w;
        s.y.w[0] = b.x;
        s.y.w[1] = b.y;
    } else {
        s.F = (int)a.x;
        s.f.w[0] = a.y;
        s.f.w[1] = a.z;
        s.f.w[2] = a.w;
        s.Y = (int)b.x;
        s.y.w[0] = b.y;
        s.y.w[1] = b.z;
        s.y.w[2] = b.w;
    }
}

// Per-lane column constants.  The LUT (two uses per cell) and the equality fields stay in
// VGPRs; the once-per-cell constants live in LDS (ColC, [k][thread]) so that K = 8 fits the
// 128-VGPR budget of occupancy 4 without spilling: LDS reads issue on the LDS pipe, not the
// (saturated) VALU.
template <int K>
struct LaneCols1 {
    uint32_t lut[K];  // w0 units by row base r: valid bit r, ts bit a1_ts_bit + r, tv bit 20 + r;
                      // bit 14 (= A1_GAP): an x-gap in column j lies in y's nucleotide span;
                      // column byte << 24
    uint32_t eqp0, eqp1, eqp2, eqp3;  // 3-bit field per column: 4 where the byte is "ACGT"[r]
};
struct ColC {
    uint32_t yn;  // A1_GAP if y[j-1] is a nucleotide
    int ox;       // doubled Ix open (end-gap open on column nB)
};

// Dynamic LDS of k_align1: [uint32 xinfo[xcap]] [RingEntry1 ring[W-1][RING]]
// [ColC colc[K][64W]] [int colex[K][64W] (non-default scores: Ix extend)]
__host__ __device__ inline size_t a1_lds_ring_off(int xcap) { return ((size_t)xcap * 4 + 15) / 16 * 16; }
__host__ __device__ inline size_t a1_lds_colc_off(int xcap, int W) {
    return a1_lds_ring_off(xcap) + (size_t)(W - 1) * RING * sizeof(RingEntry1);
}
__host__ __device__ inline size_t a1_lds_bytes(int xcap, int K, int W, bool def) {
    return a1_lds_colc_off(xcap, W) + (size_t)K * 64 * W * (sizeof(ColC) + (def ? 0 : sizeof(int)));
}

// xinfo[i-1] (LDS) for row i: byte | base code << 8 (0..3; >= 4 not a nucleotide) |
// exact "ACGT" code << 11 (4 = other byte) | (x-gap row in x's span) << 14 | nucleotide << 15
__device__ __forceinline__ uint32_t a1_xinfo(uint32_t c, int i, int fx, int lx) {
    const uint32_t bc = (uint32_t)base_code(c);
    const uint32_t ec = c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
    const uint32_t riy = (i >= fx && i + 1 <= lx) ? 1u : 0u;
    return c | (bc << 8) | (ec << 11) | (riy << 14) | ((bc < 4u ? 1u : 0u) << 15);
}

template <int K, int W, bool DEF, bool B, bool FIRST, int NW>
__device__ __forceinline__ void dp_step1(int s, int lane, int nA, S1Col<NW> (&st)[K], S1Left<NW>& pay,
                                         S1Best<NW>& carry, const LaneCols1<K>& lc, const ColC* __restrict__ colc,
                                         const int* __restrict__ colex, const uint32_t* __restrict__ xinfo,
                                         const RingEntry1* __restrict__ ring_in, RingEntry1* __restrict__ ring_out,
                                         const KScores& sc) {
    constexpr bool TRACK = !B;
    S1Left<NW> in;
    if constexpr (FIRST) {
        in = s1_shr_first(pay, s + 1, sc);
    } else {
        S1Left<NW> old;
        ring_get(ring_in + ((s + 1) & (RING - 1)), old);
        in = s1_shr_old(pay, old);
    }
    const int i = s - lane + 1;
    if (i >= 1 && i <= nA) {
        const uint32_t xi = xinfo[i - 1];
        const bool nuc = (xi >> 15) & 1u;
        const uint32_t xsh = (xi >> 8) & 3u;
        const uint32_t incm0 = nuc ? a1_inc0_mask<NW>() : 0u;
        const uint32_t incm2 = nuc ? (1u << 20) : 0u;
        const uint32_t gxrow = nuc ? A1_GAP : 0u;
        const uint32_t gyrow = ((xi >> 14) & 1u) ? ~0u : 0u;
        const uint32_t ec = (xi >> 11) & 7u;
        const uint32_t eqlo = (ec & 1u) ? lc.eqp1 : lc.eqp0;
        const uint32_t eqhi = (ec & 1u) ? lc.eqp3 : lc.eqp2;
        uint32_t eq = (ec & 2u) ? eqhi : eqlo;
        if (ec >= 4u) {  // not an exact A/C/G/T byte: compare bytes
            const uint32_t xb = xi & 0xFFu;
            eq = 0u;
#pragma unroll
            for (int k = 0; k < K; ++k) eq |= ((lc.lut[k] >> 24) == xb) ? (4u << (3 * k)) : 0u;
        }
        const bool lastrow = (i == nA);
        const int oy = lastrow ? sc.eo : sc.io;
        const int ey = lastrow ? sc.ee : sc.ie;
        S1Best<NW> d = carry;
        S1Left<NW> l = in;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t e = (eq >> (3 * k)) & 7u;
            const int sM = DEF ? sc.mi + (int)e : (e ? sc.ma : sc.mi);
            const uint32_t t = lc.lut[k] >> xsh;
            const ColC cc = colc[k * 64 * W];
            const int ex = DEF ? sc.ie : colex[k * 64 * W];
            d = s1_cell<B, TRACK>(d, st[k], l, sM, t & incm0, t & incm2, lc.lut[k] & gxrow, cc.yn & gyrow, cc.ox,
                                  ex, oy, ey);
        }
        pay = l;
        if (W > 1 && ring_out != nullptr && lane == 63) ring_put(ring_out + (i & (RING - 1)), pay);
    }
    carry = s1_best_left<B, TRACK>(in);
}

template <int NW>
__device__ __forceinline__ void a1_write(double* o, const MetricSpec& ms, const Cnt<NW>& c) {
    uint32_t valid, ts, tv, gap;
    if constexpr (NW == 2) {
        valid = c.w[0] & 0x3FFu;
        ts = (c.w[0] >> 10) & 0x3FFu;
        tv = (c.w[0] >> 20) & 0x3FFu;
        gap = (c.w[1] >> 14) & 0xFFFu;
    } else {
        valid = c.w[0] & 0xFFFFu;
        ts = c.w[0] >> 16;
        tv = c.w[2] >> 20;
        gap = c.w[1] >> 14;
    }
    for (int m = 0; m < ms.n; ++m) o[m] = metric_value(ms.code[m], valid, ts, tv, gap);
}

// Pass 1 (B = false): every pair of `ps` in orientation A (rows = the shorter sequence);
// writes A's slot, and B's slot too when A's path has no divergent tie, else appends the pair
// to wlist.  Pass 2 (B = true): the pairs of wlist[0, *wcount) in orientation B, B's slot.
template <int K, int W, bool DEF, int OCC, bool B, int NW>
__global__ void __launch_bounds__(64 * W, OCC)
k_align1(SetView XS, SetView YS, PairSrc ps, KScores scin, MetricSpec ms, int xcap, int out_mode,
         double* __restrict__ out, int32_t* __restrict__ sout, uint32_t* __restrict__ wlist,
         uint32_t* __restrict__ wcount, unsigned long long* __restrict__ next) {
    static_assert(K <= A1_MAX_K, "equality fields hold at most 10 columns");
    const KScores sc0 = DEF ? KScores{1, -1, -8, -1, -1, -1} : scin;  // align.py:20-27 defaults
    const KScores sc = doubled(sc0);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* xinfo = reinterpret_cast<uint32_t*>(smem);
    RingEntry1* rings = reinterpret_cast<RingEntry1*>(smem + a1_lds_ring_off(xcap));
    ColC* colc = reinterpret_cast<ColC*>(smem + a1_lds_colc_off(xcap, W)) + threadIdx.x;
    int* colex = reinterpret_cast<int*>(reinterpret_cast<ColC*>(smem + a1_lds_colc_off(xcap, W)) + K * 64 * W) +
                 threadIdx.x;

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int nm = ms.n;
    const int64_t total = B ? (int64_t)*wcount : ps.count;
    __shared__ int64_t s_next;

    // Persistent workgroups pull pairs from a device counter: the per-lane prologue runs once
    // per workgroup, and ragged lengths balance dynamically.
    for (;;) {
        __syncthreads();  // previous pair is done with xinfo / rings / s_next
        if (threadIdx.x == 0) s_next = (int64_t)atomicAdd(next, 1ull);
        __syncthreads();
        const int64_t q = s_next;
        if (q >= total) break;
        const int64_t p = B ? (int64_t)wlist[q] : q;
        int64_t a, b;
        decode_pair(ps, p, a, b);
        const int4 ma = XS.meta[a];
        const int4 mb = YS.meta[b];
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
        // orientation A = (rows, cols): the (a, b) slot unless swapped
        double* slot_a = swp ? o_ba : o_ab;
        double* slot_b = swp ? o_ab : o_ba;

        if (nA == 0 || nB == 0) {  // one side empty (pass 1 only): no nucleotide column
            if (threadIdx.x == 0) {
                for (int m = 0; m < nm; ++m) {
                    o_ab[m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                    if (o_ba) o_ba[m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                }
                if (sout) {
                    const int n = nA + nB;
                    sout[p] = n == 0 ? 0 : sc0.eo + sc0.ee * (n - 1);
                }
            }
            continue;
        }

        for (int i = threadIdx.x; i < nA; i += 64 * W) xinfo[i] = a1_xinfo(rseq[i], i, fx, lx);
        __syncthreads();

        const int j0 = (w * 64 + lane) * K + 1;
        LaneCols1<K> lc;
        lc.eqp0 = lc.eqp1 = lc.eqp2 = lc.eqp3 = 0u;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = j0 + k;
            uint32_t l = 0, yn = 0;
            if (j <= nB) {
                const uint32_t c = cseq[j - 1];
                const int yb = base_code(c);
                if (yb < 4) {
#pragma unroll
                    for (int xb = 0; xb < 4; ++xb) {
                        const int dd = xb ^ yb;
                        l |= 1u << xb;                      // valid
                        if (dd == 2) l |= 1u << (a1_ts_bit<NW>() + xb);  // transition
                        else if (dd) l |= 1u << (20 + xb);  // transversion
                    }
                    yn = A1_GAP;
                }
                l |= c << 24;
                if (c == 'A') lc.eqp0 |= 4u << (3 * k);
                if (c == 'C') lc.eqp1 |= 4u << (3 * k);
                if (c == 'G') lc.eqp2 |= 4u << (3 * k);
                if (c == 'T') lc.eqp3 |= 4u << (3 * k);
                if (j - 1 >= fy && j <= ly) l |= A1_GAP;
            }
            lc.lut[k] = l;
            colc[k * 64 * W] = ColC{yn, (j == nB) ? sc.eo : sc.io};
            if (!DEF) colex[k * 64 * W] = (j == nB) ? sc.ee : sc.ie;
        }

        S1Col<NW> st[K];
#pragma unroll
        for (int k = 0; k < K; ++k) st[k] = s1_col_row0<NW>(j0 + k, sc);
        S1Left<NW> pay = s1_left_row0<NW>(j0 + K - 1, sc);
        S1Best<NW> carry = s1_best_col<B, false>(s1_col_row0<NW>(j0 - 1, sc));

        const RingEntry1* ring_in = (w > 0) ? rings + (size_t)(w - 1) * RING : nullptr;
        RingEntry1* ring_out = (w < W - 1) ? rings + (size_t)w * RING : nullptr;

        const int nsteps = nA + 63;
        const int nblk = (nsteps + INTERVAL - 1) / INTERVAL;
        const int nint = (W > 1) ? nblk + WAVE_LAG * (W - 1) : 1;
        for (int it = 0; it < nint; ++it) {
            const int blk = (W > 1) ? it - WAVE_LAG * w : 0;
            const int s0 = (W > 1) ? blk * INTERVAL : 0;
            const int s1 = (W > 1) ? min(s0 + INTERVAL, nsteps) : nsteps;
            if (W == 1 || (blk >= 0 && blk < nblk)) {
                if (w == 0) {
                    for (int s = s0; s < s1; ++s)
                        dp_step1<K, W, DEF, B, true, NW>(s, lane, nA, st, pay, carry, lc, colc, colex, xinfo, ring_in, ring_out, sc);
                } else {
                    for (int s = s0; s < s1; ++s)
                        dp_step1<K, W, DEF, B, false, NW>(s, lane, nA, st, pay, carry, lc, colc, colex, xinfo, ring_in, ring_out, sc);
                }
            }
            if (W > 1) __syncthreads();
        }

        const int jl = nB - 1;
        if (w == jl / (64 * K) && lane == ((jl / K) & 63)) {
            const int kk = jl % K;
            S1Col<NW> e = st[0];
#pragma unroll
            for (int k = 1; k < K; ++k)
                if (k == kk) e = st[k];
            const S1Best<NW> fin = s1_best_col<B, !B>(e);
            if (B) {
                a1_write(slot_b, ms, fin.c);
            } else {
                const bool diverges = (fin.c.w[1] & 0x3FFFu) != 0u;
                if (slot_a) a1_write(slot_a, ms, fin.c);
                if (slot_b) {
                    if (!diverges) a1_write(slot_b, ms, fin.c);
                    else wlist[atomicAdd(wcount, 1u)] = (uint32_t)p;
                }
                if (sout) sout[p] = fin.h >> 1;
            }
        }
    }
}

}  // namespace taxi2
