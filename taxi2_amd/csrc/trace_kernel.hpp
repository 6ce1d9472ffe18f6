// Aligned strings for pairs whose alignment itself is needed: Biopython.align(pair) returning
// the aligned SequencePair (align.py:151-157) and the aligned_pairs.txt writer
// (versus_all.py:535-544, pairs.py:51-97).  The distance hot path never needs this (it carries
// counters forward, align_kernel.hpp); this path stores the tie sets.
//
// k_trace_fill: same systolic layout as k_align (lane owns K columns, rows stream through the
//   wave, DPP wave_shr hand-off, LDS ring between waves) but each cell keeps only its scores and
//   writes a 9-bit tie set {M preds, Ix preds, Iy preds} (NW: {D, V, H}).  Storage is step-major:
//   trace[pair][s][lane_global][k] (u16), so each wave stores one contiguous 16*K-byte chunk per
//   lane per step (fully coalesced).
// k_traceback: one thread per (pair, orientation) walks from (nA, nB): end state = first of the
//   priority order among the optimal states, then each backward step takes the first tied
//   predecessor (A: M>Ix>Iy, NW H>V>D; B, i.e. the (y, x) alignment: M>Iy>Ix, NW V>H>D).
#pragma once
#include "align_kernel.hpp"

namespace taxi2 {

struct TState {
    int M, X, Y;
};

template <int K, int W, bool LINEAR>
__global__ void __launch_bounds__(64 * W, 2)
k_trace_fill(SetView XS, SetView YS, const int64_t* __restrict__ xs, const int64_t* __restrict__ ys,
             int64_t count, KScores sc, int xcap, uint16_t* __restrict__ trace, int4* __restrict__ ends) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* xinfo = reinterpret_cast<uint32_t*>(smem);
    RingEntry* rings = reinterpret_cast<RingEntry*>(smem + ((size_t)xcap * 4 + 15) / 16 * 16);
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t stride = (int64_t)(xcap + 63) * 64 * W * K;

    for (int64_t p = blockIdx.x; p < count; p += gridDim.x) {
        const int64_t a = xs[p], b = ys[p];
        const uint8_t* rseq = XS.bytes + XS.offs[a];
        const uint8_t* cseq = YS.bytes + YS.offs[b];
        const int nA = XS.meta[a].x, nB = YS.meta[b].x;
        uint16_t* tr = trace + p * stride;
        if (nA == 0 || nB == 0) {
            if (threadIdx.x == 0) ends[p] = make_int4(0, 0, 0, 0);
            continue;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nA; i += 64 * W) xinfo[i] = rseq[i];
        __syncthreads();
        const int j0 = (w * 64 + lane) * K + 1;
        uint32_t yc[K];
        uint32_t lastbits = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = j0 + k;
            yc[k] = (j <= nB) ? (uint32_t)cseq[j - 1] : 0x100u;
            if (j == nB) lastbits |= 1u << k;
        }
        // state at row 0
        int S[K], Mv[K], Xv[K], Yv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = j0 + k;
            if constexpr (LINEAR) {
                S[k] = j * sc.ee;
            } else {
                Mv[k] = NEG_INF;
                Xv[k] = NEG_INF;
                Yv[k] = sc.eo + sc.ee * (j - 1);
            }
        }
        int dS = (j0 - 1) * sc.ee;  // diagonal of the first cell (row 0, column j0-1)
        TState dT{j0 == 1 ? 0 : NEG_INF, NEG_INF, j0 == 1 ? NEG_INF : sc.eo + sc.ee * (j0 - 2)};
        (void)Mv; (void)Xv; (void)Yv; (void)S;

        const RingEntry* ring_in = (w > 0) ? rings + (size_t)(w - 1) * RING : nullptr;
        RingEntry* ring_out = (w < W - 1) ? rings + (size_t)w * RING : nullptr;
        const int nsteps = nA + 63;
        const int nblk = (nsteps + INTERVAL - 1) / INTERVAL;
        const int nint = (W > 1) ? nblk + WAVE_LAG * (W - 1) : 1;
        for (int it = 0; it < nint; ++it) {
            const int blk = (W > 1) ? it - WAVE_LAG * w : 0;
            const int s0 = (W > 1) ? blk * INTERVAL : 0;
            const int s1 = (W > 1) ? min(s0 + INTERVAL, nsteps) : nsteps;
            if (W == 1 || (blk >= 0 && blk < nblk)) {
                for (int s = s0; s < s1; ++s) {
                    const int i = s - lane + 1;
                    // left input (row i, column j0-1)
                    int lS = 0;
                    TState lT{};
                    if constexpr (LINEAR) {
                        int old = (s + 1) * sc.ee;
                        if (w > 0) old = (int)ring_in[(s + 1) & (RING - 1)].q[0].x;
                        lS = (int)shr_old((uint32_t)S[K - 1], (uint32_t)old);
                    } else {
                        TState old{NEG_INF, sc.eo + sc.ee * s, NEG_INF};
                        if (w > 0) {
                            const uint4 q = ring_in[(s + 1) & (RING - 1)].q[0];
                            old = TState{(int)q.x, (int)q.y, (int)q.z};
                        }
                        lT.M = (int)shr_old((uint32_t)Mv[K - 1], (uint32_t)old.M);
                        lT.X = (int)shr_old((uint32_t)Xv[K - 1], (uint32_t)old.X);
                        lT.Y = (int)shr_old((uint32_t)Yv[K - 1], (uint32_t)old.Y);
                    }
                    uint32_t codes[K];
                    if (i >= 1 && i <= nA) {
                        const uint32_t xb = xinfo[i - 1];
                        const bool lastrow = i == nA;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const int sv = (xb == yc[k]) ? sc.ma : sc.mi;
                            const bool lastcol = (lastbits >> k) & 1u;
                            if constexpr (LINEAR) {
                                const int l = k == 0 ? lS : S[k - 1];
                                const int cd = dS + sv;
                                const int cv = S[k] + (lastcol ? sc.ee : sc.ie);
                                const int ch = l + (lastrow ? sc.ee : sc.ie);
                                const int best = imax3(cd, cv, ch);
                                codes[k] = (cd == best ? 1u : 0u) | (cv == best ? 2u : 0u) | (ch == best ? 4u : 0u);
                                dS = S[k];
                                S[k] = best;
                            } else {
                                const int ox = lastcol ? sc.eo : sc.io, ex = lastcol ? sc.ee : sc.ie;
                                const int oy = lastrow ? sc.eo : sc.io, ey = lastrow ? sc.ee : sc.ie;
                                const int lM = k == 0 ? lT.M : Mv[k - 1];
                                const int lX = k == 0 ? lT.X : Xv[k - 1];
                                const int lY = k == 0 ? lT.Y : Yv[k - 1];
                                const int h = imax3(dT.M, dT.X, dT.Y);
                                uint32_t c = (dT.M == h ? 1u : 0u) | (dT.X == h ? 2u : 0u) | (dT.Y == h ? 4u : 0u);
                                const int xa = Mv[k] + ox, xb2 = Xv[k] + ex, xc = Yv[k] + ox;
                                const int X = imax3(xa, xb2, xc);
                                c |= (xa == X ? 8u : 0u) | (xb2 == X ? 16u : 0u) | (xc == X ? 32u : 0u);
                                const int ya = lM + oy, yb = lX + oy, ycc = lY + ey;
                                const int Y = imax3(ya, yb, ycc);
                                c |= (ya == Y ? 64u : 0u) | (yb == Y ? 128u : 0u) | (ycc == Y ? 256u : 0u);
                                codes[k] = c;
                                dT = TState{Mv[k], Xv[k], Yv[k]};
                                Mv[k] = h + sv;
                                Xv[k] = X;
                                Yv[k] = Y;
                            }
                        }
                        // step-major trace: [s][lane_global][k]
                        uint16_t* dst = tr + ((int64_t)s * 64 * W + (w * 64 + lane)) * K;
#pragma unroll
                        for (int k = 0; k < K; k += 2)
                            *reinterpret_cast<uint32_t*>(dst + k) = codes[k] | (codes[k + 1] << 16);
                        if (W > 1 && ring_out != nullptr && lane == 63) {
                            RingEntry* e = ring_out + (i & (RING - 1));
                            if constexpr (LINEAR) e->q[0] = make_uint4((uint32_t)S[K - 1], 0u, 0u, 0u);
                            else e->q[0] = make_uint4((uint32_t)Mv[K - 1], (uint32_t)Xv[K - 1], (uint32_t)Yv[K - 1], 0u);
                        }
                    }
                    if constexpr (LINEAR) dS = lS;
                    else dT = lT;
                }
            }
            if (W > 1) __syncthreads();
        }
        // end scores (M, X, Y at (nA, nB); NW: S in .x)
        const int jl = nB - 1;
        if (w == jl / (64 * K) && lane == ((jl / K) & 63)) {
            const int kk = jl % K;
            int4 e = make_int4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (k == kk) {
                    if constexpr (LINEAR) e = make_int4(S[k], NEG_INF, NEG_INF, 1);
                    else e = make_int4(Mv[k], Xv[k], Yv[k], 1);
                }
            ends[p] = e;
        }
    }
}

// Walk one alignment backwards.  Writes aligned target / query right-aligned into
// out_x/out_y[p*2 + o][0 .. nA+nB) and the alignment length into out_len[p*2 + o].
template <bool LINEAR>
__global__ void __launch_bounds__(256)
k_traceback(SetView XS, SetView YS, const int64_t* __restrict__ xs, const int64_t* __restrict__ ys,
            int64_t count, int K, int W, int xcap, const uint16_t* __restrict__ trace,
            const int4* __restrict__ ends, int cap, uint8_t* __restrict__ out_x, uint8_t* __restrict__ out_y,
            int32_t* __restrict__ out_len, int both) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int norient = both ? 2 : 1;
    if (t >= count * norient) return;
    const int64_t p = t / norient;
    const int o = (int)(t % norient);  // 0 = A (x, y), 1 = B (y, x) priorities
    const int64_t a = xs[p], b = ys[p];
    const uint8_t* xseq = XS.bytes + XS.offs[a];
    const uint8_t* yseq = YS.bytes + YS.offs[b];
    const int nA = XS.meta[a].x, nB = YS.meta[b].x;
    const int64_t stride = (int64_t)(xcap + 63) * 64 * W * K;
    const uint16_t* tr = trace + p * stride;
    uint8_t* ox = out_x + (p * 2 + o) * (int64_t)cap;
    uint8_t* oy = out_y + (p * 2 + o) * (int64_t)cap;
    int pos = nA + nB;
    int i = nA, j = nB;
    // state: 0 = M / D, 1 = Ix / V (consume x), 2 = Iy / H (consume y)
    int st = 0;
    if (!LINEAR && nA > 0 && nB > 0) {
        const int4 e = ends[p];
        const int h = imax3(e.x, e.y, e.z);
        const int pr[3] = {0, o ? 2 : 1, o ? 1 : 2};
        const int v[3] = {e.x, e.y, e.z};
        for (int q = 0; q < 3; ++q)
            if (v[pr[q]] == h) { st = pr[q]; break; }
    }
    while (i > 0 || j > 0) {
        uint32_t code;
        if (i == 0) {
            code = LINEAR ? 4u : (j == 1 ? (1u << 6) : (4u << 6));   // boundary row: Iy / H
            if (!LINEAR) st = 2;
        } else if (j == 0) {
            code = LINEAR ? 2u : (i == 1 ? (1u << 3) : (2u << 3));   // boundary column: Ix / V
            if (!LINEAR) st = 1;
        } else {
            const int lg = (j - 1) / K, k = (j - 1) % K;
            const int s = i - 1 + (lg & 63);
            code = tr[((int64_t)s * 64 * W + lg) * K + k];
        }
        int mv;
        if (LINEAR) {
            // A: H > V > D ; B: V > H > D   (bits: 1 = D, 2 = V, 4 = H)
            if (o == 0) mv = (code & 4u) ? 2 : (code & 2u) ? 1 : 0;
            else mv = (code & 2u) ? 1 : (code & 4u) ? 2 : 0;
        } else {
            mv = st;
        }
        --pos;
        if (mv == 0) {
            ox[pos] = xseq[i - 1];
            oy[pos] = yseq[j - 1];
        } else if (mv == 1) {
            ox[pos] = xseq[i - 1];
            oy[pos] = '-';
        } else {
            ox[pos] = '-';
            oy[pos] = yseq[j - 1];
        }
        if (!LINEAR) {
            const uint32_t ts = (code >> (3 * st)) & 7u;  // predecessor tie set of the current state
            const int pr[3] = {0, o ? 2 : 1, o ? 1 : 2};
            int nxt = st;
            for (int q = 0; q < 3; ++q)
                if (ts & (1u << pr[q])) { nxt = pr[q]; break; }
            st = nxt;
        }
        if (mv == 0) { --i; --j; }
        else if (mv == 1) --i;
        else --j;
    }
    out_len[p * 2 + o] = nA + nB - pos;
}

}  // namespace taxi2
