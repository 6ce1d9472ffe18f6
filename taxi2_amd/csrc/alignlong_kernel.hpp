// Column-tiled trace-and-walk aligner for sequences of any length (Gotoh, and with LIN the
// Needleman-Wunsch fill Biopython uses when open == extend everywhere; the reference's
// PairwiseAligner.Biopython.align has no length limit: src/itaxotools/taxi2/align.py:151-157).
//
// The other aligners hold a whole row of the DP in one workgroup's registers: 64 K W columns
// (at most 2 048 packed, 4 096 forward-carry).  Here a pair's columns are cut into TILES of
// TC = 64 K W columns and the rows stream through the same systolic layout once per tile:
//
//   tile t covers columns (t TC, (t + 1) TC]; wave w, lane l owns the K columns from
//   t TC + (64 w + l) K + 1.  Tile 0's left input is the column-0 boundary (Ix(i, 0) =
//   eo + ee (i - 1), Iy = -inf); tile t > 0 reads, per row, the (F, Iy) payload that the last
//   wave's lane 63 of tile t - 1 handed to its right neighbour -- written to a per-workgroup
//   boundary column in global memory instead (bnd[row]), read back with L1-bypassing loads.
//
// Cells, tags and trace bytes are alignt_kernel.hpp's 32-bit ones (doubled scores, G / F tagged
// with "M won", one byte per cell with tagG, tagF and the three clamped signs), stored per tile
// step-major: cell (i, j) of tile t lives at
//   buf + ((t S + i - 1 + (l & 63)) NT + l) K + k,   S = nA + 63 steps, j - 1 = t TC + l K + k.
// One pair per workgroup pass (long pairs are few, no chains); two trace buffers per workgroup:
// the walker wave (wave W) traces pair p - 1 (both orientations: lanes 0 and 1) from one buffer
// while the fill waves fill pair p into the other, exactly as in alignt_kernel.hpp.  A pair's
// trace is nA x ceil(nB / TC) TC bytes (100 MB at 10 000 bp): the host sizes the persistent grid
// to the trace budget.
#pragma once
#include "alignt_kernel.hpp"

namespace taxi2 {

struct LongPair {
    const uint8_t* rseq;  // rows: X[a]
    const uint8_t* cseq;  // columns: Y[b]
    int64_t p;
    int nA, fx, lx, nB, fy, ly, ntile, fin;
};

// LIN (linear scores, oracle/restatement.py _nw): one DP value per cell, S(i, j) = max(D, V, H) with
// D = S(i-1, j-1) + s, V = S(i-1, j) + (ee on the last column, else ie), H = S(i, j-1) + (ee on the
// last row, else ie); the trace byte is the tie set D=1 | V=2 | H=4 of the cell, and each walk is
// stateless: from (nA, nB), the first set move in H > V > D (orientation (x, y)) or V > H > D
// (the (y, x) alignment), row 0 / column 0 forcing H / V -- align_kernel.hpp's NW priorities.
//
// Optional aligned strings (taxi2_align_strings for long pairs): when sx != nullptr every walk also
// writes its alignment right-aligned into slot [p][prio] of sx / sy (cap bytes each: bytes
// [nA + nB - len, nA + nB)) and len into slen[p][prio] -- prio 1 is the (y, x) alignment written
// in (x, y) column order, as k_traceback does.  out == nullptr: no metrics.
template <int K, int W, int OCC, bool LIN>
__global__ void __launch_bounds__(64 * (W + 1), OCC)
k_alignlong(SetView XS, SetView YS, PairSrc ps, KScores scin, MetricSpec ms, int out_mode, double* __restrict__ out,
            int32_t* __restrict__ sout, uint8_t* __restrict__ trace, int64_t buf_bytes, uint2* __restrict__ bnd_all,
            int64_t bnd_rows, unsigned long long* __restrict__ next, uint8_t* __restrict__ sx,
            uint8_t* __restrict__ sy, int32_t* __restrict__ slen, int cap) {
    static_assert(K <= A1_MAX_K && K % 4 == 0, "equality fields hold at most 10 columns; K bytes per store");
    constexpr int NT = 64 * W;
    constexpr int TC = NT * K;
    constexpr int XR = a1c_xr(W);
    const KScores sc = doubled(scin);
    __shared__ uint32_t xinfo[XR];
    __shared__ uint2 ring[(W > 1 ? W - 1 : 1) * RING];
    __shared__ uint8_t colb[NT * K];
    __shared__ int2 colc[K][NT];
    __shared__ LongPair lp[2];
    __shared__ int s_more, s_fill;
    __shared__ AtWalk wks[2];
    __shared__ int wpos[2];  // next string position of each walk (strings are written backwards)

    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool walker = w == W;
    const int nm = ms.n;
    const int64_t total = ps.count;
    uint8_t* const bufs = trace + (size_t)blockIdx.x * 2 * (size_t)buf_bytes;
    uint2* const bnd = bnd_all + (size_t)blockIdx.x * (size_t)bnd_rows;
    int cur = 0;
    bool have_prev = false;

    // row record of row g of the current pair: byte, ACGT code (bits 11-13, 4 = other), first /
    // last row flags
    auto row_info = [&](const LongPair& q, int g) -> uint32_t {
        if (g < 0 || g >= q.nA) return A1C_NONE;
        const uint32_t c = q.rseq[g];
        const uint32_t ec = c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
        uint32_t v = c | (ec << 11);
        if (g == 0) v |= A1C_FIRST;
        if (g == q.nA - 1) v |= A1C_LAST;
        return v;
    };

    auto walk_init = [&](int pb) {
        if (lane >= 2) return;
        AtWalk& W_ = wks[lane];
        W_ = AtWalk{0, 0, AT_DONE, 0, 0, 0, 0u, 0u, 0u, 0, 0, 0, 0};
        wpos[lane] = lp[pb].nA + lp[pb].nB - 1;
        if (!have_prev || (lane == 1 && out_mode != OUT_BOTH)) return;
        W_.prio = lane;
        W_.i = lp[pb].nA + (LIN ? 0 : 1);
        W_.j = lp[pb].nB + (LIN ? 0 : 1);
        W_.st = AT_M;
        W_.first = LIN ? 0 : 1;
    };
    auto walk_run = [&](int pb, int target) {
        AtWalk& W_ = wks[lane < 2 ? lane : 0];
        int st = lane < 2 ? W_.st : AT_DONE;
        if (!__any(st != AT_DONE)) return;
        const LongPair& q = lp[pb];
        const int fx = q.fx, lx = q.lx, fy = q.fy, ly = q.ly, nA = q.nA;
        const int prio = W_.prio;
        const uint8_t* tr = bufs + (size_t)pb * (size_t)buf_bytes;
        int i = W_.i, j = W_.j, first = W_.first;
        uint32_t cb = W_.cb, xa = W_.xa, yb = W_.yb;
        int valid = W_.valid, ts = W_.ts, tv = W_.tv, gap = W_.gap;
        int pos = lane < 2 ? wpos[lane] : 0;
        uint8_t* const ox = sx ? sx + ((size_t)q.p * 2 + prio) * (size_t)cap : nullptr;
        uint8_t* const oy = sx ? sy + ((size_t)q.p * 2 + prio) * (size_t)cap : nullptr;
        for (;;) {
            if (!__any(st != AT_DONE)) break;
            if (target > 0 && __hip_atomic_load(&s_fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target)
                break;
            if (st == AT_DONE) continue;
            if constexpr (LIN) {  // stateless NW walk: the move at (i, j) from its own tie set
                uint32_t tb = 0;
                if (i >= 1 && j >= 1) {
                    const int t = (j - 1) / TC;
                    const int jj = j - 1 - t * TC;
                    const int l = jj / K;
                    const int k = jj - l * K;
                    const size_t s = (size_t)t * (size_t)(nA + 63) + (size_t)(i - 1 + (l & 63));
                    tb = *(const volatile uint8_t*)(tr + (s * NT + l) * K + k);
                }
                // 0 = D, 1 = V (x against a gap), 2 = H (y against a gap)
                const int mv = i == 0 ? 2
                             : j == 0 ? 1
                             : prio ? ((tb & 2u) ? 1 : (tb & 4u) ? 2 : 0)
                                    : ((tb & 4u) ? 2 : (tb & 2u) ? 1 : 0);
                xa = i >= 1 ? q.rseq[i - 1] : 0u;
                yb = j >= 1 ? q.cseq[j - 1] : 0u;
                if (ox) {
                    ox[pos] = mv == 2 ? (uint8_t)'-' : (uint8_t)xa;
                    oy[pos] = mv == 1 ? (uint8_t)'-' : (uint8_t)yb;
                    --pos;
                }
                if (mv == 0) {
                    const int bx = base_code(xa), by = base_code(yb);
                    if (bx < 4 && by < 4) {
                        ++valid;
                        const int dd = bx ^ by;
                        ts += dd == 2;
                        tv += (dd != 0) & (dd != 2);
                    }
                    --i;
                    --j;
                } else if (mv == 1) {
                    if (base_code(xa) < 4 && j - 1 >= fy && j <= ly) ++gap;
                    --i;
                } else {
                    if (base_code(yb) < 4 && i - 1 >= fx && i <= lx) ++gap;
                    --j;
                }
                if (i == 0 && j == 0) {
                    const int64_t p = q.p;
                    if (out) {
                        double* o = out_mode == OUT_BOTH ? out + (p * 2 + prio) * nm : out + p * nm;
                        for (int m = 0; m < nm; ++m)
                            o[m] = metric_value(ms.code[m], (uint32_t)valid, (uint32_t)ts, (uint32_t)tv, (uint32_t)gap);
                    }
                    if (slen) slen[p * 2 + prio] = q.nA + q.nB - 1 - pos;
                    if (sout && !prio) sout[p] = q.fin >> 1;
                    st = AT_DONE;
                }
                continue;
            }
            int ni, nj;
            if (ox && !first) {  // this column of the alignment, written right to left
                ox[pos] = st == AT_IY ? (uint8_t)'-' : (uint8_t)xa;
                oy[pos] = st == AT_IX ? (uint8_t)'-' : (uint8_t)yb;
                --pos;
            }
            if (st == AT_M) {
                if (!first) {
                    const int bx = base_code(xa), by = base_code(yb);
                    if (bx < 4 && by < 4) {
                        ++valid;
                        const int dd = bx ^ by;
                        ts += dd == 2;
                        tv += (dd != 0) & (dd != 2);
                    }
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
            first = 0;
            if (ni == 0 && nj == 0) {
                const int64_t p = q.p;
                if (out) {
                    double* o = out_mode == OUT_BOTH ? out + (p * 2 + prio) * nm : out + p * nm;
                    for (int m = 0; m < nm; ++m)
                        o[m] = metric_value(ms.code[m], (uint32_t)valid, (uint32_t)ts, (uint32_t)tv, (uint32_t)gap);
                }
                if (slen) slen[p * 2 + prio] = q.nA + q.nB - 1 - pos;
                if (sout && !prio) sout[p] = q.fin >> 1;
                st = AT_DONE;
                continue;
            }
            uint32_t nb = 0;
            if (ni >= 1 && nj >= 1) {
                const int t = (nj - 1) / TC;
                const int jj = nj - 1 - t * TC;
                const int l = jj / K;
                const int k = jj - l * K;
                const size_t s = (size_t)t * (size_t)(nA + 63) + (size_t)(ni - 1 + (l & 63));
                nb = *(const volatile uint8_t*)(tr + (s * NT + l) * K + k);
            }
            xa = ni >= 1 ? q.rseq[ni - 1] : 0u;
            yb = nj >= 1 ? q.cseq[nj - 1] : 0u;
            int nst;
            if (ni == 0) {
                nst = AT_IY;
            } else if (nj == 0) {
                nst = AT_IX;
            } else if (st == AT_M) {
                const int ca = at_sign((nb >> 2) & 3u, 0);
                nst = ca > 0 ? ((nb & 1u) ? AT_M : AT_IY) : (ca == 0 ? (prio ? AT_IY : AT_IX) : AT_IX);
            } else if (st == AT_IX) {
                const int sb = at_sign((cb >> 4) & 3u, 0);
                const bool gp = prio ? sb >= 0 : sb > 0;
                nst = gp ? ((nb & 1u) ? AT_M : AT_IY) : AT_IX;
            } else {
                const int sc_ = at_sign((cb >> 6) & 3u, 0);
                const bool fp = prio ? sc_ > 0 : sc_ >= 0;
                nst = fp ? ((nb & 2u) ? AT_M : AT_IX) : AT_IY;
            }
            cb = nb;
            i = ni;
            j = nj;
            st = nst;
        }
        if (lane >= 2) return;
        wpos[lane] = pos;
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
    };

    for (;;) {
        // ---- next pair (thread 0)
        __syncthreads();
        if (tid == 0) {
            s_more = 0;
            s_fill = 0;
            for (;;) {
                const int64_t p = (int64_t)atomicAdd(next, 1ull);
                if (p >= total) break;
                int64_t a, b;
                decode_pair(ps, p, a, b);
                const int4 ma = XS.meta[a];
                const int4 mb = YS.meta[b];
                if (ma.x == 0 || mb.x == 0) {  // one side empty: no nucleotide column
                    if (slen) {  // strings: the other sequence against gaps (both slots alike)
                        const int L = ma.x + mb.x;
                        const uint8_t* xb = XS.bytes + XS.offs[a];
                        const uint8_t* yb = YS.bytes + YS.offs[b];
                        for (int o = 0; o < 2; ++o) {
                            uint8_t* ox = sx + ((size_t)p * 2 + o) * (size_t)cap;
                            uint8_t* oy = sy + ((size_t)p * 2 + o) * (size_t)cap;
                            for (int t = 0; t < L; ++t) {
                                ox[t] = ma.x ? xb[t] : (uint8_t)'-';
                                oy[t] = mb.x ? yb[t] : (uint8_t)'-';
                            }
                            slen[p * 2 + o] = L;
                        }
                    }
                    if (out) for (int m = 0; m < nm; ++m) {
                        if (out_mode == OUT_BOTH) {
                            out[(p * 2 + 0) * nm + m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                            out[(p * 2 + 1) * nm + m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                        } else {
                            out[p * nm + m] = metric_value(ms.code[m], 0u, 0u, 0u, 0u);
                        }
                    }
                    if (sout) {
                        const int ne = ma.x + mb.x;
                        sout[p] = ne == 0 ? 0 : scin.eo + scin.ee * (ne - 1);
                    }
                    continue;
                }
                lp[cur] = LongPair{XS.bytes + XS.offs[a], YS.bytes + YS.offs[b], p, ma.x, ma.y, ma.z,
                                   mb.x, mb.y, mb.z, (mb.x + TC - 1) / TC, 0};
                s_more = 1;
                break;
            }
        }
        __syncthreads();
        const int pb = cur ^ 1;
        if (walker) walk_init(pb);
        if (!s_more) {
            if (walker) walk_run(pb, 0);
            break;
        }
        const LongPair& q = lp[cur];
        const int nA = q.nA, nB = q.nB;
        const int nsteps = nA + 63;
        const int nblk = (nsteps + INTERVAL - 1) / INTERVAL;
        const int nint = nblk + WAVE_LAG * (W - 1);
        uint8_t* trb = bufs + (size_t)cur * (size_t)buf_bytes;
        int sig = 0;  // interval signals of this pair so far (walker target)
        for (int tile = 0; tile < q.ntile; ++tile) {
            const int c0 = tile * TC;
            const int j0 = c0 + (w * 64 + lane) * K + 1;
            uint32_t eqp0 = 0, eqp1 = 0, eqp2 = 0, eqp3 = 0;
            if (!walker) {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int j = j0 + k;
                    uint32_t c = 0x100u;
                    if (j <= nB) {
                        c = q.cseq[j - 1];
                        if (c == 'A') eqp0 |= 4u << (3 * k);
                        if (c == 'C') eqp1 |= 4u << (3 * k);
                        if (c == 'G') eqp2 |= 4u << (3 * k);
                        if (c == 'T') eqp3 |= 4u << (3 * k);
                    }
                    colb[tid * K + k] = c > 0xFFu ? 0 : (uint8_t)c;
                    colc[k][tid] = make_int2((j == nB) ? sc.eo : sc.io, (j == nB) ? sc.ee : sc.ie);
                }
            }
            if (tid < 64) xinfo[tid] = row_info(q, tid);
            else if (tid < 128) xinfo[XR - 128 + tid] = A1C_NONE;
            int stG[K], stX[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                stG[k] = sc.eo + sc.ee * (j0 + k - 1);
                stX[k] = NEG_INF;
            }
            int payF = NEG_INF, payY = NEG_INF, carry = NEG_INF;
            const uint2* ring_in = (w > 0 && !walker) ? ring + (size_t)(w - 1) * RING : nullptr;
            uint2* ring_out = (w < W - 1) ? ring + (size_t)w * RING : nullptr;
            uint8_t* trt = trb + (size_t)tile * (size_t)nsteps * NT * K;
            __syncthreads();  // xinfo block 0, column tables

            for (int it = 0; it < nint; ++it) {
                if (walker) {
                    walk_run(pb, sig + W * (it + 1));
                } else {
                    const int blk = it - WAVE_LAG * w;
                    if (blk >= 0 && blk < nblk) {
                        const int s0 = blk * INTERVAL;
                        const int s1 = min(s0 + INTERVAL, nsteps);
                        for (int s = s0; s < s1; ++s) {
                            const int g = s - lane;
                            const uint32_t xi = xinfo[g & (XR - 1)];
                            int inF, inY;
                            if (w == 0) {
                                // column c0 of row g + 1: the boundary (tile 0) or the previous
                                // tile's hand-off (an L2 read of what wave W-1 stored)
                                uint2 o = make_uint2((uint32_t)NEG_INF, (uint32_t)NEG_INF);
                                if (lane == 0 && g < nA) {
                                    if (tile == 0) o = make_uint2((uint32_t)(sc.eo + sc.ee * g), (uint32_t)NEG_INF);
                                    else {
                                        const unsigned long long v = *(const volatile unsigned long long*)(bnd + g);
                                        o = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
                                    }
                                }
                                inF = (int)shr_old((uint32_t)payF, o.x);
                                inY = (int)shr_old((uint32_t)payY, o.y);
                            } else {
                                const uint2 o = ring_in[(s + 1) & (RING - 1)];
                                inF = (int)shr_old((uint32_t)payF, o.x);
                                inY = (int)shr_old((uint32_t)payY, o.y);
                            }
                            if (!(xi & A1C_NONE)) {
                                if (xi & A1C_FIRST) {  // row 1: row-0 states and the diagonal (0, j0 - 1)
                                    int jb = c0 + tid * K;
                                    asm volatile("" : "+v"(jb));
#pragma unroll
                                    for (int k = 0; k < K; ++k) {
                                        stG[k] = sc.eo + sc.ee * (jb + k);
                                        stX[k] = NEG_INF;
                                    }
                                    carry = jb == 0 ? (LIN ? 0 : 1) : sc.eo + sc.ee * (jb - 1);
                                }
                                const uint32_t ec = (xi >> 11) & 7u;
                                const uint32_t eqlo = (ec & 1u) ? eqp1 : eqp0;
                                const uint32_t eqhi = (ec & 1u) ? eqp3 : eqp2;
                                uint32_t eq = (ec & 2u) ? eqhi : eqlo;
                                if (ec >= 4u) {  // not an exact A/C/G/T byte: compare bytes
                                    const uint32_t xb = xi & 0xFFu;
                                    eq = 0u;
#pragma unroll
                                    for (int k = 0; k < K; ++k)
                                        eq |= ((uint32_t)colb[tid * K + k] == xb && xb != 0u) ? (4u << (3 * k)) : 0u;
                                }
                                const bool lastrow = (xi & A1C_LAST) != 0u;
                                const int oy = lastrow ? sc.eo : sc.io;
                                const int ey = lastrow ? sc.ee : sc.ie;
                                int d = carry;
                                int F = inF, Y = inY;
                                uint32_t acc[K / 4];
                                if constexpr (LIN) {  // NW: S only (stG), F = S(i, j - 1)
#pragma unroll
                                    for (int k = 0; k < K; ++k) {
                                        const int U = stG[k];
                                        const uint32_t e = (eq >> (3 * k)) & 7u;
                                        const int Dv = d + (e ? sc.ma : sc.mi);
                                        const int Vv = U + colc[k][tid].y;
                                        const int Hv = F + ey;
                                        const int S = max(Dv, max(Vv, Hv));
                                        const uint32_t tset = (Dv == S ? 1u : 0u) | (Vv == S ? 2u : 0u) | (Hv == S ? 4u : 0u);
                                        uint32_t a = k % 4 == 0 ? 0u : acc[k / 4];
                                        acc[k / 4] = push_bits<8>(a, (int)tset);
                                        stG[k] = S;
                                        F = S;
                                        d = U;
                                    }
                                } else
#pragma unroll
                                for (int k = 0; k < K; ++k) {
                                    const int G = stG[k], X = stX[k];
                                    const int nd = max(G, X);
                                    const uint32_t e = (eq >> (3 * k)) & 7u;
                                    const int sM = e ? sc.ma : sc.mi;
                                    const int M = (d | 1) + sM;
                                    const int2 cc2 = colc[k][tid];
                                    const int cg = G + cc2.x, cx = X + cc2.y;
                                    const int Xn = max(cg, cx) & ~1;
                                    const int cf = F + oy, cy = Y + ey;
                                    const int Yn = max(cf, cy) & ~1;
                                    const int Gn = max(M, Yn), Fn = max(M, Xn);
                                    uint32_t a = k % 4 == 0 ? 0u : acc[k / 4];
                                    a = push_bits<1>(a, Gn);
                                    a = push_bits<1>(a, Fn);
                                    a = push_bits<2>(a, sign3(Gn - Xn));
                                    a = push_bits<2>(a, sign3(cg - cx));
                                    a = push_bits<2>(a, sign3(cf - cy));
                                    acc[k / 4] = a;
                                    stG[k] = Gn;
                                    stX[k] = Xn;
                                    F = Fn;
                                    Y = Yn;
                                    d = nd;
                                }
                                payF = F;
                                payY = Y;
                                if (j0 <= nB) {
                                    uint32_t* dst = (uint32_t*)(trt + ((size_t)s * NT + tid) * K);
#pragma unroll
                                    for (int qq = 0; qq < K / 4; ++qq) dst[qq] = acc[qq];
                                }
                                if (lastrow && j0 <= nB && nB < j0 + K) {  // this lane owns column nB: the score
                                    const int out_k = (nB - 1) % K;
                                    int eG = stG[0], eX = stX[0];
#pragma unroll
                                    for (int k = 1; k < K; ++k) {
                                        uint32_t m = (k == out_k) ? ~0u : 0u;
                                        asm volatile("" : "+v"(m));
                                        eG = (int)(((uint32_t)stG[k] & m) | ((uint32_t)eG & ~m));
                                        eX = (int)(((uint32_t)stX[k] & m) | ((uint32_t)eX & ~m));
                                    }
                                    lp[cur].fin = LIN ? eG : max(eG, eX);
                                }
                            }
                            if (W > 1 && ring_out != nullptr && lane == 63)
                                ring_out[(g + 1) & (RING - 1)] = make_uint2((uint32_t)payF, (uint32_t)payY);
                            if (w == W - 1 && lane == 63 && g >= 0 && g < nA && tile + 1 < q.ntile)
                                bnd[g] = make_uint2((uint32_t)payF, (uint32_t)payY);  // hand-off to tile + 1
                            carry = LIN ? inF : max(inF, inY);
                        }
                    }
                }
                const int gpre = (it + 1) * INTERVAL + tid;
                if (tid < INTERVAL && it + 1 < nblk) xinfo[gpre & (XR - 1)] = row_info(q, gpre);
                if (it + 1 == nint) __builtin_amdgcn_s_waitcnt(0);  // trace / boundary stores landed
                if (!walker && lane == 0) atomicAdd(&s_fill, 1);
                __syncthreads();
            }
            sig += W * nint;
        }
        if (walker) walk_run(pb, 0);
        have_prev = true;
        cur ^= 1;
    }
}

}  // namespace taxi2
