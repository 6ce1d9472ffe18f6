// Trace-and-walk aligner (Gotoh, sequences <= 64*K*W columns): the fill stores one byte of
// tie information per cell, a walker wave of the same workgroup traces both orientations.
//
// Why: the forward-carry kernels (align1_kernel.hpp, align1c_kernel.hpp) select two counter
// words per state at every cell (10 v_cndmask + their compares per cell) and re-run the pairs
// whose two orientations diverge.  Storing what the traceback needs instead costs 5 bit-field
// ops per cell, one byte of HBM per cell (1 MB per 1 000 bp pair, written once, ~2 % read
// back), and serves both orientations from one fill.  The counters are then accumulated along
// the two first paths by a walker (one lane per walk).
//
// Fill (waves 0..W-1): the systolic layout and tie-tagged doubled scores of align1_kernel.hpp
// (G = max(M, Iy) and F = max(M, Ix) carry bit 0 = "M won"; Ix / Iy are even).  For cell
// (i, j) with post values G, X (= Ix), F, Y (= Iy) the byte is
//   bit 0     tagG = G & 1                   (M >= Iy at (i, j))
//   bit 1     tagF = F & 1                   (M >= Ix)
//   bits 2-3  ca = sign(G - X)               best state of (i, j), read by a diagonal move into
//                                            it: G > X -> M / Iy by tagG, G == X -> Ix = Iy
//                                            tie, G < X -> Ix
//   bits 4-5  cb = sign(cg - cx)             how Ix(i, j) was formed: G(i-1, j) + ox (G path,
//                                            M / Iy by tagG of (i-1, j)) vs Ix(i-1, j) + ex
//   bits 6-7  cc = sign(cf - cy)             how Iy(i, j) was formed: F(i, j-1) + oy (F path,
//                                            M / Ix by tagF of (i, j-1)) vs Iy(i, j-1) + ey
// each sign as the low two bits of v_med3_i32(diff, -1, 1) (one op: -1 -> 3, 0, 1).  A
// traceback step from cell c to c' reads the move's relation from c's byte and the state of
// c' from c''s tags, so one byte load per step.  The tags make every tie against M impossible
// in these differences (odd vs even), so a 0 sign always is an Ix / Iy tie: priority A
// (M > Ix > Iy, the (rows, cols) alignment) and B (M > Iy > Ix, the (cols, rows) alignment)
// read the same bytes.
//
// Storage is step-major per chain: the byte of cell (chain row g, column j) lives at
//   buf + ((g + (t & 63)) * 64W + t) * K + (j - 1) % K,   t = (j - 1) / K
// i.e. each lane stores K bytes per step at a coalesced address.  Two buffers per workgroup:
// the fill of chain c writes one while the walker traces chain c-1 from the other.
//
// Walker (wave W): lane q walks pair q of the previous chain in orientation A (and, for
// two-sided output, lane n + q in orientation B), H hops per 64-step interval of the fill
// (one byte load per hop, issued together with the two sequence bytes of the next column),
// counting valid / ts / tv / gap columns with the common-range rules of align1_kernel.hpp.
// After the fill of a chain the walker finishes its walks while the fill waves wait.
#pragma once
#include "align1c_kernel.hpp"

namespace taxi2 {

constexpr int AT_CHUNK = 8;  // pairs per cursor step (cut into chains); bounds the trace buffers

struct AtChain {
    const uint8_t* cseq;
    int n, nB, fy, ly;
};

__device__ __forceinline__ int sign3(int x) {  // v_med3_i32(x, -1, 1)
    int r;
    asm("v_med3_i32 %0, %1, -1, 1" : "=v"(r) : "v"(x));
    return r;
}
// (acc >> n) | (v << (32 - n)): one v_alignbit_b32 (opaque, so the compiler keeps the packing
// at one op per field instead of re-deriving it with and / or / shift chains)
template <int N>
__device__ __forceinline__ uint32_t push_bits(uint32_t acc, int v) {
    uint32_t r;
    asm("v_alignbit_b32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(acc), "i"(N));
    return r;
}
// low two bits of a stored sign (+ offset c) -> -1 / 0 / +1
__device__ __forceinline__ int at_sign(uint32_t bits2, int c) {
    const uint32_t v = (bits2 + (uint32_t)c) & 3u;
    return v == 3u ? -1 : (int)v;
}

__host__ __device__ inline size_t at_buf_bytes(int cap_rows, int K, int W) {
    return (((size_t)cap_rows + 64) * 64 * W * K + 255) / 256 * 256;
}

enum : int { AT_M = 0, AT_IX = 1, AT_IY = 2, AT_DONE = 3 };

struct AtWalk {  // one walk: position, state, its cell's trace byte, bytes of the column, counters
    int i, j, st, first, pi, prio;
    uint32_t cb, xa, yb;
    int valid, ts, tv, gap;
    int sc2;   // raw-difference walks (alignt2_kernel.hpp): doubled score of the moves so far
    int ncol;  // alignt2_kernel.hpp string output: alignment columns written so far
};

template <int K, int W, bool DEF, int OCC>
__global__ void __launch_bounds__(64 * (W + 1), OCC)
k_alignt(SetView XS, SetView YS, PairSrc ps, KScores scin, MetricSpec ms, int chunk_req, int out_mode,
         double* __restrict__ out, int32_t* __restrict__ sout, uint8_t* __restrict__ trace, int64_t buf_bytes,
         int cap_rows, int hops, unsigned long long* __restrict__ next) {
    static_assert(K <= A1_MAX_K && K % 4 == 0, "equality fields hold at most 10 columns; K bytes per store");
    constexpr int NT = 64 * W;  // fill threads
    constexpr int XR = a1c_xr(W);
    const KScores sc0 = DEF ? KScores{1, -1, -8, -1, -1, -1} : scin;  // align.py:20-27 defaults
    const KScores sc = doubled(sc0);
    __shared__ uint32_t xinfo[XR];
    __shared__ ChainPair tab[2][AT_CHUNK];
    __shared__ int fin[2][AT_CHUNK];
    __shared__ uint32_t fin_n;
    __shared__ AtChain chs[2];
    __shared__ uint2 ring[(W > 1 ? W - 1 : 1) * RING];
    __shared__ uint8_t colb[NT * K];
    __shared__ int2 colc[K][NT];  // per column: {Ix open, Ix extend} (end-gap scores on column nB)
    __shared__ int64_t s_qc, s_qend;
    __shared__ int s_n, s_rows;
    __shared__ int s_fill;  // fill waves done with the current interval (cumulative per chain)

    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: ring pointers etc. in SGPRs
    const bool walker = w == W;
    const int nm = ms.n;
    const int64_t total = ps.count;
    const int64_t chunk = chunk_req >= 1 ? min((int64_t)chunk_req, (int64_t)AT_CHUNK)
                                         : max((int64_t)1, min((int64_t)AT_CHUNK, total / ((int64_t)gridDim.x * 8)));
    uint8_t* const bufs = trace + (size_t)blockIdx.x * 2 * (size_t)buf_bytes;

    if (tid == 0) {
        s_qc = 0;
        s_qend = 0;
    }
    int cur = 0;         // buffer of the chain being filled
    int prev_n = 0;      // pairs of the chain in buffer cur ^ 1 awaiting their walks

    // ---- walker lane state (wave W), kept in LDS so that it occupies no registers of the fill
    // waves (all waves run one kernel body: anything live across the chain loop is allocated in
    // every wave)
    __shared__ AtWalk wks[64];

    auto walk_init = [&](int pb, int n) {
        // lanes [0, n): orientation A (or the (a, b) slot's orientation); [n, 2n): orientation B
        const int nw = out_mode == OUT_BOTH ? 2 * n : n;
        AtWalk& W_ = wks[lane];
        W_.st = AT_DONE;
        if (lane < nw) {
            const int pi = lane < n ? lane : lane - n;
            const ChainPair& cp = tab[pb][pi];
            const AtChain& ch = chs[pb];
            W_.pi = pi;
            W_.prio = out_mode == OUT_BOTH ? (lane >= n) : cp.swp;
            W_.i = cp.nA + 1;
            W_.j = ch.nB + 1;
            W_.st = AT_M;
            W_.first = 1;
            W_.valid = W_.ts = W_.tv = W_.gap = 0;
            W_.cb = W_.xa = W_.yb = 0u;
        }
    };
    // hop until `budget` hops (< 0: unbounded) or, with target > 0, until the fill waves have
    // signalled `target` interval completions: the walker uses exactly the time the fill waves
    // spend on their interval and delays the barrier by at most one hop
    auto walk_run = [&](int pb, int budget, int target) {
        AtWalk& W_ = wks[lane];
        int st = W_.st;
        if (!__any(st != AT_DONE)) return;
        const int pi = W_.pi;
        const ChainPair& cp = tab[pb][pi];
        const AtChain& ch = chs[pb];
        const int fx = cp.fx, lx = cp.lx, fy = ch.fy, ly = ch.ly, r0 = cp.r0;
        const int prio = W_.prio;
        const uint8_t* rs = cp.rseq;
        const uint8_t* cs = ch.cseq;
        const uint8_t* tr = bufs + (size_t)pb * (size_t)buf_bytes;
        int i = W_.i, j = W_.j, first = W_.first;
        uint32_t cb = W_.cb, xa = W_.xa, yb = W_.yb;
        int valid = W_.valid, ts = W_.ts, tv = W_.tv, gap = W_.gap;
        for (int h = 0; budget < 0 || h < budget; ++h) {
            if (!__any(st != AT_DONE)) break;
            if (target > 0 && *(volatile int*)&s_fill >= target) break;
            if (st == AT_DONE) continue;
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
            if (ni == 0 && nj == 0) {  // the walk is complete: metrics of its ordered pair
                const int64_t p = cp.p;
                double* o;
                if (out_mode == OUT_BOTH) o = out + (p * 2 + ((prio ^ cp.swp) ? 1 : 0)) * nm;
                else o = out + p * nm;
                for (int m = 0; m < nm; ++m)
                    o[m] = metric_value(ms.code[m], (uint32_t)valid, (uint32_t)ts, (uint32_t)tv, (uint32_t)gap);
                if (sout && (out_mode != OUT_BOTH || !prio)) sout[p] = fin[pb][pi] >> 1;
                st = AT_DONE;
                continue;
            }
            uint32_t nb = 0;
            if (ni >= 1 && nj >= 1) {
                const int t = (nj - 1) / K;
                const int k = nj - 1 - t * K;
                const int s = r0 + ni - 1 + (t & 63);
                // volatile: an L2 (not L1) read of bytes the fill waves stored
                nb = *(const volatile uint8_t*)(tr + ((size_t)s * NT + t) * K + k);
            }
            xa = ni >= 1 ? rs[ni - 1] : 0u;
            yb = nj >= 1 ? cs[nj - 1] : 0u;
            int nst;
            if (ni == 0) {
                nst = AT_IY;  // row 0: only Iy is finite (and Ix(1, j) came from G = Iy)
            } else if (nj == 0) {
                nst = AT_IX;
            } else if (st == AT_M) {  // best state of (ni, nj)
                const int ca = at_sign((nb >> 2) & 3u, 0);
                nst = ca > 0 ? ((nb & 1u) ? AT_M : AT_IY) : (ca == 0 ? (prio ? AT_IY : AT_IX) : AT_IX);
            } else if (st == AT_IX) {  // how Ix(i, j) was formed: G path or extend
                const int sb = at_sign((cb >> 4) & 3u, 0);
                const bool gp = prio ? sb >= 0 : sb > 0;
                nst = gp ? ((nb & 1u) ? AT_M : AT_IY) : AT_IX;
            } else {  // how Iy(i, j) was formed: F path or extend
                const int sc_ = at_sign((cb >> 6) & 3u, 0);
                const bool fp = prio ? sc_ > 0 : sc_ >= 0;
                nst = fp ? ((nb & 2u) ? AT_M : AT_IX) : AT_IY;
            }
            cb = nb;
            i = ni;
            j = nj;
            st = nst;
        }
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
        // ---- cut the next chain (thread 0): pairs with the same column sequence
        __syncthreads();  // the previous chain is done with tab[cur] / xinfo / s_*
        if (tid == 0) {
            int n = 0, rows = 0;
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
                    const int64_t p = q;
                    int64_t a, b;
                    decode_pair(ps, p, a, b);
                    const int4 ma = XS.meta[a];
                    const int4 mb = YS.meta[b];
                    if (ma.x == 0 || mb.x == 0) {  // one side empty: no nucleotide column
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
                        continue;
                    }
                    const uint8_t* xa_ = XS.bytes + XS.offs[a];
                    const uint8_t* yb_ = YS.bytes + YS.offs[b];
                    const bool swp = at_swap(xa_, yb_, ma.x, mb.x, ccol, n);  // rows = b, columns = a
                    const uint8_t* cseq = swp ? xa_ : yb_;
                    const int4 rm = swp ? mb : ma;
                    if (n > 0 && (cseq != ccol || rows + rm.x > cap_rows)) break;
                    if (n == 0) {
                        const int4 cm = swp ? ma : mb;
                        ccol = cseq;
                        chs[cur] = AtChain{cseq, 0, cm.x, cm.y, cm.z};
                    }
                    tab[cur][n] = ChainPair{swp ? YS.bytes + YS.offs[b] : XS.bytes + XS.offs[a], p, rm.x, rm.y,
                                            rm.z, rows, swp ? 1 : 0, 0};
                    rows += rm.x;
                    ++n;
                }
                s_qc = q;
            }
            if (n > 0) chs[cur].n = n;
            s_n = n;
            s_rows = rows;
            fin_n = 0u;
            s_fill = 0;
        }
        __syncthreads();
        const int n = s_n;
        const int rows = s_rows;
        const int pb = cur ^ 1;  // buffer of the chain being walked
        if (walker) walk_init(pb, prev_n);
        if (n == 0) {
            // no more chains: finish the last chain's walks and leave
            if (walker) walk_run(pb, -1, 0);
            break;
        }
        const int nB = chs[cur].nB;

        // ---- fill-lane column constants (once per chain)
        const int j0 = (w * 64 + lane) * K + 1;
        uint32_t eqp0 = 0, eqp1 = 0, eqp2 = 0, eqp3 = 0;
        if (!walker) {
            const uint8_t* cseq = chs[cur].cseq;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int j = j0 + k;
                uint32_t c = 0x100u;
                if (j <= nB) {
                    c = cseq[j - 1];
                    if (c == 'A') eqp0 |= 4u << (3 * k);
                    if (c == 'C') eqp1 |= 4u << (3 * k);
                    if (c == 'G') eqp2 |= 4u << (3 * k);
                    if (c == 'T') eqp3 |= 4u << (3 * k);
                }
                colb[tid * K + k] = (uint8_t)(c & 0xFFu);
                if (c > 0xFFu) colb[tid * K + k] = 0;  // padding column: never equal to a row byte
                colc[k][tid] = make_int2((j == nB) ? sc.eo : sc.io, (j == nB) ? sc.ee : sc.ie);
            }
        }
        if (tid < 64) xinfo[tid] = a1c_row_info(tab[cur], n, rows, tid);
        // column states at row 0 (reset again on every pair's first row)
        int stG[K], stX[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            stG[k] = sc.eo + sc.ee * (j0 + k - 1);
            stX[k] = NEG_INF;
        }
        int payF = NEG_INF, payY = sc.eo + sc.ee * (j0 + K - 2);
        int carry = j0 == 1 ? 1 : sc.eo + sc.ee * (j0 - 2);
        const uint2* ring_in = (w > 0 && !walker) ? ring + (size_t)(w - 1) * RING : nullptr;
        uint2* ring_out = (w < W - 1) ? ring + (size_t)w * RING : nullptr;
        uint8_t* trb = bufs + (size_t)cur * (size_t)buf_bytes;
        __syncthreads();  // xinfo block 0, colb

        const int nsteps = rows + 63;
        const int nblk = (nsteps + INTERVAL - 1) / INTERVAL;
        const int nint = nblk + WAVE_LAG * (W - 1);
        for (int it = 0; it < nint; ++it) {
            if (walker) {
                walk_run(pb, hops, W * (it + 1));
            } else {
                const int blk = it - WAVE_LAG * w;
                if (blk >= 0 && blk < nblk) {
                    const int s0 = blk * INTERVAL;
                    const int s1 = min(s0 + INTERVAL, nsteps);
                    for (int s = s0; s < s1; ++s) {
                        const int g = s - lane;
                        const uint32_t xi = g >= 0 ? xinfo[g & (XR - 1)] : A1C_NONE;
                        int inF, inY;
                        if (w == 0) {
                            const int ir = (int)((xi >> 18) & 0xFFFu);  // Ix(i, 0) = eo + ee (i - 1)
                            inF = (int)shr_old((uint32_t)payF, (uint32_t)(sc.eo + sc.ee * (ir - 1)));
                            inY = (int)shr_old((uint32_t)payY, (uint32_t)NEG_INF);
                        } else {
                            const uint2 o = ring_in[(s + 1) & (RING - 1)];
                            inF = (int)shr_old((uint32_t)payF, o.x);
                            inY = (int)shr_old((uint32_t)payY, o.y);
                        }
                        if (!(xi & A1C_NONE)) {
                            if (xi & A1C_FIRST) {  // a new pair starts at this lane: row-0 states
                                int jb = tid * K;
                                asm volatile("" : "+v"(jb));
#pragma unroll
                                for (int k = 0; k < K; ++k) {
                                    stG[k] = sc.eo + sc.ee * (jb + k);
                                    stX[k] = NEG_INF;
                                }
                                carry = jb == 0 ? 1 : sc.eo + sc.ee * (jb - 1);
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
#pragma unroll
                            for (int k = 0; k < K; ++k) {
                                const int G = stG[k], X = stX[k];
                                const int nd = max(G, X);
                                const uint32_t e = (eq >> (3 * k)) & 7u;
                                const int sM = DEF ? sc.mi + (int)e : (e ? sc.ma : sc.mi);
                                const int M = (d | 1) + sM;
                                const int2 cc2 = colc[k][tid];
                                const int ex = DEF ? sc.ie : cc2.y;
                                const int cg = G + cc2.x, cx = X + ex;
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
                                uint32_t* dst = (uint32_t*)(trb + ((size_t)s * NT + tid) * K);
                                if constexpr (K == 8) {
                                    *(uint2*)dst = make_uint2(acc[0], acc[1]);
                                } else {
#pragma unroll
                                    for (int q = 0; q < K / 4; ++q) dst[q] = acc[q];
                                }
                            }
                            if (W > 1 && ring_out != nullptr && lane == 63)
                                ring_out[(g + 1) & (RING - 1)] = make_uint2((uint32_t)payF, (uint32_t)payY);
                            if (lastrow && tid == (nB - 1) / K) {  // this lane owns column nB: final score
                                const int out_k = (nB - 1) % K;
                                int eG = stG[0], eX = stX[0];
#pragma unroll
                                for (int k = 1; k < K; ++k) {
                                    uint32_t m = (k == out_k) ? ~0u : 0u;
                                    asm volatile("" : "+v"(m));
                                    eG = (int)(((uint32_t)stG[k] & m) | ((uint32_t)eG & ~m));
                                    eX = (int)(((uint32_t)stX[k] & m) | ((uint32_t)eX & ~m));
                                }
                                fin[cur][fin_n++] = max(eG, eX);
                            }
                        }
                        carry = max(inF, inY);
                    }
                }
            }
            // block it+1's new rows (its lane-0 rows); the barrier publishes them
            const int gpre = (it + 1) * INTERVAL + tid;
            if (tid < INTERVAL && it + 1 < nblk) xinfo[gpre & (XR - 1)] = a1c_row_info(tab[cur], n, rows, gpre);
            if (it + 1 == nint) __builtin_amdgcn_s_waitcnt(0);  // this chain's trace stores have landed
            if (!walker && lane == 0) atomicAdd(&s_fill, 1);  // this fill wave is done with interval it
            __syncthreads();
        }
        // ---- the walker finishes the previous chain (the fill waves wait at the next barrier)
        if (walker) walk_run(pb, -1, 0);
        prev_n = n;
        cur ^= 1;
    }
}

}  // namespace taxi2
