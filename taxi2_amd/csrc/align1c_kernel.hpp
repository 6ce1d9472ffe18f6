// Chained single-orientation aligner: k_align1 with the rows of consecutive pairs streamed back
// to back through the same systolic lanes.
//
// In the versusAll triangle (pairs (a, b), b = a+1, a+2, ...) and the versusReference rectangle
// (query-major) consecutive pairs share their first sequence.  Making that shared sequence the
// COLUMN sequence (orientation A = (b, a) when len(b) <= len(a), so rows stay the shorter side)
// leaves every lane's column constants unchanged from one pair to the next: only the rows
// change.  A workgroup therefore takes a chunk of consecutive pairs from the cursor, cuts it
// into chains of pairs with the same column sequence, and feeds each chain's rows to the
// wavefront as one stream.  Each lane meets a pair boundary one step after its left neighbour
// (it is simply the next row of the stream): on a pair's first row it resets its column states
// to row 0 and its diagonal to the row-0 boundary; after the last row the lane that owns column
// nB writes the pair's counters.  The 63-step fill / drain skew of the systolic wavefront (6 % at
// 1 000 rows) and the per-pair prologue are paid once per chain instead of once per pair.
//
// Rows reach the lanes through a ring in LDS (xinfo[g % XR] for global row g of the chain): each
// 64-step block, wave 0 prefetches the next block's 64 rows (byte class, span flags, the row's
// index in its pair, first / last-row flags) while the waves compute; the block barrier
// publishes them.  XR = 256 * W covers every row between the prefetch and the slowest wave
// (WAVE_LAG blocks behind per wave).  Per-cell arithmetic is s1_cell of align1_kernel.hpp,
// unchanged: the results are bit-identical to k_align1.
#pragma once
#include "align1_kernel.hpp"

namespace taxi2 {

constexpr int A1C_CHUNK = 16;  // pairs pulled from the cursor at a time (cut into chains)

// xinfo ring entry: a1_xinfo bits 0-15 | first row of its pair << 16 | last row << 17 |
// row index in its pair (1-based) << 18 | no row << 31
constexpr uint32_t A1C_FIRST = 1u << 16;
constexpr uint32_t A1C_LAST = 1u << 17;
constexpr uint32_t A1C_NONE = 1u << 31;

struct ChainPair {
    const uint8_t* rseq;  // row sequence
    int64_t p;            // pair index
    int nA, fx, lx;       // rows, first / last nucleotide index of the row sequence
    int r0;               // first global row of the pair in the chain
    int swp;              // orientation A = (rows, cols) is the (b, a) ordered pair
    int pad;
};

__host__ __device__ constexpr int a1c_xr(int W) { return 256 * W; }
__host__ __device__ inline size_t a1c_table_off(int W) { return (size_t)a1c_xr(W) * 4; }
__host__ __device__ inline size_t a1c_fin_off(int W) { return a1c_table_off(W) + A1C_CHUNK * sizeof(ChainPair); }
__host__ __device__ inline size_t a1c_ring_off(int W) { return a1c_fin_off(W) + A1C_CHUNK * sizeof(uint4); }
__host__ __device__ inline size_t a1c_colc_off(int W) { return a1c_ring_off(W) + (size_t)(W - 1) * RING * sizeof(RingEntry1); }
// [.. colc / colex] [u32 fin count].  K = 8, W = 2: 19.3 KB, 8 workgroups (4 waves / SIMD) per CU.
__host__ __device__ inline size_t a1c_fin_n_off(int K, int W, bool def) {
    return a1c_colc_off(W) + (size_t)K * 64 * W * (sizeof(ColC) + (def ? 0 : sizeof(int)));
}
__host__ __device__ inline size_t a1c_lds_bytes(int K, int W, bool def) { return a1c_fin_n_off(K, W, def) + 16; }

// xinfo entry of global row g of a chain with n pairs and `rows` rows in total.
__device__ __forceinline__ uint32_t a1c_row_info(const ChainPair* __restrict__ tab, int n, int rows, int g) {
    if (g >= rows) return A1C_NONE;
    int k = 0;
    for (int t = 1; t < n; ++t)
        if (tab[t].r0 <= g) k = t;
    const ChainPair& cp = tab[k];
    const int i = g - cp.r0;  // 0-based row of the pair
    uint32_t v = a1_xinfo(cp.rseq[i], i, cp.fx, cp.lx);
    if (i == 0) v |= A1C_FIRST;
    if (i == cp.nA - 1) v |= A1C_LAST;
    return v | ((uint32_t)(i + 1) << 18);
}

template <int K, int W, bool DEF, bool B, bool FIRST, int NW>
__device__ __forceinline__ void dp_step1c(int s, int lane, S1Col<NW> (&st)[K], S1Left<NW>& pay, S1Best<NW>& carry,
                                          const LaneCols1<K>& lc, const ColC* __restrict__ colc,
                                          const int* __restrict__ colex, const uint32_t* __restrict__ xinfo,
                                          const RingEntry1* __restrict__ ring_in, RingEntry1* __restrict__ ring_out,
                                          const KScores& sc, uint4* __restrict__ fin_tab, uint32_t* fin_n, int nB) {
    constexpr bool TRACK = !B;
    const int g = s - lane;
    const uint32_t xi = g >= 0 ? xinfo[g & (a1c_xr(W) - 1)] : A1C_NONE;
    S1Left<NW> in;
    if constexpr (FIRST) {
        in = s1_shr_first(pay, (int)((xi >> 18) & 0xFFFu), sc);
    } else {
        S1Left<NW> old;
        ring_get(ring_in + ((s + 1) & (RING - 1)), old);
        in = s1_shr_old(pay, old);
    }
    if (!(xi & A1C_NONE)) {
        if (xi & A1C_FIRST) {  // a new pair starts at this lane: row-0 states and diagonal
            // j0 - 1 behind an opaque copy: the K row-0 values are recomputed here, not hoisted out
            // of the loop into K more live registers
            int jb = (int)threadIdx.x * K;
            asm volatile("" : "+v"(jb));
#pragma unroll
            for (int k = 0; k < K; ++k) {
                st[k].G = sc.eo + sc.ee * (jb + k);  // row 0, column j = jb + k + 1 >= 1
                st[k].X = NEG_INF;
                st[k].g = st[k].x = cnt_zero<NW>();
            }
            carry.h = jb == 0 ? 1 : sc.eo + sc.ee * (jb - 1);  // best of the row-0 state of column jb
            carry.c = cnt_zero<NW>();
        }
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
        const bool lastrow = (xi & A1C_LAST) != 0u;
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
        if (W > 1 && ring_out != nullptr && lane == 63) ring_put(ring_out + ((g + 1) & (RING - 1)), pay);
        if (lastrow) {
            const int jl = nB - 1;
            const int tid = (int)threadIdx.x;
            if (tid == jl / K) {  // this lane owns column nB: the pair is complete
                const int out_k = jl % K;
                // bitwise select with an opaque mask: a plain `if (k == out_k) e = st[k]` is folded into
                // st[out_k], and a dynamic index inside the loop moves the whole st array to scratch
                S1Col<NW> e = st[0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    uint32_t m = (k == out_k) ? ~0u : 0u;
                    asm volatile("" : "+v"(m));
                    e.G = (int)(((uint32_t)st[k].G & m) | ((uint32_t)e.G & ~m));
                    e.X = (int)(((uint32_t)st[k].X & m) | ((uint32_t)e.X & ~m));
#pragma unroll
                    for (int q = 0; q < NW; ++q) {
                        e.g.w[q] = (st[k].g.w[q] & m) | (e.g.w[q] & ~m);
                        e.x.w[q] = (st[k].x.w[q] & m) | (e.x.w[q] & ~m);
                    }
                }
                const S1Best<NW> fin = s1_best_col<B, !B>(e);
                fin_tab[(*fin_n)++] = make_uint4((uint32_t)fin.h, fin.c.w[0], fin.c.w[1], NW == 3 ? fin.c.w[NW - 1] : 0u);
            }
        }
    }
    carry = s1_best_left<B, TRACK>(in);
}

// Orientation of a pair cut into a chain (true: columns = X[a], rows = Y[b]).  A pair that
// contains the chain's column sequence keeps it on the columns, so the chain goes on.  A chain
// starts with X[a] on the columns (the sequence consecutive pairs share: a triangle row, a
// query against its references) unless Y[b] is more than 1/8 longer (then the shorter rows
// save more steps than the chain would).  Equal lengths: X[a] always.
__device__ __forceinline__ bool at_swap(const uint8_t* xa, const uint8_t* yb, int la, int lb, const uint8_t* ccol,
                                        int n) {
    if (n > 0 && xa == ccol) return true;
    if (n > 0 && yb == ccol) return false;
    return 8 * lb <= 9 * la;
}

// Pass 1 (B = false) over ps / pass 2 (B = true) over wlist[0, *wcount), as k_align1.
template <int K, int W, bool DEF, int OCC, bool B, int NW>
__global__ void __launch_bounds__(64 * W, OCC)
k_align1c(SetView XS, SetView YS, PairSrc ps, KScores scin, MetricSpec ms, int chunk_req, int out_mode,
          double* __restrict__ out, int32_t* __restrict__ sout, uint32_t* __restrict__ wlist,
          uint32_t* __restrict__ wcount, unsigned long long* __restrict__ next) {
    static_assert(K <= A1_MAX_K, "equality fields hold at most 10 columns");
    const KScores sc0 = DEF ? KScores{1, -1, -8, -1, -1, -1} : scin;  // align.py:20-27 defaults
    const KScores sc = doubled(sc0);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* xinfo = reinterpret_cast<uint32_t*>(smem);
    ChainPair* tab = reinterpret_cast<ChainPair*>(smem + a1c_table_off(W));
    uint4* fin_tab = reinterpret_cast<uint4*>(smem + a1c_fin_off(W));
    RingEntry1* rings = reinterpret_cast<RingEntry1*>(smem + a1c_ring_off(W));
    ColC* colc = reinterpret_cast<ColC*>(smem + a1c_colc_off(W)) + threadIdx.x;
    int* colex = reinterpret_cast<int*>(reinterpret_cast<ColC*>(smem + a1c_colc_off(W)) + K * 64 * W) + threadIdx.x;
    uint32_t* fin_n = reinterpret_cast<uint32_t*>(smem + a1c_fin_n_off(K, W, DEF));

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int nm = ms.n;
    const int64_t total = B ? (int64_t)*wcount : ps.count;
    __shared__ int64_t s_q0, s_qnext;
    __shared__ const uint8_t* s_cseq;
    __shared__ int s_n, s_rows, s_nB, s_fy, s_ly;

    // chunk: up to A1C_CHUNK pairs, but at least ~8 chunks per workgroup so that the pass's tail
    // stays balanced (pass 2 sees a few percent of the pairs); chunk_req in [1, A1C_CHUNK] forces it
    const int64_t chunk = chunk_req >= 1 ? min((int64_t)chunk_req, (int64_t)A1C_CHUNK)
                                         : max((int64_t)1, min((int64_t)A1C_CHUNK, total / ((int64_t)gridDim.x * 8)));
    for (;;) {
        __syncthreads();  // the previous chunk is done with s_q0
        if (threadIdx.x == 0) s_q0 = (int64_t)atomicAdd(next, (unsigned long long)chunk);
        __syncthreads();
        const int64_t q0 = s_q0;
        if (q0 >= total) break;
        const int64_t qend = min(q0 + chunk, total);
        for (int64_t qc = q0; qc < qend;) {
            // ---- cut the next chain (thread 0): pairs with the same column sequence
            __syncthreads();  // the previous chain is done with tab / xinfo / s_*
            if (threadIdx.x == 0) {
                int n = 0, rows = 0;
                int64_t q = qc;
                const uint8_t* ccol = nullptr;
                for (; q < qend; ++q) {
                    // pass 2 entries carry pass 1's orientation in bit 31 (pair index < 2^31, host-checked)
                    const uint32_t wq = B ? wlist[q] : 0u;
                    const int64_t p = B ? (int64_t)(wq & 0x7FFFFFFFu) : q;
                    int64_t a, b;
                    decode_pair(ps, p, a, b);
                    const int4 ma = XS.meta[a];
                    const int4 mb = YS.meta[b];
                    if (ma.x == 0 || mb.x == 0) {  // one side empty (pass 1 only): no nucleotide column
                        if (n > 0) break;          // (keeps output order simple: flush the chain first)
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
                    // orientation (swp: rows = b, columns = a): the chain rule at_swap (keep
                    // the shared sequence on the columns; rows may then be up to 1/8 longer than
                    // columns, within the variant's capacity, which covers both sets).  It depends on
                    // the chain being cut, so pass 2 -- which cuts its own chains -- must not re-decide
                    // it: it reuses pass 1's choice from the worklist entry (a re-decided orientation
                    // wrote the unwritten orientation's slot: a null slot in single-orientation mode)
                    const bool swp = B ? (wq >> 31) != 0u
                                       : at_swap(XS.bytes + XS.offs[a], YS.bytes + YS.offs[b], ma.x, mb.x, ccol, n);
                    const uint8_t* cseq = swp ? XS.bytes + XS.offs[a] : YS.bytes + YS.offs[b];
                    if (n > 0 && cseq != ccol) break;
                    const int4 rm = swp ? mb : ma;
                    if (n == 0) {
                        const int4 cm = swp ? ma : mb;
                        ccol = cseq;
                        s_cseq = cseq;
                        s_nB = cm.x;
                        s_fy = cm.y;
                        s_ly = cm.z;
                    }
                    tab[n] = ChainPair{swp ? YS.bytes + YS.offs[b] : XS.bytes + XS.offs[a], p, rm.x, rm.y, rm.z,
                                       rows, swp ? 1 : 0, 0};
                    rows += rm.x;
                    ++n;
                }
                s_n = n;
                s_rows = rows;
                s_qnext = q;
            }
            __syncthreads();
            qc = s_qnext;
            const int n = s_n;
            if (n == 0) continue;
            const int rows = s_rows;
            const int nB = s_nB;

            // ---- per-lane column constants (once per chain)
            const uint8_t* cseq = s_cseq;
            const int fy = s_fy, ly = s_ly;
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
                            l |= 1u << xb;                                   // valid
                            if (dd == 2) l |= 1u << (a1_ts_bit<NW>() + xb);  // transition
                            else if (dd) l |= 1u << (20 + xb);               // transversion
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
            if (threadIdx.x == 0) *fin_n = 0u;
            if (threadIdx.x < 64) xinfo[threadIdx.x] = a1c_row_info(tab, n, rows, threadIdx.x);

            S1Col<NW> st[K];
#pragma unroll
            for (int k = 0; k < K; ++k) st[k] = s1_col_row0<NW>(j0 + k, sc);
            S1Left<NW> pay = s1_left_row0<NW>(j0 + K - 1, sc);
            S1Best<NW> carry = s1_best_col<B, false>(s1_col_row0<NW>(j0 - 1, sc));

            const RingEntry1* ring_in = (w > 0) ? rings + (size_t)(w - 1) * RING : nullptr;
            RingEntry1* ring_out = (w < W - 1) ? rings + (size_t)w * RING : nullptr;
            __syncthreads();  // xinfo block 0, colc

            const int nsteps = rows + 63;
            const int nblk = (nsteps + INTERVAL - 1) / INTERVAL;
            const int nint = nblk + WAVE_LAG * (W - 1);
            for (int it = 0; it < nint; ++it) {
                const int blk = it - WAVE_LAG * w;
                if (blk >= 0 && blk < nblk) {
                    const int s0 = blk * INTERVAL;
                    const int s1 = min(s0 + INTERVAL, nsteps);
                    if (w == 0) {
                        for (int s = s0; s < s1; ++s)
                            dp_step1c<K, W, DEF, B, true, NW>(s, lane, st, pay, carry, lc, colc, colex, xinfo,
                                                              ring_in, ring_out, sc, fin_tab, fin_n, nB);
                    } else {
                        for (int s = s0; s < s1; ++s)
                            dp_step1c<K, W, DEF, B, false, NW>(s, lane, st, pay, carry, lc, colc, colex, xinfo,
                                                               ring_in, ring_out, sc, fin_tab, fin_n, nB);
                    }
                }
                // block it+1's new rows (its lane-0 rows); the barrier publishes them
                const int gpre = (it + 1) * INTERVAL + (int)threadIdx.x;
                if (threadIdx.x < INTERVAL && it + 1 < nblk) xinfo[gpre & (a1c_xr(W) - 1)] = a1c_row_info(tab, n, rows, gpre);
                __syncthreads();
            }

            // ---- outputs of the chain's pairs, one thread each (fin_tab: score, counter words)
            if (threadIdx.x < n) {
                const ChainPair& cp = tab[threadIdx.x];
                const uint4 f = fin_tab[threadIdx.x];
                Cnt<NW> c;
                c.w[0] = f.y;
                c.w[1] = f.z;
                if constexpr (NW == 3) c.w[2] = f.w;
                const int64_t p = cp.p;
                double* o_ab;
                double* o_ba = nullptr;
                if (out_mode == OUT_BOTH) {
                    o_ab = out + (p * 2 + 0) * nm;
                    o_ba = out + (p * 2 + 1) * nm;
                } else {
                    o_ab = out + p * nm;
                }
                double* slot_a = cp.swp ? o_ba : o_ab;  // orientation A = (rows, cols)
                double* slot_b = cp.swp ? o_ab : o_ba;
                if (B) {
                    if (slot_b) a1_write(slot_b, ms, c);
                } else {
                    const bool diverges = (c.w[1] & 0x3FFFu) != 0u;
                    if (slot_a) a1_write(slot_a, ms, c);
                    if (slot_b) {
                        if (!diverges) a1_write(slot_b, ms, c);
                        else wlist[atomicAdd(wcount, 1u)] = (uint32_t)p | ((uint32_t)cp.swp << 31);
                    }
                    if (sout) sout[p] = (int)f.x >> 1;
                }
            }
        }
    }
}

}  // namespace taxi2
