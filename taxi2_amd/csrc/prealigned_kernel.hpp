// Pre-aligned distances (params.pairs.align == False): calc.seq_distances_* on the raw
// strings (distances.py:319-348), for every pair of a launch.
//
// Each sequence is stored as bit-planes, 32 columns per uint4 word {base lo, base hi,
// ACGT-valid, '-'} (pack_kernels.hpp).  Per pair the common range
// [max(first ACGT), min(last ACGT)] is walked a word at a time:
//   both  = valid_x & valid_y & range
//   ts    = both &  (hi_x ^ hi_y) & ~(lo_x ^ lo_y)   (A<->G, C<->T: only the high bit differs)
//   tv    = both &  (lo_x ^ lo_y)
//   gap   = ((gap_x & valid_y) | (gap_y & valid_x)) & range
// and the four counters are popcounts.  The counters are symmetric, so one value per
// unordered pair serves both ordered rows of versusAll.
//
// k_prealigned: one thread per pair, operands straight from L2 (pair lists, small launches).
// k_prealigned_tile: the triangle and the rectangle, PT x PT pair tiles with both sides' planes
// staged in LDS (below).
#pragma once
#include "common.hpp"

namespace taxi2 {

__device__ __forceinline__ void count_words(const uint4* __restrict__ px, const uint4* __restrict__ py,
                                            int lo, int hi, uint32_t& valid, uint32_t& ts,
                                            uint32_t& tv, uint32_t& gap) {
    valid = ts = tv = gap = 0;
    if (lo > hi) return;
    const int w0 = lo >> 5, w1 = hi >> 5;
    for (int wd = w0; wd <= w1; ++wd) {
        uint32_t m = 0xFFFFFFFFu;
        if (wd == w0) m &= 0xFFFFFFFFu << (lo & 31);
        if (wd == w1) m &= 0xFFFFFFFFu >> (31 - (hi & 31));
        const uint4 a = px[wd];
        const uint4 b = py[wd];
        const uint32_t both = a.z & b.z & m;
        const uint32_t dlo = a.x ^ b.x;
        const uint32_t dhi = a.y ^ b.y;
        valid += __popc(both);
        ts += __popc(both & dhi & ~dlo);
        tv += __popc(both & dlo);
        gap += __popc(((a.w & b.z) | (b.w & a.z)) & m);
    }
}

// Generic pair-list form (LIST; TRI / RECT too small for a tile); one thread per pair, operands
// from L2.
__global__ void __launch_bounds__(256)
k_prealigned(SetView XS, SetView YS, PairSrc ps, MetricSpec ms, double* __restrict__ out) {
    const int nm = ms.n;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < ps.count;
         p += (int64_t)gridDim.x * blockDim.x) {
        int64_t a, b;
        decode_pair(ps, p, a, b);
        const int4 ma = XS.meta[a];
        const int4 mb = YS.meta[b];
        const int lo = max(ma.y, mb.y);
        const int hi = min(ma.z, mb.z);
        uint32_t v, ts, tv, g;
        count_words(XS.planes + ma.w, YS.planes + mb.w, lo, hi, v, ts, tv, g);
        for (int m = 0; m < nm; ++m) out[p * nm + m] = metric_value(ms.code[m], v, ts, tv, g);
    }
}

// Tiled form for the versusAll triangle and the rectangle (round 3).  The one-thread-per-pair
// kernel gathers 2 x ceil(L/32) words of planes per pair from L2 (1 KB per 1 000 bp pair): at
// config 5 (N = 200 000, a 100 MB plane set that does not stay in L2) the operand gathers, not
// the arithmetic, bound it.  Here a workgroup takes a tile of PT x-sequences x PT y-sequences,
// stages both sides' planes in LDS PWC words at a time (coalesced 16-byte loads, zero beyond a
// sequence's end) and each thread accumulates a 4 x 4 block of pairs from registers: per word
// 8 LDS reads feed 16 pair updates, so every plane word fetched from memory serves PT pairs.
//
// No per-pair range mask: a valid bit lies inside its own sequence's [first, last ACGT] by
// definition, and k_planes keeps gap bits only inside that range, so
//   both = vx & vy,   gap = (gx & vy) | (gy & vx)
// are already restricted to the pair's common range [max(first), min(last)] (count_words masks it
// explicitly; the two agree bit for bit, tests/test_gpu_parity.py).
constexpr int PT = 64;        // sequences per tile side
constexpr int PWC = 16;       // plane words staged per chunk
constexpr int PWS = PWC + 1;  // padded LDS row (uint4): 16 lanes reading 16 rows hit 64 distinct banks
constexpr int TILE_STAGE_NM = 4;  // metrics per pair the epilogue's LDS stage holds (16 x PT x 4 f64 = 32 KB)

// Row-block epilogue of the streamed versusAll (config 5; taxi2_rect_block_dev): every value x scale
// (the task's x100, the same f64 multiply as D * 100), the diagonal rule's NaN on x == y (one set on
// both sides), and per (x row, tile) the first minimum of metric rmin_k over the tile's defined values
// (-0.0 == 0.0, ties to the lower y), reduced per row by k_rowmin_finish.
struct TileBlock {
    double scale;
    int diag, rmin_k;
    double* rmin_v;   // [nx][tiles_y]: tile minimum (+inf: none)
    int64_t* rmin_y;  // its column (-1: none)
    // column y of the Y set is the task's column ynat[y] (a permuted copy of the X set: config 5's
    // columns in subset order); nullptr: y itself.  The diagonal and the row minima use it.
    const int64_t* ynat = nullptr;
};
struct RowMin {
    double v;
    int64_t y;
};
__device__ __forceinline__ bool rowmin_less(double a, int64_t ya, double b, int64_t yb) {
    return a < b || (a == b && ya < yb);
}

// Tile grid: x rows [x0, x0 + nx), y columns [y0, y0 + ny); tiles_y tiles per tile row.
// MODE PAIRS_TRI: pair (a, b) exists for b > a, output slot tri(a, b) - ps.k0 when that lies in
// [0, ps.count); PAIRS_RECT: output slot (a * ps.R + b) - ps.k0 (b indexes YS).  GAP: some metric
// reads the gap counter (p-gaps); without it the gap popcount (4 of ~14 ops per pair-word) is skipped.
template <int MODE, bool GAP>
__global__ void __launch_bounds__(256)
k_prealigned_tile(SetView XS, SetView YS, PairSrc ps, int64_t x0, int64_t nx, int64_t y0, int64_t ny,
                  int64_t tiles_y, int nwords, MetricSpec ms, double* __restrict__ out, TileBlock tb) {
    __shared__ uint4 sxy[2 * PT * PWS];  // both sides' plane stages; the epilogue's output / row-min stage
    uint4* const sx = sxy;
    uint4* const sy = sxy + PT * PWS;
    const int tid = (int)threadIdx.x;
    const int tx = tid & 15, ty = tid >> 4;
    const int64_t bx = (int64_t)blockIdx.x / tiles_y, by = (int64_t)blockIdx.x - bx * tiles_y;
    const int64_t xa = x0 + bx * PT, ya = y0 + by * PT;
    // the whole tile at or below the diagonal: nothing to do (uniform, before any barrier)
    if (MODE == PAIRS_TRI && ya + PT - 1 <= xa) return;
    const int64_t xe = min(x0 + nx, xa + PT), ye = min(y0 + ny, ya + PT);
    uint32_t c[4][4][4];  // [i][j][valid, ts, tv, gap]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) c[i][j][q] = 0u;
    for (int w0 = 0; w0 < nwords; w0 += PWC) {
        __syncthreads();  // the previous chunk's readers are done
        // stage: PT sequences x PWC words per side, one uint4 per thread and pass
        for (int e = tid; e < PT * PWC; e += 256) {
            const int r = e / PWC, wd = e - r * PWC;
            uint4 vx = make_uint4(0u, 0u, 0u, 0u), vy = vx;
            const int64_t s = xa + r, t = ya + r;
            if (s < xe) {
                const int4 m = XS.meta[s];
                if (w0 + wd < (m.x + 31) / 32) vx = XS.planes[m.w + w0 + wd];
            }
            if (t < ye) {
                const int4 m = YS.meta[t];
                if (w0 + wd < (m.x + 31) / 32) vy = YS.planes[m.w + w0 + wd];
            }
            sx[r * PWS + wd] = vx;
            sy[r * PWS + wd] = vy;
        }
        __syncthreads();
        const int wn = min(PWC, nwords - w0);
        for (int wd = 0; wd < wn; ++wd) {
            uint4 a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = sx[(tx + 16 * i) * PWS + wd];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = sy[(ty + 16 * j) * PWS + wd];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    // c[1] counts all mismatches (ts + tv; ts = c[1] - c[2] in the epilogue).  Two
                    // three-input v_bitop3 (truth tables symmetric in the outer operands):
                    //   tvb  = both & (x.lo ^ y.lo)   (0x48: S1 & (S0 ^ S2))  -- a transversion
                    //   mism = both & (tvb | dhi)     (0xc8: S1 & (S0 | S2))  -- any base bit differs
                    const uint32_t both = a[i].z & b[j].z;
                    const uint32_t dhi = a[i].y ^ b[j].y;
                    uint32_t tvb, mism;
                    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x48" : "=v"(tvb) : "v"(a[i].x), "v"(both), "v"(b[j].x));
                    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xc8" : "=v"(mism) : "v"(tvb), "v"(both), "v"(dhi));
                    c[i][j][0] += __popc(both);
                    c[i][j][1] += __popc(mism);
                    c[i][j][2] += __popc(tvb);
                    if constexpr (GAP) c[i][j][3] += __popc((a[i].w & b[j].z) | (b[j].w & a[i].z));
                }
        }
    }
    const int nm = ms.n;
    double rv[4];
    int64_t ry[4];
    // Output through LDS, 16 rows at a time: a thread's pairs are spread over 16 rows, so direct
    // stores would write 16 short strided pieces per instruction; staged, the workgroup writes
    // each row's run of slots (nm values per pair, up to 64 pairs) as one contiguous stretch.
    double* stg = (double*)sxy;  // [16 rows][PT cols][nm] (24 KB at nm = 3; the stages hold 34 KB)
    const bool staged = nm <= TILE_STAGE_NM;
    if (staged) __syncthreads();  // the plane stages are free
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        rv[i] = __builtin_inf();
        ry[i] = -1;
        const int64_t x = xa + tx + 16 * i;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t y = ya + ty + 16 * j;
            bool ok = x < xe && y < ye;
            int64_t slot = 0;
            if (MODE == PAIRS_TRI) {
                ok = ok && y > x;
                slot = x * (2 * ps.N - x - 1) / 2 + (y - x - 1) - ps.k0;
            } else {
                slot = x * ps.R + y - ps.k0;  // a launch may start / end inside a row
            }
            ok = ok && slot >= 0 && slot < ps.count;
            const int64_t yn = tb.ynat ? (ok ? tb.ynat[y] : -1) : y;  // the task's column
            const uint32_t ts = c[i][j][1] - c[i][j][2];
            const bool none = tb.diag && x == yn;
            const double pd = c[i][j][0] ? (double)c[i][j][1] / (double)c[i][j][0] : __builtin_nan("");
            for (int m = 0; m < nm; ++m) {
                const double v = none ? __builtin_nan("")
                                      : metric_value_p(ms.code[m], c[i][j][0], ts, c[i][j][2], c[i][j][3], pd) * tb.scale;
                if (staged) stg[(tx * PT + ty + 16 * j) * nm + m] = v;
                else if (ok) out[slot * nm + m] = v;
                // the first (lowest task column) of equal values stays
                if (ok && m == tb.rmin_k && __builtin_isfinite(v) && (ry[i] < 0 || rowmin_less(v, yn, rv[i], ry[i]))) {
                    rv[i] = v;
                    ry[i] = yn;
                }
            }
        }
        if (staged) {
            __syncthreads();
            // rows xa + r + 16 i (r = 0..15): the row's pairs y in [ya, ye) (TRI: y > x) are consecutive
            // slots; element e of the row's run is pair y = y_lo + e / nm, metric e % nm
            for (int r = tid >> 4; r < 16; r += 16) {
                const int64_t x = xa + r + 16 * i;
                if (x >= xe) continue;
                const int64_t ylo = MODE == PAIRS_TRI ? max(ya, x + 1) : ya;
                if (ylo >= ye) continue;
                const int64_t s0 = MODE == PAIRS_TRI ? x * (2 * ps.N - x - 1) / 2 + (ylo - x - 1) - ps.k0
                                                     : x * ps.R + ylo - ps.k0;
                const int64_t lo = max((int64_t)0, -s0), hi = min(ye - ylo, ps.count - s0);  // pairs in the launch
                for (int64_t e = lo * nm + (tid & 15); e < hi * nm; e += 16)
                    out[s0 * nm + e] = stg[(r * PT + (ylo - ya)) * nm + e];
            }
            __syncthreads();  // the stage is rewritten by the next i
        }
    }
    if (tb.rmin_v) {  // per (row, tile): the 16 threads of a row (ty = 0..15) through LDS, in y order
        __syncthreads();  // the plane / output stages are free
        RowMin* red = (RowMin*)sx;  // [ty][64 rows]
#pragma unroll
        for (int i = 0; i < 4; ++i) red[ty * PT + tx + 16 * i] = RowMin{rv[i], ry[i]};
        __syncthreads();
        if (tid < PT) {
            double v = __builtin_inf();
            int64_t y = -1;
            for (int t = 0; t < 16; ++t) {
                const RowMin r = red[t * PT + tid];
                if (r.y >= 0 && (y < 0 || rowmin_less(r.v, r.y, v, y))) {
                    v = r.v;
                    y = r.y;
                }
            }
            const int64_t x = xa + tid;
            if (x < xe) {
                tb.rmin_v[(x - x0) * tiles_y + by] = v;
                tb.rmin_y[(x - x0) * tiles_y + by] = y;
            }
        }
    }
}

// Per row of a block: the first minimum over its tiles (in y order) -> idx (-1: none) and value (NaN).
__global__ void __launch_bounds__(256) k_rowmin_finish(int64_t nx, int64_t tiles_y, const double* __restrict__ tv,
                                                        const int64_t* __restrict__ ty_, int64_t* __restrict__ idx,
                                                        double* __restrict__ val) {
    const int lane = threadIdx.x & 63;
    const int64_t x = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (x >= nx) return;
    double v = __builtin_inf();
    int64_t y = -1;
    for (int64_t t = lane; t < tiles_y; t += 64) {
        const double a = tv[x * tiles_y + t];
        const int64_t ya = ty_[x * tiles_y + t];
        if (ya >= 0 && (y < 0 || rowmin_less(a, ya, v, y))) {
            v = a;
            y = ya;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double a = __shfl_xor(v, o);
        const int64_t ya = __shfl_xor(y, o);
        if (ya >= 0 && (y < 0 || rowmin_less(a, ya, v, y))) {
            v = a;
            y = ya;
        }
    }
    if (lane == 0) {
        idx[x] = y;
        val[x] = y >= 0 ? v : __builtin_nan("");
    }
}

}  // namespace taxi2
