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
// One thread per pair; the planes of a whole set are small (N x L/8 bytes: 2 000 x 600 bp is
// 150 KB) and stay resident in L2 / the Infinity Cache, so operands are read straight from
// there.  Work per pair is ~6 VALU ops per 32 columns, so the kernel is bounded by its f64
// output stream (HBM write).
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

// Generic pair-list form (TRI / RECT / LIST); one thread per pair, operands from L2.
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

}  // namespace taxi2
