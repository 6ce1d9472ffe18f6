// Set packing on the GPU: per-sequence meta (length, first / last ACGT index) and the
// PREALIGNED bit-planes.  Replaces the per-call str -> native conversion the reference pays
// for every pair (distances.py:323-347, align.py:152).
#pragma once
#include "common.hpp"

namespace taxi2 {

// One wave per sequence: first / last ACGT index by ballot over 64-byte chunks.
__global__ void __launch_bounds__(256)
k_meta(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ offs, const int64_t* __restrict__ woffs,
       int64_t n, int4* __restrict__ meta) {
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (s >= n) return;
    const int64_t o = offs[s];
    const int len = (int)(offs[s + 1] - o);
    int first = len + 1, last = -1;
    for (int c0 = 0; c0 < len; c0 += 64) {
        const int c = c0 + lane;
        const bool nuc = c < len && base_code(bytes[o + c]) < 4;
        const unsigned long long bal = __ballot(nuc);
        if (bal) {
            if (first == len + 1) first = c0 + __builtin_ctzll(bal);
            last = c0 + 63 - __builtin_clzll(bal);
        }
    }
    if (lane == 0) meta[s] = make_int4(len, first, last, woffs ? (int)woffs[s] : 0);
}

// One workgroup per sequence, one thread per 32-column word.  The '-' plane keeps only the gaps
// inside the sequence's own [first, last ACGT] (k_meta runs first): a gap column counts only
// inside the pair's common range, and with both sides' gap bits pre-restricted (and valid bits
// inside their range by definition) the tiled kernel needs no per-pair mask.
__global__ void __launch_bounds__(256)
k_planes(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ offs,
         const int4* __restrict__ meta, int64_t n, uint4* __restrict__ planes) {
    const int64_t s = blockIdx.x;
    if (s >= n) return;
    const int4 m = meta[s];
    const int64_t o = offs[s];
    const int len = m.x;
    const int nw = (len + 31) / 32;
    for (int wd = threadIdx.x; wd < nw; wd += blockDim.x) {
        uint32_t lo = 0, hi = 0, nv = 0, gp = 0;
        const int c0 = wd * 32;
        for (int t = 0; t < 32; ++t) {
            const int c = c0 + t;
            if (c >= len) break;
            const unsigned ch = bytes[o + c];
            const int bc = base_code(ch);
            if (bc < 4) {
                nv |= 1u << t;
                lo |= (uint32_t)(bc & 1) << t;
                hi |= (uint32_t)(bc >> 1) << t;
            } else if (ch == '-' && c >= m.y && c <= m.z) {
                gp |= 1u << t;
            }
        }
        planes[m.w + wd] = make_uint4(lo, hi, nv, gp);
    }
}

// Row argmin for versusReference closest (versus_reference.py:184-188): first minimum over
// defined values of scale * d (the reference multiplies by 100 before min() when
// percentage_multiply is set, versus_reference.py:232); -1 when every value is undefined.
__global__ void __launch_bounds__(256)
k_row_argmin(const double* __restrict__ d, int64_t rows, int64_t R, double scale,
             int64_t* __restrict__ idx, double* __restrict__ best) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (q >= rows) return;
    const double* row = d + q * R;
    double bv = 0.0;
    int64_t bi = -1;
    for (int64_t r = lane; r < R; r += 64) {
        const double v = row[r] * scale;
        if (v == v && v != __builtin_inf() && v != -__builtin_inf()) {
            if (bi < 0 || v < bv) { bv = v; bi = r; }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(bv, off);
        const int64_t oi = __shfl_xor(bi, off);
        if (oi >= 0 && (bi < 0 || ov < bv || (ov == bv && oi < bi))) { bv = ov; bi = oi; }
    }
    if (lane == 0) {
        idx[q] = bi;
        best[q] = bi >= 0 ? row[bi] : __builtin_nan("");
    }
}

// TAXI2_METRIC_COUNTS slots -> metrics: out[k][m] = metric m of counts[k], times `scale` (the x100 of
// percentage_multiply, versus_all.py:554-562, one IEEE multiply like the reference's d * 100).
__global__ void __launch_bounds__(256) k_counts_metrics(const uint64_t* __restrict__ counts, int64_t n, MetricSpec ms,
                                                      double scale, double* __restrict__ out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t c = counts[k];
        const uint32_t valid = (uint32_t)(c & 0xFFFFu), ts = (uint32_t)((c >> 16) & 0xFFFFu);
        const uint32_t tv = (uint32_t)((c >> 32) & 0xFFFFu), gap = (uint32_t)(c >> 48);
        for (int m = 0; m < ms.n; ++m) {
            const double v = metric_value(ms.code[m], valid, ts, tv, gap);
            out[k * ms.n + m] = scale == 1.0 ? v : v * scale;
        }
    }
}

// A column view's meta: view[c] = meta[perm[c]] (taxi2_set_permuted; the plane offsets keep
// pointing into the parent's planes).
__global__ void __launch_bounds__(256) k_meta_gather(const int4* __restrict__ meta, const int64_t* __restrict__ perm,
                                                     int64_t n, int4* __restrict__ view) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n) view[c] = meta[perm[c]];
}

}  // namespace taxi2
