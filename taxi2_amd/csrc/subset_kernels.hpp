// Subset aggregation on the GPU, exact and parallel (round 3): DistanceAggregator
// (versus_all.py:57-96) fed x-major by _aggregate_distances (:617-640).  Per key (subset x a,
// subset y b, metric k) the reference keeps a running `sum += v` over the key's values in x-major
// order, so the mean is a function of that order (floating-point addition is not associative).
// The round-2 kernel summed each key in one thread: with few subsets (a two-genus partition) a
// handful of threads did all N^2 additions.
//
// Exact parallel summation.  While the running sum s stays inside one binade [2^(E-1), 2^E), the
// representable values are the multiples of u = 2^(E-53), and for v >= 0 that keeps s + v inside
// the binade, fl(s + v) = s + R u with R = v / u rounded to the nearest integer -- INDEPENDENT of
// s, unless v / u lies exactly halfway (then the even neighbour of s + v wins, which depends on
// s).  So over a run of values with no tie, no negative value and no binade change, the
// sequential result is s + (sum of the R) u, and the R are exact integers (< 2^53) whose sum is
// the same in any order.  Per block of rows:
//   k_subset_cofs     chunk offsets: subset b's columns in chunks of SUB_CH (a 2-genus partition at
//                     N = 200 000 is 98 chunks per row instead of 2 waves per row)
//   k_subset_rows     one wave per (row x, chunk of column subset b): for each metric, R of every value of
//                     the row's key at SUB_J grids -- u, 2u, 4u, 8u with u from the key's sum at
//                     block start (binades e0 .. e0 + 3) -- the row's integer sums, count, first
//                     minimum, maximum, and flags (tie at each grid / negative / no grid: s = 0)
//   (few subsets, ns <= 4: k_subset_rows_nat reads each row in natural column order instead, one
//                     wave per (row, 2 048 consecutive columns), values routed to per-subset
//                     accumulators in registers: no gather)
//   k_subset_rowmerge one thread per (row x, b, metric): the row's chunk partials in column order
//                     (integer sums are exact in any order; the first minimum stays the first)
//   k_subset_combine  one thread per (row group a, b, metric): walks the block's rows of subset a
//                     in ascending x, adds the integer sums while S + sum <= 2^53 - 1 (the binade
//                     holds) and nothing is flagged, merges count / min / max (in row order, so the
//                     first minimum and the sign of a zero minimum are the sequential ones); at the
//                     first row it cannot take, it queues the key with that row
//   k_subset_fixup    one wave per queued key: that row in order, 64 values at a time (the integer
//                     step when the chunk qualifies, else 64 sequential f64 adds); each later row
//                     from its partial at the binade the sum has reached (e0 .. e0 + 3) when that
//                     partial qualifies, else again 64 values at a time
// Binade changes are rare (the sum of non-negative values doubles ~log2(N^2) times per key), and
// each costs one row walked value by value: the fixup's work no longer grows with the rows left in
// the block after the change (round 3: a 2-genus partition at N = 50 000 spent 84 % of its kernel
// time re-walking those rows).  None (non-finite)
// values are skipped as SimpleAggregator.add does (in the sums they add +0.0, an exact no-op:
// the running sum starts at +0.0 and never becomes -0.0).
#pragma once
#include "common.hpp"

namespace taxi2 {

constexpr int SUB_J = 4;  // grids per row partial: binades e0 .. e0 + SUB_J - 1
constexpr int SUB_NOE = -32768;  // no grid at block start (the key's sum was 0)
struct SubPart {            // one (block row, column subset b, metric k)
    double rsum[SUB_J];     // sum of R = rint(v / (2^j u)) over the row's values of the key (exact)
    double mn, mx;          // first minimum (from +inf), maximum (from 0.0)
    long long cnt;          // defined values
    uint32_t flags;         // SP_*: where the integer step does not reproduce the sequential sum
    int32_t mnp;            // the minimum's column (ties between chunks: the lower one is first)
};
// SP_TIE << j: some value lies exactly halfway between two multiples of 2^j u
enum : uint32_t { SP_NOGRID = 1, SP_NEG = 2, SP_TIE = 4 };
struct SubWork {  // a key the combine could not finish: its rows from grp_rows[r0] on
    int64_t key;
    int32_t g, r0;
    int32_t e0;   // binade of the key's sum at block start (the partials' grid), SUB_NOE: none
    int32_t pad;
};
constexpr double SUB_TOP = 9007199254740991.0;  // 2^53 - 1: largest integer multiple of u below 2^E
constexpr int SUB_MAX_ROWS = 8192;              // rows per k_subset_groups call (LDS sort)
constexpr int SUB_CH = 2048;                    // columns per k_subset_rows wave (a subset's chunk)
constexpr int SUB_FU = 8;                       // fixup: 64-value groups per iteration

// The grid of running sum s: true with s in [2^(e-1), 2^e) when s is a positive normal number.
__device__ __forceinline__ bool sub_grid(double s, int& e) {
    e = 0;
    if (!(s >= 2.2250738585072014e-308) || !(s <= 1.7976931348623157e308)) return false;
    (void)frexp(s, &e);
    return true;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__global__ void __launch_bounds__(256) k_subset_init(int64_t nk, double* __restrict__ sum, double* __restrict__ mn,
                                                     double* __restrict__ mx, int64_t* __restrict__ count) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nk; t += (int64_t)gridDim.x * blockDim.x) {
        sum[t] = 0.0;  // SimpleAggregator.__init__
        mn[t] = __builtin_inf();
        mx[t] = 0.0;
        count[t] = 0;
    }
}

// The block's rows grouped by subset: rows sorted by (code, row) (bitonic sort of 64-bit keys in
// LDS, nrows <= SUB_MAX_ROWS), groups [grp_start[g], grp_start[g + 1]) of equal code grp_code[g].
__global__ void __launch_bounds__(1024) k_subset_groups(const int32_t* __restrict__ row_code, int nrows,
                                                        int32_t* __restrict__ grp_rows, int32_t* __restrict__ grp_code,
                                                        int32_t* __restrict__ grp_start, int32_t* __restrict__ ngrp) {
    __shared__ unsigned long long keys[SUB_MAX_ROWS];
    if (nrows <= (int)blockDim.x) {
        // few rows (a config-5 block holds ~450): each row's rank among the (code, row) keys by
        // counting, one pass and two barriers instead of the sort's log^2 barrier stages
        __shared__ uint32_t rc[1024];
        if ((int)threadIdx.x < nrows) rc[threadIdx.x] = (uint32_t)row_code[threadIdx.x];
        for (int i = threadIdx.x; i < SUB_MAX_ROWS; i += blockDim.x) keys[i] = ~0ull;
        __syncthreads();
        if ((int)threadIdx.x < nrows) {
            const uint32_t c = rc[threadIdx.x];
            int rank = 0;
            for (int j = 0; j < nrows; ++j) rank += rc[j] < c || (rc[j] == c && j < (int)threadIdx.x);
            keys[rank] = ((unsigned long long)c << 32) | (uint32_t)threadIdx.x;
        }
        __syncthreads();
    } else {
        int P = 1;
        while (P < nrows) P <<= 1;
        for (int i = threadIdx.x; i < P; i += blockDim.x)
            keys[i] = i < nrows ? ((unsigned long long)(uint32_t)row_code[i] << 32) | (uint32_t)i : ~0ull;
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = threadIdx.x; i < P; i += blockDim.x) {
                    const int l = i ^ j;
                    if (l > i) {
                        const unsigned long long a = keys[i], b = keys[l];
                        if (((i & k) == 0) == (a > b)) {
                            keys[i] = b;
                            keys[l] = a;
                        }
                    }
                }
                __syncthreads();
            }
    }
    // group index of a boundary = boundaries before it: each thread counts its SUB_MAX_ROWS / 1024
    // consecutive positions, then a scan over the threads' counts (Hillis-Steele in LDS)
    __shared__ int part[1024];
    constexpr int PER = SUB_MAX_ROWS / 1024;
    const int t = threadIdx.x;
    auto boundary = [&](int i) { return i < nrows && (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32)); };
    int cnt = 0;
    for (int q = 0; q < PER; ++q) cnt += boundary(t * PER + q);
    part[t] = cnt;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int g = part[t] - cnt;  // boundaries before this thread's first position
    for (int q = 0; q < PER; ++q) {
        const int i = t * PER + q;
        if (i < nrows) grp_rows[i] = (int32_t)(uint32_t)keys[i];
        if (boundary(i)) {
            grp_code[g] = (int32_t)(keys[i] >> 32);
            grp_start[g] = i;
            ++g;
        }
    }
    if (t == 1023) {
        grp_start[part[1023]] = nrows;
        *ngrp = part[1023];
    }
}

// cofs[b] = chunks of the subsets before b (subset b: max(1, ceil(size / SUB_CH)) chunks), cofs[ns]
// = chunks per row.  One workgroup of 1024 threads: per-thread runs of subsets, then a scan.
__global__ void __launch_bounds__(1024) k_subset_cofs(const int64_t* __restrict__ col_start, int ns,
                                                      int32_t* __restrict__ cofs) {
    __shared__ int part[1024];
    const int t = threadIdx.x;
    const int per = (ns + 1023) / 1024;
    const int b0 = min(ns, t * per), b1 = min(ns, b0 + per);
    auto nch = [&](int b) {
        const int64_t sz = col_start[b + 1] - col_start[b];
        return sz <= SUB_CH ? 1 : (int)((sz + SUB_CH - 1) / SUB_CH);
    };
    int cnt = 0;
    for (int b = b0; b < b1; ++b) cnt += nch(b);
    part[t] = cnt;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - cnt;
    for (int b = b0; b < b1; ++b) {
        cofs[b] = run;
        run += nch(b);
    }
    if (t == 1023) cofs[ns] = part[1023];
}

// Running partial of one (row, subset, metric) inside a wave's lanes.
struct SubAcc {
    double rs[SUB_J], mn, mx;
    long long c, mnp;
    uint32_t fl;
    int sc;
    bool grid;
    __device__ __forceinline__ void init(double key_sum) {
        int e = 0;
        grid = sub_grid(key_sum, e);
        sc = 53 - e;
#pragma unroll
        for (int q = 0; q < SUB_J; ++q) rs[q] = 0.0;
        mn = __builtin_inf();
        mx = 0.0;
        c = 0;
        mnp = 0x7FFFFFFFFFFFFFFFll;
        fl = grid ? 0u : SP_NOGRID;
    }
    __device__ __forceinline__ void add(double v, int64_t j) {
        if (!isfinite(v)) return;
        ++c;
        if (v < mn) {
            mn = v;
            mnp = j;
        }
        if (v > mx) mx = v;
        if (grid) {
            if (v < 0.0) fl |= SP_NEG;
#pragma unroll
            for (int q = 0; q < SUB_J; ++q) {
                const double r = ldexp(v, sc - q);
                const double R = rint(r);
                if (fabs(r - R) == 0.5) fl |= (uint32_t)SP_TIE << q;
                rs[q] += R;
            }
        }
    }
    // the wave's lanes merged; lane 0 holds the partial
    __device__ __forceinline__ SubPart reduce() {
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int q = 0; q < SUB_J; ++q) rs[q] += __shfl_xor(rs[q], o);
            c += __shfl_xor(c, o);
            fl |= (uint32_t)__shfl_xor((int)fl, o);
            const double omx = __shfl_xor(mx, o);
            if (omx > mx) mx = omx;
            const double omn = __shfl_xor(mn, o);
            const long long omp = __shfl_xor(mnp, o);
            if (omn < mn || (omn == mn && omp < mnp)) {  // the first position among equal minima
                mn = omn;
                mnp = omp;
            }
        }
        SubPart P;
#pragma unroll
        for (int q = 0; q < SUB_J; ++q) P.rsum[q] = rs[q];
        P.mn = mn;
        P.mx = mx;
        P.cnt = c;
        P.flags = fl;
        P.mnp = (int32_t)min(mnp, (long long)INT32_MAX);
        return P;
    }
};

// chunk t -> its subset b (cofs[b] <= t < cofs[b + 1]), -1 past the last chunk: one load per wave
// in k_subset_rows instead of a binary search of dependent loads.
__global__ void __launch_bounds__(256) k_subset_t2b(const int32_t* __restrict__ cofs, int ns, int tmax,
                                                    int32_t* __restrict__ t2b) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < tmax && i >= cofs[ns]) t2b[i] = -1;  // (every chunk below cofs[ns] has its subset)
    if (i < ns)
        for (int t = cofs[i]; t < cofs[i + 1]; ++t) t2b[t] = (int32_t)i;
}

// One wave per (block row x, chunk t of the row's chunks; tmax >= cofs[ns] bounds the grid), every
// metric: up to SUB_MG metrics per pass over the chunk, each column's values read together (one
// gather of m consecutive values per column instead of one per metric).  Chunk t belongs to subset
// b = t2b[t].
constexpr int SUB_MG = 4;
__global__ void __launch_bounds__(256) k_subset_rows(const double* __restrict__ vals, int64_t nrows, int64_t ncols,
                                                     int m, const int32_t* __restrict__ row_code,
                                                     const int64_t* __restrict__ col_start,
                                                     const int32_t* __restrict__ col_idx, int ns,
                                                     const int32_t* __restrict__ cofs, int tmax,
                                                     const double* __restrict__ sum, SubPart* __restrict__ part,
                                                     const int32_t* __restrict__ t2b) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= nrows * tmax) return;
    const int64_t x = w / tmax;
    const int t = (int)(w - x * tmax);
    const int b = t2b[t];
    if (b < 0) return;
    const int a = row_code[x];
    const int64_t j0 = col_start[b] + (int64_t)(t - cofs[b]) * SUB_CH;
    const int64_t j1 = min(col_start[b + 1], j0 + SUB_CH);
    const double* row = vals + x * ncols * m;
    for (int k0 = 0; k0 < m; k0 += SUB_MG) {
        const int g = min(SUB_MG, m - k0);
        SubAcc acc[SUB_MG];
#pragma unroll
        for (int q = 0; q < SUB_MG; ++q)
            if (q < g) acc[q].init(sum[((int64_t)a * ns + b) * m + k0 + q]);
        for (int64_t j = j0 + lane; j < j1; j += 64) {
            const double* vp = row + (int64_t)col_idx[j] * m + k0;
#pragma unroll
            for (int q = 0; q < SUB_MG; ++q)
                if (q < g) acc[q].add(vp[q], j);
        }
#pragma unroll
        for (int q = 0; q < SUB_MG; ++q) {
            if (q >= g) break;
            const SubPart P = acc[q].reduce();
            if (lane == 0) part[(x * tmax + t) * m + k0 + q] = P;
        }
    }
}

// cofs[b] = b * nch (k_subset_rows_nat's chunk slots: ns subsets x nch chunks per row).
__global__ void k_subset_natcofs(int ns, int nch, int32_t* __restrict__ cofs) {
    for (int b = threadIdx.x; b <= ns; b += blockDim.x) cofs[b] = b * nch;
}

// Column codes from the sorted layout: code[col_idx[j]] = b for j in [col_start[b], col_start[b+1]).
__global__ void __launch_bounds__(256) k_subset_colcode(const int64_t* __restrict__ col_start,
                                                        const int32_t* __restrict__ col_idx, int ns, int64_t ncols,
                                                        uint8_t* __restrict__ code) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= ncols) return;
    int lo = 0, hi = ns;  // the last b with col_start[b] <= j
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (col_start[mid] <= j) lo = mid;
        else hi = mid;
    }
    code[col_idx[j]] = (uint8_t)lo;
}

// Few subsets (ns <= NSB): one wave per (block row x, chunk of SUB_CH CONSECUTIVE columns), the
// row read in natural order (coalesced, no gather) and every value routed to its subset's
// accumulators in registers; the partial of (x, chunk c, subset b) goes to slot b * nch + c, so
// k_subset_rowmerge (cofs[b] = b * nch) merges each subset's chunks in column order.  Same
// partial contents as k_subset_rows: the subset's values of the chunk in ascending column order.
template <int NSB>
__global__ void __launch_bounds__(256) k_subset_rows_nat(const double* __restrict__ vals, int64_t nrows,
                                                         int64_t ncols, int m, const int32_t* __restrict__ row_code,
                                                         const uint8_t* __restrict__ col_code, int ns, int nch,
                                                         const double* __restrict__ sum, SubPart* __restrict__ part,
                                                         const int64_t* __restrict__ nat) {
    constexpr int MG = NSB <= 2 ? 2 : 1;  // metrics per pass (NSB x MG accumulators in registers)
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= nrows * nch) return;
    const int64_t x = w / nch;
    const int c = (int)(w - x * nch);
    const int a = row_code[x];
    const int64_t j0 = (int64_t)c * SUB_CH, j1 = min(ncols, j0 + SUB_CH);
    const double* row = vals + x * ncols * m;
    const int tmax = ns * nch;
    for (int k0 = 0; k0 < m; k0 += MG) {
        const int g = min(MG, m - k0);
        SubAcc acc[NSB][MG];
#pragma unroll
        for (int b = 0; b < NSB; ++b)
#pragma unroll
            for (int q = 0; q < MG; ++q)
                acc[b][q].init(b < ns && q < g ? sum[((int64_t)a * ns + b) * m + k0 + q] : 0.0);
        for (int64_t j = j0 + lane; j < j1; j += 64) {
            const double* vp = row + j * m + k0;
            const int cb = col_code[j];
            const int64_t jn = nat ? nat[j] : j;  // the task's column of stored column j
#pragma unroll
            for (int q = 0; q < MG; ++q) {
                if (q >= g) break;
                const double v = vp[q];
#pragma unroll
                for (int b = 0; b < NSB; ++b)
                    if (cb == b) acc[b][q].add(v, jn);
            }
        }
#pragma unroll
        for (int b = 0; b < NSB; ++b) {
            if (b >= ns) break;
#pragma unroll
            for (int q = 0; q < MG; ++q) {
                if (q >= g) break;
                const SubPart P = acc[b][q].reduce();
                if (lane == 0) part[(x * tmax + (int64_t)b * nch + c) * m + k0 + q] = P;
            }
        }
    }
}

// One thread per (block row x, subset b, metric k): the row's chunk partials merged in column order.
__global__ void __launch_bounds__(256) k_subset_rowmerge(int64_t nrows, int ns, int m, const int32_t* __restrict__ cofs,
                                                         int tmax, const SubPart* __restrict__ cpart,
                                                         SubPart* __restrict__ part) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= nrows * ns * m) return;
    const int k = (int)(i % m);
    const int64_t xb = i / m;
    const int b = (int)(xb % ns);
    const int64_t x = xb / ns;
    SubPart R = cpart[(x * tmax + cofs[b]) * m + k];
    for (int t = cofs[b] + 1; t < cofs[b + 1]; ++t) {
        const SubPart& P = cpart[(x * tmax + t) * m + k];
        for (int q = 0; q < SUB_J; ++q) R.rsum[q] += P.rsum[q];  // integers: exact in any order
        if (P.mn < R.mn || (P.mn == R.mn && P.mnp < R.mnp)) {  // ties: the lower column (-0.0 vs 0.0)
            R.mn = P.mn;
            R.mnp = P.mnp;
        }
        if (P.mx > R.mx) R.mx = P.mx;
        R.cnt += P.cnt;
        R.flags |= P.flags;
    }
    part[i] = R;
}

// One thread per (row group g, column subset b, metric k).
__global__ void __launch_bounds__(256) k_subset_combine(int64_t maxg, int ns, int m, const int32_t* __restrict__ ngrp,
                                                        const int32_t* __restrict__ grp_code,
                                                        const int32_t* __restrict__ grp_start,
                                                        const int32_t* __restrict__ grp_rows,
                                                        const SubPart* __restrict__ part, double* __restrict__ sum,
                                                        double* __restrict__ mn, double* __restrict__ mx,
                                                        int64_t* __restrict__ count, SubWork* __restrict__ work,
                                                        unsigned int* __restrict__ wcount) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= maxg * ns * m) return;
    const int g = (int)(t / ((int64_t)ns * m));
    if (g >= *ngrp) return;
    const int b = (int)((t / m) % ns);
    const int k = (int)(t % m);
    const int64_t key = ((int64_t)grp_code[g] * ns + b) * m + k;
    double s = sum[key], lo = mn[key], hi = mx[key];
    long long c = count[key];
    int e;
    const bool grid = sub_grid(s, e);
    double S = grid ? ldexp(s, 53 - e) : 0.0;
    int resume = -1;
    for (int r = grp_start[g]; r < grp_start[g + 1]; ++r) {
        const SubPart P = part[((int64_t)grp_rows[r] * ns + b) * m + k];
        c += P.cnt;
        if (P.mn < lo) lo = P.mn;
        if (P.mx > hi) hi = P.mx;
        if (resume < 0) {
            if (grid && (P.flags & (SP_NOGRID | SP_NEG | SP_TIE)) == 0u && S + P.rsum[0] <= SUB_TOP) S += P.rsum[0];
            else resume = r;
        }
    }
    if (grid) s = ldexp(S, e - 53);
    sum[key] = s;
    mn[key] = lo;
    mx[key] = hi;
    count[key] = c;
    if (resume >= 0) work[atomicAdd(wcount, 1u)] = SubWork{key, g, resume, grid ? e : SUB_NOE, 0};
}

// Persistent waves over the queued keys: row r0 of the key value by value (64 at a time), then each
// later row from its partial at the grid of the binade the sum has reached, or value by value.
__global__ void __launch_bounds__(256) k_subset_fixup(const double* __restrict__ vals, int64_t ncols, int m, int ns,
                                                      const int64_t* __restrict__ col_start,
                                                      const int32_t* __restrict__ col_idx,
                                                      const int32_t* __restrict__ grp_start,
                                                      const int32_t* __restrict__ grp_rows,
                                                      const SubPart* __restrict__ part,
                                                      const SubWork* __restrict__ work,
                                                      const unsigned int* __restrict__ wcount,
                                                      double* __restrict__ sum) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t total = *wcount;
    for (int64_t q = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); q < total; q += nw) {
        const SubWork it = work[q];
        const int k = (int)(it.key % m);
        const int b = (int)((it.key / m) % ns);
        const int64_t j0 = col_start[b], j1 = col_start[b + 1];
        double s = sum[it.key];
        for (int r = it.r0; r < grp_start[it.g + 1]; ++r) {
            const int64_t x = grp_rows[r];
            int e;
            if (r > it.r0 && it.e0 != SUB_NOE && sub_grid(s, e) && e >= it.e0 && e < it.e0 + SUB_J) {
                const SubPart& P = part[(x * ns + b) * m + k];
                const int jq = e - it.e0;
                const double S = ldexp(s, 53 - e);
                if ((P.flags & (SP_NOGRID | SP_NEG | ((uint32_t)SP_TIE << jq))) == 0u && S + P.rsum[jq] <= SUB_TOP) {
                    s = ldexp(S + P.rsum[jq], e - 53);  // the whole row in the binade: exact
                    continue;
                }
            }
            const double* row = vals + x * ncols * m;
            // SUB_FU x 64 values per iteration (SUB_FU loads per lane in flight): one integer step
            // for all of them when they qualify, else 64 at a time, else one by one
            for (int64_t c0 = j0; c0 < j1; c0 += 64 * SUB_FU) {
                double v[SUB_FU];
#pragma unroll
                for (int u = 0; u < SUB_FU; ++u) {
                    const int64_t j = c0 + 64 * u + lane;
                    const double w = j < j1 ? row[(int64_t)col_idx[j] * m + k] : 0.0;
                    v[u] = isfinite(w) ? w : 0.0;  // None: skipped (+0.0 adds nothing)
                }
                if (sub_grid(s, e)) {
                    bool bad = false;
                    double tot = 0.0;
#pragma unroll
                    for (int u = 0; u < SUB_FU; ++u) {
                        const double rr = ldexp(v[u], 53 - e);
                        const double R = rint(rr);
                        bad |= v[u] < 0.0 || fabs(rr - R) == 0.5;
                        tot += R;  // integers < 2^53: exact
                    }
                    if (!__any(bad)) {
                        tot = wave_sum_f64(tot);
                        const double S = ldexp(s, 53 - e);
                        if (S + tot <= SUB_TOP) {
                            s = ldexp(S + tot, e - 53);
                            continue;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < SUB_FU; ++u) {
                    const int64_t cu = c0 + 64 * u;
                    if (cu >= j1) break;
                    if (sub_grid(s, e)) {  // the integer step, when these 64 qualify
                        const double rr = ldexp(v[u], 53 - e);
                        const double R = rint(rr);
                        const bool bad = v[u] < 0.0 || fabs(rr - R) == 0.5;
                        if (!__any(bad)) {
                            const double tot = wave_sum_f64(R);
                            const double S = ldexp(s, 53 - e);
                            if (S + tot <= SUB_TOP) {
                                s = ldexp(S + tot, e - 53);
                                continue;
                            }
                        }
                    }
                    const int n = (int)min((int64_t)64, j1 - cu);
                    for (int l = 0; l < n; ++l) s = s + __shfl(v[u], l);  // the reference's own additions
                }
            }
        }
        if (lane == 0) sum[it.key] = s;
    }
}

}  // namespace taxi2
