// Shared device-side definitions for the MI355X all-pairs distance engine (gfx950).
//
// Data layout in HBM (one "set" = one uploaded Sequences container):
//   bytes  : uint8  [total]      raw (ALIGN: normalized) sequence bytes, concatenated
//   offs   : int64  [n + 1]      byte offset of each sequence
//   meta   : int32  [n][4]       {len, first ACGT index, last ACGT index, plane word offset}
//   planes : uint4  [words]      PREALIGNED only: per 32 columns {base lo bit, base hi bit,
//                                 ACGT-valid bit, '-' bit}; sequence s owns words
//                                 [meta[s].w, meta[s].w + ceil(len/32))
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace taxi2 {

constexpr int NEG_INF = -(1 << 28);  // "minus infinity" for int DP; never the max of a cell

struct SetView {
    const uint8_t* bytes;
    const int64_t* offs;
    const int4* meta;    // x = len, y = first ACGT, z = last ACGT, w = plane word offset
    const uint4* planes; // PREALIGNED only
    int64_t n;
};

// Which pairs a launch covers.  The launch processes linear indices g = k0 + k for
// k in [0, count).
enum PairMode : int { PAIRS_TRI = 0, PAIRS_RECT = 1, PAIRS_LIST = 2 };

struct PairSrc {
    int mode;
    int64_t k0;
    int64_t count;
    int64_t N;  // TRI: set size
    int64_t R;  // RECT: reference count (g = q * R + r)
    const int64_t* la;  // LIST
    const int64_t* lb;
    // k_alignt2's second pass only: the launch covers the queued pairs sel[0 .. *dcount) (indices
    // into this source's own pairs, outputs at those indices)
    const int64_t* sel = nullptr;
    const unsigned long long* dcount = nullptr;
};

struct KScores {
    int ma, mi, io, ie, eo, ee;
};

constexpr int MAX_METRICS = 8;
// Pseudo-metric (TAXI2_METRIC_COUNTS): a launch writes the four column counters of each ordered pair
// packed into the 8 bytes of its f64 slot (valid | ts << 16 | tv << 32 | gap << 48); every metric
// is a function of them (metric_value), evaluated later by k_counts_metrics.
constexpr int METRIC_COUNTS = 16;
struct MetricSpec {
    int n;
    int code[MAX_METRICS];
};

// Row-major upper triangle of an N-set: row a holds pairs (a, b), b = a+1 .. N-1,
// S(a) = a*(2N-a-1)/2 pairs precede row a.
__device__ __forceinline__ int64_t tri_row_start(int64_t a, int64_t N) {
    return a * (2 * N - a - 1) / 2;
}

__device__ __forceinline__ void decode_pair(const PairSrc& ps, int64_t k, int64_t& a, int64_t& b) {
    const int64_t g = ps.k0 + k;
    if (ps.mode == PAIRS_TRI) {
        const double n2 = 2.0 * (double)ps.N - 1.0;
        const double disc = n2 * n2 - 8.0 * (double)g;
        int64_t r = (int64_t)((n2 - sqrt(disc > 0.0 ? disc : 0.0)) * 0.5);
        if (r < 0) r = 0;
        if (r > ps.N - 2) r = ps.N - 2;
        while (r > 0 && tri_row_start(r, ps.N) > g) --r;
        while (r + 1 <= ps.N - 2 && tri_row_start(r + 1, ps.N) <= g) ++r;
        a = r;
        b = r + 1 + (g - tri_row_start(r, ps.N));
    } else if (ps.mode == PAIRS_RECT) {
        a = g / ps.R;
        b = g - a * ps.R;
    } else {
        a = ps.la[g];
        b = ps.lb[g];
    }
}

// ACGT/acgt -> 0..3, anything else -> 4 (distances.py:319-348 counting alphabet; see
// oracle/restatement.py counts()).
__device__ __forceinline__ int base_code(unsigned c) {
    const unsigned u = c & 0xDFu;
    return u == 'A' ? 0 : u == 'C' ? 1 : u == 'G' ? 2 : u == 'T' ? 3 : 4;
}

// Natural log for the jc / k2p transforms: ~50 VALU (31 of them f64) instead of the ~98 (76 f64) of
// the library's f64 log (ocml), which dominated the pre-aligned tile kernel's epilogue (three logs
// per pair; an f64 op issues at a quarter of the f32 rate).  x = 2^e m,
// m in [sqrt(1/2), sqrt(2)); log m = 2 atanh(s) = 2 s + 2 s (s^2 / 3 + s^4 / 5 + ... + s^20 / 21),
// s = (m - 1) / (m + 1), |s| <= 0.1716 (the first omitted term is < 1e-19 relative); log x = e ln2_hi +
// (2 s + (2 s R + e ln2_lo)) with ln2 split so that e ln2_hi is exact.  Within a few ulp of a correctly
// rounded log (absolute error < 1e-15 on every argument the metrics form, which are >= ~1e-17): the
// 1e-12 bound north_star sets for jc / k2p against the reference's glibc log holds with a wide
// margin (tests/test_gpu_parity.py, tests/test_gpu_prealigned.py).  Special values as log's:
// log(1) = +0 (so -0.75 log(1) is -0.0, "-0.0000"), log(0) = -inf, log(x < 0) = log(NaN) = NaN.
__device__ __forceinline__ double metric_log(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -__builtin_inf() : __builtin_nan("");
    int e = __builtin_amdgcn_frexp_exp(x);
    double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
    if (m < 0.70710678118654752440) {
        m = m * 2.0;
        e -= 1;
    }
    // s = (m - 1) / (m + 1) from the hardware reciprocal, one Newton step and one residual
    // correction (a few ulp at most; the division's exact rounding is not needed here)
    const double d = m + 1.0, n1 = m - 1.0;
    double rc = __builtin_amdgcn_rcp(d);
    rc = fma(rc, fma(-d, rc, 1.0), rc);
    double s = n1 * rc;
    s = fma(rc, fma(-d, s, n1), s);
    const double t = s * s;
    double r = 1.0 / 21.0;
    r = fma(r, t, 1.0 / 19.0);
    r = fma(r, t, 1.0 / 17.0);
    r = fma(r, t, 1.0 / 15.0);
    r = fma(r, t, 1.0 / 13.0);
    r = fma(r, t, 1.0 / 11.0);
    r = fma(r, t, 1.0 / 9.0);
    r = fma(r, t, 1.0 / 7.0);
    r = fma(r, t, 1.0 / 5.0);
    r = fma(r, t, 1.0 / 3.0);
    const double s2 = 2.0 * s;
    const double de = (double)e;
    constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    return fma(de, LN2_HI, s2 + fma(s2 * t, r, de * LN2_LO));
}

// f64 metric from the four column counters (itaxotools.calculate_distances semantics,
// restated in oracle/restatement.py metric_value).  Compiled with -ffp-contract=off so the
// operation sequence matches the C restatement exactly (p / p-gaps bit for bit; jc / k2p through
// metric_log); NaN / inf = undefined (None).
__device__ __forceinline__ double metric_value(int code, uint32_t valid, uint32_t ts, uint32_t tv,
                                               uint32_t gap) {
    const double v = (double)valid;
    const double mism = (double)(ts + tv);
    switch (code) {
        case 0:
            return valid ? mism / v : __builtin_nan("");
        case 1:
            return (valid + gap) ? (mism + (double)gap) / (v + (double)gap) : __builtin_nan("");
        case 2: {
            if (!valid) return __builtin_nan("");
            const double p = mism / v;
            return -0.75 * metric_log(1.0 - (4.0 / 3.0) * p);
        }
        case 3: {
            if (!valid) return __builtin_nan("");
            const double P = (double)ts / v;
            const double Q = (double)tv / v;
            return -0.5 * metric_log(1.0 - 2.0 * P - Q) - 0.25 * metric_log(1.0 - 2.0 * Q);
        }
        case METRIC_COUNTS:  // the counters themselves, 16 bits each (max_len <= 32767 checked by the host)
            return __longlong_as_double((long long)((uint64_t)valid | (uint64_t)ts << 16 | (uint64_t)tv << 32 |
                                                    (uint64_t)gap << 48));
        default:
            return __builtin_nan("");
    }
}

// metric_value with the pair's p-distance (mism / valid, NaN without valid columns) already formed:
// the p and jc metrics share its division (the pre-aligned tile kernel's epilogue evaluates every
// requested metric of 16 pairs per thread).  Same values as metric_value, bit for bit.
__device__ __forceinline__ double metric_value_p(int code, uint32_t valid, uint32_t ts, uint32_t tv, uint32_t gap,
                                                 double p) {
    if (code == 0) return p;
    if (code == 2) return valid ? -0.75 * metric_log(1.0 - (4.0 / 3.0) * p) : __builtin_nan("");
    return metric_value(code, valid, ts, tv, gap);
}

}  // namespace taxi2
