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

// f64 metric from the four column counters (itaxotools.calculate_distances semantics,
// restated in oracle/restatement.py metric_value).  Compiled with -ffp-contract=off so the
// operation sequence matches the C restatement exactly; NaN / inf = undefined (None).
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
            return -0.75 * log(1.0 - (4.0 / 3.0) * p);
        }
        case 3: {
            if (!valid) return __builtin_nan("");
            const double P = (double)ts / v;
            const double Q = (double)tv / v;
            return -0.5 * log(1.0 - 2.0 * P - Q) - 0.25 * log(1.0 - 2.0 * Q);
        }
        case METRIC_COUNTS:  // the counters themselves, 16 bits each (max_len <= 32767 checked by the host)
            return __longlong_as_double((long long)((uint64_t)valid | (uint64_t)ts << 16 | (uint64_t)tv << 32 |
                                                    (uint64_t)gap << 48));
        default:
            return __builtin_nan("");
    }
}

}  // namespace taxi2
