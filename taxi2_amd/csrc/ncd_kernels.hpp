// NCD on the GPU (TaxI2 distances.py:351-358 -> alfpy 1.0.6 ncd.Distance.pairwise_distance):
//   NCD(x, y) = (C(X + Y) - min(C(X), C(Y))) / max(C(X), C(Y)),  X = x.upper(), Y = y.upper(),
//   C(s) = len(zlib.compress(s))  (zlib 1.2.11, level 6; deflate_len.hpp).
// x, y are what VersusAll hands the metric: the Biopython aligned strings of the ordered pair in
// align mode (versus_all.py:532 -> :546), the raw sequences otherwise.
//
// One thread per compressed stream: the lazy-match parse is a serial chain walk per byte, so the
// work unit is the stream, not the byte.  Each thread owns a zeroed 64 KiB hash-head table and a
// window / prev / tree scratch slab in HBM (the head table is cleaned per stream, never re-zeroed);
// the 64 KiB window slides as zlib's does, so streams have no length limit.
#pragma once
#include "common.hpp"
#include "deflate_len.hpp"
#include "zlen_wave.hpp"

namespace taxi2 {

struct ZStream {
    const uint8_t* a;
    const uint8_t* b;
    int32_t na, nb;  // na < 0: a skipped stream (its length is ZLEN_SKIPPED)
};
constexpr int32_t ZLEN_SKIPPED = -2;

// Per-thread scratch slab after the head tables: [window][prev][Trees]
constexpr size_t ZS_WIN = ((size_t)zl::WIN_BYTES + 255) / 256 * 256;
constexpr size_t ZS_PREV = (size_t)zl::WSIZE * 2;
constexpr size_t ZS_TREES = (sizeof(zl::Trees) + 255) / 256 * 256;
constexpr size_t ZS_SLAB = ZS_WIN + ZS_PREV + ZS_TREES;
constexpr size_t ZS_HEAD = (size_t)zl::HASH_SIZE * 2;

__global__ void __launch_bounds__(64, 4)
k_zlen(const ZStream* __restrict__ st, int64_t n, uint16_t* __restrict__ heads, uint8_t* __restrict__ slabs,
       int32_t* __restrict__ out, int latin1, int redo, int first_only) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    uint8_t* slab = slabs + tid * ZS_SLAB;
    zl::Scratch z{slab, reinterpret_cast<uint16_t*>(slab + ZS_WIN), heads + tid * zl::HASH_SIZE};
    zl::Trees* t = reinterpret_cast<zl::Trees*>(slab + ZS_WIN + ZS_PREV);
    for (int64_t s = tid; s < n; s += nthreads) {
        if (redo && out[s] != -1) continue;  // a second pass: only the streams the first one declined
        const ZStream d = st[s];
        out[s] = d.na < 0 ? ZLEN_SKIPPED
                          : zl::compressed_len(d.a, d.na, d.b, first_only ? 0 : d.nb, z, *t, latin1 != 0);
    }
}

// One wave per stream, all state in LDS (zlen_wave.hpp): for launches whose streams are at most
// `nmax` bytes (dynamic LDS sized for nmax); a longer stream gets -1.  Persistent: each workgroup
// (one wave) takes streams blockIdx.x, + gridDim.x, ...  redo: a second pass with a larger nmax over
// the streams a first pass (sized for the likely lengths, more waves per CU) left at -1.
__global__ void __launch_bounds__(64)
k_zlen_wave(const ZStream* __restrict__ st, int64_t n, int nmax, int32_t* __restrict__ out, int redo) {
    extern __shared__ __attribute__((aligned(16))) uint8_t zsm[];
    const int lane = (int)threadIdx.x;
    for (int64_t s = blockIdx.x; s < n; s += gridDim.x) {
        if (redo && out[s] != -1) continue;  // wave-uniform
        const ZStream d = st[s];
        if (d.na < 0) {  // skipped (wave-uniform: one wave per workgroup)
            if (lane == 0) out[s] = ZLEN_SKIPPED;
            continue;
        }
        const int r = d.na + d.nb <= nmax ? zlw::compressed_len_wave(d.a, d.na, d.b, d.nb, zsm, nmax, lane) : -1;
        if (lane == 0) out[s] = r;  // -1: longer than the launch promised (the host checks)
        __syncthreads();
    }
}

// The fused form (zlen_wave.hpp compressed_len_wave2): out[s] = C(a + b) and out_a[s] = C(a) of the
// same stream descriptor, one sort and a shared parse prefix.
__global__ void __launch_bounds__(64)
k_zlen_wave2(const ZStream* __restrict__ st, int64_t n, int nmax, int32_t* __restrict__ out, int32_t* __restrict__ out_a,
             int redo) {
    extern __shared__ __attribute__((aligned(16))) uint8_t zsm[];
    const int lane = (int)threadIdx.x;
    for (int64_t s = blockIdx.x; s < n; s += gridDim.x) {
        if (redo && out[s] != -1) continue;  // wave-uniform
        const ZStream d = st[s];
        int ca = -1, r = -1;
        if (d.na + d.nb <= nmax) r = zlw::compressed_len_wave2(d.a, d.na, d.b, d.nb, zsm, nmax, lane, &ca);
        if (lane == 0) {
            out[s] = r;  // -1: longer than the launch promised (a redo pass takes it)
            out_a[s] = ca;
        }
        __syncthreads();
    }
}

// Three streams per (pair, orientation): C(first), C(second), C(first + second).
// Orientation 0 = ordered pair (x, y); 1 = (y, x).  Aligned mode reads the traceback slots
// (ax / ay right-aligned in [0, nA + nB) of slot p*2 + o; orientation 1 holds (bx, by) in (x, y)
// column order, and the (y, x) metric sees (by, bx)).
__global__ void __launch_bounds__(256)
k_ncd_streams(SetView XS, SetView YS, const int64_t* __restrict__ xs, const int64_t* __restrict__ ys, int64_t n,
              int both, const uint8_t* __restrict__ ax, const uint8_t* __restrict__ ay,
              const int32_t* __restrict__ alen, int cap, ZStream* __restrict__ st) {
    const int no = both ? 2 : 1;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * no) return;
    const int64_t p = t / no;
    const int o = (int)(t % no);
    const int64_t a = xs[p], b = ys[p];
    const uint8_t *sx, *sy;
    int32_t lx, ly;
    if (ax != nullptr) {
        const int total = XS.meta[a].x + YS.meta[b].x;
        const int32_t len = alen[p * 2 + o];
        const int64_t off = (p * 2 + o) * (int64_t)cap + (total - len);
        sx = ax + off;
        sy = ay + off;
        lx = ly = len;
    } else {
        sx = XS.bytes + XS.offs[a];
        sy = YS.bytes + YS.offs[b];
        lx = XS.meta[a].x;
        ly = YS.meta[b].x;
    }
    const uint8_t* f = o ? sy : sx;
    const uint8_t* s = o ? sx : sy;
    const int32_t lf = o ? ly : lx, ls = o ? lx : ly;
    ZStream* d = st + t * 3;
    d[0] = ZStream{f, nullptr, lf, 0};
    d[1] = ZStream{s, nullptr, ls, 0};
    d[2] = ZStream{f, s, lf, ls};
}

__global__ void __launch_bounds__(256)
k_ncd_finish(const int32_t* __restrict__ c, int64_t m, double* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    const double c1 = c[t * 3], c2 = c[t * 3 + 1], c12 = c[t * 3 + 2];
    const double mn = c1 < c2 ? c1 : c2, mx = c1 < c2 ? c2 : c1;
    out[t] = (c12 - mn) / mx;
}

// Raw mode with per-sequence C(x): one stream per set member (C of the sequence alone) ...
__global__ void __launch_bounds__(256) k_seq_streams(SetView S, int64_t n, ZStream* __restrict__ st) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    st[t] = ZStream{S.bytes + S.offs[t], nullptr, S.meta[t].x, 0};
}

// ... and one concatenation stream per (pair, orientation): x+y for (x, y), y+x for (y, x).
__global__ void __launch_bounds__(256)
k_ncd_concat_streams(SetView XS, SetView YS, const int64_t* __restrict__ xs, const int64_t* __restrict__ ys,
                     int64_t n, int both, ZStream* __restrict__ st) {
    const int no = both ? 2 : 1;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * no) return;
    const int64_t p = t / no;
    const int o = (int)(t % no);
    const int64_t a = xs[p], b = ys[p];
    const uint8_t* sx = XS.bytes + XS.offs[a];
    const uint8_t* sy = YS.bytes + YS.offs[b];
    const int32_t lx = XS.meta[a].x, ly = YS.meta[b].x;
    st[t] = o ? ZStream{sy, sx, ly, lx} : ZStream{sx, sy, lx, ly};
}

__global__ void __launch_bounds__(256)
k_ncd_finish_cached(const int32_t* __restrict__ c12, const int32_t* __restrict__ cx, const int32_t* __restrict__ cy,
                    const int64_t* __restrict__ xs, const int64_t* __restrict__ ys, int64_t n, int both,
                    double* __restrict__ out) {
    const int no = both ? 2 : 1;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * no) return;
    const int64_t p = t / no;
    const double c1 = cx[xs[p]], c2 = cy[ys[p]], c = c12[t];
    const double mn = c1 < c2 ? c1 : c2, mx = c1 < c2 ? c2 : c1;
    out[t] = (c - mn) / mx;
}

// ---- NCD from the aligners' own string slots (one fill per pair for every metric) ------------
// versus_all.py:546-552 hands ONE alignment per ordered pair to every metric in the list, NCD
// included (distances.py:351-358).  The packed aligners' walkers write each alignment while they
// walk it (StrOut): slot s = p * nslot + o holds it right-aligned at byte end(p) = len(a) + len(b),
// slen[s] bytes.  Orientation 0 is the ordered pair (a, b): x = sx, y = sy.  Orientation 1 is
// Biopython's alignment of (b, a) written in (a, b) column order, so its metric sees x = sy, y = sx.
//
// Jobs per pair: fused[p][o] = (x_o, y_o), o < no, each giving C(x_o + y_o) and C(x_o) in one pass
// (k_zlen_wave2), and singles[p][2] = C(y0), C(x1) (x_o, y_o: the metric's first and second string of
// orientation o).  One wave per pair compares the two orientations' strings: when they are the same
// alignment (no Ix / Iy tie on the path, most pairs) x1 = y0 and y1 = x0, so C(y0) and C(x1) ARE the
// fused jobs' C(x1) and C(x0) and both singles are marked skipped (na = -1): two fused jobs per pair
// instead of six separate streams.
__device__ __forceinline__ void ncd_slot(const uint8_t* sx, const uint8_t* sy, const int32_t* slen, int64_t cap,
                                         int nslot, int o, int64_t p, int64_t end, const uint8_t*& x,
                                         const uint8_t*& y, int32_t& len) {
    const int64_t s = p * nslot + o;
    len = slen[s];
    const int64_t off = s * cap + (end - len);
    x = sx + off;
    y = sy + off;
}

__global__ void __launch_bounds__(256)
k_ncd_slot_streams(const uint8_t* __restrict__ sx, const uint8_t* __restrict__ sy, const int32_t* __restrict__ slen,
                   int64_t cap, int nslot, int no, const int64_t* __restrict__ d_end, SetView XS, SetView YS,
                   PairSrc ps, int64_t n, ZStream* __restrict__ fused, ZStream* __restrict__ singles) {
    const int lane = (int)(threadIdx.x & 63);
    const int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (p >= n) return;  // wave-uniform
    int64_t end;
    if (d_end != nullptr) {
        end = d_end[p];
    } else {
        int64_t a, b;
        decode_pair(ps, p, a, b);
        end = (int64_t)XS.meta[a].x + YS.meta[b].x;
    }
    const uint8_t *x0, *y0;
    int32_t l0;
    ncd_slot(sx, sy, slen, cap, nslot, 0, p, end, x0, y0, l0);
    if (no == 1) {
        if (lane == 0) {
            fused[p] = ZStream{x0, y0, l0, l0};
            singles[p * 2] = ZStream{y0, nullptr, l0, 0};
            singles[p * 2 + 1] = ZStream{y0, nullptr, -1, 0};
        }
        return;
    }
    const uint8_t *x1, *y1;
    int32_t l1;
    ncd_slot(sx, sy, slen, cap, nslot, 1, p, end, x1, y1, l1);
    bool diff = l1 != l0;
    if (!diff) {
        bool d = false;
        for (int i = lane; i < l0; i += 64) d |= (x0[i] != x1[i]) | (y0[i] != y1[i]);
        diff = __ballot(d) != 0;
    }
    if (lane == 0) {
        fused[p * 2] = ZStream{x0, y0, l0, l0};      // (a, b): x = a's string, y = b's
        fused[p * 2 + 1] = ZStream{y1, x1, l1, l1};  // (b, a): x = b's string (sy), y = a's (sx)
        singles[p * 2] = ZStream{y0, nullptr, diff ? l0 : -1, 0};
        singles[p * 2 + 1] = ZStream{x1, nullptr, diff ? l1 : -1, 0};
    }
}

// out[(p * no + o) * ostride + ocol] = NCD of orientation o from the fused jobs' C(x_o + y_o) (cab) and
// C(x_o) (ca) and C(y_o): the single's, or -- skipped: both orientations hold the same alignment -- the
// other orientation's fused C(x).
__global__ void __launch_bounds__(256)
k_ncd_slot_finish(const int32_t* __restrict__ cab, const int32_t* __restrict__ ca, const int32_t* __restrict__ cs,
                  int64_t n, int no, double* __restrict__ out, int64_t ostride, int ocol) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * no) return;
    const int64_t p = t / no;
    const int o = (int)(t - p * no);
    const int32_t c1 = ca[t];
    int32_t c2 = cs[p * 2 + o];
    if (c2 == ZLEN_SKIPPED) c2 = ca[p * no + (o ^ 1)];
    const double d1 = c1, d2 = c2, d12 = cab[t];
    const double mn = d1 < d2 ? d1 : d2, mx = d1 < d2 ? d2 : d1;
    out[t * ostride + ocol] = (d12 - mn) / mx;
}

// Raw-mode streams for taxi2_zlib_lengths: upper(x_a) (+ upper(y_b) when ys != nullptr).
__global__ void __launch_bounds__(256)
k_zlen_streams(SetView XS, SetView YS, const int64_t* __restrict__ xs, const int64_t* __restrict__ ys, int64_t n,
               ZStream* __restrict__ st) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int64_t a = xs[t];
    ZStream d{XS.bytes + XS.offs[a], nullptr, XS.meta[a].x, 0};
    if (ys != nullptr) {
        const int64_t b = ys[t];
        d.b = YS.bytes + YS.offs[b];
        d.nb = YS.meta[b].x;
    }
    st[t] = d;
}

}  // namespace taxi2
