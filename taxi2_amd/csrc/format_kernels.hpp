// Text for the distance writers (TaxI2 distances.py:59-279 DistanceHandler.Linear / .WithExtras /
// .Matrix, fed by versus_all.py:564-603 and versus_reference.py:131-178): every value is
// formatter.format(d) with formatter "{:.Nf}" (params.format.float = "{:.4f}", handler default
// "{:f}" = 6 decimals), None -> params.format.missing.
//
// fmt_fixed reproduces Python's '%.Nf' exactly: the decimal rounding is decided on the exact binary
// value (m * 2^e * 10^N, 128-bit integer arithmetic), ties to even, sign kept for -0.0 and for
// negatives that round to zero ("-0.0000").  Valid for |x| * 10^N < 2^63 (the host checks).
//
// Layout of one chunk of rows: one workgroup per row, tokens = the row's columns; token lengths
// are block-scanned in LDS and each thread writes its token at the row base + its offset.
//   linear: token (r, c) = row_pre[r] '\t' col_pre[c] ('\t' value(r, c, m)){nm} '\n'
//   matrix: token (r, c) = [row_pre[r] if c == 0] '\t' value(r, c) ['\n' if c == ncols-1]
// Ragged rows (taxi2_format_ragged, Dereplicate's surviving pairs): row r's tokens are an explicit
// column list instead of every column.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace taxi2 {

constexpr int FMT_MAX_DECIMALS = 17;

__host__ __device__ __forceinline__ uint64_t pow10_u64(int n) {
    uint64_t p = 1;
    for (int i = 0; i < n; ++i) p *= 10u;
    return p;
}

// Python "%.{N}f" % x for finite x; writes to dst (nullable: length only); returns the length.
__host__ __device__ inline int fmt_fixed(double x, int N, char* dst) {
    uint64_t bits;
    __builtin_memcpy(&bits, &x, 8);
    const bool neg = (bits >> 63) != 0;
    const int bexp = (int)((bits >> 52) & 0x7FF);
    const uint64_t frac = bits & ((1ull << 52) - 1);
    const uint64_t m = bexp ? (frac | (1ull << 52)) : frac;
    const int e = bexp ? bexp - 1075 : -1074;
    const unsigned __int128 P = (unsigned __int128)m * pow10_u64(N);
    uint64_t q;
    if (e >= 0) {
        q = (uint64_t)(P << e);
    } else {
        const int s = -e;
        if (s >= 128) {
            q = 0;  // P < 2^110 < 2^(s-1): rounds to 0
        } else {
            q = (uint64_t)(P >> s);
            const unsigned __int128 rem = P & ((((unsigned __int128)1) << s) - 1);
            const unsigned __int128 half = ((unsigned __int128)1) << (s - 1);
            if (rem > half || (rem == half && (q & 1u))) ++q;
        }
    }
    const uint64_t p10 = pow10_u64(N);
    uint64_t ip = q / p10;
    const uint64_t fp = q - ip * p10;
    char tmp[24];
    int nd = 0;
    do {
        tmp[nd++] = (char)('0' + ip % 10u);
        ip /= 10u;
    } while (ip);
    const int len = (neg ? 1 : 0) + nd + (N > 0 ? 1 + N : 0);
    if (dst) {
        int o = 0;
        if (neg) dst[o++] = '-';
        while (nd) dst[o++] = tmp[--nd];
        if (N > 0) {
            dst[o++] = '.';
            uint64_t f = fp;
            for (int k = N - 1; k >= 0; --k) {
                dst[o + k] = (char)('0' + f % 10u);
                f /= 10u;
            }
        }
    }
    return len;
}

#ifdef __HIPCC__
struct FmtArgs {
    int mode;  // 0 linear, 1 matrix, 2 summary
    const double* vals;  // [nrows][ncols][nm], or [rstart[nrows]][nm] when ragged
    int64_t nrows, ncols;
    int nm, decimals;
    const uint8_t* row_pre;
    const int64_t* row_offs;  // [nrows + 1] relative to the chunk
    const uint8_t* col_pre;
    const int64_t* col_offs;  // [ncols + 1]
    const uint8_t* missing;
    int missing_len;
    // ragged rows (nullable): row r holds tokens g in [rstart[r], rstart[r+1]) (relative to the
    // chunk), column cols[g]; rectangular otherwise (token t of row r = column t)
    const int64_t* rstart;
    const int32_t* cols;
    // mode 2 (versusAll summary.tsv, versus_all.py:278-350 SummaryHandler): after the values, row
    // suffix 2r (x extras), column suffix 2c (y extras), row suffix 2r+1 (x genus, species),
    // column suffix 2c+1 (y genus, species), each carrying its own leading TABs, then TAB and the
    // comparison label chosen from the (genus, species) codes (equal code = same subset)
    const uint8_t* rsuf;
    const int64_t* rsuf_offs;  // [2 * nrows + 1]
    const uint8_t* csuf;
    const int64_t* csuf_offs;  // [2 * ncols + 1]
    const int32_t* rcode;  // [2 * nrows]: genus code, species code
    const int32_t* ccode;  // [2 * ncols]
    int has_g, has_s;
    const uint8_t* lab;
    const int64_t* lab_offs;  // [6]: no info, intra-species, inter-species, intra-genus, inter-genus
    int64_t vstride;  // doubles between consecutive value slots (nm for a packed block; more when the
                      // values are a column range of a wider device array)
    double vlim;      // |value| bound of exact fixed-point text: a row holding a larger finite value
                      // gets a length of 2^60 or more from k_fmt_row_len (the host then fails)
};

__device__ __forceinline__ bool fmt_defined(double v) { return __builtin_isfinite(v); }

// SubsetDistance.get_comparison_type (versus_all.py:255-271): (same genus?, same species?) with
// None when that partition is absent.
__device__ __forceinline__ int fmt_comparison(const FmtArgs& a, int64_t r, int64_t c) {
    const int sg = a.has_g ? (a.rcode[2 * r] == a.ccode[2 * c] ? 1 : 0) : -1;
    const int ss = a.has_s ? (a.rcode[2 * r + 1] == a.ccode[2 * c + 1] ? 1 : 0) : -1;
    if (sg == 0) return 4;
    if (ss == 1) return 1;
    if (ss == 0) return 2;
    return sg == 1 ? 3 : 0;
}

__device__ __forceinline__ int64_t fmt_span(const int64_t* offs, int64_t k) { return offs[k + 1] - offs[k]; }

__device__ __forceinline__ int64_t fmt_ntok(const FmtArgs& a, int64_t r) {
    return a.rstart ? a.rstart[r + 1] - a.rstart[r] : a.ncols;
}

// Token t of row r: its value slot g and column c.
__device__ __forceinline__ void fmt_token_at(const FmtArgs& a, int64_t r, int64_t t, int64_t& g, int64_t& c) {
    if (a.rstart) {
        g = a.rstart[r] + t;
        c = a.cols[g];
    } else {
        g = r * a.ncols + t;
        c = t;
    }
}

// A token holding a value too large for fixed-point text adds FMT_OVERSIZE to its length, once: a
// chunk's sum (<= FMT_BLOCK tokens) stays below 2^63 and at or above FMT_OVERSIZE, which the host
// reports as an error.  Real token lengths stay far below it.
constexpr int64_t FMT_OVERSIZE = (int64_t)1 << 40;

__device__ __forceinline__ int64_t fmt_token_len(const FmtArgs& a, int64_t r, int64_t t, int64_t nt) {
    int64_t g, c;
    fmt_token_at(a, r, t, g, c);
    const double* v = a.vals + g * a.vstride;
    int64_t len = 0;
    bool over = false;
    if (a.mode != 1) {
        len = (a.row_offs[r + 1] - a.row_offs[r]) + 1 + (a.col_offs[c + 1] - a.col_offs[c]) + 1;  // + '\n'
        for (int m = 0; m < a.nm; ++m) {
            len += 1 + (fmt_defined(v[m]) ? fmt_fixed(v[m], a.decimals, nullptr) : a.missing_len);
            if (fmt_defined(v[m]) && !(__builtin_fabs(v[m]) < a.vlim)) over = true;
        }
        if (a.mode == 2)
            len += fmt_span(a.rsuf_offs, 2 * r) + fmt_span(a.csuf_offs, 2 * c) + fmt_span(a.rsuf_offs, 2 * r + 1) +
                   fmt_span(a.csuf_offs, 2 * c + 1) + 1 + fmt_span(a.lab_offs, fmt_comparison(a, r, c));
    } else {
        if (t == 0) len += a.row_offs[r + 1] - a.row_offs[r];
        len += 1 + (fmt_defined(v[0]) ? fmt_fixed(v[0], a.decimals, nullptr) : a.missing_len);
        if (fmt_defined(v[0]) && !(__builtin_fabs(v[0]) < a.vlim)) over = true;
        if (t == nt - 1) len += 1;
    }
    return over ? len + FMT_OVERSIZE : len;
}

__device__ __forceinline__ void fmt_token_write(const FmtArgs& a, int64_t r, int64_t t, int64_t nt, char* o) {
    int64_t g, c;
    fmt_token_at(a, r, t, g, c);
    const double* v = a.vals + g * a.vstride;
    auto put = [&](const uint8_t* s, int64_t n) {
        for (int64_t k = 0; k < n; ++k) *o++ = (char)s[k];
    };
    auto value = [&](double x) {
        *o++ = '\t';
        if (fmt_defined(x)) o += fmt_fixed(x, a.decimals, o);
        else put(a.missing, a.missing_len);
    };
    if (a.mode != 1) {
        put(a.row_pre + a.row_offs[r], a.row_offs[r + 1] - a.row_offs[r]);
        *o++ = '\t';
        put(a.col_pre + a.col_offs[c], a.col_offs[c + 1] - a.col_offs[c]);
        for (int m = 0; m < a.nm; ++m) value(v[m]);
        if (a.mode == 2) {
            put(a.rsuf + a.rsuf_offs[2 * r], fmt_span(a.rsuf_offs, 2 * r));
            put(a.csuf + a.csuf_offs[2 * c], fmt_span(a.csuf_offs, 2 * c));
            put(a.rsuf + a.rsuf_offs[2 * r + 1], fmt_span(a.rsuf_offs, 2 * r + 1));
            put(a.csuf + a.csuf_offs[2 * c + 1], fmt_span(a.csuf_offs, 2 * c + 1));
            *o++ = '\t';
            const int k = fmt_comparison(a, r, c);
            put(a.lab + a.lab_offs[k], fmt_span(a.lab_offs, k));
        }
        *o++ = '\n';
    } else {
        if (t == 0) put(a.row_pre + a.row_offs[r], a.row_offs[r + 1] - a.row_offs[r]);
        value(v[0]);
        if (t == nt - 1) *o++ = '\n';
    }
}

constexpr int FMT_BLOCK = 256;

// The work unit of both passes is a chunk: FMT_BLOCK consecutive tokens of one row (block b = row
// b / nch, chunk b % nch), so that a launch has rows x nch workgroups -- one workgroup per row left
// most of the chip idle on the few-hundred-row blocks of the dense task.
// Pass 1: text length of each chunk.
__global__ void __launch_bounds__(FMT_BLOCK) k_fmt_row_len(FmtArgs a, int nch, int64_t* __restrict__ chunk_len) {
    __shared__ int64_t red[FMT_BLOCK];
    const int64_t r = blockIdx.x / nch;
    const int64_t t = (int64_t)(blockIdx.x - r * nch) * FMT_BLOCK + threadIdx.x;
    const int64_t nt = fmt_ntok(a, r);
    red[threadIdx.x] = t < nt ? fmt_token_len(a, r, t, nt) : 0;
    __syncthreads();
    for (int w = FMT_BLOCK / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) chunk_len[blockIdx.x] = red[0];
}

constexpr int FMT_STAGE = 16384;  // LDS bytes a chunk's text is assembled in before it goes out

// Pass 2: write; chunk_base[b] = byte offset of chunk b in `out`.  Each thread renders its token
// (a few to a few dozen bytes) into LDS; the workgroup then stores the chunk with 16-byte stores
// from its first 16-aligned byte on -- the text goes to pinned host memory over the link, where a
// byte store per thread per character wasted most of the bandwidth.  A chunk longer than the
// stage (very long ids or suffixes) is written token by token.
__global__ void __launch_bounds__(FMT_BLOCK)
k_fmt_rows(FmtArgs a, int nch, const int64_t* __restrict__ chunk_base, char* __restrict__ out) {
    __shared__ int64_t scan[FMT_BLOCK];
    __shared__ __attribute__((aligned(16))) char stage[FMT_STAGE + 16];
    const int64_t r = blockIdx.x / nch;
    const int64_t t = (int64_t)(blockIdx.x - r * nch) * FMT_BLOCK + threadIdx.x;
    const int64_t nt = fmt_ntok(a, r);
    const int64_t len = t < nt ? fmt_token_len(a, r, t, nt) : 0;
    scan[threadIdx.x] = len;
    __syncthreads();
    for (int w = 1; w < FMT_BLOCK; w <<= 1) {  // inclusive Hillis-Steele scan
        const int64_t add = threadIdx.x >= w ? scan[threadIdx.x - w] : 0;
        __syncthreads();
        scan[threadIdx.x] += add;
        __syncthreads();
    }
    const int64_t b0 = chunk_base[blockIdx.x];
    const int64_t total = scan[FMT_BLOCK - 1];
    if (total > FMT_STAGE) {
        if (t < nt) fmt_token_write(a, r, t, nt, out + b0 + scan[threadIdx.x] - len);
        return;
    }
    // stage byte k + sh holds output byte b0 + k: 16-byte output words are 16-byte stage words
    const int sh = (int)(b0 & 15);
    if (t < nt) fmt_token_write(a, r, t, nt, stage + sh + scan[threadIdx.x] - len);
    __syncthreads();
    const int tot = (int)total;
    const int h = min(tot, (16 - sh) & 15);  // bytes before the first 16-aligned output byte
    const int nw = (tot - h) >> 4;
    if ((int)threadIdx.x < h) out[b0 + threadIdx.x] = stage[sh + threadIdx.x];
    const uint4* sw = reinterpret_cast<const uint4*>(stage + sh + h);
    uint4* ow = reinterpret_cast<uint4*>(out + b0 + h);
    for (int w = threadIdx.x; w < nw; w += FMT_BLOCK) ow[w] = sw[w];
    const int tb = h + 16 * nw;
    if (tb + (int)threadIdx.x < tot) out[b0 + tb + threadIdx.x] = stage[sh + tb + threadIdx.x];
}

// ---- aligned_pairs.txt (pairs.py:51-97 SequencePairHandler.Formatted, fed x-major by
// versus_all.py:746-750): per ordered pair
//   idx " / " idy LF  X LF  pattern LF  Y LF
// blocks separated by one LF (none before the file's first pair); pattern[c] = '|' for equal
// non-gap bytes, '-' when either side is a gap, '.' otherwise (Formatted._format_char).  The
// aligned strings come from the packed aligner's walkers (alignt2_kernel.hpp StrOut, one slot per
// pair): right-aligned, the alignment of (x, y) ends at byte len(x) + len(y) of its slot.
struct PairFmtArgs {
    const uint8_t* sx;
    const uint8_t* sy;
    const int32_t* slen;
    int64_t cap;
    const int4* qmeta;  // lengths of the row set, from q0
    const int4* rmeta;  // lengths of the column set
    int64_t ncols;
    const uint8_t* rid;  // ids: concatenated bytes + offsets (row ids start at row q0)
    const int64_t* roffs;
    const uint8_t* cid;
    const int64_t* coffs;
    int first;  // 1: the block's pair (0, 0) opens the file (no separator before it)
    // pointer mode (px != nullptr): pair k's aligned strings start at px[k] / py[k] (slen[k] bytes
    // each) instead of right-aligned slots -- strings kept from another block's fill
    const uint64_t* px = nullptr;
    const uint64_t* py = nullptr;
};

__device__ __forceinline__ int64_t pair_fmt_len(const PairFmtArgs& a, int64_t r, int64_t c) {
    const int64_t L = a.slen[r * a.ncols + c];
    const int64_t lx = a.roffs[r + 1] - a.roffs[r], ly = a.coffs[c + 1] - a.coffs[c];
    return ((r | c) || !a.first ? 1 : 0) + lx + 3 + ly + 1 + 3 * (L + 1);
}

// Pass 1: text length of each chunk of pairs (FMT_BLOCK columns of one row, as k_fmt_row_len).
__global__ void __launch_bounds__(FMT_BLOCK) k_pairs_row_len(PairFmtArgs a, int nch, int64_t* __restrict__ chunk_len) {
    __shared__ int64_t red[FMT_BLOCK];
    const int64_t r = blockIdx.x / nch;
    const int64_t c = (int64_t)(blockIdx.x - r * nch) * FMT_BLOCK + threadIdx.x;
    red[threadIdx.x] = c < a.ncols ? pair_fmt_len(a, r, c) : 0;
    __syncthreads();
    for (int w = FMT_BLOCK / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) chunk_len[blockIdx.x] = red[0];
}

// Asynchronous form: exclusive prefix of the row lengths on the device (one workgroup; rows in
// chunks of FMT_BLOCK), total in *total; cap_ok = total <= cap (else k_pairs_text writes nothing).
__global__ void __launch_bounds__(FMT_BLOCK) k_pairs_row_base(const int64_t* __restrict__ row_len, int64_t nrows,
                                                              int64_t cap, int64_t* __restrict__ row_base,
                                                              int64_t* __restrict__ total) {
    __shared__ int64_t scan[FMT_BLOCK];
    int64_t run = 0;
    for (int64_t r0 = 0; r0 < nrows; r0 += FMT_BLOCK) {
        const int64_t r = r0 + threadIdx.x;
        const int64_t v = r < nrows ? row_len[r] : 0;
        scan[threadIdx.x] = v;
        __syncthreads();
        for (int w = 1; w < FMT_BLOCK; w <<= 1) {
            const int64_t add = threadIdx.x >= w ? scan[threadIdx.x - w] : 0;
            __syncthreads();
            scan[threadIdx.x] += add;
            __syncthreads();
        }
        if (r < nrows) row_base[r] = run + scan[threadIdx.x] - v;
        run += scan[FMT_BLOCK - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        total[0] = run;
        total[1] = run <= cap ? 1 : 0;
    }
}

// Pass 2: one workgroup per chunk (FMT_BLOCK columns of a row); the pair offsets by an LDS scan, then
// each wave writes whole pairs, its lanes striding over the pair's bytes (coalesced stores).
//
// A pair's two aligned strings are first staged in the wave's LDS (PT_STAGE bytes each): every lane
// issues its share of 4-byte loads of the strings' aligned windows at once and waits once.  Read
// byte by byte from global memory, as the text needs them, every byte was a load, a wait and a use
// in sequence (~80 waits per 16 output bytes of a lane): latency-bound, and with the chip shared
// with the next block's fill the text kernel ran at a fifth of the host link's rate.  Longer pairs
// (more than PT_STAGE aligned columns) read global memory directly.
constexpr int PT_STAGE = 2304;  // staged bytes per string and wave (aligned pairs of up to 2 300 columns)
constexpr int PT_WORDS = (PT_STAGE + 8) / 4;
constexpr int PT_LOADS = (PT_WORDS + 63) / 64;  // 4-byte loads per lane and string
constexpr int PT_HDR = 192;  // staged header bytes (separator, "idx / idy", LF) per wave

__global__ void __launch_bounds__(FMT_BLOCK)
k_pairs_text(PairFmtArgs a, int nch, const int64_t* __restrict__ chunk_base, char* __restrict__ out,
             const int64_t* __restrict__ cap_ok = nullptr) {
    __shared__ int64_t scan[FMT_BLOCK];
    __shared__ __attribute__((aligned(16))) uint32_t stg[FMT_BLOCK / 64][2][PT_WORDS];
    __shared__ uint8_t hdr[FMT_BLOCK / 64][PT_HDR];
    if (cap_ok && cap_ok[1] == 0) return;  // asynchronous form: the text would not fit the buffer
    const int64_t r = blockIdx.x / nch;
    const int64_t c0 = (int64_t)(blockIdx.x - r * nch) * FMT_BLOCK;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t base = chunk_base[blockIdx.x];
    const int lx = (int)(a.roffs[r + 1] - a.roffs[r]);
    const uint8_t* idx = a.rid + a.roffs[r];
    const int nx = a.px ? 0 : a.qmeta[r].x;
    const uint8_t* sxb = reinterpret_cast<const uint8_t*>(stg[wv][0]);
    const uint8_t* syb = reinterpret_cast<const uint8_t*>(stg[wv][1]);
    {
        const int64_t c = c0 + threadIdx.x;
        const int64_t len = c < a.ncols ? pair_fmt_len(a, r, c) : 0;
        scan[threadIdx.x] = len;
        __syncthreads();
        for (int w = 1; w < FMT_BLOCK; w <<= 1) {
            const int64_t add = threadIdx.x >= w ? scan[threadIdx.x - w] : 0;
            __syncthreads();
            scan[threadIdx.x] += add;
            __syncthreads();
        }
        const int nc = (int)min((int64_t)FMT_BLOCK, a.ncols - c0);
        for (int q = wv; q < nc; q += FMT_BLOCK / 64) {
            const int64_t cc = c0 + q;
            const int64_t k = r * a.ncols + cc;
            const int64_t plen = scan[q] - (q ? scan[q - 1] : 0);
            char* o = out + base + scan[q] - plen;
            const int sep = ((r | cc) || !a.first) ? 1 : 0;
            const int ly = (int)(a.coffs[cc + 1] - a.coffs[cc]);
            const uint8_t* idy = a.cid + a.coffs[cc];
            const int L = a.slen[k];
            const uint8_t *X, *Y;
            if (a.px) {
                X = (const uint8_t*)a.px[k];
                Y = (const uint8_t*)a.py[k];
            } else {
                const int64_t end = (int64_t)nx + a.rmeta[cc].x;
                X = a.sx + k * a.cap + end - L;
                Y = a.sy + k * a.cap + end - L;
            }
            // the strings' aligned 4-byte windows into the wave's stage (wave-uniform branch)
            const int xo = (int)((uintptr_t)X & 3u), yo = (int)((uintptr_t)Y & 3u);
            const int h = sep + lx + 3 + ly + 1;  // header with its separator
            auto hdr_at = [&](int t) -> uint32_t {
                const int u = t - sep;
                return u < 0 ? '\n' : u < lx ? idx[u] : u < lx + 3 ? (uint32_t)" / "[u - lx] : u < lx + 3 + ly ? idy[u - lx - 3] : '\n';
            };
            const bool staged = L <= PT_STAGE && h <= PT_HDR;
            if (staged) {
                const uint32_t* xw = reinterpret_cast<const uint32_t*>(X - xo);
                const uint32_t* yw = reinterpret_cast<const uint32_t*>(Y - yo);
                const int nwx = (xo + L + 3) >> 2, nwy = (yo + L + 3) >> 2;
                uint32_t rx[PT_LOADS], ry[PT_LOADS];
#pragma unroll
                for (int i = 0; i < PT_LOADS; ++i) {
                    const int w = lane + 64 * i;
                    rx[i] = w < nwx ? xw[w] : 0u;
                    ry[i] = w < nwy ? yw[w] : 0u;
                }
                uint32_t hb[PT_HDR / 64];
#pragma unroll
                for (int i = 0; i < PT_HDR / 64; ++i) hb[i] = lane + 64 * i < h ? hdr_at(lane + 64 * i) : 0u;
                __builtin_amdgcn_wave_barrier();  // the previous pair's reads of the stage are done
#pragma unroll
                for (int i = 0; i < PT_LOADS; ++i) {
                    const int w = lane + 64 * i;
                    if (w < nwx) stg[wv][0][w] = rx[i];
                    if (w < nwy) stg[wv][1][w] = ry[i];
                }
#pragma unroll
                for (int i = 0; i < PT_HDR / 64; ++i) hdr[wv][lane + 64 * i] = (uint8_t)hb[i];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            const int L1 = L + 1;
            const int pl = (int)plen;
            // 16-byte stores from the first 16-aligned byte of the pair's text (1 KB per wave store: the
            // text goes straight to pinned host memory, where the write size sets the link rate --
            // tools/d2h_probe's 54.7 GB/s is 16-byte stores), bytes at both ends
            const int a0 = min(pl, (int)((16u - (uint32_t)((uintptr_t)o & 15u)) & 15u));
            const int nw = (pl - a0) >> 4;
            const int tb = a0 + 16 * nw;
            // the text from the stage (LDS reads) or, for a long pair, from global memory: two
            // instantiations, so that the staged form's reads are ds_read and not flat loads
            auto emit = [&](auto STG) {
                constexpr bool S = decltype(STG)::value;
                // byte t of the pair's text: the header, then three lines of L + 1 bytes (no division).
                // Staged: branch-free -- both string bytes and the header byte are read from LDS at
                // clamped positions and selected, so a lane's 16 bytes issue their reads together
                auto byte_at = [&](int t) -> uint32_t {
                    if constexpr (S) {
                        const uint32_t hbyte = hdr[wv][min(t, PT_HDR - 1)];
                        int v = t - h;
                        const int line = (v >= L1) + (v >= 2 * L1);
                        v -= line * L1;
                        const int vc = max(0, min(v, L - 1));
                        const uint32_t p = sxb[xo + vc], q2 = syb[yo + vc];
                        const uint32_t pat = (p == q2 && p != '-') ? '|' : (p == '-' || q2 == '-') ? '-' : '.';
                        const uint32_t body = v == L ? '\n' : line == 0 ? p : line == 2 ? q2 : pat;
                        return t < h ? hbyte : body;
                    } else {
                        if (t < h) return hdr_at(t);
                        int v = t - h;
                        const int line = v < L1 ? 0 : v < 2 * L1 ? 1 : 2;
                        v -= line * L1;
                        if (v == L) return '\n';
                        if (line == 0) return X[v];
                        if (line == 2) return Y[v];
                        const uint32_t p = X[v], q2 = Y[v];
                        return (p == q2 && p != '-') ? '|' : (p == '-' || q2 == '-') ? '-' : '.';
                    }
                };
                auto word_at = [&](int t) {
                    return byte_at(t) | byte_at(t + 1) << 8 | byte_at(t + 2) << 16 | byte_at(t + 3) << 24;
                };
                if (lane < a0) o[lane] = (char)byte_at(lane);
                for (int wi = lane; wi < nw; wi += 64) {
                    const int t = a0 + 16 * wi;
                    *(uint4*)__builtin_assume_aligned(o + t, 16) =
                        make_uint4(word_at(t), word_at(t + 4), word_at(t + 8), word_at(t + 12));
                }
                if (tb + lane < pl) o[tb + lane] = (char)byte_at(tb + lane);
            };
            if (staged) emit(std::true_type{});
            else emit(std::false_type{});
        }
    }
}

// Device text -> pinned host text: 16-byte loads and stores over the whole buffer (dst 16-aligned;
// the link rate of kernel stores needs whole 16-byte writes, tools/d2h_probe), the last total % 16
// bytes one per lane.
__global__ void __launch_bounds__(256) k_copy_text(const char* __restrict__ src, char* __restrict__ dst, int64_t total) {
    const int64_t n16 = total >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
        d4[i] = s4[i];
    if (blockIdx.x == 0 && threadIdx.x < (total & 15)) dst[16 * n16 + threadIdx.x] = src[16 * n16 + threadIdx.x];
}

// Compaction of one orientation's aligned strings out of the walkers' slots (StrOut): pair k's
// string is the last slen[k * nslot + slot] bytes before byte end[k] of its slot, copied to
// dst + off[k].  One wave per pair, lanes striding over the bytes (coalesced loads and stores).
__global__ void __launch_bounds__(256) k_pack_slots(const uint8_t* __restrict__ sx, const uint8_t* __restrict__ sy,
                                                    const int32_t* __restrict__ slen, int64_t cap, int nslot, int slot,
                                                    const int64_t* __restrict__ end, const int64_t* __restrict__ off,
                                                    int64_t count, uint8_t* __restrict__ dx, uint8_t* __restrict__ dy) {
    const int lane = threadIdx.x & 63;
    for (int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); k < count; k += (int64_t)gridDim.x * 4) {
        const int64_t L = slen[k * nslot + slot];
        const int64_t src = (k * nslot + slot) * cap + end[k] - L, dst = off[k];
        for (int64_t b = lane; b < L; b += 64) {
            dx[dst + b] = sx[src + b];
            dy[dst + b] = sy[src + b];
        }
    }
}

#endif

}  // namespace taxi2
