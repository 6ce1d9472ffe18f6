// C ABI implementation (include/taxi2_mi355x.h): contexts, device-resident sequence sets,
// kernel-variant selection and chunked launches.  Single translation unit: every kernel
// template is instantiated here for gfx950.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "../../include/taxi2_mi355x.h"
#include "align1_kernel.hpp"
#include "align1c_kernel.hpp"
#include "align_kernel.hpp"
#include "alignt_kernel.hpp"
#include "alignt2_kernel.hpp"
#include "alignr_kernel.hpp"
#include "alignlong_kernel.hpp"
#include "ncd_kernels.hpp"
#include "format_kernels.hpp"
#include "common.hpp"
#include "pack_kernels.hpp"
#include "prealigned_kernel.hpp"
#include "subset_kernels.hpp"
#include "trace_kernel.hpp"

using namespace taxi2;

namespace {

// Environment switches.  test_env: the parity tests' switches, kept in the product library -- each
// forces another kernel family or launch shape over the same pairs so that two paths can be compared
// (TAXI2_NO_ALIGNR / NO_PACKED / NO_ALIGNT / NO_ALIGN1 / LONG / LONG_TILE, AT_BAND, AT_CHUNK, AT_HOPS,
// A1_CHUNK, A1_NOCHAIN, AR_SWAP, PRE_NOTILE, ZLEN_SERIAL, SUB_GATHER, NO_WALK_STRINGS; AT_BAND_STATS prints
// the queued-pair count the band tests assert on).
// probe_env: tuning probes and diagnostics (occupancy caps, variant forcing, band statistics, trace
// budget, ...), read only by the variant builds (make variant VFLAGS=-DTAXI2_PROBES ...): the
// product library ignores them.
const char* test_env(const char* name) { return getenv(name); }
#ifdef TAXI2_PROBES
const char* probe_env(const char* name) { return getenv(name); }
#else
const char* probe_env(const char*) { return nullptr; }
#endif

struct DevSet {
    bool live = false;
    int mode = 0;
    int64_t n = 0;
    int32_t max_len = 0;
    bool high = false;  // holds a byte >= 0x80 (latin-1 text: NCD compresses its UTF-8 upper case)
    int64_t nbytes = 0;
    int64_t nwords = 0;
    uint8_t* bytes = nullptr;
    int64_t* offs = nullptr;
    int4* meta = nullptr;
    uint4* planes = nullptr;
    // a column view (taxi2_set_permuted): its own meta, the parent's planes; no bytes / offsets, so
    // only the pre-aligned row-block entry (taxi2_rect_block_dev) accepts it
    bool view = false;
};

}  // namespace

struct taxi2_ctx {
    int device = 0;
    int num_cus = 0;
    size_t total_mem = 0;  // device memory (bytes)
    int reserve_cus = 0;  // packed aligner launches leave this many CUs' worth of workgroups free
    int text_copy = 0;    // pair text into pinned host memory: 0 kernel stores, 1 HBM + DMA, 2 HBM + copy kernel
    hipStream_t stream = nullptr;
    std::string err;
    std::vector<DevSet> sets;
    // reusable device staging
    void* d_out = nullptr;
    size_t d_out_bytes = 0;
    void* d_aux = nullptr;
    size_t d_aux_bytes = 0;
    void* d_work = nullptr;  // single-orientation aligner: [count][worklist...]
    size_t d_work_bytes = 0;
    void* d_trace = nullptr;  // trace-and-walk aligner: two chain trace buffers per workgroup
    size_t d_trace_bytes = 0;
    void* d_bnd = nullptr;  // column-tiled aligner: per-workgroup tile boundary columns
    size_t d_bnd_bytes = 0;
    void* d_fmt = nullptr;  // text formatter staging
    size_t d_fmt_bytes = 0;
    void* d_sub = nullptr;  // subset aggregation scratch (row partials, groups, worklist)
    size_t d_sub_bytes = 0;
    void* d_ncd = nullptr;  // NCD from string slots: stream descriptors + compressed lengths
    size_t d_ncd_bytes = 0;
    void* d_nslots = nullptr;  // all-metrics versusAll: the walkers' string slots of one chunk
    size_t d_nslots_bytes = 0;
    void* d_zheads = nullptr;  // NCD: per-thread deflate hash heads (kept zero) and scratch slabs
    void* d_zslabs = nullptr;
    int64_t z_threads = 0;
    // The aligners' shared buffers (d_trace, d_work) are used on ctx->stream by the host-buffer
    // entry points and on the CALLER's stream by the *_dev ones: the last stream that used them
    // and an event recorded after that use order the next launch on another stream behind it.
    hipStream_t shared_st = nullptr;
    hipEvent_t shared_ev = nullptr;
    // row-shared aligner (alignr_kernel.hpp): the launch's segment table, staged through two pinned
    // host buffers used alternately (an event per buffer: its last copy has completed before the
    // buffer is refilled) into one device buffer (stream-ordered, under shared_acquire)
    void* d_seg = nullptr;
    size_t d_seg_bytes = 0;
    ArSeg* h_seg[2] = {nullptr, nullptr};
    size_t h_seg_cap[2] = {0, 0};
    hipEvent_t seg_ev[2] = {nullptr, nullptr};
    int seg_flip = 0;
    // k_alignr's bounded pacing wait (alignr_kernel.hpp AR_SPIN_CAP): a host-mapped word the kernel
    // sets (never clears) when a fill wave gave up waiting; read by pace_check
    unsigned int* h_pace = nullptr;
};

namespace {

int fail(taxi2_ctx* ctx, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return -1;
}

#define HIP_TRY(ctx, expr)                                                                    \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(ctx, "%s failed (capi.hip:%d): %s", #expr, __LINE__, hipGetErrorString(e_)); \
    } while (0)

int ensure(taxi2_ctx* ctx, void** p, size_t* cap, size_t need) {
    if (*cap >= need) return 0;
    // regrowth: nothing enqueued on any stream (a *_dev caller's included) may still use the old
    // buffer when it is released
    if (*p) HIP_TRY(ctx, hipDeviceSynchronize());
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    size_t want = std::max(need, (size_t)1 << 20);
    HIP_TRY(ctx, hipMalloc(p, want));
    *cap = want;
    return 0;
}

// Before a launch on `st` that uses d_trace / d_work: wait for their last use on another stream.
int shared_acquire(taxi2_ctx* ctx, hipStream_t st) {
    if (ctx->shared_st && ctx->shared_st != st) HIP_TRY(ctx, hipStreamWaitEvent(st, ctx->shared_ev, 0));
    return 0;
}
// After it: remember the stream and mark the point the next user on another stream waits for.
int shared_release(taxi2_ctx* ctx, hipStream_t st) {
    if (!ctx->shared_ev) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->shared_ev, hipEventDisableTiming));
    HIP_TRY(ctx, hipEventRecord(ctx->shared_ev, st));
    ctx->shared_st = st;
    return 0;
}

// A k_alignr launch whose fill waves gave up a pacing wait (alignr_kernel.hpp AR_SPIN_CAP) set
// ctx->h_pace: its results are invalid.  Checked after the blocking entry points' synchronisation
// and before the next row-shared launch (the *_dev calls' asynchronous launches report there).
int pace_check(taxi2_ctx* ctx) {
    const unsigned int e = ctx->h_pace ? __atomic_load_n(ctx->h_pace, __ATOMIC_ACQUIRE) : 0u;
    if (e) {
        __atomic_store_n(ctx->h_pace, 0u, __ATOMIC_RELEASE);
        if (e & 2u)  // (alignr_kernel.hpp: a launch with no queued pass, esc_list null)
            return fail(ctx, "k_alignr: a walk failed its score check in a launch without a full-trace pass; "
                             "the launch's results are invalid");
        return fail(ctx, "k_alignr: a fill wave's pacing wait exceeded its bound (AR_SPIN_CAP); the launch was "
                         "abandoned and its results are invalid");
    }
    return 0;
}

DevSet* get_set(taxi2_ctx* ctx, int id) {
    if (id < 0 || id >= (int)ctx->sets.size() || !ctx->sets[id].live || ctx->sets[id].view) return nullptr;
    return &ctx->sets[id];
}

SetView view(const DevSet& s) { return SetView{s.bytes, s.offs, s.meta, s.planes, s.n}; }

// allow_counts: the pair entry points also accept TAXI2_METRIC_COUNTS, alone, for sequences of at
// most 32 767 bp (every counter then fits its 16-bit field).
// allow_ncd: TAXI2_METRIC_NCD too (taxi2_all_pairs[_dev] on ALIGN sets: NCD from the same fill's
// aligned strings, all_pairs_ncd).
int check_metrics(taxi2_ctx* ctx, const int32_t* metrics, int nm, MetricSpec& ms, bool allow_counts = false,
                  int max_len = 0, bool allow_ncd = false) {
    if (nm < 1 || nm > MAX_METRICS) return fail(ctx, "nmetrics must be in [1, %d]", MAX_METRICS);
    ms.n = nm;
    for (int m = 0; m < nm; ++m) {
        if (metrics[m] == TAXI2_METRIC_NCD && allow_ncd) {
        } else if (metrics[m] == TAXI2_METRIC_COUNTS && allow_counts) {
            if (nm != 1) return fail(ctx, "TAXI2_METRIC_COUNTS must be the only metric of a call");
            if (max_len > 32767) return fail(ctx, "TAXI2_METRIC_COUNTS needs sequences of at most 32767 bp");
        } else if (metrics[m] < TAXI2_METRIC_P || metrics[m] > TAXI2_METRIC_K2P) {
            return fail(ctx, "unknown metric code %d", metrics[m]);
        }
        ms.code[m] = metrics[m];
    }
    return 0;
}

KScores kscores(const taxi2_scores* s) {
    return KScores{s->match_score, s->mismatch_score, s->internal_open_gap_score,
                   s->internal_extend_gap_score, s->end_open_gap_score, s->end_extend_gap_score};
}

bool is_linear(const KScores& k) { return k.io == k.ie && k.eo == k.ee; }

// ---------------------------------------------------------------- align variant table
struct Variant {
    int K, W, occ;
    bool linear, def;
    const void* fn;
    void (*launch)(dim3, dim3, size_t, hipStream_t, SetView, SetView, PairSrc, KScores, MetricSpec,
                   int, int, double*, int32_t*);
};

template <int K, int W, bool LIN, bool DEF, int OCC>
void launch_align(dim3 g, dim3 b, size_t lds, hipStream_t st, SetView x, SetView y, PairSrc ps,
                  KScores sc, MetricSpec ms, int xcap, int om, double* out, int32_t* so) {
    hipLaunchKernelGGL((k_align<K, W, LIN, DEF, OCC>), g, b, lds, st, x, y, ps, sc, ms, xcap, om, out, so);
}

#define T2_VARIANT(K, W, LIN, DEF, OCC)                                                   \
    Variant{K, W, OCC, LIN, DEF, (const void*)&k_align<K, W, LIN, DEF, OCC>,             \
            &launch_align<K, W, LIN, DEF, OCC>}

// Ordered by column capacity (64 * K * W); the first one that fits the longest sequence wins.
// DEF = the default TaxI2 scores (align.py:20-27) as compile-time constants; OCC = waves per
// SIMD the register allocation targets.
const Variant kGotohDef[] = {
    T2_VARIANT(4, 1, false, true, 3), T2_VARIANT(6, 1, false, true, 3), T2_VARIANT(8, 1, false, true, 3),
    T2_VARIANT(6, 2, false, true, 3), T2_VARIANT(8, 2, false, true, 3), T2_VARIANT(6, 4, false, true, 3),
    T2_VARIANT(8, 4, false, true, 3), T2_VARIANT(8, 8, false, true, 3),
};
const Variant kGotoh[] = {
    T2_VARIANT(4, 1, false, false, 3), T2_VARIANT(6, 1, false, false, 3), T2_VARIANT(8, 1, false, false, 3),
    T2_VARIANT(6, 2, false, false, 3), T2_VARIANT(8, 2, false, false, 3), T2_VARIANT(6, 4, false, false, 3),
    T2_VARIANT(8, 4, false, false, 3), T2_VARIANT(8, 8, false, false, 3),
};
const Variant kLinear[] = {
    T2_VARIANT(4, 1, true, false, 2), T2_VARIANT(8, 1, true, false, 2), T2_VARIANT(8, 2, true, false, 2),
    T2_VARIANT(8, 4, true, false, 2), T2_VARIANT(8, 8, true, false, 2),
};
// Experimental shapes for tuning (selected only through TAXI2_VARIANT="K,W,OCC").
const Variant kSweep[] = {
    T2_VARIANT(8, 2, false, true, 2), T2_VARIANT(8, 1, false, true, 2), T2_VARIANT(8, 1, false, true, 4),
    T2_VARIANT(8, 2, false, true, 4), T2_VARIANT(6, 3, false, true, 3), T2_VARIANT(4, 4, false, true, 4),
    T2_VARIANT(4, 4, false, true, 3),
};

bool is_default(const KScores& k) {
    return k.ma == 1 && k.mi == -1 && k.io == -8 && k.ie == -1 && k.eo == -1 && k.ee == -1;
}

template <size_t N>
const Variant* find_variant(const Variant (&tab)[N], int K, int W, int occ, bool lin, bool def) {
    for (size_t i = 0; i < N; ++i)
        if (tab[i].K == K && tab[i].W == W && tab[i].occ == occ && tab[i].linear == lin && tab[i].def == def)
            return &tab[i];
    return nullptr;
}

const Variant* pick_variant(const KScores& k, int max_len) {
    const bool lin = is_linear(k), def = !lin && is_default(k);
    if (const char* force = probe_env("TAXI2_VARIANT")) {  // tuning hook: "K,W,OCC"
        int K = 0, W = 0, occ = 0;
        if (sscanf(force, "%d,%d,%d", &K, &W, &occ) == 3 && 64 * K * W >= max_len) {
            const Variant* v = find_variant(kSweep, K, W, occ, lin, def);
            if (!v) v = find_variant(kGotohDef, K, W, occ, lin, def);
            if (!v) v = find_variant(kGotoh, K, W, occ, lin, def);
            if (!v) v = find_variant(kLinear, K, W, occ, lin, def);
            if (v) return v;
        }
    }
    const Variant* tab;
    int n;
    if (lin) {
        tab = kLinear;
        n = (int)(sizeof kLinear / sizeof kLinear[0]);
    } else if (def) {
        tab = kGotohDef;
        n = (int)(sizeof kGotohDef / sizeof kGotohDef[0]);
    } else {
        tab = kGotoh;
        n = (int)(sizeof kGotoh / sizeof kGotoh[0]);
    }
    for (int i = 0; i < n; ++i)
        if (64 * tab[i].K * tab[i].W >= max_len) return &tab[i];
    return nullptr;
}

size_t align_lds_bytes(const Variant& v, int xcap) {
    return ((size_t)xcap * 4 + 15) / 16 * 16 + (size_t)(v.W - 1) * RING * sizeof(RingEntry);
}

// ---------------------------------------------------------------- single-orientation variants
struct Variant1 {
    int K, W, occ;
    bool def;
    int nw;  // counter words: 2 (<= 1023 bp), 3 (<= 4095 bp)
    const void* fn[2];  // pass 1 (orientation A + divergence flag), pass 2 (orientation B)
    void (*launch[2])(dim3, dim3, size_t, hipStream_t, SetView, SetView, PairSrc, KScores, MetricSpec, int,
                      int, double*, int32_t*, uint32_t*, uint32_t*, unsigned long long*);
    const void* fnc[2];  // chained kernel (k_align1c), same passes
    void (*launchc[2])(dim3, dim3, size_t, hipStream_t, SetView, SetView, PairSrc, KScores, MetricSpec, int,
                       int, double*, int32_t*, uint32_t*, uint32_t*, unsigned long long*);
};

template <int K, int W, bool DEF, int OCC, bool B, int NW>
void launch_align1(dim3 g, dim3 b, size_t lds, hipStream_t st, SetView x, SetView y, PairSrc ps, KScores sc,
                   MetricSpec ms, int xcap, int om, double* out, int32_t* so, uint32_t* wl, uint32_t* wc,
                   unsigned long long* nx) {
    hipLaunchKernelGGL((k_align1<K, W, DEF, OCC, B, NW>), g, b, lds, st, x, y, ps, sc, ms, xcap, om, out, so, wl, wc,
                       nx);
}

template <int K, int W, bool DEF, int OCC, bool B, int NW>
void launch_align1c(dim3 g, dim3 b, size_t lds, hipStream_t st, SetView x, SetView y, PairSrc ps, KScores sc,
                    MetricSpec ms, int xcap, int om, double* out, int32_t* so, uint32_t* wl, uint32_t* wc,
                    unsigned long long* nx) {
    hipLaunchKernelGGL((k_align1c<K, W, DEF, OCC, B, NW>), g, b, lds, st, x, y, ps, sc, ms, xcap, om, out, so, wl,
                       wc, nx);
}

#define T2_VARIANT1N(K, W, DEF, OCC, NW)                                                                 \
    Variant1{K, W, OCC, DEF, NW,                                                                          \
             {(const void*)&k_align1<K, W, DEF, OCC, false, NW>, (const void*)&k_align1<K, W, DEF, OCC, true, NW>}, \
             {&launch_align1<K, W, DEF, OCC, false, NW>, &launch_align1<K, W, DEF, OCC, true, NW>},      \
             {(const void*)&k_align1c<K, W, DEF, OCC, false, NW>,                                           \
              (const void*)&k_align1c<K, W, DEF, OCC, true, NW>},                                           \
             {&launch_align1c<K, W, DEF, OCC, false, NW>, &launch_align1c<K, W, DEF, OCC, true, NW>}}
#define T2_VARIANT1(K, W, DEF, OCC) T2_VARIANT1N(K, W, DEF, OCC, 2)

// Ordered by column capacity 64 * K * W.  Two-word counters up to A1_MAX_LEN, three-word counters
// up to A1_MAX_LEN_LONG.
const Variant1 kAlign1Def[] = {
    T2_VARIANT1(4, 1, true, 4),      T2_VARIANT1(8, 1, true, 4),      T2_VARIANT1(6, 2, true, 4),
    T2_VARIANT1(8, 2, true, 4),      T2_VARIANT1N(10, 2, true, 3, 3), T2_VARIANT1N(6, 4, true, 3, 3),
    T2_VARIANT1N(8, 4, true, 3, 3),  T2_VARIANT1N(10, 4, true, 2, 3), T2_VARIANT1N(6, 8, true, 2, 3),
    T2_VARIANT1N(8, 8, true, 2, 3),
};
const Variant1 kAlign1[] = {
    T2_VARIANT1(4, 1, false, 4),      T2_VARIANT1(8, 1, false, 4),      T2_VARIANT1(6, 2, false, 4),
    T2_VARIANT1(8, 2, false, 4),      T2_VARIANT1N(10, 2, false, 3, 3), T2_VARIANT1N(6, 4, false, 3, 3),
    T2_VARIANT1N(8, 4, false, 3, 3),  T2_VARIANT1N(10, 4, false, 2, 3), T2_VARIANT1N(6, 8, false, 2, 3),
    T2_VARIANT1N(8, 8, false, 2, 3),
};
// Tuning shapes (TAXI2_VARIANT1="K,W,OCC").
const Variant1 kAlign1Sweep[] = {
    T2_VARIANT1(8, 2, true, 3), T2_VARIANT1(8, 2, true, 5), T2_VARIANT1(4, 4, true, 4), T2_VARIANT1(4, 4, true, 6),
    T2_VARIANT1(10, 2, true, 3), T2_VARIANT1(10, 2, true, 4), T2_VARIANT1N(8, 4, true, 4, 3),
    T2_VARIANT1N(8, 4, true, 2, 3), T2_VARIANT1N(10, 2, true, 2, 3), T2_VARIANT1N(6, 4, true, 2, 3),
    T2_VARIANT1N(10, 4, true, 3, 3), T2_VARIANT1N(6, 8, true, 3, 3),
};

const Variant1* pick_variant1(const KScores& k, int max_len) {
    const bool def = is_default(k);
    if (const char* force = probe_env("TAXI2_VARIANT1")) {
        int K = 0, W = 0, occ = 0;
        if (sscanf(force, "%d,%d,%d", &K, &W, &occ) == 3 && 64 * K * W >= max_len) {
            for (const auto* tab : {kAlign1Sweep, kAlign1Def, kAlign1}) {
                const size_t n = tab == kAlign1Sweep ? sizeof kAlign1Sweep / sizeof kAlign1Sweep[0]
                                 : tab == kAlign1Def ? sizeof kAlign1Def / sizeof kAlign1Def[0]
                                                     : sizeof kAlign1 / sizeof kAlign1[0];
                for (size_t i = 0; i < n; ++i)
                    if (tab[i].K == K && tab[i].W == W && tab[i].occ == occ && tab[i].def == def &&
                        (tab[i].nw == 2) == (max_len <= A1_MAX_LEN))
                        return &tab[i];
            }
        }
    }
    const Variant1* tab = def ? kAlign1Def : kAlign1;
    const int n = (int)(def ? sizeof kAlign1Def / sizeof kAlign1Def[0] : sizeof kAlign1 / sizeof kAlign1[0]);
    const int nw = max_len <= A1_MAX_LEN ? 2 : 3;
    for (int i = 0; i < n; ++i)
        if (tab[i].nw == nw && 64 * tab[i].K * tab[i].W >= max_len) return &tab[i];
    return nullptr;
}

// Both passes of the single-orientation aligner, stream-ordered (no host synchronisation).
int launch_align1_pairs(taxi2_ctx* ctx, const Variant1& v, const DevSet& X, const DevSet& Y, const PairSrc& ps,
                        const KScores& k, const MetricSpec& ms, int out_mode, double* d_out, int32_t* d_scores,
                        hipStream_t st, int xcap) {
    // chained kernel (consecutive pairs sharing their column sequence stream through the lanes);
    // TAXI2_A1_NOCHAIN=1 selects the one-pair-at-a-time kernel
    const bool chain = !test_env("TAXI2_A1_NOCHAIN");
    if (chain && ps.count >= ((int64_t)1 << 31))  // worklist entries: pair index | orientation << 31
        return fail(ctx, "single-orientation aligner: %lld pairs in one call (limit 2^31 - 1)", (long long)ps.count);
    const size_t lds = chain ? a1c_lds_bytes(v.K, v.W, v.def) : a1_lds_bytes(xcap, v.K, v.W, v.def);
    const void* const* fns = chain ? v.fnc : v.fn;
    auto launch = chain ? v.launchc : v.launch;
    if (lds > 160 * 1024) return fail(ctx, "LDS requirement %zu exceeds 160 KiB", lds);
    if (lds > 64 * 1024)
        for (int k = 0; k < 2; ++k)
            HIP_TRY(ctx, hipFuncSetAttribute(fns[k], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (shared_acquire(ctx, st)) return -1;
    // d_work: [u32 worklist count, pad] [u64 pass-1 cursor] [u64 pass-2 cursor] [u32 worklist...]
    if (ensure(ctx, &ctx->d_work, &ctx->d_work_bytes, 32 + (size_t)ps.count * 4)) return -1;
    uint32_t* wcount = (uint32_t*)ctx->d_work;
    unsigned long long* next = (unsigned long long*)((char*)ctx->d_work + 8);
    uint32_t* wlist = (uint32_t*)((char*)ctx->d_work + 32);
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_work, 0, 32, st));
    // persistent grids: the workgroups resident at the variant's occupancy (pairs are pulled from
    // a device cursor; pass 2's length is known only on the device)
    const int64_t resident = (int64_t)ctx->num_cus * std::max(1, 4 * v.occ / v.W);
    const int64_t grid = std::min<int64_t>(ps.count, resident);
    // the int argument is xcap for k_align1 and the chunk request for k_align1c (0 = automatic;
    // TAXI2_A1_CHUNK forces 1..16 pairs per cursor step, e.g. to test long chains on small inputs)
    int arg = xcap;
    if (chain) {
        const char* c = test_env("TAXI2_A1_CHUNK");
        arg = c ? std::max(0, std::min(A1C_CHUNK, atoi(c))) : 0;
    }
    launch[0](dim3((unsigned)grid), dim3(64 * v.W), lds, st, view(X), view(Y), ps, k, ms, arg, out_mode, d_out,
              d_scores, wlist, wcount, next);
    HIP_TRY(ctx, hipGetLastError());
    launch[1](dim3((unsigned)grid), dim3(64 * v.W), lds, st, view(X), view(Y), ps, k, ms, arg, out_mode, d_out,
              nullptr, wlist, wcount, next + 1);
    HIP_TRY(ctx, hipGetLastError());
    if (shared_release(ctx, st)) return -1;
    if (probe_env("TAXI2_A1_STATS")) {  // diagnostics: share of pairs re-run in orientation B
        uint32_t n2 = 0;
        HIP_TRY(ctx, hipMemcpyAsync(&n2, wcount, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(ctx, hipStreamSynchronize(st));
        fprintf(stderr, "taxi2: single-orientation pass 2 re-ran %u of %lld pairs\n", n2, (long long)ps.count);
    }
    return 0;
}

// ---------------------------------------------------------------- trace-and-walk variants
// trace band of the packed kernel (alignt2_kernel.hpp a2_band_blocks) and its escape queue
struct BandArgs {
    int band;
    int64_t* esc_list;
    unsigned long long* esc_n;
};

struct VariantT {
    int K, W, occ;
    bool def;
    const void* fn;
    void (*launch)(dim3, dim3, hipStream_t, SetView, SetView, PairSrc, KScores, MetricSpec, int, int, double*,
                   int32_t*, uint8_t*, int64_t, int, int, unsigned long long*, BandArgs, StrOut);
    bool raw = false;  // packed kernels: best-open fill + raw-difference trace (4 K bytes per lane-step)
};

template <int K, int W, bool DEF, int OCC>
void launch_alignt(dim3 g, dim3 b, hipStream_t st, SetView x, SetView y, PairSrc ps, KScores sc, MetricSpec ms,
                   int chunk, int om, double* out, int32_t* so, uint8_t* tr, int64_t bb, int cap, int hops,
                   unsigned long long* nx, BandArgs, StrOut) {  // no string output (launch_packed_strings)
    hipLaunchKernelGGL((k_alignt<K, W, DEF, OCC>), g, b, 0, st, x, y, ps, sc, ms, chunk, om, out, so, tr, bb, cap,
                       hops, nx);
}

#define T2_VARIANTT(K, W, DEF, OCC) \
    VariantT{K, W, OCC, DEF, (const void*)&k_alignt<K, W, DEF, OCC>, &launch_alignt<K, W, DEF, OCC>}

// Ordered by column capacity 64 * K * W (waves per SIMD in `occ`).
const VariantT kAlignT[] = {
    T2_VARIANTT(4, 1, true, 6),  T2_VARIANTT(8, 1, true, 6),  T2_VARIANTT(8, 2, true, 6),
    T2_VARIANTT(4, 1, false, 6), T2_VARIANTT(8, 1, false, 6), T2_VARIANTT(8, 2, false, 6),
};

const VariantT* pick_variantt(const KScores& k, int max_len) {
    const bool def = is_default(k);
    for (const auto& v : kAlignT)
        if (v.def == def && 64 * v.K * v.W >= max_len) return &v;
    return nullptr;
}

// Packed variants (two pairs per lane in 16-bit halves, alignt2_kernel.hpp); same launch shape.
#define T2_VARIANTT2(K, W, DEF, OCC) \
    VariantT{K, W, OCC, DEF, (const void*)&k_alignt2<K, W, DEF, OCC>, &launch_alignt2<K, W, DEF, OCC>, a2_raw<W, DEF>()}
// other scores on the best-open fill (opens no better than extends: bopen_ok)
#define T2_VARIANTT2R(K, W, OCC) \
    VariantT{K, W, OCC, false, (const void*)&k_alignt2<K, W, false, OCC, true>, &launch_alignt2<K, W, false, OCC, true>, true}

template <int K, int W, bool DEF, int OCC, bool RAWT = a2_raw<W, DEF>()>
void launch_alignt2(dim3 g, dim3 b, hipStream_t st, SetView x, SetView y, PairSrc ps, KScores sc, MetricSpec ms,
                    int chunk, int om, double* out, int32_t* so, uint8_t* tr, int64_t bb, int cap, int hops,
                    unsigned long long* nx, BandArgs ba, StrOut str) {
    if (ps.sel)  // the queued pairs of a band pass, full trace
        hipLaunchKernelGGL((k_alignt2_queued<K, W, DEF, OCC>), g, b, 0, st, x, y, ps, sc, ms, chunk, om, out, so, tr,
                           bb, cap, hops, nx, str);
    else
        hipLaunchKernelGGL((k_alignt2<K, W, DEF, OCC, RAWT>), g, b, 0, st, x, y, ps, sc, ms, chunk, om, out, so, tr, bb, cap,
                           hops, nx, ba.band, ba.esc_list, ba.esc_n, str);
}

// A2_OCC: waves per SIMD the one- and two-fill-wave shapes are compiled for (the VGPR budget:
// 6 -> 80, 5 -> 96, 4 -> 128 registers per lane)
#ifndef A2_OCC
#define A2_OCC 6
#endif
// The same for other scores (the sign-digit trace + per-column extend constants): asked for 6 waves,
// the compiler gave up at 144 VGPRs (3 waves per SIMD); 4 fits in 128 VGPRs with its spills in cold code
#ifndef A2_OCC_GEN
#define A2_OCC_GEN 4
#endif
const VariantT kAlignT2[] = {
    T2_VARIANTT2(4, 1, true, A2_OCC),  T2_VARIANTT2(8, 1, true, A2_OCC),
    T2_VARIANTT2(6, 2, true, A2_OCC),  T2_VARIANTT2(8, 2, true, A2_OCC),
    T2_VARIANTT2(4, 1, false, A2_OCC_GEN), T2_VARIANTT2(8, 1, false, A2_OCC_GEN),
    T2_VARIANTT2(6, 2, false, A2_OCC_GEN), T2_VARIANTT2(8, 2, false, A2_OCC_GEN),
    // 1 025 - 2 048 columns: four fill waves + the walker (5 waves per workgroup)
    T2_VARIANTT2(6, 4, true, 5), T2_VARIANTT2(8, 4, true, 5), T2_VARIANTT2(6, 4, false, 5), T2_VARIANTT2(8, 4, false, 5),
};
// other scores, best-open fill (at 6 waves per SIMD the compiler ends at 4 with 117 VGPRs)
const VariantT kAlignT2R[] = {
    T2_VARIANTT2R(4, 1, A2_OCC_GEN), T2_VARIANTT2R(8, 1, A2_OCC_GEN),
    T2_VARIANTT2R(6, 2, A2_OCC_GEN), T2_VARIANTT2R(8, 2, A2_OCC_GEN),
};

// The best-open recurrences (alignt2_kernel.hpp) need every open no better than its extend (an Ix / Iy
// open from its own state is then never better than the extend); the raw trace keeps the cell's
// state differences as int8 (CPU model: within [-16, 25] for scores up to 10 with one extend; the
// walkers' score check is a second net, but it cannot see a wrapped difference that flips a tie
// between two optimal moves, so the bound itself must hold)
// The kernel drifts by the extend (cells store V - (i + j) ie), which needs ONE extend for internal and
// end gaps: then neighbouring cells differ by amounts bounded by the scores and the int8 differences
// are exact (with ie != ee they grow with the length of end gaps: tools/proto_bopen.c).
bool bopen_ok(const KScores& k) {
    auto ab = [](int v) { return v < 0 ? -v : v; };
    const int big = std::max({ab(k.ma), ab(k.mi), ab(k.io), ab(k.ie), ab(k.eo), ab(k.ee)});
    return k.ie == k.ee && k.io <= k.ie && k.eo <= k.ee && big <= 12 && !probe_env("TAXI2_NO_BOPEN");
}

const VariantT* pick_variantt2(const KScores& k, int max_len) {
    const bool def = is_default(k);
    if (!def && bopen_ok(k))
        for (const auto& v : kAlignT2R)
            if (64 * v.K * v.W >= max_len) return &v;
    for (const auto& v : kAlignT2)
        if (v.def == def && 64 * v.K * v.W >= max_len) return &v;
    return nullptr;
}

// packed: two streams per chain, two trace bytes per lane-column and step
int launch_alignt_pairs(taxi2_ctx* ctx, const VariantT& v, const DevSet& X, const DevSet& Y, const PairSrc& ps,
                        const KScores& k, const MetricSpec& ms, int out_mode, double* d_out, int32_t* d_scores,
                        hipStream_t st, int max_len, bool packed, StrOut str = StrOut{}) {
    // resident workgroups of the kernel (VGPR and LDS limits), persistent grid; a caller overlapping
    // other work with this launch leaves ctx->reserve_cus CUs' worth of workgroups unlaunched
    int per_cu = 0;
    HIP_TRY(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, v.fn, 64 * (v.W + 1), 0));
    const int64_t resident =
        (int64_t)std::max(1, ctx->num_cus - std::max(0, std::min(ctx->reserve_cus, ctx->num_cus - 1))) *
        std::max(1, per_cu);
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(ps.count, resident));
    // chunk (pairs per cursor step): TAXI2_AT_CHUNK forces 1..AT_CHUNK, else the kernel's automatic
    // rule (at least ~8 chunks per workgroup); it bounds the rows of a chain, hence the buffers
    const int cmax = packed ? AT2_CHUNK : AT_CHUNK;
    int chunk = 0;
    if (const char* c = test_env("TAXI2_AT_CHUNK")) chunk = std::max(0, std::min(cmax, atoi(c)));
    int64_t eff = chunk >= 1 ? chunk : std::max<int64_t>(1, std::min<int64_t>(cmax, ps.count / (grid * 8)));
    // two trace buffers per resident workgroup: shrink the chunk (hence the chain rows) until they
    // fit the budget (TAXI2_AT_TRACE_GB, default 40 GB of the 288 GB HBM; 80 GB for the packed
    // default-score kernel, whose raw-difference trace takes 4 bytes per lane-column and step)
    const bool raw = packed && v.raw;  // best-open fill + raw-difference trace (alignt2_kernel.hpp)
    double budget_gb = raw ? 80.0 : 40.0;
    if (const char* b = probe_env("TAXI2_AT_TRACE_GB")) budget_gb = std::max(1.0, atof(b));
    auto buf_bytes = [&](int64_t e) {
        const int64_t per_stream = packed ? (e + 1) / 2 : e;  // a stream takes every other pair of a chain
        return at_buf_bytes((int)per_stream * std::max(1, max_len), packed ? (raw ? 4 : 2) * v.K : v.K, v.W);
    };
    while (eff > 1 && (double)grid * 2.0 * (double)buf_bytes(eff) > budget_gb * 1e9) eff = eff / 2;
    if (shared_acquire(ctx, st)) return -1;
    chunk = (int)eff;  // the kernel must cut chains with the same bound the buffers were sized for
    const int cap_rows = (int)(packed ? (eff + 1) / 2 : eff) * std::max(1, max_len);
    const size_t bb = buf_bytes(eff);
    if (ensure(ctx, &ctx->d_trace, &ctx->d_trace_bytes, (size_t)grid * 2 * bb)) return -1;
    int hops = 4096;  // per-interval cap; the packed kernel stops at the fill waves' signal
    if (const char* h = test_env("TAXI2_AT_HOPS")) hops = std::max(1, atoi(h));
    // Packed kernel: the fill stores only a diagonal strip of each pair's trace (band half-width in
    // columns: TAXI2_AT_BAND, 0 = everything; default 3 sqrt(max_len), at least 32: wider than the
    // first paths of synthetic families measured at 200-2 000 bp); walks that leave
    // it queue their pair and a second launch redoes exactly those pairs with the full trace.
    int band = 0;
    if (packed) {
        band = std::max(32, (int)std::ceil(3.0 * std::sqrt((double)std::max(1, max_len))));
        if (4 * band >= max_len) band = 0;  // the strip would be most of the row
        if (const char* e = test_env("TAXI2_AT_BAND")) band = std::max(0, atoi(e));
    }
    // d_work: [u64 pad] [u64 pass-1 cursor] [u64 pass-2 cursor] [u64 queue count] [pad] [i64 queue...]
    // (the queue also takes raw-difference walks whose score check failed, so it exists whenever
    // the band pass can queue anything)
    const bool queue = band > 0 || raw;
    if (ensure(ctx, &ctx->d_work, &ctx->d_work_bytes, 64 + (queue ? (size_t)ps.count * 8 : 0))) return -1;
    unsigned long long* next = (unsigned long long*)((char*)ctx->d_work + 8);
    unsigned long long* next2 = (unsigned long long*)((char*)ctx->d_work + 16);
    unsigned long long* esc_n = (unsigned long long*)((char*)ctx->d_work + 24);
    int64_t* esc_list = (int64_t*)((char*)ctx->d_work + 64);
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_work, 0, 64, st));
    v.launch(dim3((unsigned)grid), dim3(64 * (v.W + 1)), st, view(X), view(Y), ps, k, ms, chunk, out_mode, d_out,
             d_scores, (uint8_t*)ctx->d_trace, (int64_t)bb, cap_rows, hops, next,
             BandArgs{band, queue ? esc_list : nullptr, esc_n}, str);
    HIP_TRY(ctx, hipGetLastError());
    if (queue) {  // the queued pairs (usually none: the workgroups exit at once), full trace
        PairSrc p2 = ps;
        p2.sel = esc_list;
        p2.dcount = esc_n;
        v.launch(dim3((unsigned)grid), dim3(64 * (v.W + 1)), st, view(X), view(Y), p2, k, ms, chunk, out_mode, d_out,
                 d_scores, (uint8_t*)ctx->d_trace, (int64_t)bb, cap_rows, hops, next2, BandArgs{0, nullptr, nullptr}, str);
        HIP_TRY(ctx, hipGetLastError());
        if (test_env("TAXI2_AT_BAND_STATS")) {  // diagnostics: queued pairs of this call on stderr
            unsigned long long q = 0;
            HIP_TRY(ctx, hipMemcpyAsync(&q, esc_n, sizeof q, hipMemcpyDeviceToHost, st));
            HIP_TRY(ctx, hipStreamSynchronize(st));
            fprintf(stderr, "taxi2 band: k_alignt2<%d,%d,%d> band %d: %llu of %lld pairs took the full-trace pass\n",
                    v.K, v.W, (int)v.def, band, q, (long long)ps.count);
        }
    }
    if (shared_release(ctx, st)) return -1;
#ifdef TAXI2_GUARD
    if (packed) {  // debug build: report (and clear) out-of-range accesses the guards skipped
        unsigned int e = 0;
        HIP_TRY(ctx, hipStreamSynchronize(st));
        HIP_TRY(ctx, hipMemcpyFromSymbol(&e, HIP_SYMBOL(at_guard_err), sizeof e));
        unsigned int dg[8] = {0}, z8[8] = {0};
        HIP_TRY(ctx, hipMemcpyFromSymbol(dg, HIP_SYMBOL(at_diag), sizeof dg));
        HIP_TRY(ctx, hipMemcpyToSymbol(HIP_SYMBOL(at_diag), z8, sizeof z8));
        fprintf(stderr, "taxi2 diag: k_alignt2<%d,%d,%d> grid %lld chunk %d count %lld: chains %u pairs %u t0stores %u "
                "fin %u walks %u t0first %u steps %u nB %u\n", v.K, v.W, (int)v.def, (long long)grid, chunk,
                (long long)ps.count, dg[0], dg[1], dg[2], dg[3], dg[4], dg[5], dg[6], dg[7]);
        if (e) {
            fprintf(stderr, "taxi2 guard: k_alignt2<%d,%d,%d> codes 0x%x (grid %lld, chunk %d, cap_rows %d, buf %zu, "
                    "count %lld)\n", v.K, v.W, (int)v.def, e, (long long)grid, chunk, cap_rows, bb, (long long)ps.count);
            const unsigned int z = 0;
            HIP_TRY(ctx, hipMemcpyToSymbol(HIP_SYMBOL(at_guard_err), &z, sizeof z));
            return fail(ctx, "guard build: k_alignt2<%d,%d,%d> guard codes 0x%x (see alignt2_kernel.hpp AG_*)", v.K,
                        v.W, (int)v.def, e);
        }
    }
#endif
    return 0;
}

// ---------------------------------------------------------------- row-shared packed aligner
// (alignr_kernel.hpp): the default scores (constants folded in) and one-extend user sets
// (ar_scores_ok), triangle and rectangle launches up to 1 024 columns and rows.
struct VariantR {
    int K, W, occ;
    bool def;
    const void* fn;
    void (*launch)(dim3, dim3, hipStream_t, SetView, SetView, KScores, const ArSeg*, int, int64_t, int64_t, MetricSpec, int,
                   int, double*, int32_t*, uint8_t*, int64_t, int, unsigned long long*, int, int64_t*,
                   unsigned long long*, StrOut, unsigned int*);
};

template <int K, int W, int OCC, bool DEF>
void launch_alignr(dim3 g, dim3 b, hipStream_t st, SetView x, SetView y, KScores k, const ArSeg* segs, int nseg,
                   int64_t units, int64_t npairs, MetricSpec ms, int chunk, int om, double* out, int32_t* so, uint8_t* tr,
                   int64_t bb, int cap, unsigned long long* nx, int band, int64_t* el, unsigned long long* en, StrOut str,
                   unsigned int* perr) {
    hipLaunchKernelGGL((k_alignr<K, W, OCC, DEF>), g, b, 0, st, x, y, k, segs, nseg, units, npairs, ms, chunk, om, out, so,
                       tr, bb, cap, nx, band, el, en, str, perr);
}

// waves per SIMD the row-shared shapes are compiled for: LDS (~23.5 KB per workgroup of three waves)
// allows six workgroups per CU, i.e. 4.5 waves per SIMD, so 5 (96 VGPRs) costs no occupancy
#ifndef AR_OCC
#define AR_OCC 5
#endif
#define T2_VARIANTR(K, W, D) \
    VariantR{K, W, AR_OCC, D, (const void*)&k_alignr<K, W, AR_OCC, D>, &launch_alignr<K, W, AR_OCC, D>}
const VariantR kAlignR[] = {T2_VARIANTR(4, 1, true), T2_VARIANTR(8, 1, true), T2_VARIANTR(6, 2, true),
                            T2_VARIANTR(8, 2, true)};
const VariantR kAlignRG[] = {T2_VARIANTR(4, 1, false), T2_VARIANTR(8, 1, false), T2_VARIANTR(6, 2, false),
                             T2_VARIANTR(8, 2, false)};

static int64_t tri_row_host(int64_t g, int64_t N);

// A run of row intervals: pairs (x, b) for lo <= b < hi, launch index pbase + b.
struct RowIv {
    int64_t x, lo, hi, pbase;
};

// Cut the launch's pairs into segments of units (x0, x1, b): a sweep over b keeps the rows active
// on each elementary b-interval paired in x order (x1 = -1 for an odd one out), and a pair of rows
// stays one segment for as long as the pairing keeps it.  Rows enter and leave the active set only
// at their interval ends, and in the triangle they enter in x order at the end of the order, so the
// pairing of earlier rows persists: few segments, few single units.
// swap_ok: a row whose pairs no second row shares (an odd number of rows over those columns) becomes a
// swapped segment -- units of two of its pairs sharing the row's sequence -- instead of units that
// idle one half (needs the aligner shape to hold the column set's sequences as columns too)
void build_segments(std::vector<RowIv>& rows, std::vector<ArSeg>& segs, int64_t& units, bool swap_ok) {
    segs.clear();
    units = 0;
    std::sort(rows.begin(), rows.end(), [](const RowIv& a, const RowIv& b) { return a.x < b.x; });
    std::vector<int64_t> pts;
    for (const auto& r : rows)
        if (r.hi > r.lo) {
            pts.push_back(r.lo);
            pts.push_back(r.hi);
        }
    std::sort(pts.begin(), pts.end());
    pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
    struct Open {
        int r0, r1;  // row slots (r1 = -1: single)
        int64_t b0, b1;
    };
    const int R = (int)rows.size();
    std::vector<Open> open(R, Open{-1, -1, 0, 0});  // open segment by its first row slot
    std::vector<int> act;
    auto close = [&](const Open& o) {
        const RowIv& a = rows[o.r0];
        const int64_t nb = o.b1 - o.b0;
        if (nb <= 0) return;
        ArSeg sg{};
        sg.x0 = a.x;
        sg.p0 = a.pbase + o.b0;
        if (o.r1 >= 0) {
            sg.x1 = rows[o.r1].x;
            sg.p1 = rows[o.r1].pbase + o.b0;
        } else {
            sg.x1 = -1;
            sg.p1 = -1;
        }
        sg.b0 = o.b0;
        sg.nb = nb;
        if (o.r1 < 0 && swap_ok && nb > 1) {  // one row alone: pairs of its own columns per unit
            sg.sw = nb;
            sg.nb = (nb + 1) / 2;
        }
        sg.u0 = units;
        units += sg.nb;
        segs.push_back(sg);
    };
    for (size_t e = 0; e + 1 < pts.size(); ++e) {
        const int64_t b0 = pts[e], b1 = pts[e + 1];
        act.clear();
        for (int r = 0; r < R; ++r)
            if (rows[r].lo <= b0 && rows[r].hi >= b1) act.push_back(r);
        // pairs of this interval: continue an open segment of the same two rows ending at b0
        std::vector<char> cont(R, 0);
        for (size_t q = 0; q < act.size(); q += 2) {
            const int r0 = act[q], r1 = q + 1 < act.size() ? act[q + 1] : -1;
            Open& o = open[r0];
            if (o.r0 == r0 && o.r1 == r1 && o.b1 == b0) {
                o.b1 = b1;
            } else {
                if (o.r0 >= 0) close(o);
                o = Open{r0, r1, b0, b1};
            }
            cont[r0] = 1;
        }
        for (int r = 0; r < R; ++r)
            if (open[r].r0 >= 0 && !cont[r]) {
                close(open[r]);
                open[r].r0 = -1;
            }
    }
    for (int r = 0; r < R; ++r)
        if (open[r].r0 >= 0) close(open[r]);
}

const VariantR* pick_variantr(const KScores& k, const DevSet& X, const DevSet& Y, const PairSrc& ps) {
    if (test_env("TAXI2_NO_ALIGNR") || test_env("TAXI2_NO_PACKED") || ps.sel) return nullptr;
    if (ps.mode != PAIRS_TRI && ps.mode != PAIRS_RECT) return nullptr;
    if (X.max_len > 1024 || Y.max_len > 1024) return nullptr;  // the f16-maximum3 value range (BIAS16)
    // the walker addresses sequence bytes by 32-bit offsets from the sets' bases
    if (X.nbytes >= ((int64_t)1 << 32) || Y.nbytes >= ((int64_t)1 << 32)) return nullptr;
    const bool def = is_default(k);
    // user sets: one extend and best opens (the queued pass's kAlignT2R recurrences, bopen_ok), and
    // their fill values in the f16 range at this length (ar_scores_ok)
    if (!def && !(bopen_ok(k) && ar_scores_ok(k.ma, k.mi, k.io, k.ie, k.eo, k.ee, std::max(X.max_len, Y.max_len)) &&
                  !test_env("TAXI2_NO_ALIGNR_GEN")))
        return nullptr;
    const VariantR* tab = def ? kAlignR : kAlignRG;
    for (int i = 0; i < 4; ++i)
        if (64 * tab[i].K * tab[i].W >= X.max_len) return &tab[i];
    return nullptr;
}

int launch_alignr_pairs(taxi2_ctx* ctx, const VariantR& v, const DevSet& X, const DevSet& Y, const PairSrc& ps,
                        const KScores& k, const MetricSpec& ms, int out_mode, double* d_out, int32_t* d_scores,
                        hipStream_t st, StrOut str = StrOut{}, bool queue = true) {
    if (pace_check(ctx)) return -1;  // an earlier asynchronous launch failed
    // ---- segments of the launch's pairs (host), staged through a pinned buffer
    std::vector<RowIv> rows;
    if (ps.mode == PAIRS_TRI) {
        auto start = [&](int64_t a) { return a * (2 * ps.N - a - 1) / 2; };
        const int64_t g0 = ps.k0, g1 = ps.k0 + ps.count - 1;
        const int64_t a0 = tri_row_host(g0, ps.N), a1 = tri_row_host(g1, ps.N);
        for (int64_t a = a0; a <= a1; ++a) {
            const int64_t lo = a == a0 ? a + 1 + (g0 - start(a)) : a + 1;
            const int64_t hi = a == a1 ? a + 2 + (g1 - start(a)) : ps.N;
            rows.push_back(RowIv{a, lo, hi, start(a) - a - 1 - ps.k0});
        }
    } else {
        const int64_t g0 = ps.k0, g1 = ps.k0 + ps.count - 1;
        const int64_t q0 = g0 / ps.R, q1 = g1 / ps.R;
        for (int64_t q = q0; q <= q1; ++q) {
            const int64_t lo = q == q0 ? g0 - q * ps.R : 0;
            const int64_t hi = q == q1 ? g1 - q * ps.R + 1 : ps.R;
            rows.push_back(RowIv{q, lo, hi, q * ps.R - ps.k0});
        }
    }
    std::vector<ArSeg> segs;
    int64_t units = 0;
    // swapped units (TAXI2_AR_SWAP=1) put the column set's sequences on the columns: the shape must
    // hold them.  Off by default: each swapped unit is a chain of its own, whose walks (latency-bound,
    // four per chain instead of up to 32) outlast its fill, so the fill waves wait at the chain's end
    // barrier -- 94.6 vs 93.6 ms per config-3 launch although the units drop by 4.4 %
    build_segments(rows, segs, units, 64 * v.K * v.W >= Y.max_len && test_env("TAXI2_AR_SWAP"));
    if (segs.empty()) return 0;
    const int f = ctx->seg_flip;
    ctx->seg_flip ^= 1;
    if (!ctx->seg_ev[f]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->seg_ev[f], hipEventDisableTiming));
    else HIP_TRY(ctx, hipEventSynchronize(ctx->seg_ev[f]));  // this buffer's previous copy is done
    if (ctx->h_seg_cap[f] < segs.size()) {
        if (ctx->h_seg[f]) (void)hipHostFree(ctx->h_seg[f]);
        ctx->h_seg[f] = nullptr;
        ctx->h_seg_cap[f] = 0;
        const size_t want = std::max(segs.size(), (size_t)4096);
        HIP_TRY(ctx, hipHostMalloc((void**)&ctx->h_seg[f], want * sizeof(ArSeg), hipHostMallocDefault));
        ctx->h_seg_cap[f] = want;
    }
    std::memcpy(ctx->h_seg[f], segs.data(), segs.size() * sizeof(ArSeg));

    // ---- resident grid, chunk (units per cursor step) and trace buffers, as launch_alignt_pairs
    int per_cu = 0;
    HIP_TRY(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, v.fn, 64 * (v.W + 1), 0));
    if (const char* e = probe_env("TAXI2_AR_PERCU")) per_cu = std::max(1, std::min(per_cu, atoi(e)));  // scaling probe
    const int64_t resident =
        (int64_t)std::max(1, ctx->num_cus - std::max(0, std::min(ctx->reserve_cus, ctx->num_cus - 1))) *
        std::max(1, per_cu);
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(units, resident));
    const int max_len = std::max(1, std::max(X.max_len, Y.max_len));
    int chunk = 0;
    if (const char* c = test_env("TAXI2_AT_CHUNK")) chunk = std::max(0, std::min(AR_UNITS, (atoi(c) + 1) / 2));
    int64_t eff = chunk >= 1 ? chunk : std::max<int64_t>(1, std::min<int64_t>(AR_UNITS, units / (grid * 8)));
    // trace buffers: two per resident workgroup, AR_UNITS rows of sequences each (8 x 1 000 bp: 33 MB);
    // up to 120 GB of the 288 GB HBM, at most 45 % of the device's memory (TAXI2_AT_TRACE_GB overrides)
    double budget_gb = std::min(120.0, 0.45 * (double)ctx->total_mem / 1e9);
    if (const char* b = probe_env("TAXI2_AT_TRACE_GB")) budget_gb = std::max(1.0, atof(b));
    // chain rows: row sequences of the row set, or (swapped units) one of the column set's
    const int rmax = std::max(1, std::max(X.max_len, Y.max_len));
    auto buf_bytes = [&](int64_t e) { return at_buf_bytes(ar_trace_rows((int)e * rmax) - 64, 4 * v.K, v.W); };
    while (eff > 1 && (double)grid * 2.0 * (double)buf_bytes(eff) > budget_gb * 1e9) eff = eff / 2;
    chunk = (int)eff;
    const int cap_rows = (int)eff * rmax;
    const size_t bb = buf_bytes(eff);
    // trace band: 2.5 sqrt(L) (80 at 1 000 bp: the widest measured excursion is 67; escapes requeue
    // exactly).  Narrower bands cut the trace writes (337 KB per pair at 80, 275 at 64) but the
    // requeued pairs' full-trace pass costs more than the writes save
    // User one-extend sets take more paths off the diagonal at that width (1 000 bp, config 3: 5.4 %
    // of generic1's pairs and 13.8 % of (1, -2, -4, -1, -2, -1)'s requeued at band 80): 3 sqrt(L) for
    // them, 3.5 sqrt(L) when a mismatch scores no better than two gap columns (s - 2 ie <= 0 in drift
    // coordinates: a pair of gap runs then replaces a run of mismatches for the two opens alone).
    // Measured optima (tools/bench_scores.py, profiles/r6/scores/): 80 / 96 / 112.
    const ArSc asc = ar_sc(k.ma, k.mi, k.io, k.ie, k.eo, k.ee);
    const double bf = v.def ? 2.5 : asc.eqx > 0 ? 3.0 : 3.5;
    int band = std::max(32, (int)std::ceil(bf * std::sqrt((double)max_len)));
    if (4 * band >= max_len) band = 0;
    if (const char* e = test_env("TAXI2_AT_BAND")) band = std::max(0, atoi(e));
    // the queued pass (k_alignt2_queued over the launch's PairSrc, sign-digit full trace); scores
    // outside its 16-bit range (queue = false): no band, nothing to requeue
    const VariantT* vq = queue ? pick_variantt2(k, max_len) : nullptr;
    if (queue && !vq) return fail(ctx, "no packed variant for the queued pass at length %d", max_len);
    if (!vq) band = 0;
    int per_cu_q = 0;
    if (vq) HIP_TRY(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_q, vq->fn, 64 * (vq->W + 1), 0));
    const int64_t grid_q = std::max<int64_t>(1, std::min<int64_t>(ps.count, (int64_t)ctx->num_cus * std::max(1, per_cu_q)));
    const int chunk_q = 2;  // one pair per stream: the queue is usually empty or a handful of pairs
    const int cap_rows_q = max_len;
    const size_t bb_q = vq ? at_buf_bytes(cap_rows_q, 2 * vq->K, vq->W) : 0;

    if (shared_acquire(ctx, st)) return -1;
    if (ensure(ctx, &ctx->d_trace, &ctx->d_trace_bytes, std::max((size_t)grid * 2 * bb, (size_t)grid_q * 2 * bb_q)))
        return -1;
    if (ensure(ctx, &ctx->d_seg, &ctx->d_seg_bytes, segs.size() * sizeof(ArSeg))) return -1;
    if (ensure(ctx, &ctx->d_work, &ctx->d_work_bytes, 64 + (size_t)ps.count * 8)) return -1;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_seg, ctx->h_seg[f], segs.size() * sizeof(ArSeg), hipMemcpyHostToDevice, st));
    HIP_TRY(ctx, hipEventRecord(ctx->seg_ev[f], st));
    unsigned long long* next = (unsigned long long*)((char*)ctx->d_work + 8);
    unsigned long long* next2 = (unsigned long long*)((char*)ctx->d_work + 16);
    unsigned long long* esc_n = (unsigned long long*)((char*)ctx->d_work + 24);
    int64_t* esc_list = (int64_t*)((char*)ctx->d_work + 64);
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_work, 0, 64, st));
    v.launch(dim3((unsigned)grid), dim3(64 * (v.W + 1)), st, view(X), view(Y), k, (const ArSeg*)ctx->d_seg, (int)segs.size(),
             units, ps.count, ms, chunk, out_mode, d_out, d_scores, (uint8_t*)ctx->d_trace, (int64_t)bb, cap_rows, next,
             band, vq ? esc_list : nullptr, esc_n, str, ctx->h_pace);
    HIP_TRY(ctx, hipGetLastError());
    PairSrc p2 = ps;
    p2.sel = esc_list;
    p2.dcount = esc_n;
    if (vq) vq->launch(dim3((unsigned)grid_q), dim3(64 * (vq->W + 1)), st, view(X), view(Y), p2, k, ms, chunk_q, out_mode, d_out,
               d_scores, (uint8_t*)ctx->d_trace, (int64_t)bb_q, cap_rows_q, 4096, next2, BandArgs{0, nullptr, nullptr}, str);
    HIP_TRY(ctx, hipGetLastError());
    if (test_env("TAXI2_AT_BAND_STATS")) {
        unsigned long long q = 0;
        HIP_TRY(ctx, hipMemcpyAsync(&q, esc_n, sizeof q, hipMemcpyDeviceToHost, st));
        HIP_TRY(ctx, hipStreamSynchronize(st));
        int64_t single = 0;  // units of one pair (x1 = -1): the other half of every lane idles
        for (const auto& sg : segs)
            if (sg.x1 < 0) single += sg.sw ? (sg.sw & 1) : sg.nb;
        fprintf(stderr, "taxi2 band: k_alignr<%d,%d> band %d: %llu of %lld pairs took the full-trace pass (%zu segments, "
                "%lld units, %lld single-pair units = %.2f %%, grid %lld, chunk %d)\n", v.K, v.W, band, q,
                (long long)ps.count, segs.size(), (long long)units, (long long)single,
                units ? 100.0 * (double)single / (double)units : 0.0, (long long)grid, chunk);
    }
#ifdef AR_PROF
    {  // profiling build: the launch's per-wave phase totals (alignr_kernel.hpp AR_PROF)
        unsigned long long pf[12] = {0}, z[12] = {0};
        HIP_TRY(ctx, hipStreamSynchronize(st));
        HIP_TRY(ctx, hipMemcpyFromSymbol(pf, HIP_SYMBOL(ar_prof), sizeof pf));
        HIP_TRY(ctx, hipMemcpyToSymbol(HIP_SYMBOL(ar_prof), z, sizeof z));
        fprintf(stderr, "taxi2 arprof: k_alignr<%d,%d> grid %lld units %lld chains %llu | fill steps %llu waits %llu barrier %llu"
                " setup %llu | walker walking %llu barrier %llu | polls %llu walker iterations %llu fill steps %llu\n", v.K, v.W,
                (long long)grid, (long long)units, pf[6], pf[0], pf[4], pf[1], pf[2], pf[3], pf[5], pf[7], pf[8], pf[9]);
    }
#endif
    if (shared_release(ctx, st)) return -1;
    return 0;
}

// ---------------------------------------------------------------- column-tiled (any length)
struct VariantL {
    int K, W, occ;
    bool lin;
    const void* fn;
    void (*launch)(dim3, dim3, hipStream_t, SetView, SetView, PairSrc, KScores, MetricSpec, int, double*, int32_t*,
                   uint8_t*, int64_t, uint2*, int64_t, unsigned long long*, uint8_t*, uint8_t*, int32_t*, int);
};

template <int K, int W, int OCC, bool LIN>
void launch_alignlong(dim3 g, dim3 b, hipStream_t st, SetView x, SetView y, PairSrc ps, KScores sc, MetricSpec ms,
                      int om, double* out, int32_t* so, uint8_t* tr, int64_t bb, uint2* bnd, int64_t brows,
                      unsigned long long* nx, uint8_t* sx, uint8_t* sy, int32_t* slen, int cap) {
    hipLaunchKernelGGL((k_alignlong<K, W, OCC, LIN>), g, b, 0, st, x, y, ps, sc, ms, om, out, so, tr, bb, bnd, brows, nx,
                       sx, sy, slen, cap);
}

#define T2_VARIANTL(K, W, OCC, LIN) \
    VariantL{K, W, OCC, LIN, (const void*)&k_alignlong<K, W, OCC, LIN>, &launch_alignlong<K, W, OCC, LIN>}
// tile widths 64 K W: 2 048 (production), 1 024 and 256 (TAXI2_LONG_TILE: tests cover many tiles
// with short sequences); Gotoh and linear (NW) scores
const VariantL kAlignLong[] = {T2_VARIANTL(8, 4, 2, false), T2_VARIANTL(8, 2, 2, false), T2_VARIANTL(4, 1, 2, false),
                               T2_VARIANTL(8, 4, 2, true),  T2_VARIANTL(8, 2, 2, true),  T2_VARIANTL(4, 1, 2, true)};

// Pairs of any length (alignlong_kernel.hpp): rows = X sequences, columns = Y sequences; Gotoh, or
// Biopython's NW fill and traceback order when the scores are linear (open == extend).
int launch_alignlong_pairs(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, const PairSrc& ps, const KScores& k,
                           const MetricSpec& ms, int out_mode, double* d_out, int32_t* d_scores, hipStream_t st,
                           uint8_t* sx = nullptr, uint8_t* sy = nullptr, int32_t* slen = nullptr, int cap = 0) {
    if (ps.count <= 0) return 0;
    const bool lin = is_linear(k);
    const VariantL* v = lin ? &kAlignLong[3] : &kAlignLong[0];
    if (const char* t = test_env("TAXI2_LONG_TILE")) {
        const int tc = atoi(t);
        for (const auto& c : kAlignLong)
            if (64 * c.K * c.W == tc && c.lin == lin) v = &c;
    }
    const int64_t TC = 64 * v->K * v->W;
    const int64_t rows = std::max(1, X.max_len), cols = std::max(1, Y.max_len);
    const int64_t ntile = (cols + TC - 1) / TC;
    const size_t bb = ((size_t)ntile * (size_t)(rows + 63) * (size_t)TC + 255) / 256 * 256;
    int per_cu = 0;
    HIP_TRY(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, v->fn, 64 * (v->W + 1), 0));
    // trace budget: 40 GB, grown up to 96 GB (a third of the HBM) when that keeps every resident
    // workgroup busy (pairs past ~6 500 bp need > 80 MB of trace each); TAXI2_AT_TRACE_GB fixes it
    const int64_t resident = (int64_t)ctx->num_cus * std::max(1, per_cu);
    double budget_gb = std::max(40.0, std::min(96.0, (double)std::min<int64_t>(ps.count, resident) * 2.0 * (double)bb / 1e9));
    if (const char* b = probe_env("TAXI2_AT_TRACE_GB")) budget_gb = std::max(1.0, atof(b));
    const int64_t fit = (int64_t)(budget_gb * 1e9 / (2.0 * (double)bb));
    if (2.0 * (double)bb > 200e9)
        return fail(ctx, "pair trace of %lld x %lld bp needs %.1f GB (limit 200 GB)", (long long)rows,
                    (long long)cols, 2.0 * (double)bb / 1e9);
    const int64_t grid = std::max<int64_t>(1, std::min({ps.count, resident, fit}));
    if (shared_acquire(ctx, st)) return -1;
    if (ensure(ctx, &ctx->d_trace, &ctx->d_trace_bytes, (size_t)grid * 2 * bb)) return -1;
    const int64_t brows = rows + 64;
    if (ensure(ctx, &ctx->d_bnd, &ctx->d_bnd_bytes, (size_t)grid * (size_t)brows * sizeof(uint2))) return -1;
    if (ensure(ctx, &ctx->d_work, &ctx->d_work_bytes, 32)) return -1;
    unsigned long long* next = (unsigned long long*)((char*)ctx->d_work + 8);
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_work, 0, 32, st));
    v->launch(dim3((unsigned)grid), dim3(64 * (v->W + 1)), st, view(X), view(Y), ps, k, ms, out_mode, d_out, d_scores,
              (uint8_t*)ctx->d_trace, (int64_t)bb, (uint2*)ctx->d_bnd, brows, next, sx, sy, slen, cap);
    HIP_TRY(ctx, hipGetLastError());
    if (shared_release(ctx, st)) return -1;
    return 0;
}

int launch_align_pairs(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, const PairSrc& ps,
                       const taxi2_scores* sc, const MetricSpec& ms, int out_mode, double* d_out,
                       int32_t* d_scores, hipStream_t st) {
    const KScores k = kscores(sc);
    const int max_len = std::max(X.max_len, Y.max_len);
    // int DP range check (32-bit, doubled and tie-tagged): every finite score stays far above NEG_INF
    {
        const long long mag = std::max({std::llabs(k.ma), std::llabs(k.mi), std::llabs(k.io),
                                        std::llabs(k.ie), std::llabs(k.eo), std::llabs(k.ee)});
        if (mag * (2LL * max_len + 2) >= (1LL << 26))
            return fail(ctx, "score magnitudes too large for 32-bit DP at length %d", max_len);
    }
    // past every register-resident shape (and on request, TAXI2_LONG=1): the column-tiled aligner
    if (max_len > 4095 || test_env("TAXI2_LONG"))
        return launch_alignlong_pairs(ctx, X, Y, ps, k, ms, out_mode, d_out, d_scores, st);
    const Variant* v = pick_variant(k, max_len);
    if (!v) return fail(ctx, "sequence length %d exceeds the aligner's column capacity", max_len);
    // int DP range check: every finite (doubled, tie-tagged) score stays far above NEG_INF
    const long long mag = std::max({std::llabs(k.ma), std::llabs(k.mi), std::llabs(k.io),
                                    std::llabs(k.ie), std::llabs(k.eo), std::llabs(k.ee)});
    if (mag * (2LL * max_len + 2) >= (1LL << 26))
        return fail(ctx, "score magnitudes too large for 32-bit DP at length %d", max_len);
    const int xcap = std::max(max_len, 1);
    // linear gaps with one extend: the row-shared aligner, its walker in the single-matrix tie order;
    // the full trace (no band: the queued pass, k_alignt2_queued, walks in the Gotoh order)
    if (is_linear(k) && !test_env("TAXI2_NO_ALIGNT"))
        if (const VariantR* vr = pick_variantr(k, X, Y, ps)) {
            if (ps.count <= 0) return 0;
            return launch_alignr_pairs(ctx, *vr, X, Y, ps, k, ms, out_mode, d_out, d_scores, st, StrOut{}, false);
        }
    if (!is_linear(k) && !test_env("TAXI2_NO_ALIGNT")) {
        // packed 16-bit fill when every difference fits int16 (TAXI2_NO_PACKED=1: 32-bit fill)
        const bool packed = at_fits16(k, max_len) && !test_env("TAXI2_NO_PACKED");
        // the row-shared aligner has its own value range (ar_scores_ok); when the packed queued pass's
        // (at_fits16) is exceeded it stores the full trace and requeues nothing
        if (const VariantR* vr = pick_variantr(k, X, Y, ps)) {
            if (ps.count <= 0) return 0;
            return launch_alignr_pairs(ctx, *vr, X, Y, ps, k, ms, out_mode, d_out, d_scores, st, StrOut{}, packed);
        }
        const VariantT* vt = packed ? pick_variantt2(k, max_len) : pick_variantt(k, max_len);
        if (vt) {
            if (ps.count <= 0) return 0;
            return launch_alignt_pairs(ctx, *vt, X, Y, ps, k, ms, out_mode, d_out, d_scores, st, max_len, packed);
        }
    }
    if (!is_linear(k) && max_len <= A1_MAX_LEN_LONG && !test_env("TAXI2_NO_ALIGN1")) {
        if (ps.count <= 0) return 0;
        const Variant1* v1 = pick_variant1(k, max_len);
        if (v1) return launch_align1_pairs(ctx, *v1, X, Y, ps, k, ms, out_mode, d_out, d_scores, st, xcap);
    }
    const size_t lds = align_lds_bytes(*v, xcap);
    if (lds > 160 * 1024) return fail(ctx, "LDS requirement %zu exceeds 160 KiB", lds);
    if (lds > 64 * 1024)
        HIP_TRY(ctx, hipFuncSetAttribute(v->fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t grid = std::min<int64_t>(ps.count, (int64_t)1 << 30);
    if (grid <= 0) return 0;
    v->launch(dim3((unsigned)grid), dim3(64 * v->W), lds, st, view(X), view(Y), ps, k, ms, xcap,
              out_mode, d_out, d_scores);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

// Metrics (optional) AND aligned strings from one fill per launched pair: the packed trace-and-walk
// kernel's walkers write each alignment as they walk it (alignt2_kernel.hpp StrOut).  Returns 1
// without launching when that kernel does not cover the shape (linear scores, past 2 048 columns,
// scores outside int16); the caller then uses the trace kernels (Tracer) or the column-tiled aligner.
int launch_packed_strings(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, const PairSrc& ps, const taxi2_scores* sc,
                          const MetricSpec& ms, int out_mode, double* d_out, int32_t* d_scores, hipStream_t st,
                          StrOut str) {
    const KScores k = kscores(sc);
    const int max_len = std::max(X.max_len, Y.max_len);
    if (is_linear(k) || !at_fits16(k, max_len) || test_env("TAXI2_NO_ALIGNT") || test_env("TAXI2_NO_PACKED") ||
        test_env("TAXI2_LONG") || test_env("TAXI2_NO_WALK_STRINGS"))
        return 1;
    const VariantT* vt = pick_variantt2(k, max_len);
    if (!vt) return 1;
    if (ps.count <= 0) return 0;
    if (str.cap < X.max_len + Y.max_len)
        return fail(ctx, "string slots of %d bytes < longest x + longest y (%d)", str.cap, X.max_len + Y.max_len);
    if (const VariantR* vr = pick_variantr(k, X, Y, ps))
        return launch_alignr_pairs(ctx, *vr, X, Y, ps, k, ms, out_mode, d_out, d_scores, st, str) ? -1 : 0;
    const int rc = launch_alignt_pairs(ctx, *vt, X, Y, ps, k, ms, out_mode, d_out, d_scores, st, max_len, true, str);
    return rc ? -1 : 0;
}

// host copy of the triangle row of linear pair index g (common.hpp decode_pair)
static int64_t tri_row_host(int64_t g, int64_t N) {
    auto start = [N](int64_t a) { return a * (2 * N - a - 1) / 2; };
    const double n2 = 2.0 * (double)N - 1.0;
    const double disc = n2 * n2 - 8.0 * (double)g;
    int64_t r = (int64_t)((n2 - std::sqrt(disc > 0.0 ? disc : 0.0)) * 0.5);
    r = std::max<int64_t>(0, std::min<int64_t>(r, N - 2));
    while (r > 0 && start(r) > g) --r;
    while (r + 1 <= N - 2 && start(r + 1) <= g) ++r;
    return r;
}

int launch_prealigned(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, const PairSrc& ps,
                      const MetricSpec& ms, double* d_out, hipStream_t st, TileBlock tb = TileBlock{1.0, 0, -1, nullptr, nullptr}) {
    if (ps.count <= 0) return 0;
    // triangle / rectangle blocks: PT x PT pair tiles with LDS-staged planes (prealigned_kernel.hpp);
    // TAXI2_PRE_NOTILE=1 keeps the one-thread-per-pair kernel (A/B and parity tests)
    // (the row-block epilogue of taxi2_rect_block_dev exists only in the tiled kernel)
    const bool epi = tb.rmin_v || tb.diag || tb.scale != 1.0 || tb.ynat;
    if (ps.mode != PAIRS_LIST && (epi || (ps.count >= 4096 && !test_env("TAXI2_PRE_NOTILE")))) {
        int64_t x0, nx, y0, ny;
        if (ps.mode == PAIRS_TRI) {
            const int64_t a0 = tri_row_host(ps.k0, ps.N), a1 = tri_row_host(ps.k0 + ps.count - 1, ps.N);
            x0 = a0;
            nx = a1 - a0 + 1;
            y0 = a0 + 1;
            ny = ps.N - y0;
        } else {
            x0 = ps.k0 / ps.R;
            nx = (ps.k0 + ps.count - 1) / ps.R + 1 - x0;
            y0 = 0;
            ny = ps.R;
        }
        const int64_t tiles_x = (nx + PT - 1) / PT, tiles_y = (ny + PT - 1) / PT;
        if (tiles_x * tiles_y > ((int64_t)1 << 31) - 1) return fail(ctx, "pre-aligned tile grid too large");
        const int nwords = (std::max(X.max_len, Y.max_len) + 31) / 32;
        bool gap = false;  // p-gaps (or anything but p / jc / k2p) reads the gap counter
        for (int m = 0; m < ms.n; ++m) gap |= ms.code[m] != TAXI2_METRIC_P && ms.code[m] != TAXI2_METRIC_JC &&
                                              ms.code[m] != TAXI2_METRIC_K2P;
        const dim3 g((unsigned)(tiles_x * tiles_y)), b(256);
        if (ps.mode == PAIRS_TRI) {
            if (gap) hipLaunchKernelGGL((k_prealigned_tile<PAIRS_TRI, true>), g, b, 0, st, view(X), view(Y), ps, x0, nx, y0,
                                        ny, tiles_y, nwords, ms, d_out, tb);
            else hipLaunchKernelGGL((k_prealigned_tile<PAIRS_TRI, false>), g, b, 0, st, view(X), view(Y), ps, x0, nx, y0,
                                    ny, tiles_y, nwords, ms, d_out, tb);
        } else {
            if (gap) hipLaunchKernelGGL((k_prealigned_tile<PAIRS_RECT, true>), g, b, 0, st, view(X), view(Y), ps, x0, nx,
                                        y0, ny, tiles_y, nwords, ms, d_out, tb);
            else hipLaunchKernelGGL((k_prealigned_tile<PAIRS_RECT, false>), g, b, 0, st, view(X), view(Y), ps, x0, nx,
                                    y0, ny, tiles_y, nwords, ms, d_out, tb);
        }
        HIP_TRY(ctx, hipGetLastError());
        return 0;
    }
    if (epi) return fail(ctx, "row-block epilogue needs a triangle or rectangle launch");
    const int64_t blocks = std::min<int64_t>((ps.count + 255) / 256, (int64_t)ctx->num_cus * 64);
    hipLaunchKernelGGL(k_prealigned, dim3((unsigned)blocks), dim3(256), 0, st, view(X), view(Y), ps,
                       ms, d_out);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

// Generic chunked driver: pairs [0, count) described by `base` (k0 advanced per chunk),
// device results copied back into host `out` (+ `scores_out`).
int run_pairs(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, PairSrc base, const taxi2_scores* sc,
              const MetricSpec& ms, int out_mode, double* out, int32_t* scores_out) {
    const bool align = X.mode == TAXI2_MODE_ALIGN;
    const int per_pair = (align && out_mode == OUT_BOTH) ? 2 * ms.n : ms.n;
    const int64_t chunk_cap = std::max<int64_t>(1, ((int64_t)256 << 20) / (8 * per_pair + 4));
    for (int64_t done = 0; done < base.count; done += chunk_cap) {
        const int64_t n = std::min(chunk_cap, base.count - done);
        if (ensure(ctx, &ctx->d_out, &ctx->d_out_bytes, (size_t)n * per_pair * 8)) return -1;
        int32_t* d_sc = nullptr;
        if (scores_out) {
            if (ensure(ctx, &ctx->d_aux, &ctx->d_aux_bytes, (size_t)n * 4)) return -1;
            d_sc = (int32_t*)ctx->d_aux;
        }
        PairSrc ps = base;
        ps.k0 = base.k0 + done;
        ps.count = n;
        int rc = align ? launch_align_pairs(ctx, X, Y, ps, sc, ms, out_mode, (double*)ctx->d_out, d_sc,
                                            ctx->stream)
                       : launch_prealigned(ctx, X, Y, ps, ms, (double*)ctx->d_out, ctx->stream);
        if (rc) return rc;
        HIP_TRY(ctx, hipMemcpyAsync(out + done * per_pair, ctx->d_out, (size_t)n * per_pair * 8,
                                    hipMemcpyDeviceToHost, ctx->stream));
        if (scores_out)
            HIP_TRY(ctx, hipMemcpyAsync(scores_out + done, d_sc, (size_t)n * 4, hipMemcpyDeviceToHost,
                                        ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (pace_check(ctx)) return -1;
    }
    return 0;
}


int check_pair_indices(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, const int64_t* xs, const int64_t* ys,
                       int64_t count) {
    for (int64_t k = 0; k < count; ++k)
        if (xs[k] < 0 || xs[k] >= X.n || ys[k] < 0 || ys[k] >= Y.n)
            return fail(ctx, "pair %lld index out of bounds", (long long)k);
    return 0;
}

// Aligned strings on the device (k_trace_fill + k_traceback), chunked: slots [chunk][2][cap] for
// x and for y, right-aligned, plus lengths [chunk][2].
struct Tracer {
    uint16_t* d_trace = nullptr;
    int4* d_ends = nullptr;
    int64_t* d_idx = nullptr;
    uint8_t* d_out = nullptr;
    int32_t* d_len = nullptr;
    int64_t chunk = 0, stride = 0;
    int K = 8, W = 1, xcap = 1, cap = 0;
    size_t lds = 0;
    KScores k{};
    bool lin = false;
    bool longp = false;  // pairs past 4 095 bp (or TAXI2_LONG): the column-tiled aligner's walkers

    ~Tracer() {
        if (d_trace) (void)hipFree(d_trace);
        if (d_ends) (void)hipFree(d_ends);
        if (d_idx) (void)hipFree(d_idx);
        if (d_out) (void)hipFree(d_out);
        if (d_len) (void)hipFree(d_len);
    }

    int setup(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, const KScores& ks, int cap_) {
        if (X.mode != TAXI2_MODE_ALIGN || Y.mode != TAXI2_MODE_ALIGN) return fail(ctx, "aligned strings need ALIGN sets");
        const int max_len = std::max(X.max_len, Y.max_len);
        k = ks;
        lin = is_linear(k);
        cap = cap_;
        longp = max_len > 4095 || test_env("TAXI2_LONG");
        if (longp) {  // strings from k_alignlong's walkers: only the index and output staging
            chunk = std::max<int64_t>(1, std::min<int64_t>(4096, ((int64_t)1 << 30) / (4 * (int64_t)std::max(cap, 1))));
            HIP_TRY(ctx, hipMalloc(&d_idx, (size_t)chunk * 2 * sizeof(int64_t)));
            HIP_TRY(ctx, hipMalloc(&d_out, (size_t)chunk * 2 * cap * 2));
            HIP_TRY(ctx, hipMalloc(&d_len, (size_t)chunk * 2 * sizeof(int32_t)));
            return 0;
        }
        if (max_len <= 256) K = 4, W = 1;
        else if (max_len <= 512) W = 1;
        else if (max_len <= 1024) W = 2;
        else if (max_len <= 2048) W = 4;
        else W = 8;
        xcap = std::max(max_len, 1);
        lds = ((size_t)xcap * 4 + 15) / 16 * 16 + (size_t)(W - 1) * RING * sizeof(RingEntry);
        stride = (int64_t)(xcap + 63) * 64 * W * K;  // u16 per pair
        chunk = std::max<int64_t>(1, std::min<int64_t>(4096, ((int64_t)1 << 30) / (stride * 2)));
        HIP_TRY(ctx, hipMalloc(&d_trace, (size_t)chunk * stride * 2));
        HIP_TRY(ctx, hipMalloc(&d_ends, (size_t)chunk * sizeof(int4)));
        HIP_TRY(ctx, hipMalloc(&d_idx, (size_t)chunk * 2 * sizeof(int64_t)));
        HIP_TRY(ctx, hipMalloc(&d_out, (size_t)chunk * 2 * cap * 2));
        HIP_TRY(ctx, hipMalloc(&d_len, (size_t)chunk * 2 * sizeof(int32_t)));
        if (K == 8 && W == 8 && lds > 64 * 1024)
            HIP_TRY(ctx, hipFuncSetAttribute(lin ? (const void*)&k_trace_fill<8, 8, true>
                                                 : (const void*)&k_trace_fill<8, 8, false>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        return 0;
    }

    // pairs (xs[0..n), ys[0..n)) host indices, n <= chunk; stream-ordered, no synchronisation
    int run(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, const int64_t* xs, const int64_t* ys, int64_t n,
            int both) {
        HIP_TRY(ctx, hipMemcpyAsync(d_idx, xs, n * 8, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(d_idx + chunk, ys, n * 8, hipMemcpyHostToDevice, ctx->stream));
        if (longp) {  // both slots, whatever `both` asks (slot 1 is then simply not read)
            PairSrc ps{PAIRS_LIST, 0, n, 0, 0, d_idx, d_idx + chunk};
            MetricSpec none{};
            return launch_alignlong_pairs(ctx, X, Y, ps, k, none, OUT_BOTH, nullptr, nullptr, ctx->stream, d_out,
                                          d_out + chunk * 2 * cap, d_len, cap);
        }
        const dim3 grid((unsigned)n), block(64 * W);
#define T2_FILL(KK, WW, LIN)                                                                         \
    hipLaunchKernelGGL((k_trace_fill<KK, WW, LIN>), grid, block, lds, ctx->stream, view(X), view(Y), d_idx, \
                       d_idx + chunk, n, k, xcap, d_trace, d_ends)
        if (K == 4) {
            if (lin) T2_FILL(4, 1, true); else T2_FILL(4, 1, false);
        } else if (W == 1) {
            if (lin) T2_FILL(8, 1, true); else T2_FILL(8, 1, false);
        } else if (W == 2) {
            if (lin) T2_FILL(8, 2, true); else T2_FILL(8, 2, false);
        } else if (W == 4) {
            if (lin) T2_FILL(8, 4, true); else T2_FILL(8, 4, false);
        } else {
            if (lin) T2_FILL(8, 8, true); else T2_FILL(8, 8, false);
        }
#undef T2_FILL
        HIP_TRY(ctx, hipGetLastError());
        const int64_t threads = n * (both ? 2 : 1);
        const dim3 g2((unsigned)((threads + 255) / 256));
        if (lin)
            hipLaunchKernelGGL(k_traceback<true>, g2, dim3(256), 0, ctx->stream, view(X), view(Y), d_idx, d_idx + chunk,
                               n, K, W, xcap, d_trace, d_ends, cap, d_out, d_out + chunk * 2 * cap, d_len, both);
        else
            hipLaunchKernelGGL(k_traceback<false>, g2, dim3(256), 0, ctx->stream, view(X), view(Y), d_idx,
                               d_idx + chunk, n, K, W, xcap, d_trace, d_ends, cap, d_out, d_out + chunk * 2 * cap,
                               d_len, both);
        HIP_TRY(ctx, hipGetLastError());
        return 0;
    }
};

// first_only: the one-thread path compresses each descriptor's first part alone (launch_zlen2)
// Workgroups of `lds` bytes the 160 KiB of a gfx950 CU's LDS hold: the LDS is allocated in 256-byte
// granules, which hipOccupancyMaxActiveBlocksPerMultiprocessor does not round to (it answered 14
// for 11 568-byte workgroups that fit 13 at a time).  A persistent grid sized for one workgroup too
// many per CU runs its extra workgroups as a second round behind the whole first one.
static int lds_fit_per_cu(size_t lds) {
    const size_t g = (lds + 255) / 256 * 256;
    return g ? (int)((size_t)160 * 1024 / g) : 1 << 20;
}

int launch_zlen(taxi2_ctx* ctx, const ZStream* d_st, int64_t n, int32_t* d_out, int max_n, bool latin1,
                hipStream_t st = nullptr, int likely_n = 0, int first_only = 0);

// Raw-mode NCD with C(x) computed once per set member (when the pairs outnumber the sequences).
int ncd_raw_cached(taxi2_ctx* ctx, const DevSet& X, const DevSet& Y, const int64_t* xs, const int64_t* ys,
                   int64_t count, int both, double* out) {
    const int no = both ? 2 : 1;
    const bool same = &X == &Y;
    const int64_t chunk = std::min<int64_t>(count, (int64_t)1 << 18);
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t b_single = al((size_t)X.n * 4) + (same ? 0 : al((size_t)Y.n * 4));
    const size_t b_sst = al((size_t)std::max(X.n, Y.n) * sizeof(ZStream));
    const size_t b_idx = al((size_t)chunk * 16);
    const size_t b_cst = al((size_t)chunk * no * sizeof(ZStream)), b_c = al((size_t)chunk * no * 4);
    const size_t b_v = al((size_t)chunk * no * 8);
    if (ensure(ctx, &ctx->d_aux, &ctx->d_aux_bytes, b_single + b_sst + b_idx + b_cst + b_c + b_v)) return -1;
    char* base = (char*)ctx->d_aux;
    int32_t* d_cx = (int32_t*)base;
    int32_t* d_cy = same ? d_cx : (int32_t*)(base + al((size_t)X.n * 4));
    ZStream* d_sst = (ZStream*)(base + b_single);
    int64_t* d_idx = (int64_t*)((char*)d_sst + b_sst);
    ZStream* d_cst = (ZStream*)((char*)d_idx + b_idx);
    int32_t* d_c = (int32_t*)((char*)d_cst + b_cst);
    double* d_v = (double*)((char*)d_c + b_c);
    const DevSet* sets[2] = {&X, &Y};
    int32_t* singles[2] = {d_cx, d_cy};
    for (int k = 0; k < (same ? 1 : 2); ++k) {
        const DevSet& S = *sets[k];
        if (S.n == 0) continue;
        hipLaunchKernelGGL(k_seq_streams, dim3((unsigned)((S.n + 255) / 256)), dim3(256), 0, ctx->stream, view(S), S.n,
                           d_sst);
        HIP_TRY(ctx, hipGetLastError());
        if (launch_zlen(ctx, d_sst, S.n, singles[k], S.max_len, S.high)) return -1;
    }
    for (int64_t c0 = 0; c0 < count; c0 += chunk) {
        const int64_t n = std::min(chunk, count - c0);
        HIP_TRY(ctx, hipMemcpyAsync(d_idx, xs + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(d_idx + chunk, ys + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
        const int64_t m = n * no;
        hipLaunchKernelGGL(k_ncd_concat_streams, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, ctx->stream, view(X),
                           view(Y), d_idx, d_idx + chunk, n, both, d_cst);
        HIP_TRY(ctx, hipGetLastError());
        if (launch_zlen(ctx, d_cst, m, d_c, X.max_len + Y.max_len, X.high || Y.high)) return -1;
        hipLaunchKernelGGL(k_ncd_finish_cached, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, ctx->stream, d_c, d_cx,
                           d_cy, d_idx, d_idx + chunk, n, both, d_v);
        HIP_TRY(ctx, hipGetLastError());
        HIP_TRY(ctx, hipMemcpyAsync(out + c0 * no, d_v, (size_t)m * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    return 0;
}

// Compressed lengths of `n` device stream descriptors, every stream at most max_n bytes.  Streams
// up to zlw::NMAX bytes of ASCII: one wave per stream with its state in LDS (k_zlen_wave,
// zlen_wave.hpp); longer ones, latin-1 text (each byte -> 1-2 UTF-8 bytes) or TAXI2_ZLEN_SERIAL=1:
// one thread per stream with per-thread HBM scratch slabs kept in the context (the head tables
// are zeroed once at allocation), any length (the window slides as zlib's does).
int launch_zlen(taxi2_ctx* ctx, const ZStream* d_st, int64_t n, int32_t* d_out, int max_n, bool latin1,
                hipStream_t st, int likely_n, int first_only) {
    if (n <= 0) return 0;
    if (!st) st = ctx->stream;
    bool wave_ok = !latin1 && !test_env("TAXI2_ZLEN_SERIAL");
    auto wave_pass = [&](int nmax_in, int redo) -> int {
        const int nmax = std::max(nmax_in, 4);
        const size_t lds = zlw::lds_bytes(nmax);
        if (lds > 64 * 1024)
            HIP_TRY(ctx, hipFuncSetAttribute((const void*)k_zlen_wave, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int per_cu = 0;
        HIP_TRY(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_zlen_wave, 64, lds));
        per_cu = std::min(per_cu, lds_fit_per_cu(lds));
        const int64_t grid = std::min<int64_t>(n, (int64_t)ctx->num_cus * std::max(1, per_cu));
        hipLaunchKernelGGL(k_zlen_wave, dim3((unsigned)grid), dim3(64), lds, st, d_st, n, nmax, d_out, redo);
        HIP_TRY(ctx, hipGetLastError());
        return 0;
    };
    int redo = 0;
    if (first_only) wave_ok = false;  // (only the fused fallback asks for it)
    if (wave_ok && likely_n > 0 && likely_n < max_n && likely_n <= zlw::NMAX) {
        // most streams fit `likely_n`: a first pass sized for them (smaller LDS, more waves per CU),
        // then the pass below over the streams it declined (-1) only
        if (wave_pass(likely_n, 0)) return -1;
        redo = 1;
    }
    if (max_n <= zlw::NMAX && wave_ok) return wave_pass(max_n, redo);
    // waves per SIMD of the one-thread-per-stream parse (TAXI2_ZLEN_WAVES, 1..4: VGPRs cap it at 4);
    // each thread owns 113 KB of HBM scratch
    int wps = 2;
    if (const char* e = probe_env("TAXI2_ZLEN_WAVES")) wps = std::max(1, std::min(4, atoi(e)));
    const int64_t want = std::min<int64_t>(n, (int64_t)ctx->num_cus * 4 * 64 * wps);
    const int64_t threads = (want + 63) / 64 * 64;
    if (ctx->z_threads < threads) {
        if (ctx->d_zheads) (void)hipFree(ctx->d_zheads);
        if (ctx->d_zslabs) (void)hipFree(ctx->d_zslabs);
        ctx->d_zheads = nullptr;
        ctx->d_zslabs = nullptr;
        ctx->z_threads = 0;
        HIP_TRY(ctx, hipMalloc(&ctx->d_zheads, (size_t)threads * ZS_HEAD));
        HIP_TRY(ctx, hipMalloc(&ctx->d_zslabs, (size_t)threads * ZS_SLAB));
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_zheads, 0, (size_t)threads * ZS_HEAD, st));
        ctx->z_threads = threads;
    }
    hipLaunchKernelGGL(k_zlen, dim3((unsigned)(threads / 64)), dim3(64), 0, st, d_st, n,
                       (uint16_t*)ctx->d_zheads, (uint8_t*)ctx->d_zslabs, d_out, (int)latin1, redo, first_only);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

// The fused lengths of `n` descriptors: d_out[s] = C(a + b), d_out_a[s] = C(a) (k_zlen_wave2: one sort
// and a shared parse prefix, zlen_wave.hpp); where the one-wave path does not apply, two one-thread
// passes (a + b, then a alone).
int launch_zlen2(taxi2_ctx* ctx, const ZStream* d_st, int64_t n, int32_t* d_out, int32_t* d_out_a, int max_n,
                 bool latin1, hipStream_t st, int likely_n) {
    if (n <= 0) return 0;
    if (!st) st = ctx->stream;
    if (latin1 || test_env("TAXI2_ZLEN_SERIAL") || max_n > zlw::NMAX) {
        if (launch_zlen(ctx, d_st, n, d_out, max_n, latin1, st)) return -1;
        return launch_zlen(ctx, d_st, n, d_out_a, max_n, latin1, st, 0, 1);
    }
    auto wave_pass = [&](int nmax_in, int redo) -> int {
        const int nmax = std::max(nmax_in, 4);
        const size_t lds = zlw::lds_bytes(nmax);
        if (lds > 64 * 1024)
            HIP_TRY(ctx, hipFuncSetAttribute((const void*)k_zlen_wave2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int per_cu = 0;
        HIP_TRY(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_zlen_wave2, 64, lds));
        per_cu = std::min(per_cu, lds_fit_per_cu(lds));
        if (const char* e = probe_env("TAXI2_ZLEN_PERCU")) per_cu = std::max(1, std::min(per_cu, atoi(e)));  // scaling probe
        const int64_t grid = std::min<int64_t>(n, (int64_t)ctx->num_cus * std::max(1, per_cu));
        hipLaunchKernelGGL(k_zlen_wave2, dim3((unsigned)grid), dim3(64), lds, st, d_st, n, nmax, d_out, d_out_a, redo);
        HIP_TRY(ctx, hipGetLastError());
        return 0;
    };
    if (likely_n > 0 && likely_n < max_n) {
        if (wave_pass(likely_n, 0)) return -1;
        return wave_pass(max_n, 1);
    }
    return wave_pass(max_n, 0);
}

// Where the aligned strings of `n` pairs sit (the walkers' StrOut slots) and which ordered pairs
// want NCD: slot p * nslot + o, right-aligned at d_end[p] (or len(a) + len(b) of pair p of `ps`
// when d_end is null), `no` orientations (1: (a, b) only; 2: and (b, a)).
struct SlotSrc {
    const uint8_t* sx;
    const uint8_t* sy;
    const int32_t* slen;
    int64_t cap;
    int nslot, no;
    const int64_t* d_end;
    PairSrc ps;
};

// NCD (distances.py:351-358) of every (pair, orientation) from the aligned strings already in HBM:
// k_ncd_slot_streams (per pair one fused job per orientation -- C(x + y) and C(x) in one pass -- and
// C(y0), C(x1) only where the two orientations' alignments differ), k_zlen_wave2 over the fused jobs,
// k_zlen_wave over the singles, k_ncd_slot_finish into out[(p * no + o) * ostride + ocol].  max_str
// bounds every stream (2 x the longest aligned string); latin1: the set holds bytes >= 0x80
// (compressed as their UTF-8 upper case, one-thread path).  Stream-ordered on `st`, no host sync.
int ncd_from_slots(taxi2_ctx* ctx, const SlotSrc& ss, const DevSet& X, const DevSet& Y, int64_t n, int max_str,
                   bool latin1, double* out, int64_t ostride, int ocol, hipStream_t st) {
    if (n <= 0) return 0;
    const int64_t nf = n * ss.no, ns = n * 2;
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t b_f = al((size_t)nf * sizeof(ZStream)), b_s = al((size_t)ns * sizeof(ZStream));
    const size_t b_c = al((size_t)(2 * nf + ns) * 4);
    if (ensure(ctx, &ctx->d_ncd, &ctx->d_ncd_bytes, b_f + b_s + b_c)) return -1;
    ZStream* d_fused = (ZStream*)ctx->d_ncd;
    ZStream* d_single = (ZStream*)((char*)ctx->d_ncd + b_f);
    int32_t* d_cab = (int32_t*)((char*)ctx->d_ncd + b_f + b_s);
    int32_t* d_ca = d_cab + nf;
    int32_t* d_cs = d_ca + nf;
    // d_ncd (and the caller's d_nslots) are per-context scratch: a call on another stream than the
    // last user's is ordered behind it (the aligners' shared-buffer event)
    if (shared_acquire(ctx, st)) return -1;
    hipLaunchKernelGGL(k_ncd_slot_streams, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, ss.sx, ss.sy, ss.slen,
                       ss.cap, ss.nslot, ss.no, ss.d_end, view(X), view(Y), ss.ps, n, d_fused, d_single);
    HIP_TRY(ctx, hipGetLastError());
    // each launch first sized for the likely length (an aligned string is rarely much longer than
    // the longer sequence: +1/16 + 32 bytes), a second pass over the streams that did not fit
    // The fused pass's occupancy is set by its LDS (~5 B per stream byte): among first-pass sizes
    // from the longer sequence + 1/32 + 16 to + 1/16 + 32 bytes per string, the largest that keeps
    // the most waves per CU (at 1 000 bp: 14 instead of 13 waves, all metrics 5.1e5 -> 6.8e5 pairs/s;
    // the few longer alignments take the redo pass).  TAXI2_NCD_MARGIN fixes the margin instead.
    const int lmax = std::max(X.max_len, Y.max_len);
    int likely = lmax + lmax / 16 + 32;
    if (const char* e = probe_env("TAXI2_NCD_MARGIN")) {
        likely = lmax + std::max(0, atoi(e));
    } else {
        int best_w = -1;
        for (int L = lmax + lmax / 32 + 16; L <= lmax + lmax / 16 + 32; L += 2) {
            const int w = lds_fit_per_cu(zlw::lds_bytes(std::max(2 * L, 4)));
            if (w >= best_w) {  // ties: the larger size (fewer redos)
                best_w = w;
                likely = L;
            }
        }
    }
    likely = std::min(max_str / 2, likely);
    if (launch_zlen2(ctx, d_fused, nf, d_cab, d_ca, max_str, latin1, st, 2 * likely)) return -1;
    if (launch_zlen(ctx, d_single, ns, d_cs, max_str / 2, latin1, st, likely)) return -1;
    hipLaunchKernelGGL(k_ncd_slot_finish, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, st, d_cab, d_ca, d_cs, n,
                       ss.no, out, ostride, ocol);
    HIP_TRY(ctx, hipGetLastError());
    return shared_release(ctx, st);
}

bool has_ncd(const MetricSpec& ms) {
    for (int m = 0; m < ms.n; ++m)
        if (ms.code[m] == TAXI2_METRIC_NCD) return true;
    return false;
}

// versusAll with every metric incl. NCD from ONE fill per unordered pair (versus_all.py:546-552): the
// packed aligner writes the counter metrics (NCD's columns get a NaN placeholder) and both
// orientations' aligned strings of a chunk of pairs into slots; ncd_from_slots overwrites the NCD
// columns.  d_out[k][2][nm] on the device (h_out == nullptr, stream-ordered on st) or h_out on the
// host (chunk by chunk through ctx->d_out).  Returns 1 without launching when the packed aligner
// does not cover the shape (linear scores, past 2 048 bp, scores outside int16).
int all_pairs_ncd(taxi2_ctx* ctx, const DevSet& S, int64_t k0, int64_t count, const taxi2_scores* sc,
                  const MetricSpec& ms, double* d_out, double* h_out, int32_t* scores_out, hipStream_t st) {
    const int cap = std::max(2 * S.max_len, 1);
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(count, ((int64_t)2 << 30) / (4 * (int64_t)cap + 16)));
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t b_slots = al((size_t)chunk * 2 * cap), b_len = al((size_t)chunk * 2 * 4);
    const size_t b_out = h_out ? al((size_t)chunk * 2 * ms.n * 8) : 0, b_sc = scores_out && h_out ? al((size_t)chunk * 4) : 0;
    if (ensure(ctx, &ctx->d_nslots, &ctx->d_nslots_bytes, 2 * b_slots + b_len + b_out + b_sc)) return -1;
    uint8_t* d_sx = (uint8_t*)ctx->d_nslots;
    uint8_t* d_sy = d_sx + b_slots;
    int32_t* d_len = (int32_t*)(d_sy + b_slots);
    double* d_tmp = h_out ? (double*)((char*)d_len + b_len) : nullptr;
    int32_t* d_stmp = b_sc ? (int32_t*)((char*)d_len + b_len + b_out) : nullptr;
    if (shared_acquire(ctx, st)) return -1;  // d_nslots: per-context scratch, ordered across streams
    for (int64_t c0 = 0; c0 < count; c0 += chunk) {
        const int64_t n = std::min(chunk, count - c0);
        PairSrc ps{PAIRS_TRI, k0 + c0, n, S.n, 0, nullptr, nullptr};
        double* o = h_out ? d_tmp : d_out + c0 * 2 * ms.n;
        int32_t* so = scores_out ? (h_out ? d_stmp : scores_out + c0) : nullptr;
        const int rc = launch_packed_strings(ctx, S, S, ps, sc, ms, OUT_BOTH, o, so, st, StrOut{d_sx, d_sy, d_len, cap, 2});
        if (rc) return rc;
        SlotSrc ss{d_sx, d_sy, d_len, cap, 2, 2, nullptr, ps};
        for (int m = 0; m < ms.n; ++m)
            if (ms.code[m] == TAXI2_METRIC_NCD && ncd_from_slots(ctx, ss, S, S, n, 2 * cap, S.high, o, ms.n, m, st))
                return -1;
        if (h_out) {
            HIP_TRY(ctx, hipMemcpyAsync(h_out + c0 * 2 * ms.n, o, (size_t)n * 2 * ms.n * 8, hipMemcpyDeviceToHost, st));
            if (scores_out)
                HIP_TRY(ctx, hipMemcpyAsync(scores_out + c0, so, (size_t)n * 4, hipMemcpyDeviceToHost, st));
            HIP_TRY(ctx, hipStreamSynchronize(st));
        }
    }
    return shared_release(ctx, st);
}

}  // namespace

extern "C" {

#ifndef TAXI2_SRC_HASH
#define TAXI2_SRC_HASH "unknown"
#endif
// "... src:<hash>": TAXI2_SRC_HASH is taxi2_amd/srchash.py's hash of the sources the library was
// built from (Makefile); bench.py and smoke() compare it with the hash of the tree they run in
const char* taxi2_version(void) {
    return "taxi2_mi355x 0.2 (gfx950; packed trace-and-walk Gotoh, column-tiled Gotoh / NW, "
           "tiled bit-plane pre-aligned counter) src:" TAXI2_SRC_HASH;
}

int taxi2_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int taxi2_ctx_create(int device, taxi2_ctx** out) {
    if (!out) return -1;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return -2;
    if (device < 0 || device >= n) return -3;
    if (hipSetDevice(device) != hipSuccess) return -4;
    taxi2_ctx* ctx = new taxi2_ctx();
    ctx->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete ctx;
        return -5;
    }
    ctx->num_cus = prop.multiProcessorCount;
    ctx->total_mem = prop.totalGlobalMem;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return -6;
    }
    if (hipHostMalloc((void**)&ctx->h_pace, sizeof(unsigned int), hipHostMallocMapped) != hipSuccess) {
        (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return -7;
    }
    *ctx->h_pace = 0;
    *out = ctx;
    return 0;
}

void taxi2_ctx_destroy(taxi2_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();  // *_dev work on caller streams may still use the buffers
    for (int i = 0; i < (int)ctx->sets.size(); ++i) taxi2_set_destroy(ctx, i);
    if (ctx->d_out) (void)hipFree(ctx->d_out);
    if (ctx->d_aux) (void)hipFree(ctx->d_aux);
    if (ctx->d_work) (void)hipFree(ctx->d_work);
    if (ctx->d_trace) (void)hipFree(ctx->d_trace);
    if (ctx->d_seg) (void)hipFree(ctx->d_seg);
    for (int f = 0; f < 2; ++f) {
        if (ctx->h_seg[f]) (void)hipHostFree(ctx->h_seg[f]);
        if (ctx->seg_ev[f]) (void)hipEventDestroy(ctx->seg_ev[f]);
    }
    if (ctx->d_bnd) (void)hipFree(ctx->d_bnd);
    if (ctx->d_fmt) (void)hipFree(ctx->d_fmt);
    if (ctx->d_sub) (void)hipFree(ctx->d_sub);
    if (ctx->d_zheads) (void)hipFree(ctx->d_zheads);
    if (ctx->d_zslabs) (void)hipFree(ctx->d_zslabs);
    if (ctx->d_ncd) (void)hipFree(ctx->d_ncd);
    if (ctx->d_nslots) (void)hipFree(ctx->d_nslots);
    if (ctx->shared_ev) (void)hipEventDestroy(ctx->shared_ev);
    if (ctx->h_pace) (void)hipHostFree(ctx->h_pace);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* taxi2_last_error(const taxi2_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int taxi2_set_create(taxi2_ctx* ctx, const uint8_t* bytes, const int64_t* offsets, int64_t n,
                     int mode, int* set_id) {
    if (!ctx || !offsets || !set_id || n < 0) return fail(ctx, "invalid arguments to taxi2_set_create");
    if (mode != TAXI2_MODE_PREALIGNED && mode != TAXI2_MODE_ALIGN) return fail(ctx, "bad mode %d", mode);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    DevSet s;
    s.mode = mode;
    s.n = n;
    s.nbytes = offsets[n] - offsets[0];
    int32_t maxlen = 0;
    std::vector<int64_t> woffs(mode == TAXI2_MODE_PREALIGNED ? n : 0);
    std::vector<int64_t> offs0(n + 1);
    int64_t nwords = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t len = offsets[i + 1] - offsets[i];
        if (len < 0) return fail(ctx, "offsets must be non-decreasing");
        if (len > (1 << 20)) return fail(ctx, "sequence %lld longer than 1 MiB", (long long)i);
        maxlen = std::max<int32_t>(maxlen, (int32_t)len);
        if (mode == TAXI2_MODE_PREALIGNED) {
            woffs[i] = nwords;
            nwords += (len + 31) / 32;
        }
    }
    for (int64_t i = 0; i <= n; ++i) offs0[i] = offsets[i] - offsets[0];
    if (nwords > INT32_MAX) return fail(ctx, "set too large");
    {
        const uint8_t* p = bytes + offsets[0];
        uint64_t acc = 0;
        int64_t k = 0;
        for (; k + 8 <= s.nbytes; k += 8) {
            uint64_t w;
            memcpy(&w, p + k, 8);
            acc |= w;
        }
        for (; k < s.nbytes; ++k) acc |= p[k];
        s.high = (acc & 0x8080808080808080ull) != 0;
    }
    s.max_len = maxlen;
    s.nwords = nwords;
    HIP_TRY(ctx, hipMalloc(&s.bytes, std::max<int64_t>(s.nbytes, 16)));
    HIP_TRY(ctx, hipMalloc(&s.offs, (n + 1) * sizeof(int64_t)));
    HIP_TRY(ctx, hipMalloc(&s.meta, std::max<int64_t>(n, 1) * sizeof(int4)));
    if (s.nbytes)
        HIP_TRY(ctx, hipMemcpyAsync(s.bytes, bytes + offsets[0], s.nbytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s.offs, offs0.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice,
                                ctx->stream));
    int64_t* d_woffs = nullptr;
    if (mode == TAXI2_MODE_PREALIGNED && n) {
        HIP_TRY(ctx, hipMalloc(&d_woffs, n * sizeof(int64_t)));
        HIP_TRY(ctx, hipMemcpyAsync(d_woffs, woffs.data(), n * sizeof(int64_t), hipMemcpyHostToDevice,
                                    ctx->stream));
        HIP_TRY(ctx, hipMalloc(&s.planes, std::max<int64_t>(nwords, 1) * sizeof(uint4)));
    }
    if (n) {
        hipLaunchKernelGGL(k_meta, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, ctx->stream, s.bytes,
                           s.offs, d_woffs, n, s.meta);
        HIP_TRY(ctx, hipGetLastError());
        if (mode == TAXI2_MODE_PREALIGNED) {
            hipLaunchKernelGGL(k_planes, dim3((unsigned)n), dim3(64), 0, ctx->stream, s.bytes, s.offs,
                               s.meta, n, s.planes);
            HIP_TRY(ctx, hipGetLastError());
        }
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (d_woffs) (void)hipFree(d_woffs);
    s.live = true;
    ctx->sets.push_back(s);
    *set_id = (int)ctx->sets.size() - 1;
    return 0;
}

int taxi2_set_permuted(taxi2_ctx* ctx, int set_id, const int64_t* d_perm, int64_t n, int* view_id) {
    if (!ctx || !view_id) return -1;
    DevSet* P = get_set(ctx, set_id);
    if (!P) return fail(ctx, "unknown set %d", set_id);
    if (P->mode != TAXI2_MODE_PREALIGNED) return fail(ctx, "taxi2_set_permuted: PREALIGNED sets only");
    if (n != P->n || (n && !d_perm)) return fail(ctx, "taxi2_set_permuted: the permutation must cover the set");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    DevSet v = *P;  // the parent's planes and sizes
    v.view = true;
    v.bytes = nullptr;
    v.offs = nullptr;
    v.meta = nullptr;
    HIP_TRY(ctx, hipMalloc(&v.meta, std::max<int64_t>(n, 1) * sizeof(int4)));
    if (n) {
        hipLaunchKernelGGL(k_meta_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, P->meta, d_perm,
                           n, v.meta);
        HIP_TRY(ctx, hipGetLastError());
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->sets.push_back(v);
    *view_id = (int)ctx->sets.size() - 1;
    return 0;
}

int taxi2_set_destroy(taxi2_ctx* ctx, int set_id) {
    if (!ctx) return -1;
    if (set_id >= 0 && set_id < (int)ctx->sets.size() && ctx->sets[set_id].live && ctx->sets[set_id].view) {
        (void)hipSetDevice(ctx->device);
        if (ctx->sets[set_id].meta) (void)hipFree(ctx->sets[set_id].meta);
        ctx->sets[set_id] = DevSet();
        return 0;
    }
    DevSet* s = get_set(ctx, set_id);
    if (!s) return 0;
    (void)hipSetDevice(ctx->device);
    if (s->bytes) (void)hipFree(s->bytes);
    if (s->offs) (void)hipFree(s->offs);
    if (s->meta) (void)hipFree(s->meta);
    if (s->planes) (void)hipFree(s->planes);
    *s = DevSet();
    return 0;
}

int taxi2_set_info(taxi2_ctx* ctx, int set_id, int64_t* n, int32_t* max_len, int* mode) {
    DevSet* s = ctx ? get_set(ctx, set_id) : nullptr;
    if (!s) return fail(ctx, "unknown set %d", set_id);
    if (n) *n = s->n;
    if (max_len) *max_len = s->max_len;
    if (mode) *mode = s->mode;
    return 0;
}

static int ncd_pairs_impl(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys, int64_t count,
                          const taxi2_scores* sc, int both, double* out, bool try_packed);

int taxi2_all_pairs(taxi2_ctx* ctx, int set, int64_t k0, int64_t count, const taxi2_scores* sc,
                    const int32_t* metrics, int nmetrics, double* out, int32_t* scores_out) {
    if (!ctx) return -1;
    DevSet* s = get_set(ctx, set);
    if (!s) return fail(ctx, "unknown set %d", set);
    MetricSpec ms;
    if (check_metrics(ctx, metrics, nmetrics, ms, true, s->max_len, s->mode == TAXI2_MODE_ALIGN)) return -1;
    const int64_t total = s->n * (s->n - 1) / 2;
    if (k0 < 0 || count < 0 || k0 + count > total) return fail(ctx, "pair range out of bounds");
    if (s->mode == TAXI2_MODE_ALIGN && !sc) return fail(ctx, "scores required in ALIGN mode");
    if (s->mode == TAXI2_MODE_PREALIGNED && scores_out) return fail(ctx, "no scores in PREALIGNED mode");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    PairSrc ps{PAIRS_TRI, k0, count, s->n, 0, nullptr, nullptr};
    if (has_ncd(ms)) {
        if (count == 0) return 0;
        const int rc = all_pairs_ncd(ctx, *s, k0, count, sc, ms, nullptr, out, scores_out, ctx->stream);
        if (rc <= 0) return rc;
        // not the packed aligner's shape: the counter metrics (NCD columns NaN), then NCD of the
        // trace kernels' strings per chunk of host pair lists (taxi2_ncd_pairs)
        if (run_pairs(ctx, *s, *s, ps, sc, ms, OUT_BOTH, out, scores_out)) return -1;
        const int64_t step = (int64_t)1 << 16;
        std::vector<int64_t> xa, yb;
        std::vector<double> v;
        for (int64_t c0 = 0; c0 < count; c0 += step) {
            const int64_t n = std::min(step, count - c0);
            xa.resize(n);
            yb.resize(n);
            v.resize(2 * n);
            int64_t a = tri_row_host(k0 + c0, s->n), b = a + 1 + (k0 + c0 - a * (2 * s->n - a - 1) / 2);
            for (int64_t k = 0; k < n; ++k) {
                xa[k] = a;
                yb[k] = b;
                if (++b == s->n) b = ++a + 1;
            }
            if (ncd_pairs_impl(ctx, set, set, xa.data(), yb.data(), n, sc, 1, v.data(), false)) return -1;
            for (int64_t k = 0; k < n; ++k)
                for (int m = 0; m < ms.n; ++m)
                    if (ms.code[m] == TAXI2_METRIC_NCD) {
                        out[((c0 + k) * 2) * ms.n + m] = v[2 * k];
                        out[((c0 + k) * 2 + 1) * ms.n + m] = v[2 * k + 1];
                    }
        }
        return 0;
    }
    return run_pairs(ctx, *s, *s, ps, sc, ms, OUT_BOTH, out, scores_out);
}

int taxi2_all_pairs_dev(taxi2_ctx* ctx, int set, int64_t k0, int64_t count, const taxi2_scores* sc,
                        const int32_t* metrics, int nmetrics, double* d_out, int32_t* d_scores,
                        void* stream) {
    if (!ctx) return -1;
    DevSet* s = get_set(ctx, set);
    if (!s) return fail(ctx, "unknown set %d", set);
    MetricSpec ms;
    if (check_metrics(ctx, metrics, nmetrics, ms, true, s->max_len, s->mode == TAXI2_MODE_ALIGN)) return -1;
    const int64_t total = s->n * (s->n - 1) / 2;
    if (k0 < 0 || count < 0 || k0 + count > total) return fail(ctx, "pair range out of bounds");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    PairSrc ps{PAIRS_TRI, k0, count, s->n, 0, nullptr, nullptr};
    if (s->mode == TAXI2_MODE_ALIGN) {
        if (!sc) return fail(ctx, "scores required in ALIGN mode");
        if (has_ncd(ms)) {
            if (count == 0) return 0;
            const int rc = all_pairs_ncd(ctx, *s, k0, count, sc, ms, d_out, nullptr, d_scores, st);
            if (rc > 0)
                return fail(ctx, "NCD on the device path needs the packed aligner (Gotoh scores within int16, "
                                 "<= 2 048 bp): use taxi2_all_pairs");
            return rc;
        }
        return launch_align_pairs(ctx, *s, *s, ps, sc, ms, OUT_BOTH, d_out, d_scores, st);
    }
    return launch_prealigned(ctx, *s, *s, ps, ms, d_out, st);
}

int taxi2_counts_metrics_dev(taxi2_ctx* ctx, const uint64_t* d_counts, int64_t n, const int32_t* metrics,
                             int nmetrics, double scale, double* d_out, void* stream) {
    if (!ctx) return -1;
    if (n < 0 || (n > 0 && (!d_counts || !d_out))) return fail(ctx, "invalid arguments to taxi2_counts_metrics_dev");
    MetricSpec ms;
    if (check_metrics(ctx, metrics, nmetrics, ms)) return -1;
    if (n == 0) return 0;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, (int64_t)ctx->num_cus * 32);
    hipLaunchKernelGGL(k_counts_metrics, dim3((unsigned)blocks), dim3(256), 0, st, d_counts, n, ms, scale, d_out);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int taxi2_rect_pairs(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1, const taxi2_scores* sc,
                     const int32_t* metrics, int nmetrics, double* out, int32_t* scores_out) {
    if (!ctx) return -1;
    DevSet* Q = get_set(ctx, set_q);
    DevSet* R = get_set(ctx, set_r);
    if (!Q || !R) return fail(ctx, "unknown set");
    if (Q->mode != R->mode) return fail(ctx, "query and reference sets differ in mode");
    MetricSpec ms;
    if (check_metrics(ctx, metrics, nmetrics, ms, true, std::max(Q->max_len, R->max_len))) return -1;
    if (q0 < 0 || q1 < q0 || q1 > Q->n) return fail(ctx, "query range out of bounds");
    if (Q->mode == TAXI2_MODE_ALIGN && !sc) return fail(ctx, "scores required in ALIGN mode");
    if (Q->mode == TAXI2_MODE_PREALIGNED && scores_out) return fail(ctx, "no scores in PREALIGNED mode");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    PairSrc ps{PAIRS_RECT, q0 * R->n, (q1 - q0) * R->n, 0, R->n, nullptr, nullptr};
    return run_pairs(ctx, *Q, *R, ps, sc, ms, OUT_AB, out, scores_out);
}

int taxi2_rect_strings_dev(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1, const taxi2_scores* sc,
                           const int32_t* metrics, int nmetrics, double* d_out, int32_t cap, uint8_t* d_sx,
                           uint8_t* d_sy, int32_t* d_slen, void* stream) {
    if (!ctx) return -1;
    DevSet* Q = get_set(ctx, set_q);
    DevSet* R = get_set(ctx, set_r);
    if (!Q || !R) return fail(ctx, "unknown set");
    if (Q->mode != TAXI2_MODE_ALIGN || R->mode != TAXI2_MODE_ALIGN) return fail(ctx, "aligned strings need ALIGN sets");
    if (!sc) return fail(ctx, "scores required");
    MetricSpec ms{};
    if (nmetrics > 0 && check_metrics(ctx, metrics, nmetrics, ms, true, std::max(Q->max_len, R->max_len), true))
        return -1;
    if (q0 < 0 || q1 < q0 || q1 > Q->n) return fail(ctx, "query range out of bounds");
    if ((q1 - q0) * R->n > 0 && (!d_sx || !d_sy || !d_slen || (nmetrics > 0 && !d_out))) return fail(ctx, "null output");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    PairSrc ps{PAIRS_RECT, q0 * R->n, (q1 - q0) * R->n, 0, R->n, nullptr, nullptr};
    const int rc = launch_packed_strings(ctx, *Q, *R, ps, sc, ms, OUT_AB, d_out, nullptr, st,
                                         StrOut{d_sx, d_sy, d_slen, cap, 1});
    if (rc > 0) return fail(ctx, "walker strings need the packed aligner (Gotoh scores within int16, <= 2 048 bp)");
    if (rc == 0 && has_ncd(ms) && ps.count > 0) {  // NCD of the strings this fill just wrote
        SlotSrc ss{d_sx, d_sy, d_slen, cap, 1, 1, nullptr, ps};
        for (int m = 0; m < ms.n; ++m)
            if (ms.code[m] == TAXI2_METRIC_NCD &&
                ncd_from_slots(ctx, ss, *Q, *R, ps.count, 2 * (Q->max_len + R->max_len), Q->high || R->high, d_out,
                               ms.n, m, st))
                return -1;
    }
    return rc;
}

int taxi2_tri_strings_dev(taxi2_ctx* ctx, int set, int64_t k0, int64_t count, const taxi2_scores* sc,
                          const int32_t* metrics, int nmetrics, double* d_out, int32_t cap, uint8_t* d_sx,
                          uint8_t* d_sy, int32_t* d_slen, int reserve_cus, void* stream) {
    if (!ctx) return -1;
    DevSet* S = get_set(ctx, set);
    if (!S) return fail(ctx, "unknown set");
    if (S->mode != TAXI2_MODE_ALIGN) return fail(ctx, "aligned strings need an ALIGN set");
    if (!sc) return fail(ctx, "scores required");
    MetricSpec ms{};
    if (nmetrics > 0 && check_metrics(ctx, metrics, nmetrics, ms, true, S->max_len, true)) return -1;
    const int64_t total = S->n * (S->n - 1) / 2;
    if (k0 < 0 || count < 0 || k0 + count > total) return fail(ctx, "pair range out of bounds");
    if (count > 0 && (!d_sx || !d_sy || !d_slen || (nmetrics > 0 && !d_out))) return fail(ctx, "null output");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    PairSrc ps{PAIRS_TRI, k0, count, S->n, 0, nullptr, nullptr};
    ctx->reserve_cus = std::max(0, reserve_cus);
    const int rc = launch_packed_strings(ctx, *S, *S, ps, sc, ms, OUT_BOTH, d_out, nullptr, st,
                                         StrOut{d_sx, d_sy, d_slen, cap, 2});
    ctx->reserve_cus = 0;
    if (rc > 0) return fail(ctx, "walker strings need the packed aligner (Gotoh scores within int16, <= 2 048 bp)");
    if (rc == 0 && has_ncd(ms) && count > 0) {  // NCD of both orientations' strings this fill just wrote
        SlotSrc ss{d_sx, d_sy, d_slen, cap, 2, 2, nullptr, ps};
        for (int m = 0; m < ms.n; ++m)
            if (ms.code[m] == TAXI2_METRIC_NCD &&
                ncd_from_slots(ctx, ss, *S, *S, count, 4 * S->max_len, S->high, d_out, ms.n, m, st))
                return -1;
    }
    return rc;
}

int taxi2_rect_pairs_dev(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1, const taxi2_scores* sc,
                         const int32_t* metrics, int nmetrics, double* d_out, int32_t* d_scores, void* stream) {
    if (!ctx) return -1;
    DevSet* Q = get_set(ctx, set_q);
    DevSet* R = get_set(ctx, set_r);
    if (!Q || !R) return fail(ctx, "unknown set");
    if (Q->mode != R->mode) return fail(ctx, "query and reference sets differ in mode");
    MetricSpec ms;
    if (check_metrics(ctx, metrics, nmetrics, ms, true, std::max(Q->max_len, R->max_len))) return -1;
    if (q0 < 0 || q1 < q0 || q1 > Q->n) return fail(ctx, "query range out of bounds");
    if (Q->mode == TAXI2_MODE_PREALIGNED && d_scores) return fail(ctx, "no scores in PREALIGNED mode");
    if ((q1 - q0) * R->n > 0 && !d_out) return fail(ctx, "null output");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    PairSrc ps{PAIRS_RECT, q0 * R->n, (q1 - q0) * R->n, 0, R->n, nullptr, nullptr};
    if (Q->mode == TAXI2_MODE_ALIGN) {
        if (!sc) return fail(ctx, "scores required in ALIGN mode");
        return launch_align_pairs(ctx, *Q, *R, ps, sc, ms, OUT_AB, d_out, d_scores, st);
    }
    return launch_prealigned(ctx, *Q, *R, ps, ms, d_out, st);
}

int taxi2_rect_block_dev(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1, const int32_t* metrics,
                         int nmetrics, double scale, int diag, int rmin_metric, int64_t* d_rmin_idx, double* d_rmin_val,
                         const int64_t* d_col_nat, double* d_out, void* stream) {
    if (!ctx) return -1;
    DevSet* Q = get_set(ctx, set_q);
    // the column side may be a view of Q (taxi2_set_permuted)
    DevSet* R = (set_r >= 0 && set_r < (int)ctx->sets.size() && ctx->sets[set_r].live) ? &ctx->sets[set_r] : nullptr;
    if (!Q || !R) return fail(ctx, "unknown set");
    if (Q->mode != TAXI2_MODE_PREALIGNED || R->mode != TAXI2_MODE_PREALIGNED)
        return fail(ctx, "taxi2_rect_block_dev: PREALIGNED sets only");
    if (R->view && (!d_col_nat || R->planes != Q->planes))
        return fail(ctx, "taxi2_rect_block_dev: a column view needs its parent as the row set and the column map");
    MetricSpec ms;
    if (check_metrics(ctx, metrics, nmetrics, ms, false, std::max(Q->max_len, R->max_len))) return -1;
    if (q0 < 0 || q1 < q0 || q1 > Q->n) return fail(ctx, "query range out of bounds");
    if (rmin_metric >= nmetrics || (rmin_metric >= 0 && (!d_rmin_idx || !d_rmin_val)))
        return fail(ctx, "bad row-minimum metric or outputs");
    if (diag && set_q != set_r && !d_col_nat)
        return fail(ctx, "the diagonal rule needs one set on both sides (or the column map of a permuted copy)");
    if (d_col_nat && R->n != Q->n) return fail(ctx, "a column map needs a permuted copy of the row set");
    if ((q1 - q0) * R->n > 0 && !d_out) return fail(ctx, "null output");
    if (q1 == q0 || R->n == 0) return 0;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    PairSrc ps{PAIRS_RECT, q0 * R->n, (q1 - q0) * R->n, 0, R->n, nullptr, nullptr};
    const int64_t nx = q1 - q0, tiles_y = (R->n + PT - 1) / PT;
    TileBlock tb{scale, diag ? 1 : 0, rmin_metric, nullptr, nullptr, d_col_nat};
    if (rmin_metric >= 0) {
        if (ensure(ctx, &ctx->d_aux, &ctx->d_aux_bytes, (size_t)nx * tiles_y * 16)) return -1;
        tb.rmin_v = (double*)ctx->d_aux;
        tb.rmin_y = (int64_t*)ctx->d_aux + nx * tiles_y;
    }
    if (launch_prealigned(ctx, *Q, *R, ps, ms, d_out, st, tb)) return -1;
    if (rmin_metric >= 0) {
        hipLaunchKernelGGL(k_rowmin_finish, dim3((unsigned)((nx + 3) / 4)), dim3(256), 0, st, nx, tiles_y, tb.rmin_v,
                           tb.rmin_y, d_rmin_idx, d_rmin_val);
        HIP_TRY(ctx, hipGetLastError());
    }
    return 0;
}

int taxi2_list_pairs(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys,
                     int64_t count, const taxi2_scores* sc, const int32_t* metrics, int nmetrics,
                     double* out, int32_t* scores_out) {
    if (!ctx) return -1;
    DevSet* X = get_set(ctx, set_x);
    DevSet* Y = get_set(ctx, set_y);
    if (!X || !Y) return fail(ctx, "unknown set");
    if (X->mode != Y->mode) return fail(ctx, "sets differ in mode");
    MetricSpec ms;
    if (check_metrics(ctx, metrics, nmetrics, ms, true, std::max(X->max_len, Y->max_len))) return -1;
    if (count < 0) return fail(ctx, "negative count");
    if (count == 0) return 0;
    if (X->mode == TAXI2_MODE_ALIGN && !sc) return fail(ctx, "scores required in ALIGN mode");
    if (X->mode == TAXI2_MODE_PREALIGNED && scores_out) return fail(ctx, "no scores in PREALIGNED mode");
    for (int64_t k = 0; k < count; ++k)
        if (xs[k] < 0 || xs[k] >= X->n || ys[k] < 0 || ys[k] >= Y->n)
            return fail(ctx, "pair %lld index out of bounds", (long long)k);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int64_t* d_idx = nullptr;
    HIP_TRY(ctx, hipMalloc(&d_idx, 2 * count * sizeof(int64_t)));
    int rc = 0;
    do {
        if (hipMemcpyAsync(d_idx, xs, count * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
            hipMemcpyAsync(d_idx + count, ys, count * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
            rc = fail(ctx, "pair list upload failed");
            break;
        }
        PairSrc ps{PAIRS_LIST, 0, count, 0, 0, d_idx, d_idx + count};
        rc = run_pairs(ctx, *X, *Y, ps, sc, ms, OUT_BOTH, out, scores_out);
    } while (0);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_idx);
    return rc;
}

int taxi2_closest(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1, const taxi2_scores* sc,
                  int32_t primary, double scale, const int32_t* metrics, int nmetrics, int64_t* idx_out,
                  double* d_out, double* extra_out, double* primary_out) {
    if (!ctx) return -1;
    DevSet* Q = get_set(ctx, set_q);
    DevSet* R = get_set(ctx, set_r);
    if (!Q || !R) return fail(ctx, "unknown set");
    if (Q->mode != R->mode) return fail(ctx, "query and reference sets differ in mode");
    if (q0 < 0 || q1 < q0 || q1 > Q->n) return fail(ctx, "query range out of bounds");
    if (!idx_out || !d_out) return fail(ctx, "idx_out and d_out are required");
    MetricSpec pm;
    if (check_metrics(ctx, &primary, 1, pm)) return -1;
    MetricSpec em{};
    if (extra_out && check_metrics(ctx, metrics, nmetrics, em)) return -1;
    if (Q->mode == TAXI2_MODE_ALIGN && !sc) return fail(ctx, "scores required in ALIGN mode");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const int64_t Rn = R->n;
    if (q1 == q0) return 0;
    if (Rn == 0) {
        for (int64_t q = 0; q < q1 - q0; ++q) {
            idx_out[q] = -1;
            d_out[q] = NAN;
        }
        return 0;
    }
    // query chunks sized so the primary block stays <= 256 MiB of device memory
    const int64_t qchunk = std::max<int64_t>(1, ((int64_t)256 << 20) / (8 * Rn));
    std::vector<int64_t> all_idx;
    for (int64_t qa = q0; qa < q1; qa += qchunk) {
        const int64_t qb = std::min(q1, qa + qchunk);
        const int64_t nq = qb - qa;
        if (ensure(ctx, &ctx->d_out, &ctx->d_out_bytes, (size_t)nq * Rn * 8)) return -1;
        if (ensure(ctx, &ctx->d_aux, &ctx->d_aux_bytes, (size_t)nq * 16)) return -1;
        double* d_prim = (double*)ctx->d_out;
        int64_t* d_idx = (int64_t*)ctx->d_aux;
        double* d_best = (double*)(d_idx + nq);
        PairSrc ps{PAIRS_RECT, qa * Rn, nq * Rn, 0, Rn, nullptr, nullptr};
        int rc = Q->mode == TAXI2_MODE_ALIGN
                     ? launch_align_pairs(ctx, *Q, *R, ps, sc, pm, OUT_AB, d_prim, nullptr, ctx->stream)
                     : launch_prealigned(ctx, *Q, *R, ps, pm, d_prim, ctx->stream);
        if (rc) return rc;
        hipLaunchKernelGGL(k_row_argmin, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, ctx->stream, d_prim,
                           nq, Rn, scale, d_idx, d_best);
        HIP_TRY(ctx, hipGetLastError());
        HIP_TRY(ctx, hipMemcpyAsync(idx_out + (qa - q0), d_idx, nq * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(d_out + (qa - q0), d_best, nq * 8, hipMemcpyDeviceToHost, ctx->stream));
        if (primary_out)
            HIP_TRY(ctx, hipMemcpyAsync(primary_out + (qa - q0) * Rn, d_prim, (size_t)nq * Rn * 8,
                                        hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    if (extra_out) {
        // extras only for each query's closest reference (versus_reference.py:124-129)
        std::vector<int64_t> xs, ys, slot;
        for (int64_t q = 0; q < q1 - q0; ++q) {
            if (idx_out[q] >= 0) {
                xs.push_back(q0 + q);
                ys.push_back(idx_out[q]);
                slot.push_back(q);
            } else {
                for (int m = 0; m < em.n; ++m) extra_out[q * em.n + m] = NAN;
            }
        }
        if (!xs.empty()) {
            const bool align = Q->mode == TAXI2_MODE_ALIGN;
            const int per = align ? 2 * em.n : em.n;
            std::vector<double> tmp(xs.size() * per);
            int rc = taxi2_list_pairs(ctx, set_q, set_r, xs.data(), ys.data(), (int64_t)xs.size(), sc,
                                      em.code, em.n, tmp.data(), nullptr);
            if (rc) return rc;
            for (size_t t = 0; t < xs.size(); ++t)
                for (int m = 0; m < em.n; ++m) extra_out[slot[t] * em.n + m] = tmp[t * per + m];
        }
    }
    return 0;
}

int taxi2_align_strings(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys,
                        int64_t count, const taxi2_scores* sc, int both, int32_t cap, uint8_t* out_x,
                        uint8_t* out_y, int32_t* out_len) {
    if (!ctx) return -1;
    DevSet* X = get_set(ctx, set_x);
    DevSet* Y = get_set(ctx, set_y);
    if (!X || !Y) return fail(ctx, "unknown set");
    if (!sc) return fail(ctx, "scores required");
    if (count <= 0) return 0;
    if (cap < X->max_len + Y->max_len) return fail(ctx, "cap %d < longest x + longest y", cap);
    if (check_pair_indices(ctx, *X, *Y, xs, ys, count)) return -1;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (X->mode != TAXI2_MODE_ALIGN || Y->mode != TAXI2_MODE_ALIGN) return fail(ctx, "aligned strings need ALIGN sets");
    {  // the packed trace-and-walk kernel writes the strings while it walks (one fill per pair)
        const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(count, ((int64_t)1 << 30) / (4 * (int64_t)cap + 16)));
        const size_t bytes = (size_t)chunk * 2 * (8 + 4) + (size_t)chunk * 2 * 2 * cap;
        if (ensure(ctx, &ctx->d_aux, &ctx->d_aux_bytes, bytes)) return -1;
        int64_t* d_idx = (int64_t*)ctx->d_aux;
        int32_t* d_len = (int32_t*)(d_idx + 2 * chunk);
        uint8_t* d_sx = (uint8_t*)(d_len + 2 * chunk);
        uint8_t* d_sy = d_sx + (size_t)chunk * 2 * cap;
        MetricSpec none{};
        int rc = 1;
        for (int64_t c0 = 0; c0 < count; c0 += chunk) {
            const int64_t n = std::min(chunk, count - c0);
            HIP_TRY(ctx, hipMemcpyAsync(d_idx, xs + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(ctx, hipMemcpyAsync(d_idx + chunk, ys + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
            PairSrc ps{PAIRS_LIST, 0, n, 0, 0, d_idx, d_idx + chunk};
            rc = launch_packed_strings(ctx, *X, *Y, ps, sc, none, both ? OUT_BOTH : OUT_AB, nullptr, nullptr,
                                       ctx->stream, StrOut{d_sx, d_sy, d_len, cap, 2});
            if (rc < 0) return -1;
            if (rc > 0) break;  // not this kernel's shape: the trace kernels below
            HIP_TRY(ctx, hipMemcpyAsync(out_x + c0 * 2 * cap, d_sx, (size_t)n * 2 * cap, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipMemcpyAsync(out_y + c0 * 2 * cap, d_sy, (size_t)n * 2 * cap, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipMemcpyAsync(out_len + c0 * 2, d_len, (size_t)n * 2 * 4, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        }
        if (rc == 0) return 0;
    }
    Tracer tr;
    if (tr.setup(ctx, *X, *Y, kscores(sc), cap)) return -1;
    for (int64_t c0 = 0; c0 < count; c0 += tr.chunk) {
        const int64_t n = std::min(tr.chunk, count - c0);
        if (tr.run(ctx, *X, *Y, xs + c0, ys + c0, n, both)) return -1;
        HIP_TRY(ctx, hipMemcpyAsync(out_x + c0 * 2 * cap, tr.d_out, (size_t)n * 2 * cap, hipMemcpyDeviceToHost,
                                    ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(out_y + c0 * 2 * cap, tr.d_out + tr.chunk * 2 * cap, (size_t)n * 2 * cap,
                                    hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(out_len + c0 * 2, tr.d_len, (size_t)n * 2 * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    return 0;
}

// try_packed: aligned pairs first go through the packed aligner's string walkers (one fill each);
// false when the caller already knows the shape is not the packed aligner's (taxi2_all_pairs' NCD
// fallback), which then skips the per-chunk attempt and its staging.
static int ncd_pairs_impl(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys, int64_t count,
                          const taxi2_scores* sc, int both, double* out, bool try_packed) {
    if (!ctx) return -1;
    DevSet* X = get_set(ctx, set_x);
    DevSet* Y = get_set(ctx, set_y);
    if (!X || !Y) return fail(ctx, "unknown set");
    if (count <= 0) return 0;
    if (!out || !xs || !ys) return fail(ctx, "null argument");
    if (check_pair_indices(ctx, *X, *Y, xs, ys, count)) return -1;
    const bool aligned = sc != nullptr;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const int no = both ? 2 : 1;
    const int cap = X->max_len + Y->max_len;
    if (!aligned && X->n + (X == Y ? 0 : Y->n) <= count * no) return ncd_raw_cached(ctx, *X, *Y, xs, ys, count, both, out);
    if (try_packed && aligned && X->mode == TAXI2_MODE_ALIGN && Y->mode == TAXI2_MODE_ALIGN) {
        // the packed aligner's walkers write the strings (one fill per pair, both orientations),
        // NCD from those slots (ncd_from_slots); the trace kernels below only for other shapes
        const int scap = std::max(cap, 1);
        const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(count, ((int64_t)1 << 30) / (4 * (int64_t)scap + 16)));
        auto al = [](size_t b) { return (b + 255) / 256 * 256; };
        const size_t b_idx = al((size_t)chunk * 16), b_len = al((size_t)chunk * 8), b_v = al((size_t)chunk * 16);
        const size_t b_slots = al((size_t)chunk * 2 * scap);
        if (ensure(ctx, &ctx->d_nslots, &ctx->d_nslots_bytes, b_idx + b_len + b_v + 2 * b_slots)) return -1;
        int64_t* d_idx = (int64_t*)ctx->d_nslots;
        int32_t* d_len = (int32_t*)((char*)d_idx + b_idx);
        double* d_v = (double*)((char*)d_len + b_len);
        uint8_t* d_sx = (uint8_t*)d_v + b_v;
        uint8_t* d_sy = d_sx + b_slots;
        MetricSpec none{};
        int rc = 1;
        for (int64_t c0 = 0; c0 < count; c0 += chunk) {
            const int64_t n = std::min(chunk, count - c0);
            HIP_TRY(ctx, hipMemcpyAsync(d_idx, xs + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(ctx, hipMemcpyAsync(d_idx + chunk, ys + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
            PairSrc ps{PAIRS_LIST, 0, n, 0, 0, d_idx, d_idx + chunk};
            rc = launch_packed_strings(ctx, *X, *Y, ps, sc, none, both ? OUT_BOTH : OUT_AB, nullptr, nullptr,
                                       ctx->stream, StrOut{d_sx, d_sy, d_len, scap, 2});
            if (rc < 0) return -1;
            if (rc > 0) break;  // not this kernel's shape: the trace kernels below
            SlotSrc ss{d_sx, d_sy, d_len, scap, 2, no, nullptr, ps};
            if (ncd_from_slots(ctx, ss, *X, *Y, n, 2 * scap, X->high || Y->high, d_v, 1, 0, ctx->stream)) return -1;
            HIP_TRY(ctx, hipMemcpyAsync(out + c0 * no, d_v, (size_t)n * no * 8, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        }
        if (rc == 0) return 0;
    }
    Tracer tr;
    int64_t chunk = (int64_t)1 << 16;
    if (aligned) {
        if (tr.setup(ctx, *X, *Y, kscores(sc), std::max(cap, 1))) return -1;
        chunk = tr.chunk;
    } else {
        if (ensure(ctx, &ctx->d_aux, &ctx->d_aux_bytes, (size_t)chunk * 2 * 8)) return -1;
    }
    const int64_t nstreams = chunk * no * 3;
    if (ensure(ctx, &ctx->d_out, &ctx->d_out_bytes, (size_t)nstreams * (sizeof(ZStream) + 4) + chunk * no * 8))
        return -1;
    ZStream* d_st = (ZStream*)ctx->d_out;
    int32_t* d_c = (int32_t*)(d_st + nstreams);
    double* d_v = (double*)(((uintptr_t)(d_c + nstreams) + 7) & ~(uintptr_t)7);
    for (int64_t c0 = 0; c0 < count; c0 += chunk) {
        const int64_t n = std::min(chunk, count - c0);
        const int64_t* d_xs;
        const int64_t* d_ys;
        if (aligned) {
            if (tr.run(ctx, *X, *Y, xs + c0, ys + c0, n, both)) return -1;
            d_xs = tr.d_idx;
            d_ys = tr.d_idx + tr.chunk;
        } else {
            int64_t* di = (int64_t*)ctx->d_aux;
            HIP_TRY(ctx, hipMemcpyAsync(di, xs + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(ctx, hipMemcpyAsync(di + chunk, ys + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
            d_xs = di;
            d_ys = di + chunk;
        }
        const int64_t m = n * no;
        hipLaunchKernelGGL(k_ncd_streams, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, ctx->stream, view(*X),
                           view(*Y), d_xs, d_ys, n, both, aligned ? tr.d_out : nullptr,
                           aligned ? tr.d_out + tr.chunk * 2 * tr.cap : nullptr, aligned ? tr.d_len : nullptr,
                           aligned ? tr.cap : 0, d_st);
        HIP_TRY(ctx, hipGetLastError());
        if (launch_zlen(ctx, d_st, m * 3, d_c, aligned ? 2 * tr.cap : X->max_len + Y->max_len, X->high || Y->high))
            return -1;
        hipLaunchKernelGGL(k_ncd_finish, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, ctx->stream, d_c, m, d_v);
        HIP_TRY(ctx, hipGetLastError());
        HIP_TRY(ctx, hipMemcpyAsync(out + c0 * no, d_v, (size_t)m * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    return 0;
}

int taxi2_ncd_pairs(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys, int64_t count,
                    const taxi2_scores* sc, int both, double* out) {
    return ncd_pairs_impl(ctx, set_x, set_y, xs, ys, count, sc, both, out, true);
}

int taxi2_ncd_slots_dev(taxi2_ctx* ctx, const uint8_t* d_sx, const uint8_t* d_sy, const int32_t* d_slen, int64_t cap,
                        int nslot, int no, const int64_t* d_end, int64_t count, int32_t max_len, int latin1,
                        double* d_out, void* stream) {
    if (!ctx) return -1;
    if (count < 0 || cap < 1 || max_len < 0 || (nslot != 1 && nslot != 2) || no < 1 || no > nslot)
        return fail(ctx, "invalid arguments to taxi2_ncd_slots_dev");
    if (count == 0) return 0;
    if (!d_sx || !d_sy || !d_slen || !d_end || !d_out) return fail(ctx, "null argument");
    if (2 * (int64_t)max_len > cap) return fail(ctx, "slots of %lld bytes < twice the longest sequence", (long long)cap);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    DevSet lens;  // no set: the slot ends come from d_end; only the length bound is read
    lens.max_len = max_len;
    SlotSrc ss{d_sx, d_sy, d_slen, cap, nslot, no, d_end, PairSrc{PAIRS_LIST, 0, count, 0, 0, nullptr, nullptr}};
    return ncd_from_slots(ctx, ss, lens, lens, count, 4 * std::max(max_len, 1), latin1 != 0, d_out, 1, 0, st);
}

int taxi2_zlib_lengths(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys, int64_t count,
                       int32_t* out) {
    if (!ctx) return -1;
    DevSet* X = get_set(ctx, set_x);
    DevSet* Y = ys ? get_set(ctx, set_y) : X;
    if (!X || !Y) return fail(ctx, "unknown set");
    if (count <= 0) return 0;
    if (!out || !xs) return fail(ctx, "null argument");
    for (int64_t k = 0; k < count; ++k) {
        if (xs[k] < 0 || xs[k] >= X->n || (ys && (ys[k] < 0 || ys[k] >= Y->n)))
            return fail(ctx, "stream %lld index out of bounds", (long long)k);
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const int64_t chunk = (int64_t)1 << 18;
    if (ensure(ctx, &ctx->d_aux, &ctx->d_aux_bytes, (size_t)chunk * 2 * 8)) return -1;
    if (ensure(ctx, &ctx->d_out, &ctx->d_out_bytes, (size_t)chunk * (sizeof(ZStream) + 4))) return -1;
    ZStream* d_st = (ZStream*)ctx->d_out;
    int32_t* d_c = (int32_t*)(d_st + chunk);
    int64_t* di = (int64_t*)ctx->d_aux;
    for (int64_t c0 = 0; c0 < count; c0 += chunk) {
        const int64_t n = std::min(chunk, count - c0);
        HIP_TRY(ctx, hipMemcpyAsync(di, xs + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
        if (ys) HIP_TRY(ctx, hipMemcpyAsync(di + chunk, ys + c0, n * 8, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_zlen_streams, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, view(*X),
                           view(*Y), di, ys ? di + chunk : nullptr, n, d_st);
        HIP_TRY(ctx, hipGetLastError());
        if (launch_zlen(ctx, d_st, n, d_c, X->max_len + (ys ? Y->max_len : 0), X->high || (ys && Y->high)))
            return -1;
        HIP_TRY(ctx, hipMemcpyAsync(out + c0, d_c, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    return 0;
}

}  // extern "C"

// Summary-mode extras (taxi2_format_summary).
struct SummaryHost {
    const uint8_t* rsuf;
    const int64_t* rsuf_offs;
    const uint8_t* csuf;
    const int64_t* csuf_offs;
    const int32_t* rcode;
    const int32_t* ccode;
    int has_g, has_s;
    const uint8_t* lab;
    const int64_t* lab_offs;
};

// Shared by taxi2_format_rows (rectangular), taxi2_format_ragged (rstart / cols non-null) and
// taxi2_format_summary (mode 2, sm non-null).
// The device address of a page-locked host buffer (hipHostMalloc, e.g. a torch pinned tensor), or
// nullptr for pageable memory.  The text kernels then store straight into host memory over the link
// (tools/d2h_probe: 54.7 GB/s from kernel stores against 27-30 GB/s for hipMemcpyAsync into the same
// pinned buffer), with no staging copy in HBM and no separate D2H.  TAXI2_TEXT_D2H=1: the copy path.
static char* host_mapped(void* out) {
    if (!out || probe_env("TAXI2_TEXT_D2H")) return nullptr;
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, out) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error of the call
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost || !at.devicePointer) return nullptr;
    return (char*)at.devicePointer;
}

static int format_impl(taxi2_ctx* ctx, int mode, const double* vals, int64_t nrows, int64_t ncols, int nm,
                       const int64_t* rstart, const int32_t* cols, const uint8_t* row_pre, const int64_t* row_offs,
                       const uint8_t* col_pre, const int64_t* col_offs, int decimals, const uint8_t* missing,
                       int32_t missing_len, uint8_t* out, int64_t cap, int64_t* out_len,
                       const SummaryHost* sm = nullptr, bool dev_vals = false, int64_t vstride = 0,
                       hipStream_t st_in = nullptr) {
    if (!ctx) return -1;
    if (!out_len || (nrows > 0 && (!vals || !row_pre || !row_offs))) return fail(ctx, "null argument");
    if (mode < 0 || mode > 2 || (mode == 2) != (sm != nullptr))
        return fail(ctx, "mode must be 0 (linear) or 1 (matrix)");
    if (mode == 1 && nm != 1) return fail(ctx, "matrix mode formats one metric");
    if (mode != 1 && (!col_pre || !col_offs)) return fail(ctx, "linear mode needs column prefixes");
    if (sm && nrows > 0 && ncols > 0 &&
        (!sm->rsuf || !sm->rsuf_offs || !sm->csuf || !sm->csuf_offs || !sm->rcode || !sm->ccode || !sm->lab ||
         !sm->lab_offs))
        return fail(ctx, "null summary argument");
    if (decimals < 0 || decimals > FMT_MAX_DECIMALS) return fail(ctx, "decimals must be in [0, %d]", FMT_MAX_DECIMALS);
    if (nrows < 0 || ncols < 0 || nm < 1 || missing_len < 0) return fail(ctx, "bad shape");
    const bool ragged = rstart != nullptr;
    *out_len = 0;
    if (nrows == 0) return 0;
    int64_t ntok = nrows * ncols;
    if (ragged) {
        if (!cols) return fail(ctx, "ragged rows need a column list");
        for (int64_t r = 0; r < nrows; ++r)
            if (rstart[r + 1] < rstart[r]) return fail(ctx, "row starts must be non-decreasing");
        ntok = rstart[nrows] - rstart[0];
        for (int64_t g = rstart[0]; g < rstart[nrows]; ++g)
            if (cols[g] < 0 || cols[g] >= ncols) return fail(ctx, "column %d out of range [0, %lld)", cols[g], (long long)ncols);
    }
    if (ntok == 0) return 0;
    // dev_vals: `vals` is device memory, slot g at vals + g * vstride (the range check runs in
    // k_fmt_row_len); host values are packed (vstride = nm), checked here and copied
    if (dev_vals && ragged) return fail(ctx, "device values are rectangular blocks");
    if (dev_vals && vstride < nm) return fail(ctx, "value stride %lld below the metric count", (long long)vstride);
    const int64_t vs = dev_vals ? vstride : nm;
    const double* v0 = ragged ? vals + rstart[0] * nm : vals;
    const int64_t nv = ntok * nm;
    const double lim = std::ldexp(1.0, 63) / (double)pow10_u64(decimals);
    if (!dev_vals)
        for (int64_t k = 0; k < nv; ++k)
            if (std::isfinite(v0[k]) && !(std::fabs(v0[k]) < lim))
                return fail(ctx, "value %g too large for fixed-point text with %d decimals", v0[k], decimals);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t fst = st_in ? st_in : ctx->stream;
    // chunks of FMT_BLOCK tokens per row (format_kernels.hpp): nch per row, nrows * nch workgroups
    int64_t max_nt = ncols;
    if (ragged) {
        max_nt = 0;
        for (int64_t r = 0; r < nrows; ++r) max_nt = std::max(max_nt, rstart[r + 1] - rstart[r]);
    }
    const int64_t nch = std::max<int64_t>(1, (max_nt + FMT_BLOCK - 1) / FMT_BLOCK), nblk = nrows * nch;
    if (nblk >= ((int64_t)1 << 31)) return fail(ctx, "text block too large (%lld chunks)", (long long)nblk);
    const int64_t rp = row_offs[nrows] - row_offs[0];
    const int64_t cp = mode != 1 ? col_offs[ncols] - col_offs[0] : 0;
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const int64_t rs_b = sm ? sm->rsuf_offs[2 * nrows] - sm->rsuf_offs[0] : 0;
    const int64_t cs_b = sm ? sm->csuf_offs[2 * ncols] - sm->csuf_offs[0] : 0;
    const int64_t lab_b = sm ? sm->lab_offs[5] - sm->lab_offs[0] : 0;
    const size_t b_vals = dev_vals ? 0 : al(nv * 8), b_roffs = al((nrows + 1) * 8), b_coffs = al((ncols + 1) * 8),
                 b_rpre = al(rp + 1), b_cpre = al(cp + 1), b_miss = al(missing_len + 1), b_len = al(nblk * 8),
                 b_rst = ragged ? al((nrows + 1) * 8) : 0, b_cols = ragged ? al(ntok * 4) : 0,
                 b_rsuf = sm ? al(rs_b + 1) + al((2 * nrows + 1) * 8) + al(2 * nrows * 4) : 0,
                 b_csuf = sm ? al(cs_b + 1) + al((2 * ncols + 1) * 8) + al(2 * ncols * 4) : 0,
                 b_lab = sm ? al(lab_b + 1) + al(6 * 8) : 0;
    const size_t fixed = b_vals + b_roffs + b_coffs + b_rpre + b_cpre + b_miss + 2 * b_len + b_rst + b_cols +
                         b_rsuf + b_csuf + b_lab;
    if (ensure(ctx, &ctx->d_fmt, &ctx->d_fmt_bytes, fixed)) return -1;
    char* base = (char*)ctx->d_fmt;
    const double* d_vals = dev_vals ? vals : (const double*)base;
    int64_t* d_roffs = (int64_t*)(base + b_vals);
    int64_t* d_coffs = (int64_t*)((char*)d_roffs + b_roffs);
    uint8_t* d_rpre = (uint8_t*)d_coffs + b_coffs;
    uint8_t* d_cpre = d_rpre + b_rpre;
    uint8_t* d_miss = d_cpre + b_cpre;
    int64_t* d_rlen = (int64_t*)(d_miss + b_miss);
    int64_t* d_rbase = (int64_t*)((char*)d_rlen + b_len);
    int64_t* d_rst = ragged ? (int64_t*)((char*)d_rbase + b_len) : nullptr;
    int32_t* d_cols = ragged ? (int32_t*)((char*)d_rbase + b_len + b_rst) : nullptr;
    char* sbase = (char*)d_rbase + b_len + b_rst + b_cols;  // summary extras
    std::vector<int64_t> roffs(nrows + 1), coffs(mode != 1 ? ncols + 1 : 1, 0), rst(ragged ? nrows + 1 : 0);
    for (int64_t r = 0; r <= nrows; ++r) roffs[r] = row_offs[r] - row_offs[0];
    if (mode != 1)
        for (int64_t c = 0; c <= ncols; ++c) coffs[c] = col_offs[c] - col_offs[0];
    uint8_t *d_rsuf = nullptr, *d_csuf = nullptr, *d_lab = nullptr;
    int64_t *d_rsoffs = nullptr, *d_csoffs = nullptr, *d_laboffs = nullptr;
    int32_t *d_rcode = nullptr, *d_ccode = nullptr;
    std::vector<int64_t> rso, cso, lo;
    if (sm) {
        d_rsuf = (uint8_t*)sbase;
        d_rsoffs = (int64_t*)(sbase + al(rs_b + 1));
        d_rcode = (int32_t*)((char*)d_rsoffs + al((2 * nrows + 1) * 8));
        sbase += b_rsuf;
        d_csuf = (uint8_t*)sbase;
        d_csoffs = (int64_t*)(sbase + al(cs_b + 1));
        d_ccode = (int32_t*)((char*)d_csoffs + al((2 * ncols + 1) * 8));
        sbase += b_csuf;
        d_lab = (uint8_t*)sbase;
        d_laboffs = (int64_t*)(sbase + al(lab_b + 1));
        rso.resize(2 * nrows + 1);
        cso.resize(2 * ncols + 1);
        lo.resize(6);
        for (int64_t k = 0; k <= 2 * nrows; ++k) rso[k] = sm->rsuf_offs[k] - sm->rsuf_offs[0];
        for (int64_t k = 0; k <= 2 * ncols; ++k) cso[k] = sm->csuf_offs[k] - sm->csuf_offs[0];
        for (int k = 0; k < 6; ++k) lo[k] = sm->lab_offs[k] - sm->lab_offs[0];
        if (rs_b) HIP_TRY(ctx, hipMemcpyAsync(d_rsuf, sm->rsuf + sm->rsuf_offs[0], rs_b, hipMemcpyHostToDevice, fst));
        if (cs_b) HIP_TRY(ctx, hipMemcpyAsync(d_csuf, sm->csuf + sm->csuf_offs[0], cs_b, hipMemcpyHostToDevice, fst));
        if (lab_b) HIP_TRY(ctx, hipMemcpyAsync(d_lab, sm->lab + sm->lab_offs[0], lab_b, hipMemcpyHostToDevice, fst));
        HIP_TRY(ctx, hipMemcpyAsync(d_rsoffs, rso.data(), rso.size() * 8, hipMemcpyHostToDevice, fst));
        HIP_TRY(ctx, hipMemcpyAsync(d_csoffs, cso.data(), cso.size() * 8, hipMemcpyHostToDevice, fst));
        HIP_TRY(ctx, hipMemcpyAsync(d_laboffs, lo.data(), 6 * 8, hipMemcpyHostToDevice, fst));
        HIP_TRY(ctx, hipMemcpyAsync(d_rcode, sm->rcode, 2 * nrows * 4, hipMemcpyHostToDevice, fst));
        HIP_TRY(ctx, hipMemcpyAsync(d_ccode, sm->ccode, 2 * ncols * 4, hipMemcpyHostToDevice, fst));
    }
    if (ragged) {
        for (int64_t r = 0; r <= nrows; ++r) rst[r] = rstart[r] - rstart[0];
        HIP_TRY(ctx, hipMemcpyAsync(d_rst, rst.data(), (nrows + 1) * 8, hipMemcpyHostToDevice, fst));
        HIP_TRY(ctx, hipMemcpyAsync(d_cols, cols + rstart[0], ntok * 4, hipMemcpyHostToDevice, fst));
    }
    if (!dev_vals) HIP_TRY(ctx, hipMemcpyAsync((double*)d_vals, v0, nv * 8, hipMemcpyHostToDevice, fst));
    HIP_TRY(ctx, hipMemcpyAsync(d_roffs, roffs.data(), (nrows + 1) * 8, hipMemcpyHostToDevice, fst));
    if (rp) HIP_TRY(ctx, hipMemcpyAsync(d_rpre, row_pre + row_offs[0], rp, hipMemcpyHostToDevice, fst));
    if (mode != 1) {
        HIP_TRY(ctx, hipMemcpyAsync(d_coffs, coffs.data(), (ncols + 1) * 8, hipMemcpyHostToDevice, fst));
        if (cp) HIP_TRY(ctx, hipMemcpyAsync(d_cpre, col_pre + col_offs[0], cp, hipMemcpyHostToDevice, fst));
    }
    if (missing_len) HIP_TRY(ctx, hipMemcpyAsync(d_miss, missing, missing_len, hipMemcpyHostToDevice, fst));
    FmtArgs a{mode, d_vals, nrows, ncols, nm, decimals, d_rpre, d_roffs, d_cpre, d_coffs, d_miss, missing_len,
              d_rst, d_cols, d_rsuf, d_rsoffs, d_csuf, d_csoffs, d_rcode, d_ccode, sm ? sm->has_g : 0,
              sm ? sm->has_s : 0, d_lab, d_laboffs, vs, lim};
    hipLaunchKernelGGL(k_fmt_row_len, dim3((unsigned)nblk), dim3(FMT_BLOCK), 0, fst, a, (int)nch, d_rlen);
    HIP_TRY(ctx, hipGetLastError());
    std::vector<int64_t> rlen(nblk), rbase(nblk);
    HIP_TRY(ctx, hipMemcpyAsync(rlen.data(), d_rlen, nblk * 8, hipMemcpyDeviceToHost, fst));
    HIP_TRY(ctx, hipStreamSynchronize(fst));
    int64_t total = 0;
    for (int64_t b = 0; b < nblk; ++b) {
        if (rlen[b] >= FMT_OVERSIZE)
            return fail(ctx, "a value of row %lld is too large for fixed-point text with %d decimals",
                        (long long)(b / nch), decimals);
        rbase[b] = total;
        total += rlen[b];
    }
    *out_len = total;
    if (total > cap) return 1;  // caller retries with a buffer of *out_len bytes
    if (!out) return fail(ctx, "null output buffer");
    char* mapped = host_mapped(out);
    if (!mapped && ensure(ctx, &ctx->d_out, &ctx->d_out_bytes, (size_t)total + 1)) return -1;
    HIP_TRY(ctx, hipMemcpyAsync(d_rbase, rbase.data(), nblk * 8, hipMemcpyHostToDevice, fst));
    hipLaunchKernelGGL(k_fmt_rows, dim3((unsigned)nblk), dim3(FMT_BLOCK), 0, fst, a, (int)nch, d_rbase,
                       mapped ? mapped : (char*)ctx->d_out);
    HIP_TRY(ctx, hipGetLastError());
    if (!mapped) HIP_TRY(ctx, hipMemcpyAsync(out, ctx->d_out, total, hipMemcpyDeviceToHost, fst));
    HIP_TRY(ctx, hipStreamSynchronize(fst));
    return 0;
}

extern "C" {

namespace {
// Both pair-text entry points: ids to the device, per-row lengths, host prefix, the text, D2H.
int format_pairs_impl(taxi2_ctx* ctx, int64_t nrows, int64_t ncols, PairFmtArgs a, const uint8_t* row_ids,
                      const int64_t* row_offs, const uint8_t* col_ids, const int64_t* col_offs, uint8_t* out,
                      int64_t out_cap, int64_t* out_len, hipStream_t st) {
    const int64_t rb = row_offs[nrows] - row_offs[0], cb = col_offs[ncols] - col_offs[0];
    const int64_t nch = (ncols + FMT_BLOCK - 1) / FMT_BLOCK, nblk = nrows * nch;  // FMT_BLOCK-column chunks
    if (nblk >= ((int64_t)1 << 31)) return fail(ctx, "pair text block too large (%lld chunks)", (long long)nblk);
    auto al = [](size_t v) { return (v + 255) / 256 * 256; };
    const size_t o_ro = 0, o_co = o_ro + al((size_t)(nrows + 1) * 8), o_rid = o_co + al((size_t)(ncols + 1) * 8);
    const size_t o_cid = o_rid + al((size_t)rb + 1), o_len = o_cid + al((size_t)cb + 1);
    const size_t o_base = o_len + al((size_t)nblk * 8), fixed = o_base + al((size_t)nblk * 8);
    if (ensure(ctx, &ctx->d_fmt, &ctx->d_fmt_bytes, fixed)) return -1;
    char* b = (char*)ctx->d_fmt;
    std::vector<int64_t> ro(nrows + 1), co(ncols + 1);
    for (int64_t r = 0; r <= nrows; ++r) ro[r] = row_offs[r] - row_offs[0];
    for (int64_t c = 0; c <= ncols; ++c) co[c] = col_offs[c] - col_offs[0];
    HIP_TRY(ctx, hipMemcpyAsync(b + o_ro, ro.data(), (nrows + 1) * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(ctx, hipMemcpyAsync(b + o_co, co.data(), (ncols + 1) * 8, hipMemcpyHostToDevice, st));
    if (rb) HIP_TRY(ctx, hipMemcpyAsync(b + o_rid, row_ids + row_offs[0], rb, hipMemcpyHostToDevice, st));
    if (cb) HIP_TRY(ctx, hipMemcpyAsync(b + o_cid, col_ids + col_offs[0], cb, hipMemcpyHostToDevice, st));
    a.ncols = ncols;
    a.rid = (const uint8_t*)(b + o_rid);
    a.roffs = (const int64_t*)(b + o_ro);
    a.cid = (const uint8_t*)(b + o_cid);
    a.coffs = (const int64_t*)(b + o_co);
    int64_t* d_rlen = (int64_t*)(b + o_len);
    int64_t* d_rbase = (int64_t*)(b + o_base);
    hipLaunchKernelGGL(k_pairs_row_len, dim3((unsigned)nblk), dim3(FMT_BLOCK), 0, st, a, (int)nch, d_rlen);
    HIP_TRY(ctx, hipGetLastError());
    std::vector<int64_t> rlen(nblk), rbase(nblk);
    HIP_TRY(ctx, hipMemcpyAsync(rlen.data(), d_rlen, nblk * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(ctx, hipStreamSynchronize(st));
    int64_t total = 0;
    for (int64_t b = 0; b < nblk; ++b) {
        rbase[b] = total;
        total += rlen[b];
    }
    *out_len = total;
    if (total > out_cap) return 1;  // caller retries with a buffer of *out_len bytes
    if (!out) return fail(ctx, "null output buffer");
    char* mapped = host_mapped(out);
    // text_copy 1 / 2: the text kernel writes HBM (its byte stores at every pair's unaligned ends
    // stay on the device) and one linear copy moves it: the DMA engine (no CUs), or a copy kernel
    // of 16-byte stores from a 16-aligned destination (only the last partial word by bytes)
    const int mode = mapped ? (ctx->text_copy == 2 && ((uintptr_t)mapped & 15u) ? 1 : ctx->text_copy) : 1;
    if (mode && ensure(ctx, &ctx->d_out, &ctx->d_out_bytes, (size_t)total + 16)) return -1;
    HIP_TRY(ctx, hipMemcpyAsync(d_rbase, rbase.data(), nblk * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_pairs_text, dim3((unsigned)nblk), dim3(FMT_BLOCK), 0, st, a, (int)nch, d_rbase,
                       mode ? (char*)ctx->d_out : mapped);
    HIP_TRY(ctx, hipGetLastError());
    if (mode == 1) {
        HIP_TRY(ctx, hipMemcpyAsync(out, ctx->d_out, total, hipMemcpyDeviceToHost, st));
    } else if (mode == 2) {
        const int64_t n16 = total >> 4;
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n16 + 255) / 256, 1024));
        hipLaunchKernelGGL(k_copy_text, dim3((unsigned)blocks), dim3(256), 0, st, (const char*)ctx->d_out, mapped, total);
        HIP_TRY(ctx, hipGetLastError());
    }
    HIP_TRY(ctx, hipStreamSynchronize(st));
    return 0;
}
}  // namespace

int taxi2_format_pairs_dev(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1, int32_t cap,
                           const uint8_t* d_sx, const uint8_t* d_sy, const int32_t* d_slen, const uint8_t* row_ids,
                           const int64_t* row_offs, const uint8_t* col_ids, const int64_t* col_offs, int first,
                           uint8_t* out, int64_t out_cap, int64_t* out_len, void* stream) {
    if (!ctx) return -1;
    DevSet* Q = get_set(ctx, set_q);
    DevSet* R = get_set(ctx, set_r);
    if (!Q || !R) return fail(ctx, "unknown set");
    if (q0 < 0 || q1 < q0 || q1 > Q->n) return fail(ctx, "query range out of bounds");
    if (!out_len || !row_offs || !col_offs) return fail(ctx, "null argument");
    const int64_t nrows = q1 - q0, ncols = R->n;
    *out_len = 0;
    if (nrows == 0 || ncols == 0) return 0;
    if (!d_sx || !d_sy || !d_slen) return fail(ctx, "null string slots");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    PairFmtArgs a{d_sx, d_sy, d_slen, (int64_t)cap, Q->meta + q0, R->meta, ncols, nullptr, nullptr, nullptr, nullptr,
                  first ? 1 : 0};
    return format_pairs_impl(ctx, nrows, ncols, a, row_ids, row_offs, col_ids, col_offs, out, out_cap, out_len, st);
}

int taxi2_format_pairs_ptr_dev(taxi2_ctx* ctx, int64_t nrows, int64_t ncols, const uint64_t* d_px,
                               const uint64_t* d_py, const int32_t* d_slen, const uint8_t* row_ids,
                               const int64_t* row_offs, const uint8_t* col_ids, const int64_t* col_offs, int first,
                               uint8_t* out, int64_t out_cap, int64_t* out_len, void* stream) {
    if (!ctx) return -1;
    if (nrows < 0 || ncols < 0) return fail(ctx, "negative size");
    if (!out_len || !row_offs || !col_offs) return fail(ctx, "null argument");
    *out_len = 0;
    if (nrows == 0 || ncols == 0) return 0;
    if (!d_px || !d_py || !d_slen) return fail(ctx, "null string pointers");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    PairFmtArgs a{nullptr, nullptr, d_slen, 0, nullptr, nullptr, ncols, nullptr, nullptr, nullptr, nullptr,
                  first ? 1 : 0, d_px, d_py};
    return format_pairs_impl(ctx, nrows, ncols, a, row_ids, row_offs, col_ids, col_offs, out, out_cap, out_len, st);
}

int taxi2_pack_slots_dev(taxi2_ctx* ctx, const uint8_t* d_sx, const uint8_t* d_sy, const int32_t* d_slen, int64_t cap,
                         int nslot, int slot, const int64_t* d_end, const int64_t* d_off, int64_t count, uint8_t* d_dx,
                         uint8_t* d_dy, void* stream) {
    if (!ctx) return -1;
    if (count < 0 || cap <= 0 || nslot < 1 || slot < 0 || slot >= nslot) return fail(ctx, "bad slot arguments");
    if (count == 0) return 0;
    if (!d_sx || !d_sy || !d_slen || !d_end || !d_off || !d_dx || !d_dy) return fail(ctx, "null device argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    const int64_t blocks = std::min<int64_t>((count + 3) / 4, (int64_t)ctx->num_cus * 32);
    hipLaunchKernelGGL(k_pack_slots, dim3((unsigned)blocks), dim3(256), 0, st, d_sx, d_sy, d_slen, cap, nslot, slot, d_end,
                       d_off, count, d_dx, d_dy);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int taxi2_stream_create_cus(taxi2_ctx* ctx, int cu_first, int cu_count, void** out_stream) {
    if (!ctx) return -1;
    if (!out_stream) return fail(ctx, "null output stream");
    *out_stream = nullptr;
    if (cu_first < 0 || cu_count < 1 || cu_first + cu_count > ctx->num_cus)
        return fail(ctx, "CU range [%d, %d) outside the device's %d CUs", cu_first, cu_first + cu_count, ctx->num_cus);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    std::vector<uint32_t> mask((ctx->num_cus + 31) / 32, 0u);
    for (int c = cu_first; c < cu_first + cu_count; ++c) mask[c >> 5] |= 1u << (c & 31);
    hipStream_t s = nullptr;
    HIP_TRY(ctx, hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    *out_stream = (void*)s;
    return 0;
}

int taxi2_stream_destroy(taxi2_ctx* ctx, void* stream) {
    if (!ctx) return -1;
    if (!stream) return 0;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(ctx, hipStreamDestroy((hipStream_t)stream));
    return 0;
}

int taxi2_num_cus(taxi2_ctx* ctx) { return ctx ? ctx->num_cus : -1; }

int taxi2_copy_text_dev(taxi2_ctx* ctx, const uint8_t* d_src, uint8_t* h_dst, int64_t nbytes, void* stream) {
    if (!ctx) return -1;
    if (nbytes < 0) return fail(ctx, "negative size");
    if (nbytes == 0) return 0;
    if (!d_src || !h_dst) return fail(ctx, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    char* mapped = host_mapped(h_dst);
    if (!mapped) return fail(ctx, "taxi2_copy_text_dev: the destination is not pinned host memory");
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    const int64_t n16 = nbytes >> 4;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n16 + 255) / 256, 1024));
    if (((uintptr_t)mapped & 15u) || ((uintptr_t)d_src & 15u)) {  // the 16-byte copy needs both aligned
        HIP_TRY(ctx, hipMemcpyAsync(h_dst, d_src, (size_t)nbytes, hipMemcpyDeviceToHost, st));
        return 0;
    }
    hipLaunchKernelGGL(k_copy_text, dim3((unsigned)blocks), dim3(256), 0, st, (const char*)d_src, mapped, nbytes);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int taxi2_set_text_copy(taxi2_ctx* ctx, int mode) {
    if (!ctx) return -1;
    if (mode < 0 || mode > 2) return fail(ctx, "text copy mode %d (0 kernel stores, 1 DMA, 2 copy kernel)", mode);
    ctx->text_copy = mode;
    return 0;
}

int taxi2_format_pairs_ptr_async(taxi2_ctx* ctx, int64_t nrows, int64_t ncols, const uint64_t* d_px,
                                 const uint64_t* d_py, const int32_t* d_slen, const uint8_t* d_row_ids,
                                 const int64_t* d_row_offs, const uint8_t* d_col_ids, const int64_t* d_col_offs,
                                 int first, uint8_t* d_text, int64_t text_cap, int64_t* d_total,
                                 int64_t* d_scratch, void* stream) {
    if (!ctx) return -1;
    if (nrows < 0 || ncols < 0) return fail(ctx, "negative size");
    if (!d_total || !d_scratch) return fail(ctx, "null total / scratch");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    if (nrows == 0 || ncols == 0) {
        HIP_TRY(ctx, hipMemsetAsync(d_total, 0, 8, st));
        return 0;
    }
    if (!d_px || !d_py || !d_slen || !d_row_ids || !d_row_offs || !d_col_ids || !d_col_offs || !d_text)
        return fail(ctx, "null device argument");
    // row lengths and bases in the caller's scratch (2 nrows int64: no context buffer that could be
    // regrown -- hipFree synchronises the whole device -- while another stream runs); ids and
    // offsets are device arrays the caller keeps: row offsets relative to d_row_ids, column
    // offsets to d_col_ids
    const int64_t nch = (ncols + FMT_BLOCK - 1) / FMT_BLOCK, nblk = nrows * nch;  // FMT_BLOCK-column chunks
    if (nblk >= ((int64_t)1 << 31)) return fail(ctx, "pair text block too large (%lld chunks)", (long long)nblk);
    int64_t* d_rlen = d_scratch;
    int64_t* d_rbase = d_rlen + nblk;
    PairFmtArgs a{nullptr, nullptr, d_slen, 0, nullptr, nullptr, ncols, d_row_ids, d_row_offs, d_col_ids, d_col_offs,
                  first ? 1 : 0, d_px, d_py};
    hipLaunchKernelGGL(k_pairs_row_len, dim3((unsigned)nblk), dim3(FMT_BLOCK), 0, st, a, (int)nch, d_rlen);
    HIP_TRY(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_pairs_row_base, dim3(1), dim3(FMT_BLOCK), 0, st, (const int64_t*)d_rlen, nblk, text_cap,
                       d_rbase, d_total);
    HIP_TRY(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_pairs_text, dim3((unsigned)nblk), dim3(FMT_BLOCK), 0, st, a, (int)nch, (const int64_t*)d_rbase,
                       (char*)d_text, (const int64_t*)d_total);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int taxi2_format_rows(taxi2_ctx* ctx, int mode, const double* vals, int64_t nrows, int64_t ncols, int nm,
                      const uint8_t* row_pre, const int64_t* row_offs, const uint8_t* col_pre,
                      const int64_t* col_offs, int decimals, const uint8_t* missing, int32_t missing_len,
                      uint8_t* out, int64_t cap, int64_t* out_len) {
    return format_impl(ctx, mode, vals, nrows, ncols, nm, nullptr, nullptr, row_pre, row_offs, col_pre, col_offs,
                       decimals, missing, missing_len, out, cap, out_len);
}

int taxi2_format_ragged(taxi2_ctx* ctx, int mode, const double* vals, int64_t nrows, const int64_t* row_start,
                        const int32_t* cols, int64_t ncols, int nm, const uint8_t* row_pre, const int64_t* row_offs,
                        const uint8_t* col_pre, const int64_t* col_offs, int decimals, const uint8_t* missing,
                        int32_t missing_len, uint8_t* out, int64_t cap, int64_t* out_len) {
    if (ctx && nrows > 0 && !row_start) return fail(ctx, "null row starts");
    return format_impl(ctx, mode, vals, nrows, ncols, nm, row_start, cols, row_pre, row_offs, col_pre, col_offs,
                       decimals, missing, missing_len, out, cap, out_len);
}

int taxi2_format_summary(taxi2_ctx* ctx, const double* vals, int64_t nrows, int64_t ncols, int nm,
                         const uint8_t* row_pre, const int64_t* row_offs, const uint8_t* col_pre,
                         const int64_t* col_offs, const uint8_t* row_suf, const int64_t* row_suf_offs,
                         const uint8_t* col_suf, const int64_t* col_suf_offs, const int32_t* row_codes,
                         const int32_t* col_codes, int has_genera, int has_species, const uint8_t* labels,
                         const int64_t* label_offs, int decimals, const uint8_t* missing, int32_t missing_len,
                         uint8_t* out, int64_t cap, int64_t* out_len) {
    const SummaryHost sm{row_suf, row_suf_offs, col_suf, col_suf_offs, row_codes, col_codes,
                         has_genera ? 1 : 0, has_species ? 1 : 0, labels, label_offs};
    return format_impl(ctx, 2, vals, nrows, ncols, nm, nullptr, nullptr, row_pre, row_offs, col_pre, col_offs,
                       decimals, missing, missing_len, out, cap, out_len, &sm);
}

int taxi2_format_rows_dev(taxi2_ctx* ctx, int mode, const double* d_vals, int64_t vstride, int64_t nrows,
                          int64_t ncols, int nm, const uint8_t* row_pre, const int64_t* row_offs, const uint8_t* col_pre,
                          const int64_t* col_offs, int decimals, const uint8_t* missing, int32_t missing_len,
                          uint8_t* out, int64_t cap, int64_t* out_len, void* stream) {
    return format_impl(ctx, mode, d_vals, nrows, ncols, nm, nullptr, nullptr, row_pre, row_offs, col_pre, col_offs,
                       decimals, missing, missing_len, out, cap, out_len, nullptr, true, vstride, (hipStream_t)stream);
}

int taxi2_format_summary_dev(taxi2_ctx* ctx, const double* d_vals, int64_t vstride, int64_t nrows, int64_t ncols,
                             int nm, const uint8_t* row_pre, const int64_t* row_offs, const uint8_t* col_pre,
                             const int64_t* col_offs, const uint8_t* row_suf, const int64_t* row_suf_offs,
                             const uint8_t* col_suf, const int64_t* col_suf_offs, const int32_t* row_codes,
                             const int32_t* col_codes, int has_genera, int has_species, const uint8_t* labels,
                             const int64_t* label_offs, int decimals, const uint8_t* missing, int32_t missing_len,
                             uint8_t* out, int64_t cap, int64_t* out_len, void* stream) {
    const SummaryHost sm{row_suf, row_suf_offs, col_suf, col_suf_offs, row_codes, col_codes,
                         has_genera ? 1 : 0, has_species ? 1 : 0, labels, label_offs};
    return format_impl(ctx, 2, d_vals, nrows, ncols, nm, nullptr, nullptr, row_pre, row_offs, col_pre, col_offs,
                       decimals, missing, missing_len, out, cap, out_len, &sm, true, vstride, (hipStream_t)stream);
}

int taxi2_subset_aggregate_dev(taxi2_ctx* ctx, const double* d_vals, int64_t nrows, int64_t ncols, int m,
                               const int32_t* d_row_code, const int64_t* d_col_start, const int32_t* d_col_idx,
                               int32_t ns, int init, double* d_sum, double* d_min, double* d_max, int64_t* d_count,
                               const int64_t* d_col_nat, void* d_scratch, int64_t scratch_bytes, void* stream) {
    if (!ctx) return -1;
    if (nrows < 0 || ncols < 0 || m < 1 || ns < 0) return fail(ctx, "invalid sizes to taxi2_subset_aggregate_dev");
    const int64_t nk = (int64_t)ns * ns * m;
    if (nk == 0) return 0;
    if (!d_sum || !d_min || !d_max || !d_count || !d_col_start || (nrows > 0 && (!d_vals || !d_row_code)) ||
        (ncols > 0 && !d_col_idx))
        return fail(ctx, "null pointer passed to taxi2_subset_aggregate_dev");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    if (init) {
        const int64_t blocks = std::min<int64_t>((nk + 255) / 256, (int64_t)ctx->num_cus * 32);
        hipLaunchKernelGGL(k_subset_init, dim3((unsigned)blocks), dim3(256), 0, st, nk, d_sum, d_min, d_max, d_count);
        HIP_TRY(ctx, hipGetLastError());
    }
    if (nrows == 0) return 0;
    // exact parallel summation (subset_kernels.hpp), rows in sub-blocks whose row partials fit
    // ~256 MB of scratch (and the groups' LDS sort), in ascending order on one stream; each row's
    // subsets in chunks of SUB_CH columns (tmax bounds the chunks per row: sum of ceil(size / CH))
    const int64_t per_row = (int64_t)ns * m;
    // few subsets: natural-order rows (k_subset_rows_nat), ns x nch chunk slots per row
    const int64_t nch = std::max<int64_t>(1, (ncols + SUB_CH - 1) / SUB_CH);
    const bool nat = ns <= 4 && !test_env("TAXI2_SUB_GATHER");
    const int64_t tmax64 = nat ? (int64_t)ns * nch : (int64_t)ns + (ncols + SUB_CH - 1) / SUB_CH;
    if (tmax64 > INT32_MAX / 2) return fail(ctx, "taxi2_subset_aggregate_dev: too many subsets");
    const int tmax = (int)tmax64;
    const int64_t row_bytes = per_row * (int64_t)(sizeof(SubPart) + sizeof(SubWork)) + tmax64 * m * (int64_t)sizeof(SubPart);
    // the row sub-block fits ~256 MB, or the caller's scratch (its per-block arrays: partials, work,
    // chunk partials, 3 ints per row; fixed: offsets, chunk map, column codes, 10 x 256 B of alignment)
    int64_t budget = (int64_t)256 << 20;
    if (d_scratch) {
        const int64_t fixed = (int64_t)(ns + 1) * 4 + (int64_t)tmax * 4 + (nat ? ncols : 0) + 1 + 4 + 10 * 256;
        budget = std::min<int64_t>(budget, scratch_bytes - fixed);
    }
    const int64_t rows_fit = budget / (row_bytes + 12);
    if (d_scratch && rows_fit < 1)
        return fail(ctx, "taxi2_subset_aggregate_dev: scratch of %lld bytes holds no row (%lld per row)",
                    (long long)scratch_bytes, (long long)(row_bytes + 12));
    const int64_t rows_per = std::max<int64_t>(1, std::min<int64_t>(SUB_MAX_ROWS, rows_fit));
    const int64_t rsub = std::min(rows_per, nrows);
    auto al = [](size_t v) { return (v + 255) / 256 * 256; };
    const size_t o_part = 0, o_work = al((size_t)rsub * per_row * sizeof(SubPart));
    const size_t o_cpart = o_work + al((size_t)rsub * per_row * sizeof(SubWork));
    const size_t o_cofs = o_cpart + al((size_t)rsub * tmax * m * sizeof(SubPart));
    const size_t o_t2b = o_cofs + al((size_t)(ns + 1) * 4);
    const size_t o_ccode = o_t2b + al((size_t)tmax * 4);
    const size_t o_rows = o_ccode + al((size_t)(nat ? ncols : 0) + 1);
    const size_t o_code = o_rows + al((size_t)rsub * 4), o_start = o_code + al((size_t)rsub * 4);
    const size_t o_n = o_start + al((size_t)(rsub + 1) * 4), total = o_n + 256;
    char* base;
    if (d_scratch) {  // the caller's scratch: aggregations of several partitions on several streams
        if (scratch_bytes < (int64_t)total)
            return fail(ctx, "taxi2_subset_aggregate_dev: scratch of %lld bytes, %lld needed", (long long)scratch_bytes,
                        (long long)total);
        base = (char*)d_scratch;
    } else {
        if (ensure(ctx, &ctx->d_sub, &ctx->d_sub_bytes, total)) return -1;
        base = (char*)ctx->d_sub;
    }
    SubPart* part = (SubPart*)(base + o_part);
    SubWork* work = (SubWork*)(base + o_work);
    SubPart* cpart = (SubPart*)(base + o_cpart);
    int32_t* cofs = (int32_t*)(base + o_cofs);
    int32_t* grows = (int32_t*)(base + o_rows);
    int32_t* gcode = (int32_t*)(base + o_code);
    int32_t* gstart = (int32_t*)(base + o_start);
    int32_t* ngrp = (int32_t*)(base + o_n);
    unsigned int* wcount = (unsigned int*)(base + o_n + 64);
    uint8_t* ccode = (uint8_t*)(base + o_ccode);
    int32_t* t2b = (int32_t*)(base + o_t2b);
    if (nat) {  // cofs[b] = b * nch, on the device (no host staging, no synchronisation)
        hipLaunchKernelGGL(k_subset_natcofs, dim3(1), dim3(64), 0, st, (int)ns, (int)nch, cofs);
        if (ncols > 0)
            hipLaunchKernelGGL(k_subset_colcode, dim3((unsigned)((ncols + 255) / 256)), dim3(256), 0, st, d_col_start,
                               d_col_idx, (int)ns, ncols, ccode);
    } else {
        hipLaunchKernelGGL(k_subset_cofs, dim3(1), dim3(1024), 0, st, d_col_start, (int)ns, cofs);
        hipLaunchKernelGGL(k_subset_t2b, dim3((unsigned)((std::max<int64_t>(tmax, ns) + 255) / 256)), dim3(256), 0, st,
                           (const int32_t*)cofs, (int)ns, tmax, t2b);
    }
    HIP_TRY(ctx, hipGetLastError());
    for (int64_t r0 = 0; r0 < nrows; r0 += rsub) {
        const int64_t nr = std::min(rsub, nrows - r0);
        const double* v = d_vals + r0 * ncols * m;
        const int32_t* rc = d_row_code + r0;
        hipLaunchKernelGGL(k_subset_groups, dim3(1), dim3(1024), 0, st, rc, (int)nr, grows, gcode, gstart, ngrp);
        HIP_TRY(ctx, hipGetLastError());
        if (nat) {
            const dim3 g((unsigned)((nr * nch + 3) / 4)), b(256);
            if (ns <= 2)
                hipLaunchKernelGGL(k_subset_rows_nat<2>, g, b, 0, st, v, nr, ncols, m, rc, (const uint8_t*)ccode, (int)ns,
                                   (int)nch, (const double*)d_sum, cpart, d_col_nat);
            else
                hipLaunchKernelGGL(k_subset_rows_nat<4>, g, b, 0, st, v, nr, ncols, m, rc, (const uint8_t*)ccode, (int)ns,
                                   (int)nch, (const double*)d_sum, cpart, d_col_nat);
        } else {
            hipLaunchKernelGGL(k_subset_rows, dim3((unsigned)((nr * tmax + 3) / 4)), dim3(256), 0, st, v, nr, ncols, m,
                               rc, d_col_start, d_col_idx, (int)ns, (const int32_t*)cofs, tmax, (const double*)d_sum,
                               cpart, (const int32_t*)t2b);
        }
        HIP_TRY(ctx, hipGetLastError());
        hipLaunchKernelGGL(k_subset_rowmerge, dim3((unsigned)((nr * per_row + 255) / 256)), dim3(256), 0, st, nr,
                           (int)ns, m, (const int32_t*)cofs, tmax, (const SubPart*)cpart, part);
        HIP_TRY(ctx, hipGetLastError());
        HIP_TRY(ctx, hipMemsetAsync(wcount, 0, 4, st));
        hipLaunchKernelGGL(k_subset_combine, dim3((unsigned)((nr * per_row + 255) / 256)), dim3(256), 0, st, nr,
                           (int)ns, m, (const int32_t*)ngrp, (const int32_t*)gcode, (const int32_t*)gstart,
                           (const int32_t*)grows, (const SubPart*)part, d_sum, d_min, d_max, d_count, work, wcount);
        HIP_TRY(ctx, hipGetLastError());
        hipLaunchKernelGGL(k_subset_fixup, dim3((unsigned)(ctx->num_cus * 8)), dim3(256), 0, st, v, ncols, m, (int)ns,
                           d_col_start, d_col_idx, (const int32_t*)gstart, (const int32_t*)grows,
                           (const SubPart*)part, (const SubWork*)work, (const unsigned int*)wcount, d_sum);
        HIP_TRY(ctx, hipGetLastError());
    }
    return 0;
}

int taxi2_format_subset_stats(int64_t ns, int m, const double* mean, const double* mn, const double* mx,
                              const int64_t* count, const uint8_t* names, const int64_t* name_offs, int decimals,
                              int part, uint8_t* out, int64_t cap, int64_t* out_len, int threads) {
    if (ns < 0 || m < 1 || decimals < 0 || decimals > FMT_MAX_DECIMALS || !out_len || part < 0 || part >= 2 + m)
        return -1;
    if (ns > 0 && (!mean || !mn || !mx || !count || !names || !name_offs)) return -1;
    // one token: Python "{:.Nf}" of a finite value, "NA" otherwise (subsets._text)
    auto tok = [&](double v, std::string& o) {
        if (!std::isfinite(v)) {
            o += "NA";
            return;
        }
        char b[400];
        const int L = fmt_fixed(v, decimals, b);
        o.append(b, (size_t)L);
    };
    auto name = [&](int64_t a, std::string& o) {
        o.append((const char*)names + name_offs[a], (size_t)(name_offs[a + 1] - name_offs[a]));
    };
    // rows of the part: pairs (a != b), identity (a == b), or the matricial rows of metric part - 2
    const int64_t nrows = part == 0 ? ns * ns : ns;
    if (threads <= 0) threads = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, std::max<int64_t>(1, nrows / 1024)));
    std::vector<std::string> chunk((size_t)threads);
    auto work = [&](int t) {
        std::string& o = chunk[(size_t)t];
        const int64_t r0 = nrows * t / threads, r1 = nrows * (t + 1) / threads;
        for (int64_t r = r0; r < r1; ++r) {
            if (part == 0 || part == 1) {
                const int64_t a = part == 0 ? r / ns : r, b = part == 0 ? r % ns : r;
                if (part == 0 && a == b) continue;
                name(a, o);
                if (part == 0) {
                    o += '\t';
                    name(b, o);
                }
                const int64_t q = (a * ns + b) * m;
                for (int k = 0; k < m; ++k) {
                    o += '\t';
                    tok(mean[q + k], o);
                    o += '\t';
                    tok(mn[q + k], o);
                    o += '\t';
                    tok(mx[q + k], o);
                }
            } else {
                const int k = part - 2;
                name(r, o);
                for (int64_t b = 0; b < ns; ++b) {
                    const int64_t q = (r * ns + b) * m + k;
                    o += '\t';
                    if (!count[q]) {
                        o += "NA";
                        continue;
                    }
                    tok(mean[q], o);
                    o += " (";
                    tok(mn[q], o);
                    o += '-';
                    tok(mx[q], o);
                    o += ')';
                }
            }
            o += '\n';
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    int64_t total = 0;
    for (const auto& c : chunk) total += (int64_t)c.size();
    *out_len = total;
    if (total > cap) return 1;
    int64_t o = 0;
    for (const auto& c : chunk) {
        std::memcpy(out + o, c.data(), c.size());
        o += (int64_t)c.size();
    }
    return 0;
}

int taxi2_subset_aggregate(const double* d, int64_t n, int m, const int32_t* code, int32_t ns, double* sum,
                           double* mn, double* mx, int64_t* count, int threads) {
    if (n < 0 || m < 1 || ns < 0 || (n > 0 && (!d || !code || !sum || !mn || !mx || !count))) return -1;
    for (int64_t i = 0; i < n; ++i)
        if (code[i] < 0 || code[i] >= ns) return -3;
    const int64_t nk = (int64_t)ns * ns * m;
    for (int64_t k = 0; k < nk; ++k) {  // SimpleAggregator.__init__
        sum[k] = 0.0;
        mn[k] = std::numeric_limits<double>::infinity();
        mx[k] = 0.0;
        count[k] = 0;
    }
    if (threads <= 0) threads = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, ns));
    // Worker t owns the keys whose x subset a has a % threads == t, and visits its rows in ascending
    // x, each row in ascending y: every key sees its values in the reference's x-major order.
    auto work = [&](int t) {
        for (int64_t x = 0; x < n; ++x) {
            const int64_t a = code[x];
            if (a % threads != t) continue;
            const double* row = d + x * n * m;
            for (int64_t y = 0; y < n; ++y) {
                const int64_t base = (a * ns + code[y]) * m;
                for (int k = 0; k < m; ++k) {
                    const double v = row[y * m + k];
                    if (!std::isfinite(v)) continue;  // None
                    const int64_t q = base + k;
                    sum[q] += v;
                    if (v < mn[q]) mn[q] = v;
                    if (v > mx[q]) mx[q] = v;
                    ++count[q];
                }
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    return 0;
}

int taxi2_dereplicate_walk(const double* d, int64_t n, const int64_t* id, const int64_t* len, double similarity,
                           int64_t* row_kept, int32_t* kept_cols, int64_t kept_cap, int64_t* n_kept,
                           int64_t* line_idx, double* line_d, int64_t line_cap, int64_t* n_lines,
                           uint8_t* excluded) {
    if (n < 0 || !n_kept || !n_lines || (n > 0 && (!d || !id || !len || !row_kept || !excluded))) return -1;
    if (n > INT32_MAX) return -2;
    for (int64_t i = 0; i < n; ++i)
        if (id[i] < 0 || id[i] >= n) return -3;
    std::vector<uint8_t> ex((size_t)n, 0);  // by id code
    const double nan = std::numeric_limits<double>::quiet_NaN();
    int64_t nk = 0, nl = 0;
    int64_t gcode = -1, gq = -1, best = -1;  // current group: id code, query row, longest member
    double bestd = nan;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t xi = id[i];
        int64_t kept_i = 0;
        for (int64_t j = 0; j < n && !ex[xi]; ++j) {  // an excluded x drops the rest of its row
            const int64_t yj = id[j];
            if (yj == xi || ex[yj]) continue;
            if (nk < kept_cap) kept_cols[nk] = (int32_t)j;
            ++nk;
            ++kept_i;
            const double v = d[i * n + j];
            const bool defined = std::isfinite(v);
            if (gq < 0 || gcode != xi) {  // groupby(id_x): a new run of equal query ids
                gcode = xi;
                gq = i;
                best = i;
                bestd = defined ? v : nan;
            }
            if (!(defined && v <= similarity)) continue;
            const bool longer = len[j] > len[best];
            const int64_t inc = longer ? j : best, exc = longer ? best : j;
            const double incd = longer ? v : bestd, excd = longer ? bestd : v;
            ex[id[exc]] = 1;
            if (nl < line_cap) {
                line_idx[nl * 3] = gq;
                line_idx[nl * 3 + 1] = inc;
                line_idx[nl * 3 + 2] = exc;
                line_d[nl * 2] = incd;
                line_d[nl * 2 + 1] = excd;
            }
            ++nl;
            if (longer) {
                best = j;
                bestd = v;
            }
        }
        row_kept[i] = kept_i;
    }
    for (int64_t i = 0; i < n; ++i) excluded[i] = ex[id[i]];
    *n_kept = nk;
    *n_lines = nl;
    return (nk > kept_cap || nl > line_cap) ? 1 : 0;
}

}  // extern "C"
