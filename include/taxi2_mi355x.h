/*
 * taxi2_mi355x.h -- C ABI of the MI355X all-pairs genetic-distance engine.
 *
 * Drop-in boundary for the TaxI2 versusAll / versusReference hot path.  Today the
 * reference crosses into native code once per pair and per metric, with the GIL held:
 *
 *   Biopython (C)  PairwiseAligner(**Scores).align(x, y)[0]
 *                  src/itaxotools/taxi2/align.py:75, 151-157   (via versus_all.py:527-533,
 *                  versus_reference.py:100-106)
 *   calc (Rust)    seq_distances_p / _p_gaps / _jukes_cantor / _kimura2p (str, str) -> f64
 *                  src/itaxotools/taxi2/distances.py:323, 331, 339, 347
 *                  (via versus_all.py:546-552, versus_reference.py:119-129)
 *
 * This library replaces both with batched entry points: one call covers a block of
 * pairs, aligns them (when requested) and evaluates every requested metric for both
 * ordered orientations on the GPU.  Every entry point is plain C: pointers and sizes,
 * no torch or HIP types.  Bind it from Python with ctypes (taxi2_amd/_native.py), which
 * releases the GIL for the duration of each call.
 *
 * Conventions
 *   - Return value: 0 on success, < 0 on error; taxi2_last_error() describes the last
 *     error of that context.  Nothing aborts the process.
 *   - Undefined distances (0/0, log of <= 0 -- the cases the reference maps to None at
 *     distances.py:291-292) are written as NaN or +/-inf; the host wrapper maps both to None.
 *   - Ownership: the caller owns every host buffer it passes (inputs and outputs); the
 *     context owns all device memory.  *_dev entry points take device pointers that the
 *     caller allocated on the context's device, plus an optional hipStream_t (void*).
 *   - Threading: one context per device; calls on one context are serialized by the
 *     caller (the Python layer holds one context per process / GPU).  A context's device
 *     scratch (e.g. the aligner's re-run worklist) is reused by its next call, so *_dev calls
 *     on one context must be stream-ordered (same stream, or synchronized in between).
 */
#ifndef TAXI2_MI355X_H
#define TAXI2_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct taxi2_ctx taxi2_ctx;

/* align.py:17-35 Scores, same field order as Scores.defaults. */
typedef struct {
    int32_t match_score;
    int32_t mismatch_score;
    int32_t internal_open_gap_score;
    int32_t internal_extend_gap_score;
    int32_t end_open_gap_score;
    int32_t end_extend_gap_score;
} taxi2_scores;

/* distances.py:319-348 metric labels p, p-gaps, jc, k2p; distances.py:351-358 ncd.
 * TAXI2_METRIC_NCD is accepted by taxi2_all_pairs[_dev] on ALIGN sets only: NCD of the same fill's
 * aligned strings (the walkers write them, one fill per unordered pair for every metric, as
 * versus_all.py:546-552 feeds one alignment to all metrics); elsewhere use taxi2_ncd_pairs.
 * TAXI2_METRIC_COUNTS is not a metric: accepted ALONE by the pair entry points (all_pairs[_dev],
 * rect_pairs, list_pairs) for sequences of at most 32 767 bp, it writes the four column counters of
 * every ordered pair packed into its 8-byte output slot (uint64: valid | ts << 16 | tv << 32 |
 * gap << 48) -- a quarter of the bytes of four f64 metrics, and every metric is a function of them
 * (taxi2_counts_metrics_dev).  Used by the streamed versusAll (taxi2_amd/streaming.py). */
enum {
    TAXI2_METRIC_P = 0,
    TAXI2_METRIC_P_GAPS = 1,
    TAXI2_METRIC_JC = 2,
    TAXI2_METRIC_K2P = 3,
    TAXI2_METRIC_NCD = 4,
    TAXI2_METRIC_COUNTS = 16
};

/* Sequence set modes.
 *   PREALIGNED: params.pairs.align == False (versus_all.py:522-533): strings are compared
 *               column by column as given (case-insensitive ACGT, '-' gaps).
 *   ALIGN:      params.pairs.align == True: strings are the normalized sequences
 *               (sequences.py:20-25, done by the caller) and every pair is globally
 *               aligned first (Gotoh; NW when every open == extend). */
enum { TAXI2_MODE_PREALIGNED = 0, TAXI2_MODE_ALIGN = 1 };

/* ---- context ----------------------------------------------------------------------- */
int taxi2_device_count(void);
int taxi2_ctx_create(int device, taxi2_ctx** out);
void taxi2_ctx_destroy(taxi2_ctx* ctx);
const char* taxi2_last_error(const taxi2_ctx* ctx);
/* Replaces nothing in the reference; reports the build (kernel variants, arch) and ends in
 * "src:<16 hex>", the hash of the sources it was built from (taxi2_amd/srchash.py). */
const char* taxi2_version(void);

/* ---- sequence sets ------------------------------------------------------------------ *
 * Replaces the per-pair str -> Rust/C conversion of each call: the set is uploaded once
 * (raw bytes, offsets[n+1]) and packed on the GPU (per-sequence length / first / last
 * ACGT index; 2-bit + validity + gap bit-planes in PREALIGNED mode). */
int taxi2_set_create(taxi2_ctx* ctx, const uint8_t* bytes, const int64_t* offsets, int64_t n,
                     int mode, int* set_id);
int taxi2_set_destroy(taxi2_ctx* ctx, int set_id);
int taxi2_set_info(taxi2_ctx* ctx, int set_id, int64_t* n, int32_t* max_len, int* mode);

/* ---- versusAll block (versus_all.py:746-752: fromProduct -> align -> calculate) ------ *
 * Unordered pairs with linear index k in [k0, k0 + count) of the row-major upper triangle
 * of `set` (a < b; k = a*(2N-a-1)/2 + (b-a-1)).
 *   ALIGN:      out[count][2][nmetrics]: [k][0][m] = metric m of (a, b) (target a, query b),
 *               [k][1][m] = metric m of (b, a).  scores_out[count] (nullable) = the optimal
 *               global alignment score.
 *   PREALIGNED: out[count][nmetrics] (the p/p-gaps/jc/k2p counters are symmetric, so one
 *               value serves both ordered pairs); scores_out must be NULL.
 * The diagonal rule of versus_all.py:549 (x == y -> None) is the caller's business. */
int taxi2_all_pairs(taxi2_ctx* ctx, int set, int64_t k0, int64_t count, const taxi2_scores* sc,
                    const int32_t* metrics, int nmetrics, double* out, int32_t* scores_out);

/* Same with device-resident outputs (d_out / d_scores on the context's device); `stream`
 * is a hipStream_t or NULL for the context's own stream.  Asynchronous. */
int taxi2_all_pairs_dev(taxi2_ctx* ctx, int set, int64_t k0, int64_t count,
                        const taxi2_scores* sc, const int32_t* metrics, int nmetrics,
                        double* d_out, int32_t* d_scores, void* stream);

/* Metrics from TAXI2_METRIC_COUNTS slots (device buffers, asynchronous on `stream` or the context's
 * own): d_out[k][m] = scale * metric m of d_counts[k] for k < n (metrics 0..3; scale 100 is
 * versus_all.py:554-562's percentage adjustment, 1 leaves the values alone).  Bit-identical to the
 * same metrics written directly by the pair entry points. */
int taxi2_counts_metrics_dev(taxi2_ctx* ctx, const uint64_t* d_counts, int64_t n, const int32_t* metrics,
                             int nmetrics, double scale, double* d_out, void* stream);

/* ---- rectangle (versus_reference.py:225-229, decontaminate.py:336-371 shape) ---------- *
 * Pairs (q, r) for q in [q0, q1) of set_q and every r of set_r, row-major:
 *   out[(q - q0) * R + r][nmetrics] -- orientation (query, reference) only.
 * scores_out[(q - q0) * R + r] (nullable, ALIGN only). */
int taxi2_rect_pairs(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1,
                     const taxi2_scores* sc, const int32_t* metrics, int nmetrics, double* out,
                     int32_t* scores_out);

/* Same with device-resident outputs on `stream` (NULL: the context's own), asynchronous.  The
 * streamed versusAll feeds its x-major row blocks [x0, x1) x [0, N) from it in PREALIGNED mode
 * (versus_all.py:732-773 drain order; set_q == set_r), where recomputing the block is cheaper
 * than storing the triangle. */
int taxi2_rect_pairs_dev(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1,
                         const taxi2_scores* sc, const int32_t* metrics, int nmetrics, double* d_out,
                         int32_t* d_scores, void* stream);

/* A column view of PREALIGNED set `set_id`: view column c is the set's sequence d_perm[c] (device,
 * n = the set's size).  It shares the set's bit-planes (destroy it before the set) and is accepted
 * only as set_r of taxi2_rect_block_dev with the same map as d_col_nat. */
int taxi2_set_permuted(taxi2_ctx* ctx, int set_id, const int64_t* d_perm, int64_t n, int* view_id);

/* Row block of the streamed pre-aligned versusAll (versus_all.py:732-773 fed block by block, the
 * reductions of config 5): as taxi2_rect_pairs_dev on PREALIGNED sets, with the task's epilogue
 * fused -- every value x scale (percentage_multiply), NaN on x == y when diag (set_q == set_r: the
 * diagonal rule for unique full tuples, versus_all.py:549) -- and, when rmin_metric >= 0, each
 * row's first minimum of that metric over its defined values (-0.0 == 0.0, ties to the lower
 * column): d_rmin_idx[q - q0] (-1: none) and d_rmin_val[q - q0] (NaN: none).  d_col_nat (device,
 * optional): set_r is a permuted copy of set_q whose column c is the task's column d_col_nat[c] --
 * the block's columns are then stored in set_r's order (config 5: subset order, so the subset
 * aggregation reads contiguous runs) while the diagonal rule and the row minima (index and tie
 * order) follow the task's columns.  Asynchronous on `stream`; uses the context's staging buffer
 * (one call at a time per context). */
int taxi2_rect_block_dev(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1, const int32_t* metrics,
                         int nmetrics, double scale, int diag, int rmin_metric, int64_t* d_rmin_idx, double* d_rmin_val,
                         const int64_t* d_col_nat, double* d_out, void* stream);

/* ---- explicit pair list (align.py:50-51 align_pairs, distances.py:297 calculate) ------- *
 * Pairs (xs[k] of set_x, ys[k] of set_y): out[count][2][nmetrics] in ALIGN mode
 * ([k][0] = (x, y), [k][1] = (y, x)), out[count][nmetrics] in PREALIGNED mode. */
int taxi2_list_pairs(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys,
                     int64_t count, const taxi2_scores* sc, const int32_t* metrics, int nmetrics,
                     double* out, int32_t* scores_out);

/* ---- versusReference closest (versus_reference.py:184-188 get_minimum_distances) ------ *
 * For each query q in [q0, q1): the reference index with the smallest `scale * primary`
 * metric (NaN/inf skipped, first minimum wins, -0.0 == +0.0; scale = 100 reproduces the
 * percentage_multiply adjustment that versus_reference.py:232 applies before min()), the
 * unscaled value, and -- for that pair only -- every metric in `metrics`
 * (versus_reference.py:124-129).  idx_out[q - q0] = -1 when all values are undefined (the
 * reference raises ValueError from min() there).
 *   idx_out[nq], d_out[nq], extra_out[nq][nmetrics] (nullable),
 *   primary_out[nq][R] (nullable: the full primary matrix for the linear/matrix writers). */
int taxi2_closest(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1,
                  const taxi2_scores* sc, int32_t primary, double scale, const int32_t* metrics,
                  int nmetrics, int64_t* idx_out, double* d_out, double* extra_out,
                  double* primary_out);

/* ---- aligned strings (align.py:151-157 Biopython.align; pairs.py:51-97 Formatted writer) -- *
 * First Biopython global alignment of (xs[k] of set_x = target, ys[k] of set_y = query), as
 * gapped strings.  Both sets must be ALIGN mode.  Outputs are right-aligned in fixed slots:
 *   out_x / out_y [count][2][cap] bytes, out_len[count][2]; slot [k][0] = alignment of
 *   (x, y); slot [k][1] (only when both != 0) = the alignment Biopython returns for (y, x),
 *   written in (x, y) column order.  The alignment of slot o occupies bytes
 *   [len(x)+len(y)-out_len[k][o], len(x)+len(y)) of its slot; cap >= len(x)+len(y) for every
 *   pair. */
int taxi2_align_strings(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys,
                        int64_t count, const taxi2_scores* sc, int both, int32_t cap, uint8_t* out_x,
                        uint8_t* out_y, int32_t* out_len);

/* Metrics (nmetrics may be 0) AND aligned strings of the rectangle's pairs from ONE fill each: the
 * packed trace-and-walk aligner's walkers write every alignment while they walk it, as
 * versus_all.py:746-750 feeds one aligned pair to both the metrics and aligned_pairs.txt.  Device
 * outputs on `stream` (asynchronous): d_out[(q - q0) * R + r][nmetrics] as taxi2_rect_pairs_dev,
 * slots d_sx / d_sy [(q - q0) * R + r][cap] (right-aligned as taxi2_align_strings' slot 0, cap >=
 * longest q + longest r) and lengths d_slen[(q - q0) * R + r].  Gotoh scores within int16, pairs up
 * to 2 048 bp (else an error: use taxi2_align_strings).  TAXI2_METRIC_NCD may be among the metrics:
 * NCD of the strings the same fill wrote (taxi2_ncd_slots_dev). */
int taxi2_rect_strings_dev(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1,
                           const taxi2_scores* sc, const int32_t* metrics, int nmetrics, double* d_out,
                           int32_t cap, uint8_t* d_sx, uint8_t* d_sy, int32_t* d_slen, void* stream);

/* Metrics and aligned strings of the unordered pairs [k0, k0 + count) of the versusAll triangle
 * (pair k = (a, b), a < b, numbered as taxi2_all_pairs) from ONE fill each: the walkers walk both
 * orientations, as the metric kernel does.  d_out[k][2][nmetrics] as taxi2_all_pairs (row (a, b),
 * then row (b, a)); slot k*2 + 0 = the alignment of (a, b), slot k*2 + 1 = the alignment Biopython
 * returns for (b, a) written in (a, b) column order (d_sx holds a's aligned string, d_sy b's), each
 * right-aligned at byte len(a) + len(b) of its cap-byte slot, lengths d_slen[k*2 + o].  Replaces
 * versus_all.py:746-750's two alignments of a pair (one per ordered pair) by one fill.  Same
 * shape limits as taxi2_rect_strings_dev; TAXI2_METRIC_NCD as there.  reserve_cus: the persistent aligner grid leaves that many
 * CUs' worth of workgroups unlaunched, so work the caller queues on another stream (the previous
 * block's text) finds room to run beside it; 0 = the whole GPU. */
int taxi2_tri_strings_dev(taxi2_ctx* ctx, int set, int64_t k0, int64_t count, const taxi2_scores* sc,
                          const int32_t* metrics, int nmetrics, double* d_out, int32_t cap, uint8_t* d_sx,
                          uint8_t* d_sy, int32_t* d_slen, int reserve_cus, void* stream);

/* aligned_pairs.txt text (pairs.py:51-97 SequencePairHandler.Formatted) of the rectangle rows
 * [q0, q1) x every r from taxi2_rect_strings_dev slots (device): per pair "idx / idy" LF, the
 * aligned x, the pattern ('|' equal non-gap, '-' gap, '.' mismatch), the aligned y, each LF-ended;
 * pairs separated by one LF, none before pair (q0, 0) when `first`.  Ids: concatenated bytes +
 * offsets (rows: [q1 - q0 + 1], columns: [R + 1]).  Writes out[0, *out_len) on the host; returns 1
 * without writing when out_cap < *out_len (retry with that capacity; the slots stay valid). */
int taxi2_format_pairs_dev(taxi2_ctx* ctx, int set_q, int set_r, int64_t q0, int64_t q1, int32_t cap,
                           const uint8_t* d_sx, const uint8_t* d_sy, const int32_t* d_slen,
                           const uint8_t* row_ids, const int64_t* row_offs, const uint8_t* col_ids,
                           const int64_t* col_offs, int first, uint8_t* out, int64_t out_cap,
                           int64_t* out_len, void* stream);

/* Same text from per-pair string pointers: pair (r, c) of the nrows x ncols block (row-major k =
 * r * ncols + c) shows the d_slen[k] bytes at device addresses d_px[k] (first line) and d_py[k]
 * (third line) -- e.g. taxi2_tri_strings_dev slots of this block and strings kept from earlier
 * blocks' fills (the (b, a) orientation of a pair filled with row a). */
int taxi2_format_pairs_ptr_dev(taxi2_ctx* ctx, int64_t nrows, int64_t ncols, const uint64_t* d_px,
                               const uint64_t* d_py, const int32_t* d_slen, const uint8_t* row_ids,
                               const int64_t* row_offs, const uint8_t* col_ids, const int64_t* col_offs, int first,
                               uint8_t* out, int64_t out_cap, int64_t* out_len, void* stream);

/* ---- NCD (distances.py:351-358 NCD._calculate -> alfpy 1.0.6 ncd.Distance) ---------------- *
 * NCD(x, y) = (C(X+Y) - min(C(X), C(Y))) / max(C(X), C(Y)), X / Y = upper-cased strings,
 * C(s) = len(zlib.compress(s)) with zlib 1.2.11 level 6 (computed exactly on the GPU).
 * For each pair k: out[k*no] = value of the ordered pair (x, y) and, when both != 0 (no = 2),
 * out[k*2+1] = value of (y, x).  With scores (ALIGN sets): x, y are the first Biopython
 * alignment's gapped strings of that ordered pair, as VersusAll feeds them to the metric
 * (versus_all.py:532, 546-552); scores == NULL: the sequences as stored.  Any length: the
 * length accounts for every deflate block and every slide of zlib's 64 KiB window
 * (deflate_len.hpp); bytes are compressed as given (the Python layer hands UTF-8). */
int taxi2_ncd_pairs(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys,
                    int64_t count, const taxi2_scores* sc, int both, double* out);

/* Asynchronous form of taxi2_format_pairs_ptr_dev for pipelines: every input is a device array
 * (ids as concatenated bytes with offsets relative to those bytes), the text goes to the device
 * buffer d_text, and d_total[0] = its length, d_total[1] = 1 if it fit text_cap (else nothing is
 * written: call again with a larger buffer); d_scratch: 2 nrows ceil(ncols / 256) int64 of device
 * scratch (per-chunk lengths and offsets, 256 columns a chunk).  Nothing
 * synchronises the host or the device: the caller copies d_text[0, d_total[0]) out when the stream
 * reaches it. */
int taxi2_format_pairs_ptr_async(taxi2_ctx* ctx, int64_t nrows, int64_t ncols, const uint64_t* d_px,
                                 const uint64_t* d_py, const int32_t* d_slen, const uint8_t* d_row_ids,
                                 const int64_t* d_row_offs, const uint8_t* d_col_ids, const int64_t* d_col_offs,
                                 int first, uint8_t* d_text, int64_t text_cap, int64_t* d_total,
                                 int64_t* d_scratch, void* stream);

/* Compaction of walker string slots (taxi2_tri_strings_dev / taxi2_rect_strings_dev output):
 * pair k's string of orientation `slot` -- the last d_slen[k * nslot + slot] bytes before byte
 * d_end[k] of slot k * nslot + slot (cap bytes each) -- is copied to d_dx / d_dy + d_off[k], for
 * both aligned strings.  Asynchronous on `stream`.  (The (b, a) strings kept for a later row
 * block of aligned_pairs.txt, versus_all.py:746-750.) */
int taxi2_pack_slots_dev(taxi2_ctx* ctx, const uint8_t* d_sx, const uint8_t* d_sy, const int32_t* d_slen, int64_t cap,
                         int nslot, int slot, const int64_t* d_end, const int64_t* d_off, int64_t count, uint8_t* d_dx,
                         uint8_t* d_dy, void* stream);

/* A stream of the context's device whose kernels run only on compute units
 * [cu_first, cu_first + cu_count) (hipExtStreamCreateWithCUMask; logical CU numbers, which the
 * driver stripes over the XCDs).  Two such streams over disjoint ranges keep a persistent fill
 * launch and the text kernels of the task pipeline on separate CUs (versus_all.py:746-769: the
 * aligned_pairs.txt writer beside the alignments) instead of sharing every CU's issue slots.
 * *out_stream receives the hipStream_t; destroy it with taxi2_stream_destroy. */
int taxi2_stream_create_cus(taxi2_ctx* ctx, int cu_first, int cu_count, void** out_stream);
int taxi2_stream_destroy(taxi2_ctx* ctx, void* stream);
/* Number of compute units of the context's device. */
int taxi2_num_cus(taxi2_ctx* ctx);
/* How the pair-text entry points (taxi2_format_pairs_dev / _ptr_dev) move the text into a pinned
 * host buffer: 0 = the text kernel stores straight into it (default), 1 = the text kernel writes
 * device memory and one DMA copy moves it (no CUs), 2 = the same with a 16-byte copy kernel.  The
 * text bytes are identical in every mode. */
int taxi2_set_text_copy(taxi2_ctx* ctx, int mode);
/* d_src[0, nbytes) (device) -> h_dst (pinned host memory), asynchronous on `stream`: a copy kernel of
 * 16-byte stores (the rate of kernel stores over the host link, beside a running fill), or the DMA
 * engine when either side is not 16-byte aligned.  The task pipeline's text transfer
 * (versus_all.py:746-750, aligned_pairs.txt). */
int taxi2_copy_text_dev(taxi2_ctx* ctx, const uint8_t* d_src, uint8_t* h_dst, int64_t nbytes, void* stream);

/* NCD of aligned-string slots already on the device -- taxi2_tri_strings_dev (nslot 2) or
 * taxi2_rect_strings_dev (nslot 1) output: pair k's alignment of orientation o is the last
 * d_slen[k * nslot + o] bytes before byte d_end[k] of slot k * nslot + o (cap bytes each).
 * Orientation 0 is the ordered pair (x = d_sx string, y = d_sy string); orientation 1 (no = 2,
 * nslot 2) the alignment of (b, a) stored in (a, b) column order, whose metric sees (d_sy, d_sx).
 * d_out[k * no + o] = NCD (distances.py:351-358) of that ordered pair.  max_len: the longest
 * sequence of the pairs (sizes the deflate working set; any aligned string is at most twice it);
 * latin1: some byte >= 0x80 (compressed as its UTF-8 upper case).  Asynchronous on `stream`; uses
 * the context's NCD staging: a call on another stream than the context's previous device work is
 * ordered behind that work (no two streams use the staging at once). */
int taxi2_ncd_slots_dev(taxi2_ctx* ctx, const uint8_t* d_sx, const uint8_t* d_sy, const int32_t* d_slen, int64_t cap,
                        int nslot, int no, const int64_t* d_end, int64_t count, int32_t max_len, int latin1,
                        double* d_out, void* stream);

/* ---- compressed length (alfpy ncd.complexity) --------------------------------------------- *
 * out[k] = len(zlib.compress(upper(x[xs[k]]) + upper(y[ys[k]]))), zlib 1.2.11 level 6;
 * ys == NULL compresses x[xs[k]] alone.  Any length. */
int taxi2_zlib_lengths(taxi2_ctx* ctx, int set_x, int set_y, const int64_t* xs, const int64_t* ys,
                       int64_t count, int32_t* out);

/* ---- writer text (distances.py:59-279 DistanceHandler.Linear[.WithExtras] / .Matrix) ------- *
 * Text rows of a float table vals[nrows][ncols][nm] (host, f64; NaN/inf -> `missing`), every
 * value as Python "%.{decimals}f" % v (= "{:.Nf}".format(v): correctly rounded, ties to even,
 * "-0.0000" kept); |v| * 10^decimals < 2^63 for finite v.
 *   mode 0 (linear): per row r, per column c:  row_pre[r] TAB col_pre[c] (TAB value){nm} LF
 *   mode 1 (matrix): per row r:                row_pre[r] (TAB value[r][c]){ncols} LF   (nm = 1)
 * row_pre / col_pre: concatenated UTF-8 bytes, offsets [n + 1].  Writes out[0, *out_len);
 * returns 1 without writing when cap < *out_len (retry with that capacity). */
int taxi2_format_rows(taxi2_ctx* ctx, int mode, const double* vals, int64_t nrows, int64_t ncols, int nm,
                      const uint8_t* row_pre, const int64_t* row_offs, const uint8_t* col_pre,
                      const int64_t* col_offs, int decimals, const uint8_t* missing, int32_t missing_len,
                      uint8_t* out, int64_t cap, int64_t* out_len);

/* Same text for ragged rows (dereplicate.py:255-287 writers fed only the pairs that survive
 * drop_excluded_pairs): row r holds tokens g in [row_start[r], row_start[r+1]) with column
 * cols[g] in [0, ncols) and values vals[g][nm] (indices absolute, row_start[0] may be > 0).  Linear:
 * row_pre[r] TAB col_pre[cols[g]] (TAB value){nm} LF per token; matrix: row_pre[r] (TAB value)* LF,
 * nothing for an empty row. */
int taxi2_format_ragged(taxi2_ctx* ctx, int mode, const double* vals, int64_t nrows, const int64_t* row_start,
                        const int32_t* cols, int64_t ncols, int nm, const uint8_t* row_pre, const int64_t* row_offs,
                        const uint8_t* col_pre, const int64_t* col_offs, int decimals, const uint8_t* missing,
                        int32_t missing_len, uint8_t* out, int64_t cap, int64_t* out_len);

/* ---- versusAll summary.tsv text (versus_all.py:278-350 SummaryHandler, fed at :754-768) ----- *
 * One line per ordered pair (r, c) of vals[nrows][ncols][nm] (host, f64, NaN/inf -> missing):
 *   row_pre[r] TAB col_pre[c] (TAB value){nm} row_suf[2r] col_suf[2c] row_suf[2r+1] col_suf[2c+1]
 *   TAB label LF
 * where row_suf / col_suf are 2 strings per row / column (offsets [2n + 1]) that carry their own
 * leading TABs (entry 2k: "\t" + extras values; entry 2k+1: "\tgenus\tspecies"), and label is
 * labels[k] (offsets [6]: "no info", "intra-species", "inter-species", "intra-genus",
 * "inter-genus") for k = SubsetDistance.get_comparison_type (versus_all.py:255-271) of
 * (genus equal?, species equal?) from row_codes / col_codes [n][2] = (genus code, species code)
 * -- equal code <=> same subset (a sequence missing from a partition gets a code of its own that
 * equals every other missing one: None == None) -- or None when has_genera / has_species is 0.
 * Values as in taxi2_format_rows; returns 1 when cap < *out_len. */
int taxi2_format_summary(taxi2_ctx* ctx, const double* vals, int64_t nrows, int64_t ncols, int nm,
                         const uint8_t* row_pre, const int64_t* row_offs, const uint8_t* col_pre,
                         const int64_t* col_offs, const uint8_t* row_suf, const int64_t* row_suf_offs,
                         const uint8_t* col_suf, const int64_t* col_suf_offs, const int32_t* row_codes,
                         const int32_t* col_codes, int has_genera, int has_species, const uint8_t* labels,
                         const int64_t* label_offs, int decimals, const uint8_t* missing, int32_t missing_len,
                         uint8_t* out, int64_t cap, int64_t* out_len);

/* taxi2_format_rows / taxi2_format_summary on values already in device memory (a row block the
 * engine produced, e.g. versusAll's adjusted rows): value slot g = r * ncols + c starts at
 * d_vals + g * vstride (vstride >= nm doubles: a metric's column of a wider block is d_vals + m with
 * vstride = the block's metric count), so the writers' values never cross the host link.  The
 * fixed-point range check runs on the device (a row with a larger finite value fails the call);
 * `stream` orders the reads after the values' producer (NULL: the context's stream).  Blocks the
 * caller until the text is in `out` (pinned host memory is written directly by the kernel). */
int taxi2_format_rows_dev(taxi2_ctx* ctx, int mode, const double* d_vals, int64_t vstride, int64_t nrows,
                          int64_t ncols, int nm, const uint8_t* row_pre, const int64_t* row_offs, const uint8_t* col_pre,
                          const int64_t* col_offs, int decimals, const uint8_t* missing, int32_t missing_len,
                          uint8_t* out, int64_t cap, int64_t* out_len, void* stream);
int taxi2_format_summary_dev(taxi2_ctx* ctx, const double* d_vals, int64_t vstride, int64_t nrows, int64_t ncols,
                             int nm, const uint8_t* row_pre, const int64_t* row_offs, const uint8_t* col_pre,
                             const int64_t* col_offs, const uint8_t* row_suf, const int64_t* row_suf_offs,
                             const uint8_t* col_suf, const int64_t* col_suf_offs, const int32_t* row_codes,
                             const int32_t* col_codes, int has_genera, int has_species, const uint8_t* labels,
                             const int64_t* label_offs, int decimals, const uint8_t* missing, int32_t missing_len,
                             uint8_t* out, int64_t cap, int64_t* out_len, void* stream);

/* Host-only (no context): the text of the subset statistics files (versus_all.py:642-684, written by
 * tasks/subsets.py write_subset_statistics) for a partition of ns subsets and m metrics, with the
 * handlers' "{:.Nf}" formatter (N = decimals) and missing text "NA".  mean / mn / mx / count are
 * [ns][ns][m] (subset of x, subset of y, metric); names: the subsets' display names, packed.
 * part 0: linear/pairs.tsv lines (a != b): name_a TAB name_b (TAB mean TAB min TAB max) per metric;
 * part 1: linear/identity.tsv lines (a == b): name_a (TAB mean TAB min TAB max) per metric;
 * part 2 + k: matricial/<metric k>.tsv rows: name_a (TAB "mean (min-max)" or "NA" when count is 0).
 * Headers are the caller's.  Returns 1 when cap < *out_len (nothing written). */
int taxi2_format_subset_stats(int64_t ns, int m, const double* mean, const double* mn, const double* mx,
                              const int64_t* count, const uint8_t* names, const int64_t* name_offs, int decimals,
                              int part, uint8_t* out, int64_t cap, int64_t* out_len, int threads);

/* ---- subset aggregation (versus_all.py:57-96 SimpleAggregator / DistanceAggregator, fed by
 * _aggregate_distances :617-640) ------------------------------------------------------------ *
 * Host-only (no context).  d[n][n][m]: the (x100-adjusted) ordered-pair values, non-finite = None;
 * code[n] in [0, ns): each sequence's subset (the partition's value, None included, numbered in
 * first-appearance order = the aggregators' key order).  For key (a, b) and metric k the values of
 * the pairs with code[x] == a, code[y] == b are accumulated in x-major order, None skipped,
 * exactly as SimpleAggregator.add: sum += v, min (from +inf), max (from 0.0), count.
 * Outputs sum / min / max / count [ns][ns][m].  threads <= 0: up to 16; keys are split by their
 * x subset, so each key's summation order is the reference's. */
int taxi2_subset_aggregate(const double* d, int64_t n, int m, const int32_t* code, int32_t ns, double* sum,
                           double* mn, double* mx, int64_t* count, int threads);

/* Same aggregation on the device, one row block at a time (the streamed versusAll,
 * taxi2_amd/streaming.py): d_vals[nrows][ncols][m] = the block's adjusted values, d_row_code[nrows]
 * the block rows' subset codes, the columns grouped by subset as a CSR (d_col_start[ns + 1],
 * d_col_idx[ncols]: each subset's columns in ascending order).  The state arrays [ns][ns][m] are
 * initialised first when init != 0, else accumulated into; blocks fed in ascending row order give
 * exactly taxi2_subset_aggregate's (= the reference's x-major) sums.  d_col_nat (optional): the block's
 * columns are stored in another order (taxi2_rect_block_dev's column map) -- d_col_idx then holds
 * stored positions and d_col_nat[c] the task's column of stored column c, which orders ties of the
 * minimum (-0.0 against 0.0).  d_scratch (optional, scratch_bytes; ~300 MB suffice): the call's working
 * memory instead of the context's, so that two partitions can be aggregated concurrently on two
 * streams.  Asynchronous on `stream`. */
int taxi2_subset_aggregate_dev(taxi2_ctx* ctx, const double* d_vals, int64_t nrows, int64_t ncols, int m,
                               const int32_t* d_row_code, const int64_t* d_col_start, const int32_t* d_col_idx,
                               int32_t ns, int init, double* d_sum, double* d_min, double* d_max, int64_t* d_count,
                               const int64_t* d_col_nat, void* d_scratch, int64_t scratch_bytes, void* stream);

/* ---- Dereplicate's greedy walk (dereplicate.py:180-196 drop_*_pairs, 289-337 find_replicates,
 * 393-425 the lazily pulled chain that interleaves them) ------------------------------------ *
 * Host-only (no context, no device): over precomputed distances d[n][n] of the ordered pairs of
 * the length-filtered sequences (x100-adjusted; non-finite = None; diagonal unused), ids as codes
 * id[n] in [0, n) (equal code <=> equal id) and unaligned lengths len[n].  Pairs are visited
 * x-major; (i, j) is kept unless id[i] == id[j] or either id is excluded at that point; runs of
 * kept pairs with equal x id form the groups of find_replicates.
 *   row_kept[n]                   kept pairs per row;
 *   kept_cols[kept_cap]           their columns, row-major (*n_kept in total);
 *   line_idx[line_cap][3]         summary lines: (query row, included row, excluded row);
 *   line_d[line_cap][2]           (included distance, excluded distance), NaN = None;
 *   excluded[n]                   1 when the sequence's id ends up excluded.
 * Returns 0; 1 when kept_cap < *n_kept or line_cap < *n_lines (outputs truncated; retry with
 * those capacities); < 0 on bad arguments (-1 null pointer / negative n, -2 n > 2^31-1,
 * -3 id code out of range). */
int taxi2_dereplicate_walk(const double* d, int64_t n, const int64_t* id, const int64_t* len, double similarity,
                           int64_t* row_kept, int32_t* kept_cols, int64_t kept_cap, int64_t* n_kept,
                           int64_t* line_idx, double* line_d, int64_t line_cap, int64_t* n_lines,
                           uint8_t* excluded);

#ifdef __cplusplus
}
#endif
#endif /* TAXI2_MI355X_H */
