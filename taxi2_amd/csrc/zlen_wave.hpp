// Compressed length of zlib.compress(s) with ONE WAVE per stream, everything in LDS.
//
// Same result as deflate_len.hpp's compressed_len (zlib 1.2.11, level 6) -- the parse, tallies
// and block flushes are that code's -- but the two latency-bound parts are restructured:
//
// * Hash chains without head / prev tables.  deflate_slow inserts every position p <= n - 3 in
//   order, so zlib's chain from p is exactly "the earlier positions with the same 15-bit hash
//   ((b0 << 10) ^ (b1 << 5) ^ b2, masked), newest first", and hash_head = the newest of them.
//   The wave sorts the keys (hash << 16 | position) once per stream (bitonic, in LDS); candidate
//   k of a query at p is then sorted[idx(p) - 1 - k] while the hash matches: one LDS read, no
//   pointer chase.  (Inputs stay below 32 768 bytes on this path, so zlib's prev[p & WMASK]
//   aliasing never applies.)
// * longest_match evaluated for 64 candidates at once, one per lane, then reduced to what zlib's
//   sequential loop returns: the chain is cut at the first candidate <= limit (the first one, the
//   hash head, only needs to be a real position: its distance was checked by the caller); the
//   loop stops at the first candidate whose length reaches nice_match AND beats prev_length (it is
//   the first improvement to reach nice); among the candidates up to there the longest wins, the
//   earliest on ties, and only if it beats prev_length (zlib's strict `len > best_len`).  zlib's
//   quick rejects (bytes best_len - 1 / best_len, 0, 1) only skip candidates that cannot improve,
//   so comparing full lengths gives the same answer.  A second round covers candidates 64-127.
//
// Everything else is uniform across the wave (every lane runs the same parse on the same values);
// lane 0 alone owns the Huffman statistics (Trees, in LDS) and the block flushes.
#pragma once
#include "deflate_len.hpp"

namespace taxi2 {
namespace zlw {

constexpr int NMAX = 16384;  // longest stream on this path (LDS: ~7 B per byte + the trees)

#ifdef ZLW_PROF  // tools/zlw_phases.hip: s_memtime ticks per phase (window, sort, parse, flush) + counts
__device__ unsigned long long zlw_prof[8];
#define ZLW_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define ZLW_ADD(k, x) do { if (lane == 0) atomicAdd(&zlw_prof[k], (unsigned long long)(x)); } while (0)
#else
#define ZLW_T(v) (void)0
#define ZLW_ADD(k, x) (void)0
#endif

__host__ __device__ inline int pow2_at_least(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}
__host__ __device__ inline size_t al16(size_t b) { return (b + 15) / 16 * 16; }
// LDS layout for streams of at most nmax bytes: [window nmax + 274][key region][tallies], and the
// Trees overlaid on the key region.  The key region holds the (hash << 16 | position) sort keys
// (npmax = nmax - 2 inserted positions at most); after the sort it is reused as the sorted positions
// (u16, first half) and each position's sorted index (u16, second half).  The sort network never
// moves a key past npos (below), so the region is sized by the positions, not by the next power of
// two (2 050-byte streams, e.g. two 1 025-column aligned strings, would otherwise need a 4 096-key
// region).  The parse only counts symbols (the tallies: lfc[0..286) and dfc[0..30) as 158 u16
// pairs); the trees are built at a flush, and a stream shorter than LIT_BUFSIZE - 1 symbols
// flushes only at its end, after its last chain walk -- so the Trees (4.5 kB) live in the key
// region and a wave needs ~5.4 B per byte instead of ~7.4 (13 waves per CU instead of 10 at 2 kB).
// Longer streams (nmax >= LIT_BUFSIZE - 1) may flush mid-stream and keep the Trees apart.
constexpr int TAL_L = zl::L_CODES / 2, TAL_W = zl::L_CODES / 2 + zl::D_CODES / 2;
__host__ __device__ inline int npos_max(int nmax) { return nmax > 4 ? nmax - 2 : 2; }
__host__ __device__ inline bool trees_overlaid(int nmax) { return nmax < zl::LIT_BUFSIZE - 1; }
__host__ __device__ inline size_t off_keys(int nmax) { return al16((size_t)nmax + zl::MAX_MATCH + 16); }
__host__ __device__ inline size_t off_idx(int nmax) { return off_keys(nmax) + (size_t)npos_max(nmax) * 2; }
__host__ __device__ inline size_t key_bytes(int nmax) {
    const size_t k = (size_t)npos_max(nmax) * 4;
    return al16(trees_overlaid(nmax) && k < sizeof(zl::Trees) ? sizeof(zl::Trees) : k);
}
__host__ __device__ inline size_t off_tal(int nmax) { return off_keys(nmax) + key_bytes(nmax); }
__host__ __device__ inline size_t off_trees(int nmax) {
    return trees_overlaid(nmax) ? off_keys(nmax) : off_tal(nmax) + al16(TAL_W * 4);
}
__host__ __device__ inline size_t lds_bytes(int nmax) {
    return off_tal(nmax) + al16(TAL_W * 4) + (trees_overlaid(nmax) ? 0 : al16(sizeof(zl::Trees)));
}

__device__ __forceinline__ uint32_t hash3(const uint8_t* w, int p) {
    return (((uint32_t)w[p] << 10) ^ ((uint32_t)w[p + 1] << 5) ^ (uint32_t)w[p + 2]) & (uint32_t)zl::HASH_MASK;
}
// the same hash from the low three bytes of a little-endian word
__device__ __forceinline__ uint32_t hash_w(uint32_t w) {
    return (((w & 0xFFu) << 10) ^ (((w >> 8) & 0xFFu) << 5) ^ ((w >> 16) & 0xFFu)) & (uint32_t)zl::HASH_MASK;
}

// bytes w[p .. p + 3] (little-endian) from two aligned LDS words: one v_alignbyte
__device__ __forceinline__ uint32_t load4(const uint8_t* w, int p) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(w) + (p >> 2);
    return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(p & 3));
}

// Maximum of a non-negative int over the wave, uniform result: DPP butterflies within each row of 16
// lanes, then the row broadcasts (lane 63 ends with the wave's maximum) -- register-to-register
// steps only, where a bisection on ballots took nine dependent compare / ballot rounds.
__device__ __forceinline__ int wave_max_nonneg(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));   // quad_perm [1, 0, 3, 2]
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));   // quad_perm [2, 3, 0, 1]
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));  // row_mirror
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false));   // row_bcast15 (rows 1, 3)
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false));   // row_bcast31 (rows 2, 3)
    return __builtin_amdgcn_readlane(v, 63);
}

// zlib's longest_match for the query at `strstart` (see the header comment); uniform in, uniform out
__device__ __forceinline__ int coop_longest_match(const uint8_t* win, const uint16_t* spos, int i0, uint32_t h,
                                                  int strstart, int lookahead, int prev_length, int& match_start,
                                                  int lane) {
    const int chain_length = prev_length >= zl::GOOD ? zl::CHAIN >> 2 : zl::CHAIN;
    const int nice = zl::NICE < lookahead ? zl::NICE : lookahead;
    const int limit = strstart > zl::MAX_DIST ? strstart - zl::MAX_DIST : 0;
    int best = prev_length, best_pos = -1;
    for (int base = 0; base < chain_length; base += 64) {
        const int k = base + lane;
        const int idx = i0 - 1 - k;
        bool ok = k < chain_length && idx >= 0;
        int cand = 0;
        uint32_t w0 = 0;
        if (ok) {  // the chain: earlier sorted positions while the hash (from the candidate's bytes) holds
            cand = spos[idx];
            w0 = load4(win, cand);
            ok = hash_w(w0) == h && (k == 0 ? cand > 0 : cand > limit);
        }
        int len = 0;
        if (ok) {
            // common prefix, four bytes per step (the window is zero-padded past the input, as
            // zlib's; lengths are capped at MAX_MATCH as its scan loop is).  zlib examines a
            // candidate only when bytes 0 and 1 match (byte 2 then matches by the hash): a shorter
            // prefix is no candidate.
            for (;;) {  // eight bytes per step: the four word reads of a step go out together
                const uint32_t x0 = load4(win, strstart + len) ^ (len ? load4(win, cand + len) : w0);
                const uint32_t x1 = load4(win, strstart + len + 4) ^ load4(win, cand + len + 4);
                if (x0) {
                    len += __builtin_ctz(x0) >> 3;
                    break;
                }
                if (x1) {
                    len += 4 + (__builtin_ctz(x1) >> 3);
                    break;
                }
                len += 8;
                if (len >= zl::MAX_MATCH) break;
            }
            len = len < zl::MAX_MATCH ? len : zl::MAX_MATCH;
            if (len < zl::MIN_MATCH) len = 0;
        }
        const uint64_t stop = __ballot(len >= nice && len > prev_length);
        // lanes up to the stop, then the longest (earliest on ties): the wave maximum by DPP, the
        // earliest lane holding it by one ballot
        const uint64_t upto = stop ? (stop ^ (stop - 1)) : ~0ull;
        const int lv = (upto >> lane) & 1ull ? len : 0;
        const int rlen = wave_max_nonneg(lv);
        if (rlen > best) {
            best = rlen;
            best_pos = __builtin_amdgcn_readlane(cand, __builtin_ctzll(__ballot(lv == rlen)));
        }
        // the chain ends inside this round, or the loop stopped: no further rounds
        if (stop || __ballot(ok) != ~0ull) break;
    }
    if (best_pos >= 0) match_start = best_pos;
    return best <= lookahead ? best : lookahead;
}

// len(zlib.compress(upper(a) + upper(b))); n = na + nb <= nmax (the caller's LDS layout).
//
// With c_a (nb > 0): len(zlib.compress(upper(a))) too, from the same sort and a shared parse prefix.
// deflate_slow's decisions at position s read the window only below s + MAX_MATCH (the match scan,
// capped at MAX_MATCH; candidates and the inserted hashes lie below s) and its lookahead caps
// (nice_match, the returned length) bind only within MAX_MATCH of the end, so while s + MIN_LOOKAHEAD
// <= na the parse of a + b and the parse of a alone are the same sequence of states.  The parse of
// a + b snapshots its state (tallies, match state, block position) at the first step past that
// point, runs to its end, and the parse of a alone resumes from the snapshot with the window zeroed
// past na (what the one-stream form loads there).  The sorted keys of a + b serve a alone: a chain
// walks only earlier positions of the same hash, and those lie below na - 2.  NCD needs C(x) and
// C(x + y) of the same x (distances.py:351-358): one sort and ~three quarters of C(x)'s parse saved.
__device__ inline int compressed_len_wave2(const uint8_t* a, int na, const uint8_t* b, int nb, uint8_t* lds, int nmax,
                                           int lane, int* c_a) {
    using namespace zl;
    const int n = na + nb;
    uint8_t* win = lds;
    uint32_t* keys = reinterpret_cast<uint32_t*>(lds + off_keys(nmax));
    uint16_t* spos = reinterpret_cast<uint16_t*>(lds + off_keys(nmax));  // after the sort
    uint16_t* idx_of = reinterpret_cast<uint16_t*>(lds + off_idx(nmax));
    Trees& t = *reinterpret_cast<Trees*>(lds + off_trees(nmax));
    uint32_t* tal = reinterpret_cast<uint32_t*>(lds + off_tal(nmax));  // the parse's symbol counts
    // empty statistics, END_BLOCK counted once (init_block's tallies)
    auto tal_reset = [&]() {
        for (int w = lane; w < TAL_W; w += 64) tal[w] = w == END_BLOCK / 2 ? 1u : 0u;
    };
    ZLW_T(tw0);
    for (int i = lane; i < n + MAX_MATCH + 12; i += 64) {
        uint8_t c = 0;
        if (i < na) c = a[i];
        else if (i < n) c = b[i - na];
        win[i] = (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
    }
    __syncthreads();
    ZLW_T(tw1);
    ZLW_ADD(0, tw1 - tw0);
    // sorted (hash, position) keys of the inserted positions 0 .. n - 3.  Bitonic network in its
    // all-ascending form (each merge starts with a flip: i against the mirror of its block), padded
    // to P2 with virtual +inf keys: every comparator puts the minimum at the lower index, so a
    // comparator touching a pad (hi >= npos) never swaps and the pads are never stored.
    const int npos = n >= MIN_MATCH ? n - (MIN_MATCH - 1) : 0;
    const int P2 = pow2_at_least(npos > 1 ? npos : 2);
    for (int i = lane; i < npos; i += 64) keys[i] = (hash3(win, i) << 16) | (uint32_t)i;
    __syncthreads();
    for (int size = 2; size <= P2; size <<= 1) {
        for (int i = lane; i < P2 / 2; i += 64) {  // flip: lo and its mirror in the size-block
            const int half = size >> 1;
            const int lo = (i / half) * size + (i & (half - 1));
            const int hi = (lo | (size - 1)) - (i & (half - 1));
            if (hi < npos) {
                const uint32_t x = keys[lo], y = keys[hi];
                if (x > y) {
                    keys[lo] = y;
                    keys[hi] = x;
                }
            }
        }
        __syncthreads();
        for (int stride = size >> 2; stride > 0; stride >>= 1) {
            for (int i = lane; i < P2 / 2; i += 64) {
                const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));  // stride is a power of 2
                const int hi = lo + stride;
                if (hi < npos) {
                    const uint32_t x = keys[lo], y = keys[hi];
                    if (x > y) {
                        keys[lo] = y;
                        keys[hi] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    // compact the sorted keys to positions in place: chunk c writes bytes [128 c, 128 c + 128),
    // i.e. keys [32 c, 32 c + 32), all read by chunk c / 2 <= c (read, barrier, write)
    for (int base = 0; base < npos; base += 64) {
        const uint32_t kv = base + lane < npos ? keys[base + lane] : 0u;
        __syncthreads();
        if (base + lane < npos) spos[base + lane] = (uint16_t)(kv & 0xFFFFu);
        __syncthreads();
    }
    // the second half of the region is free now: sorted index of every position
    for (int i = lane; i < npos; i += 64) idx_of[spos[i]] = (uint16_t)i;
    tal_reset();
    __syncthreads();
    ZLW_T(tw2);
    ZLW_ADD(1, tw2 - tw1);

    int64_t bits = 0;
    int block_start = 0, last_lit = 0;
    int strstart = 0, lookahead = n;
    int match_length = MIN_MATCH - 1, prev_length = 0, match_start = 0, prev_match = 0;
    bool match_available = false;
    auto flush = [&](bool last) {  // FLUSH_BLOCK_ONLY: the tallies into the trees, lane 0 builds them
        __syncthreads();
        uint32_t* lw = reinterpret_cast<uint32_t*>(t.lfc);
        uint32_t* dw = reinterpret_cast<uint32_t*>(t.dfc);
        for (int w = lane; w < TAL_W; w += 64) {
            if (w < TAL_L) lw[w] = tal[w];
            else dw[w - TAL_L] = tal[w];
        }
        if (lane < BL_CODES) t.bfc[lane] = 0;
        __syncthreads();
        if (lane == 0) {
            t.opt_len = t.static_len = 0;
            flush_block_inl(t, strstart - block_start, last, bits);
        }
        bits = __shfl(bits, 0);
        block_start = strstart;
        last_lit = 0;
        tal_reset();
        __syncthreads();
    };
    // The parse's per-position LDS reads, 64 positions at a time into lane registers: lane l holds
    // for position pb + l its sorted index | hash head << 16 (pinf), its hash, and the byte before
    // it (the literal a step there tallies); the serial parse then reads them with v_readlane.
    int pb = -64;
    uint32_t pinf = 0, phash = 0, pbyte = 0;
    int nn = n;  // the stream being parsed ends here (na for a alone after the fork)
    auto prefetch = [&](int s0) {
        pb = s0;
        const int p = s0 + lane;
        uint32_t v = 0, hq = 0;
        if (p < npos) {
            const int ii = idx_of[p];
            hq = hash3(win, p);
            uint32_t hh = 0;
            if (ii > 0) {
                const uint32_t q = spos[ii - 1];
                if (hash3(win, (int)q) == hq) hh = q;
            }
            v = (uint32_t)ii | (hh << 16);
        }
        pinf = v;
        phash = hq;
        pbyte = (p >= 1 && p <= nn) ? win[p - 1] : 0u;
    };
    // tallies: no-return LDS atomics on the u16 frequency pairs (lane 0), nothing waits on them
    auto tally = [&](int word0, int c) {
        if (lane == 0) atomicAdd(tal + word0 + (c >> 1), 1u << (16 * (c & 1)));
    };
    // the fork (c_a): the state at the first step with strstart + MIN_LOOKAHEAD > na
    const bool fork = c_a != nullptr && nb > 0;
    const int fork_at = na - MIN_LOOKAHEAD;
    bool snapped = !fork;
    int64_t f_bits = 0;
    int f_block_start = 0, f_last_lit = 0, f_strstart = 0, f_match_length = MIN_MATCH - 1, f_match_start = 0;
    bool f_match_available = false;
    uint32_t f_tal[3] = {0u, 0u, 0u};  // the tallies (158 u16 pairs), three words per lane
    auto parse = [&]() {
        while (lookahead != 0) {
            if (!snapped && strstart > fork_at) {  // a alone parses the same up to here: keep the state
                snapped = true;
                __syncthreads();  // lane 0's tallies are in LDS
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int w = lane + 64 * q;
                    f_tal[q] = w < TAL_W ? tal[w] : 0u;
                }
                f_bits = bits;
                f_block_start = block_start;
                f_last_lit = last_lit;
                f_strstart = strstart;
                f_match_length = match_length;
                f_match_start = match_start;
                f_match_available = match_available;
            }
            if (strstart - pb >= 64) prefetch(strstart);
            const int sl = strstart - pb;
            int hash_head = 0, i0 = 0;
            uint32_t hq = 0;
            if (lookahead >= MIN_MATCH) {  // insert(strstart): hash_head = the newest earlier same-hash position
                const uint32_t inf = __builtin_amdgcn_readlane(pinf, sl);
                i0 = (int)(inf & 0xFFFFu);
                hash_head = (int)(inf >> 16);
                hq = __builtin_amdgcn_readlane(phash, sl);
            }
            prev_length = match_length;
            prev_match = match_start;
            match_length = MIN_MATCH - 1;
            if (hash_head != 0 && prev_length < LAZY && strstart - hash_head <= MAX_DIST) {
                match_length = coop_longest_match(win, spos, i0, hq, strstart, lookahead, prev_length, match_start, lane);
                if (match_length <= 5 && match_length == MIN_MATCH && strstart - match_start > TOO_FAR)
                    match_length = MIN_MATCH - 1;
            }
            if (prev_length >= MIN_MATCH && match_length <= prev_length) {
                tally(0, length_code(prev_length - MIN_MATCH) + LITERALS + 1);  // _tr_tally_dist
                tally(TAL_L, dist_code(strstart - 1 - prev_match - 1));
                const bool bflush = ++last_lit == LIT_BUFSIZE - 1;
                lookahead -= prev_length - 1;
                strstart += prev_length - 2;  // the match's other positions (inserted by the sort)
                match_available = false;
                match_length = MIN_MATCH - 1;
                strstart++;
                if (bflush) flush(false);
            } else if (match_available) {
                tally(0, (int)__builtin_amdgcn_readlane(pbyte, sl));
                const bool bflush = ++last_lit == LIT_BUFSIZE - 1;
                if (bflush) flush(false);
                strstart++;
                lookahead--;
            } else {
                match_available = true;
                strstart++;
                lookahead--;
            }
        }
        if (match_available) tally(0, win[strstart - 1]);  // the stream's end: the caller flushes
    };
    ZLW_T(tw3);
    parse();  // a + b, up to its final flush
    ZLW_T(tw4);
    ZLW_ADD(2, tw4 - tw3);
    auto finish = [&]() {  // the final flush: the stream's length in bytes (header, blocks, adler32)
        flush(true);
        return 2 + (int)(bits >> 3) + 4;
    };
    if (!fork) {
        const int c_ab = finish();
        if (c_a) *c_a = c_ab;  // nb == 0: a + b is a
        return c_ab;
    }
    // a + b's end state (its last block's tallies, bit count, block start) waits in registers while a
    // alone resumes from the snapshot: a's final flush builds its trees over the key region, which
    // a's parse still needs until then
    uint32_t g_tal[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int w = lane + 64 * q;
        g_tal[q] = w < TAL_W ? tal[w] : 0u;
    }
    const int64_t g_bits = bits;
    const int g_block_start = block_start, g_strstart = strstart;
    // a alone from the snapshot: the window past na as the one-stream form has it (zeros)
    if (!snapped) {  // (a + b ended before the fork point: a is too short to share anything)
        f_strstart = 0;
        f_match_length = MIN_MATCH - 1;
    }
    for (int i = na + lane; i < n + MAX_MATCH + 12; i += 64) win[i] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int w = lane + 64 * q;
        if (w < TAL_W) tal[w] = snapped ? f_tal[q] : (w == END_BLOCK / 2 ? 1u : 0u);
    }
    __syncthreads();
    bits = snapped ? f_bits : 0;
    block_start = snapped ? f_block_start : 0;
    last_lit = snapped ? f_last_lit : 0;
    strstart = f_strstart;
    lookahead = na - strstart;
    match_length = f_match_length;
    match_start = snapped ? f_match_start : 0;
    match_available = snapped && f_match_available;
    nn = na;
    pb = -64;  // the prefetched literals past na changed
    parse();
    *c_a = finish();
    // a + b's final flush
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int w = lane + 64 * q;
        if (w < TAL_W) tal[w] = g_tal[q];
    }
    bits = g_bits;
    block_start = g_block_start;
    strstart = g_strstart;
    return finish();
}

// len(zlib.compress(upper(a) + upper(b))); n = na + nb <= nmax (the caller's LDS layout).
__device__ inline int compressed_len_wave(const uint8_t* a, int na, const uint8_t* b, int nb, uint8_t* lds, int nmax,
                                          int lane) {
    return compressed_len_wave2(a, na, b, nb, lds, nmax, lane, nullptr);
}

}  // namespace zlw
}  // namespace taxi2
