// Length of zlib.compress(data) (zlib 1.2.11, level -1 = 6, windowBits 15, memLevel 8, default
// strategy), computed exactly without producing the bitstream.  The NCD metric needs only
// C(s) = len(zlib.compress(s)) (alfpy 1.0.6 `ncd.complexity`, called from TaxI2
// distances.py:351-358).
//
// Restated from the DEFLATE format (RFC 1950 / 1951) and the published zlib 1.2.11 algorithm
// (deflate.c: fill_window, longest_match, deflate_slow with the level-6 configuration
// good 8 / lazy 16 / nice 128 / chain 128; trees.c: _tr_tally, build_tree with its heap order and
// depth tie-break, gen_bitlen with the length-overflow repair, scan_tree, build_bl_tree,
// _tr_flush_block's stored / fixed / dynamic choice).  Only lengths are tracked: the output size
// of one final block is 2 (zlib header) + block bytes + 4 (Adler-32).
//
// Blocks: deflate_slow flushes a block whenever _tr_tally has buffered lit_bufsize - 1 = 16 383
// symbols (literals + matches, memLevel 8), at the position zlib's FLUSH_BLOCK macros use (after
// the match's strstart++ for a match, before it for a literal), and a final block at the end; each
// block is stored, fixed or dynamic by _tr_flush_block's byte comparison, and the bits of all
// blocks are summed exactly (3-bit headers, stored blocks' byte alignment + LEN/NLEN, the final
// bi_windup).  Any length: the input streams through the 64 KiB window as fill_window moves it
// (compressed_len below).
// Pinned against Python's zlib.compress (zlib 1.2.11) by tests/test_ncd.py on random,
// low-entropy and DNA-like inputs, single- and multi-block, one window and many.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif
// The Huffman bookkeeping runs once per block.  The one-thread parse calls it out of line
// (flush_block: its own small register set, higher occupancy for that latency-bound scalar code);
// the one-wave parse (zlen_wave.hpp) inlines it (flush_block_inl), so the trees it keeps in LDS are
// addressed with LDS instructions rather than flat ones.
#define ZL_COLD __attribute__((always_inline))

namespace taxi2 {
namespace zl {

constexpr int MIN_MATCH = 3, MAX_MATCH = 258, MIN_LOOKAHEAD = MAX_MATCH + MIN_MATCH + 1;
constexpr int WSIZE = 32768, WMASK = WSIZE - 1, MAX_DIST = WSIZE - MIN_LOOKAHEAD;
constexpr int HASH_SIZE = 1 << 15, HASH_MASK = HASH_SIZE - 1, HASH_SHIFT = 5;
constexpr int GOOD = 8, LAZY = 16, NICE = 128, CHAIN = 128, TOO_FAR = 4096;
constexpr int LITERALS = 256, END_BLOCK = 256, L_CODES = 286, D_CODES = 30, BL_CODES = 19;
constexpr int HEAP_SIZE = 2 * L_CODES + 1, MAX_BITS = 15, MAX_BL_BITS = 7;
constexpr int REP_3_6 = 16, REPZ_3_10 = 17, REPZ_11_138 = 18;
constexpr int LIT_BUFSIZE = 1 << (8 + 6);  // memLevel 8
constexpr int WIN_SIZE = 2 * WSIZE, WIN_INIT = MAX_MATCH;  // s->window_size, zlib's WIN_INIT
constexpr int ZMAX_INPUT = WSIZE + MAX_DIST - 1;  // longest input the window holds without a slide
constexpr int WIN_BYTES = WIN_SIZE;

// Python's str.upper().encode() ("UTF-8") of one latin-1 character (one stored byte), as 1 or 2
// bytes: returns the first, sets `second` to the other or -1.  Non-ASCII: 0xB5 -> U+039C,
// 0xDF -> "SS", 0xFF -> U+0178, 0xE0..0xFE except 0xF7 -> minus 0x20, the rest unchanged, each
// then UTF-8 encoded (checked against Python for all 256 by tests/test_ncd.py).
__host__ __device__ __forceinline__ uint8_t upper_utf8(uint8_t c, int& second) {
    if (c < 0x80) {
        second = -1;
        return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
    }
    if (c == 0xB5) return second = 0x9C, 0xCE;
    if (c == 0xDF) return second = 'S', 'S';
    if (c == 0xFF) return second = 0xB8, 0xC5;
    const int u = (c >= 0xE0 && c != 0xF7) ? c - 0x20 : c;
    second = 0x80 | (u & 0x3F);
    return (uint8_t)(0xC0 | (u >> 6));
}

// Per-stream scratch the caller provides.  head[] must be all zero on entry; it is left all zero.
struct Scratch {
    uint8_t* win;    // WIN_BYTES (64 KiB): zlib's window
    uint16_t* prev;  // WSIZE entries (indexed pos & WMASK, as zlib's)
    uint16_t* head;  // HASH_SIZE entries
};

__host__ __device__ __forceinline__ int ilog2(uint32_t v) {
    int r = 0;
    while (v >>= 1) ++r;
    return r;
}
__host__ __device__ __forceinline__ int extra_lbits(int code) {  // length code 0..28
    return (code < 8 || code == 28) ? 0 : (code - 4) >> 2;
}
__host__ __device__ __forceinline__ int extra_dbits(int code) {  // distance code 0..29
    return code < 4 ? 0 : (code - 2) >> 1;
}
__host__ __device__ __forceinline__ int extra_blbits(int code) {
    return code == 16 ? 2 : code == 17 ? 3 : code == 18 ? 7 : 0;
}
// _length_code[lc] for lc = match length - 3 in 0..255
__host__ __device__ __forceinline__ int length_code(int lc) {
    if (lc < 8) return lc;
    if (lc == 255) return 28;
    const int e = ilog2((uint32_t)lc) - 2;
    return 4 * (e + 1) + ((lc >> e) & 3);
}
// d_code(dist) for dist = distance - 1 in 0..32767
__host__ __device__ __forceinline__ int dist_code(int d) {
    if (d < 4) return d;
    const int e = ilog2((uint32_t)d) - 1;
    return 2 * (e + 1) + ((d >> e) & 1);
}
__host__ __device__ __forceinline__ int static_llen(int n) {
    return n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8;
}

// Huffman bookkeeping for one block (trees.c).  fc = Freq, dl = Dad/Len (one union in zlib:
// gen_bitlen overwrites Dad with Len while walking the heap).
struct Trees {
    uint16_t lfc[HEAP_SIZE], ldl[HEAP_SIZE];
    uint16_t dfc[2 * D_CODES + 1], ddl[2 * D_CODES + 1];
    uint16_t bfc[2 * BL_CODES + 1], bdl[2 * BL_CODES + 1];
    int16_t heap[2 * L_CODES + 1];
    uint8_t depth[2 * L_CODES + 1];
    uint16_t bl_count[MAX_BITS + 1];
    int heap_len, heap_max;
    int64_t opt_len, static_len;
};

enum TreeKind { T_LIT = 0, T_DIST = 1, T_BL = 2 };

__host__ __device__ __forceinline__ bool smaller(const uint16_t* fc, const uint8_t* depth, int n, int m) {
    return fc[n] < fc[m] || (fc[n] == fc[m] && depth[n] <= depth[m]);
}

__host__ __device__ ZL_COLD inline void pqdownheap(Trees& t, const uint16_t* fc, int k) {
    const int v = t.heap[k];
    int j = k << 1;
    while (j <= t.heap_len) {
        if (j < t.heap_len && smaller(fc, t.depth, t.heap[j + 1], t.heap[j])) j++;
        if (smaller(fc, t.depth, v, t.heap[j])) break;
        t.heap[k] = t.heap[j];
        k = j;
        j <<= 1;
    }
    t.heap[k] = (int16_t)v;
}

__host__ __device__ ZL_COLD inline void gen_bitlen(Trees& t, int kind, uint16_t* fc, uint16_t* dl, int max_code) {
    const int max_length = kind == T_BL ? MAX_BL_BITS : MAX_BITS;
    for (int b = 0; b <= MAX_BITS; b++) t.bl_count[b] = 0;
    dl[t.heap[t.heap_max]] = 0;  // root
    int overflow = 0;
    int h;
    for (h = t.heap_max + 1; h < HEAP_SIZE; h++) {
        const int n = t.heap[h];
        int bits = dl[dl[n]] + 1;
        if (bits > max_length) bits = max_length, overflow++;
        dl[n] = (uint16_t)bits;
        if (n > max_code) continue;  // internal node
        t.bl_count[bits]++;
        int xbits = 0;
        if (kind == T_LIT) {
            if (n >= LITERALS + 1) xbits = extra_lbits(n - (LITERALS + 1));
        } else if (kind == T_DIST) {
            xbits = extra_dbits(n);
        } else {
            xbits = extra_blbits(n);
        }
        const int64_t f = fc[n];
        t.opt_len += f * (bits + xbits);
        if (kind == T_LIT) t.static_len += f * (static_llen(n) + xbits);
        else if (kind == T_DIST) t.static_len += f * (5 + xbits);
    }
    if (overflow == 0) return;
    do {
        int bits = max_length - 1;
        while (t.bl_count[bits] == 0) bits--;
        t.bl_count[bits]--;
        t.bl_count[bits + 1] += 2;
        t.bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (int bits = max_length; bits != 0; bits--) {
        int n = t.bl_count[bits];
        while (n != 0) {
            const int m = t.heap[--h];
            if (m > max_code) continue;
            if ((int)dl[m] != bits) {
                t.opt_len += ((int64_t)bits - dl[m]) * fc[m];
                dl[m] = (uint16_t)bits;
            }
            n--;
        }
    }
}

// build_tree: returns max_code.
__host__ __device__ ZL_COLD inline int build_tree(Trees& t, int kind) {
    uint16_t* fc = kind == T_LIT ? t.lfc : kind == T_DIST ? t.dfc : t.bfc;
    uint16_t* dl = kind == T_LIT ? t.ldl : kind == T_DIST ? t.ddl : t.bdl;
    const int elems = kind == T_LIT ? L_CODES : kind == T_DIST ? D_CODES : BL_CODES;
    int max_code = -1;
    t.heap_len = 0;
    t.heap_max = HEAP_SIZE;
    for (int n = 0; n < elems; n++) {
        if (fc[n] != 0) {
            t.heap[++t.heap_len] = (int16_t)(max_code = n);
            t.depth[n] = 0;
        } else {
            dl[n] = 0;
        }
    }
    while (t.heap_len < 2) {
        const int node = max_code < 2 ? ++max_code : 0;
        t.heap[++t.heap_len] = (int16_t)node;
        fc[node] = 1;
        t.depth[node] = 0;
        t.opt_len--;
        if (kind == T_LIT) t.static_len -= static_llen(node);
        else if (kind == T_DIST) t.static_len -= 5;
    }
    for (int n = t.heap_len / 2; n >= 1; n--) pqdownheap(t, fc, n);
    int node = elems;
    do {
        const int n = t.heap[1];  // pqremove
        t.heap[1] = t.heap[t.heap_len--];
        pqdownheap(t, fc, 1);
        const int m = t.heap[1];
        t.heap[--t.heap_max] = (int16_t)n;
        t.heap[--t.heap_max] = (int16_t)m;
        fc[node] = (uint16_t)(fc[n] + fc[m]);
        t.depth[node] = (uint8_t)((t.depth[n] >= t.depth[m] ? t.depth[n] : t.depth[m]) + 1);
        dl[n] = dl[m] = (uint16_t)node;
        t.heap[1] = (int16_t)node++;
        pqdownheap(t, fc, 1);
    } while (t.heap_len >= 2);
    t.heap[--t.heap_max] = t.heap[1];
    gen_bitlen(t, kind, fc, dl, max_code);
    return max_code;
}

__host__ __device__ ZL_COLD inline void scan_tree(Trees& t, uint16_t* dl, int max_code) {
    int prevlen = -1, nextlen = dl[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    dl[max_code + 1] = 0xffff;  // guard
    for (int n = 0; n <= max_code; n++) {
        const int curlen = nextlen;
        nextlen = dl[n + 1];
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            t.bfc[curlen] += (uint16_t)count;
        } else if (curlen != 0) {
            if (curlen != prevlen) t.bfc[curlen]++;
            t.bfc[REP_3_6]++;
        } else if (count <= 10) {
            t.bfc[REPZ_3_10]++;
        } else {
            t.bfc[REPZ_11_138]++;
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

// _tr_flush_block for one block of `stored_len` input bytes: adds its bits to `bits` (the
// stream's bit count so far; a stored block pads to a byte first) and, for the last block, the
// final bi_windup.  Leaves the block statistics for init_block to reset.
__host__ __device__ __forceinline__ void flush_block_inl(Trees& t, int stored_len, bool last, int64_t& bits) {
    const int lmax = build_tree(t, T_LIT);
    const int dmax = build_tree(t, T_DIST);
    scan_tree(t, t.ldl, lmax);
    scan_tree(t, t.ddl, dmax);
    build_tree(t, T_BL);
    const uint8_t bl_order[BL_CODES] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    int max_blindex;
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (t.bdl[bl_order[max_blindex]] != 0) break;
    t.opt_len += 3 * (int64_t)(max_blindex + 1) + 5 + 5 + 4;
    const int64_t dyn_b = (t.opt_len + 3 + 7) >> 3;
    const int64_t static_b = (t.static_len + 3 + 7) >> 3;
    const int64_t opt_b = static_b <= dyn_b ? static_b : dyn_b;
    if ((int64_t)stored_len + 4 <= opt_b) {  // stored: header, bi_windup, LEN, NLEN, the bytes
        bits = ((bits + 3 + 7) & ~(int64_t)7) + 32 + 8 * (int64_t)stored_len;
    } else if (static_b == opt_b) {  // fixed trees
        bits += 3 + t.static_len;
    } else {  // dynamic trees (opt_len includes the tree description)
        bits += 3 + t.opt_len;
    }
    if (last) bits = (bits + 7) & ~(int64_t)7;
}
__host__ __device__ __attribute__((noinline)) inline void flush_block(Trees& t, int stored_len, bool last, int64_t& bits) {
    flush_block_inl(t, stored_len, last, bits);
}

// init_block: empty statistics, END_BLOCK counted once.
__host__ __device__ inline void init_block(Trees& t) {
    for (int i = 0; i < L_CODES; i++) t.lfc[i] = 0;
    for (int i = 0; i < D_CODES; i++) t.dfc[i] = 0;
    for (int i = 0; i < BL_CODES; i++) t.bfc[i] = 0;
    t.lfc[END_BLOCK] = 1;
    t.opt_len = t.static_len = 0;
}

// longest_match (deflate.c) for the current position.
__host__ __device__ inline int longest_match(const uint8_t* win, const uint16_t* prev, int strstart,
                                             int lookahead, int prev_length, int cur_match, int& match_start) {
    int chain_length = CHAIN;
    const uint8_t* scan = win + strstart;
    int best_len = prev_length;
    int nice_match = NICE;
    const int limit = strstart > MAX_DIST ? strstart - MAX_DIST : 0;
    if (prev_length >= GOOD) chain_length >>= 2;
    if (nice_match > lookahead) nice_match = lookahead;
    uint8_t scan_end1 = scan[best_len - 1];
    uint8_t scan_end = scan[best_len];
    do {
        const uint8_t* match = win + cur_match;
        if (match[best_len] != scan_end || match[best_len - 1] != scan_end1 || match[0] != scan[0] ||
            match[1] != scan[1])
            continue;
        // bytes 2.. (zlib skips byte 2: equal hashes and equal bytes 0, 1 imply it)
        int len = 3;
        while (len < MAX_MATCH && scan[len] == match[len]) len++;
        if (len > best_len) {
            match_start = cur_match;
            best_len = len;
            if (len >= nice_match) break;
            scan_end1 = scan[best_len - 1];
            scan_end = scan[best_len];
        }
    } while ((cur_match = prev[cur_match & WMASK]) > limit && --chain_length != 0);
    return best_len <= lookahead ? best_len : lookahead;
}

// len(zlib.compress(upper(a[0:na]) + upper(b[0:nb]))) with level 6, for any length.
// `upper` maps a..z to A..Z (Python str.upper on the ASCII letters the sequences hold); with
// `latin1` every byte is a latin-1 character and becomes upper_utf8's bytes, i.e. the input is
// Python's (a + b).upper().encode() -- what alfpy compresses for non-ASCII text.
//
// The input streams through zlib's 64 KiB window exactly as fill_window moves it: it is read in
// as room allows, and whenever fill_window runs (lookahead < MIN_LOOKAHEAD at the top of
// deflate_slow's loop) with strstart >= WSIZE + MAX_DIST -- with or without input left -- the
// upper half moves down (the bytes past the data stay as they were: zlib zeroes WIN_INIT bytes
// past the data only up to its high-water mark, which never comes down), strstart / match_start /
// block_start drop by WSIZE and slide_hash rebases head[] and prev[] (positions below WSIZE
// become NIL = 0).  Python's zlib.compress runs deflate(Z_NO_FLUSH) over the whole input and
// then deflate(Z_FINISH) with none: the extra fill_window at that boundary is idempotent, so one
// pass with every byte available is the same parse.
__host__ __device__ inline int compressed_len(const uint8_t* a, int na, const uint8_t* b, int nb, Scratch& z,
                                              Trees& t, bool latin1 = false) {
    const int64_t n = (int64_t)na + nb;
    uint8_t* win = z.win;
    int64_t rd = 0;          // source bytes consumed
    int pend = -1;           // second byte of a two-byte character not yet in the window
    int high_water = 0;      // zlib's s->high_water
    bool slid = false;

    init_block(t);
    int64_t bits = 0;        // deflate stream bits so far (after the 2-byte zlib header)
    int block_start = 0;     // first input byte of the open block (window position; < 0 after a slide)
    int last_lit = 0;        // symbols buffered in the open block (_tr_tally's s->last_lit)

    uint32_t ins_h = 0;
    int strstart = 0, lookahead = 0;
    int match_length = MIN_MATCH - 1, prev_length, match_start = 0, prev_match;
    bool match_available = false;

    auto fill_window = [&]() {
        do {
            int more = WIN_SIZE - lookahead - strstart;
            if (strstart >= WSIZE + MAX_DIST) {
                for (int i = 0; i < WSIZE - more; i++) win[i] = win[i + WSIZE];
                match_start -= WSIZE;
                strstart -= WSIZE;
                block_start -= WSIZE;
                for (int i = 0; i < HASH_SIZE; i++) {
                    const int m = z.head[i];
                    z.head[i] = (uint16_t)(m >= WSIZE ? m - WSIZE : 0);
                }
                for (int i = 0; i < WSIZE; i++) {
                    const int m = z.prev[i];
                    z.prev[i] = (uint16_t)(m >= WSIZE ? m - WSIZE : 0);
                }
                slid = true;
                more += WSIZE;
            }
            if (rd == n && pend < 0) break;  // strm->avail_in == 0
            uint8_t* dst = win + strstart + lookahead;
            int k = 0;
            if (!latin1) {
                k = (int)(n - rd < more ? n - rd : more);
                for (int i = 0; i < k; i++, rd++) {
                    const uint8_t c = rd < na ? a[rd] : b[rd - na];
                    dst[i] = (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
                }
            } else {
                while (k < more) {
                    if (pend >= 0) {
                        dst[k++] = (uint8_t)pend;
                        pend = -1;
                        continue;
                    }
                    if (rd == n) break;
                    const uint8_t c = rd < na ? a[rd] : b[rd - na];
                    rd++;
                    dst[k++] = upper_utf8(c, pend);
                }
            }
            lookahead += k;
            if (lookahead >= MIN_MATCH)  // s->insert is 0 during the parse
                ins_h = (((uint32_t)win[strstart] << HASH_SHIFT) ^ win[strstart + 1]) & HASH_MASK;
        } while (lookahead < MIN_LOOKAHEAD && (rd != n || pend >= 0));
        if (high_water < WIN_SIZE) {  // WIN_INIT zeroing past the data
            const int curr = strstart + lookahead;
            if (high_water < curr) {
                const int init = WIN_SIZE - curr < WIN_INIT ? WIN_SIZE - curr : WIN_INIT;
                for (int i = 0; i < init; i++) win[curr + i] = 0;
                high_water = curr + init;
            } else if (high_water < curr + WIN_INIT) {
                int init = curr + WIN_INIT - high_water;
                if (init > WIN_SIZE - high_water) init = WIN_SIZE - high_water;
                for (int i = 0; i < init; i++) win[high_water + i] = 0;
                high_water += init;
            }
        }
    };
    auto insert = [&](int str) -> int {
        ins_h = ((ins_h << HASH_SHIFT) ^ win[str + (MIN_MATCH - 1)]) & HASH_MASK;
        const int head = z.head[ins_h];
        z.prev[str & WMASK] = (uint16_t)head;
        z.head[ins_h] = (uint16_t)str;
        return head;
    };
    // _tr_tally: true when the symbol buffer is full (a block must be flushed)
    auto tally_lit = [&](int c) -> bool {
        t.lfc[c]++;
        return ++last_lit == LIT_BUFSIZE - 1;
    };
    auto tally_dist = [&](int dist, int lc) -> bool {
        t.lfc[length_code(lc) + LITERALS + 1]++;
        t.dfc[dist_code(dist - 1)]++;
        return ++last_lit == LIT_BUFSIZE - 1;
    };
    auto flush = [&](bool last) {  // FLUSH_BLOCK_ONLY
        flush_block(t, strstart - block_start, last, bits);
        block_start = strstart;
        init_block(t);
        last_lit = 0;
    };

    for (;;) {
        if (lookahead < MIN_LOOKAHEAD) {
            fill_window();
            if (lookahead == 0) break;
        }
        int hash_head = 0;
        if (lookahead >= MIN_MATCH) hash_head = insert(strstart);
        prev_length = match_length;
        prev_match = match_start;
        match_length = MIN_MATCH - 1;
        if (hash_head != 0 && prev_length < LAZY && strstart - hash_head <= MAX_DIST) {
            match_length = longest_match(win, z.prev, strstart, lookahead, prev_length, hash_head, match_start);
            if (match_length <= 5 && match_length == MIN_MATCH && strstart - match_start > TOO_FAR)
                match_length = MIN_MATCH - 1;
        }
        if (prev_length >= MIN_MATCH && match_length <= prev_length) {
            const int max_insert = strstart + lookahead - MIN_MATCH;
            const bool bflush = tally_dist(strstart - 1 - prev_match, prev_length - MIN_MATCH);
            lookahead -= prev_length - 1;
            prev_length -= 2;
            do {
                if (++strstart <= max_insert) insert(strstart);
            } while (--prev_length != 0);
            match_available = false;
            match_length = MIN_MATCH - 1;
            strstart++;
            if (bflush) flush(false);
        } else if (match_available) {
            if (tally_lit(win[strstart - 1])) flush(false);
            strstart++;
            lookahead--;
        } else {
            match_available = true;
            strstart++;
            lookahead--;
        }
    }
    if (match_available) tally_lit(win[strstart - 1]);
    flush(true);

    // leave head[] all zero for the next stream
    if (slid) {
        for (int i = 0; i < HASH_SIZE; i++) z.head[i] = 0;
    } else if (strstart >= MIN_MATCH) {  // never slid: the window holds all strstart input bytes
        uint32_t h = (((uint32_t)win[0] << HASH_SHIFT) ^ win[1]) & HASH_MASK;
        for (int p = 0; p + MIN_MATCH - 1 < strstart; p++) {
            h = ((h << HASH_SHIFT) ^ win[p + 2]) & HASH_MASK;
            z.head[h] = 0;
        }
    }
    return 2 + (int)(bits >> 3) + 4;
}

}  // namespace zl
}  // namespace taxi2
