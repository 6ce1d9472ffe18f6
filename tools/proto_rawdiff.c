/*
 * CPU model of the "raw difference" trace format of the packed aligner (DEF scores), used to
 * validate the walker's decode before it goes into alignt2_kernel.hpp.  Not product code.
 *
 * The fill is the kernel's arithmetic cell by cell (doubled scores, drift coordinates
 * V - (i + j) dz, G = max(M, Iy) tagged by parity (M odd, Iy even), Ix and F = max(M, Ix) kept
 * odd).  Per cell it keeps only D = Gn - Xn1 and E = Fn1 - Yn as int8 (wrapped mod 256, as the
 * kernel's byte store keeps them).  The walker decodes class, Ix formation and Iy formation from
 * the NEXT cell's (D, E) plus row / column constants, accumulates the alignment score and
 * compares it with the fill's optimum (the kernel's escape rule).
 *
 * build: gcc -O2 -shared -fPIC -o /tmp/proto_rawdiff.so tools/proto_rawdiff.c
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { ST_M = 0, ST_IX = 1, ST_IY = 2 };

static int bcode(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
    }
    return 4;
}

static void span(const char* s, int n, int* f, int* l) {
    *f = n + 1;
    *l = -1;
    for (int k = 0; k < n; k++)
        if (bcode((unsigned char)s[k]) < 4) { *f = k; break; }
    for (int k = n - 1; k >= 0; k--)
        if (bcode((unsigned char)s[k]) < 4) { *l = k; break; }
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
static int sgn(int v) { return (v > 0) - (v < 0); }

/* stats: [0] min D, [1] max D, [2] min E, [3] max E, [4] score-check failures, [5] hops */
int proto_align(const char* x, int nA, const char* y, int nB, int* out /* [2][4] */, int* stats, int wrap) {
    /* doubled default scores: match 1, mismatch -1, open -8, extend -1, end open / extend -1 */
    const int ma = 2, mi = -2, io = -16, ie = -2, eo = -2, ee = -2, dz = ie;
    const int NEG = -16384;
    int8_t* D = (int8_t*)calloc((size_t)(nA + 1) * (nB + 1), 1);
    int8_t* E = (int8_t*)calloc((size_t)(nA + 1) * (nB + 1), 1);
    int* tD = (int*)calloc((size_t)(nA + 1) * (nB + 1), sizeof(int));
    int* tE = (int*)calloc((size_t)(nA + 1) * (nB + 1), sizeof(int));
    int* G = (int*)malloc(sizeof(int) * (nB + 1));
    int* X = (int*)malloc(sizeof(int) * (nB + 1));
    for (int j = 1; j <= nB; j++) {
        G[j] = eo + ee * (j - 1) - j * dz; /* Iy(0, j), even */
        X[j] = NEG | 1;
    }
    int fin = 0;
    for (int i = 1; i <= nA; i++) {
        const int oy1 = (i == nA ? eo : io) - dz - 1;
        int F1 = eo - dz + 1; /* column-0 boundary: odd F, constant under DEF */
        int Y = NEG;
        /* diagonal of column 1 at row i: best of (i - 1, 0) | 1 */
        int d1 = (i == 1) ? 1 : ((eo - dz + 1) | 1);
        for (int j = 1; j <= nB; j++) {
            const int Gp = G[j], X1 = X[j];
            const int G1 = Gp | 1;
            const int nd1 = G1 > X1 ? G1 : X1;
            const int sM = ((x[i - 1] == y[j - 1]) ? ma : mi) - 2 * dz;
            const int M = d1 + sM;
            const int colc = (j == nB ? eo : io) - dz;
            const int cg = G1 + colc, cx = X1;
            const int Xn1 = cg > cx ? cg : cx;
            const int cf = F1 + oy1, cy = Y;
            const int Yn = cf > cy ? cf : cy;
            const int Gn = M > Yn ? M : Yn;
            const int Fn1 = M > Xn1 ? M : Xn1;
            const size_t c = (size_t)i * (nB + 1) + j;
            tD[c] = Gn - Xn1;
            tE[c] = Fn1 - Yn;
            D[c] = (int8_t)(uint8_t)(Gn - Xn1);
            E[c] = (int8_t)(uint8_t)(Fn1 - Yn);
            if (tD[c] < stats[0]) stats[0] = tD[c];
            if (tD[c] > stats[1]) stats[1] = tD[c];
            if (tE[c] < stats[2]) stats[2] = tE[c];
            if (tE[c] > stats[3]) stats[3] = tE[c];
            G[j] = Gn;
            X[j] = Xn1;
            F1 = Fn1;
            Y = Yn;
            d1 = nd1;
            if (i == nA && j == nB) fin = Gn > Xn1 ? Gn : Xn1;
        }
    }
    const int best = (fin + (nA + nB) * dz) >> 1; /* real optimum */
    int fx, lx, fy, ly;
    span(x, nA, &fx, &lx);
    span(y, nB, &fy, &ly);
    for (int prio = 0; prio < 2; prio++) {
        int i = nA + 1, j = nB + 1, st = ST_M, first = 1;
        int valid = 0, ts = 0, tv = 0, gap = 0, score = 0;
        for (;;) {
            int ni, nj;
            if (st == ST_M) {
                if (!first) {
                    const int bx = bcode((unsigned char)x[i - 1]), by = bcode((unsigned char)y[j - 1]);
                    if (bx < 4 && by < 4) {
                        ++valid;
                        const int dd = bx ^ by;
                        ts += dd == 2;
                        tv += dd != 0 && dd != 2;
                    }
                }
                ni = i - 1;
                nj = j - 1;
            } else if (st == ST_IX) {
                if (bcode((unsigned char)x[i - 1]) < 4 && j - 1 >= fy && j <= ly) ++gap;
                ni = i - 1;
                nj = j;
            } else {
                if (bcode((unsigned char)y[j - 1]) < 4 && i - 1 >= fx && i <= lx) ++gap;
                ni = i;
                nj = j - 1;
            }
            int nst;
            if (ni == 0 && nj == 0) {
                nst = -1;
            } else if (ni == 0) {
                nst = ST_IY;
            } else if (nj == 0) {
                nst = ST_IX;
            } else {
                const size_t c = (size_t)ni * (nB + 1) + nj;
                const int d = wrap ? D[c] : tD[c], e = wrap ? E[c] : tE[c];
                const int tag = !(d & 1);
                const int sa = clampi(d, -2, 1);
                const int clsM = sa == 0 || (sa == 1 && tag);
                if (st == ST_M) {
                    nst = clsM ? ST_M : sa == 1 ? ST_IY : sa == -1 ? (prio ? ST_IY : ST_IX) : ST_IX;
                } else if (st == ST_IX) {
                    const int colc = (j == nB ? eo : io) - dz;
                    const int sb = sgn(d + (1 - tag) + colc);
                    const int gp = sb > 0 || (sb == 0 && (tag || prio));
                    nst = gp ? (tag ? ST_M : ST_IY) : ST_IX;
                } else {
                    const int oy1 = (i == nA ? eo : io) - dz - 1;
                    const int sc = sgn(e + oy1);
                    const int tagF = clsM;
                    const int fp = sc > 0 || (sc == 0 && (tagF || !prio));
                    nst = fp ? (tagF ? ST_M : ST_IX) : ST_IY;
                }
            }
            /* score of the move just made (real units) */
            if (!first) {
                if (st == ST_M) {
                    score += x[i - 1] == y[j - 1] ? ma / 2 : mi / 2;
                } else if (st == ST_IX) {
                    const int end = (j == nB || j == 0);
                    score += (nst == ST_IX) ? (end ? ee : ie) / 2 : (end ? eo : io) / 2;
                } else {
                    const int end = (i == nA || i == 0);
                    score += (nst == ST_IY) ? (end ? ee : ie) / 2 : (end ? eo : io) / 2;
                }
            }
            first = 0;
            stats[5]++;
            if (nst < 0) break;
            i = ni;
            j = nj;
            st = nst;
        }
        if (score != best) stats[4]++;
        out[prio * 4 + 0] = valid;
        out[prio * 4 + 1] = ts;
        out[prio * 4 + 2] = tv;
        out[prio * 4 + 3] = gap;
    }
    free(D); free(E); free(tD); free(tE); free(G); free(X);
    return best;
}
