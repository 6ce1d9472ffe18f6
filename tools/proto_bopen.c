/*
 * CPU model of the "best-open" fill of the packed aligner (default scores), used to validate the
 * formulation and the walker's decode before they go into alignt2_kernel.hpp.  Not product code.
 *
 * Default scores open no cheaper than they extend (io <= ie, eo <= ee), so the gap recurrences
 * may open from the cell's best state B = max(M, Ix, Iy) instead of max(M, Iy) / max(M, Ix):
 *   Ix(i, j) = max(M + o, Iy + o, Ix + e)(i-1, j) = max(B(i-1, j) + o, Ix(i-1, j) + e)   (Ix + o <= Ix + e)
 *   (Iy may likewise open from B(i, j-1); the kernel keeps Biopython's F = max(M, Ix) there)
 * and the diagonal input of the next column is B itself, so per cell the fill is
 *   M = B(i-1, j-1) + s,  X = max(B_up + co_j, X_up),  F = max(M, X),
 *   Y = max(F_left + ro_i, Y_left),  B = max(F, Y)
 * (drift coordinates V - (i + j) ie: both extends vanish, co_j / ro_i = open - ie; plain, untagged
 * scores).  The values of M, Ix and Iy are Biopython's, so the first path is decided exactly from
 * D1 = M - X and D2 = M - Y of each cell (int8: the trace bytes), whatever tie set a cell holds.
 *
 * build: gcc -O2 -shared -fPIC -o /tmp/proto_bopen.so tools/proto_bopen.c
 */
#include <stdint.h>
#include <stdlib.h>

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

static int max2(int a, int b) { return a > b ? a : b; }

/* first state in priority order (prio 0: M, Ix, Iy; prio 1: M, Iy, Ix) among those at the maximum */
static int pick(int vM, int vX, int vY, int prio) {
    const int m = max2(vM, max2(vX, vY));
    if (vM == m) return ST_M;
    if (prio == 0) return vX == m ? ST_IX : ST_IY;
    return vY == m ? ST_IY : ST_IX;
}

/* stats: [0] min D1, [1] max D1, [2] min D2, [3] max D2, [4] score-check failures, [5] hops */
int proto_align_sc(const char* x, int nA, const char* y, int nB, int* out /* [2][4] */, int* stats, int wrap,
                   const int* scv /* ma, mi, io, ie, eo, ee; NULL = TaxI2 defaults */) {
    static const int def[6] = {1, -1, -8, -1, -1, -1};
    if (!scv) scv = def;
    const int ma = scv[0], mi = scv[1], io = scv[2], ie = scv[3], eo = scv[4], ee = scv[5];
    /* drift only when every extend is the same (the default scores); otherwise plain values */
    const int dz = (ie == ee) ? ie : 0;  /* as the kernel: drift whenever one extend serves both (best-open sets) */
    const int NEG = -16384;
    int8_t* D1 = (int8_t*)calloc((size_t)(nA + 1) * (nB + 1), 1);
    int8_t* D2 = (int8_t*)calloc((size_t)(nA + 1) * (nB + 1), 1);
    int* t1 = (int*)calloc((size_t)(nA + 1) * (nB + 1), sizeof(int));
    int* t2 = (int*)calloc((size_t)(nA + 1) * (nB + 1), sizeof(int));
    int* B = (int*)malloc(sizeof(int) * (nB + 1));
    int* X = (int*)malloc(sizeof(int) * (nB + 1));
    for (int j = 1; j <= nB; j++) {
        B[j] = eo + ee * (j - 1) - j * dz; /* Iy(0, j) */
        X[j] = NEG;
    }
    int fin = 0;
    for (int i = 1; i <= nA; i++) {
        const int ro = (i == nA ? eo : io) - dz, re = (i == nA ? ee : ie) - dz;
        int Fl = eo + ee * (i - 1) - i * dz; /* Ix(i, 0) = F(i, 0) */
        int Yl = NEG;
        int d = (i == 1) ? 0 : eo + ee * (i - 2) - (i - 1) * dz; /* B(i - 1, 0) */
        for (int j = 1; j <= nB; j++) {
            const int Bu = B[j], Xu = X[j];
            const int co = (j == nB ? eo : io) - dz, ce = (j == nB ? ee : ie) - dz;
            const int M = d + ((x[i - 1] == y[j - 1]) ? ma : mi) - 2 * dz;
            const int Xn = max2(Bu + co, Xu + ce);
            const int Fn = max2(M, Xn);
            const int Yn = max2(Fl + ro, Yl + re); /* Iy opens from F = max(M, Ix) (Biopython's recurrence) */
            const int Bn = max2(Fn, Yn);
            const size_t c = (size_t)i * (nB + 1) + j;
            t1[c] = M - Xn;
            t2[c] = M - Yn;
            D1[c] = (int8_t)(uint8_t)(M - Xn);
            D2[c] = (int8_t)(uint8_t)(M - Yn);
            if (t1[c] < stats[0]) stats[0] = t1[c];
            if (t1[c] > stats[1]) stats[1] = t1[c];
            if (t2[c] < stats[2]) stats[2] = t2[c];
            if (t2[c] > stats[3]) stats[3] = t2[c];
            d = Bu;
            B[j] = Bn;
            X[j] = Xn;
            Fl = Fn;
            Yl = Yn;
            if (i == nA && j == nB) fin = Bn;
        }
    }
    const int best = fin + (nA + nB) * dz; /* real optimum */
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
                const int a = wrap ? D1[c] : t1[c], b = wrap ? D2[c] : t2[c];
                if (st == ST_M) {          /* best state of (ni, nj); relative to X */
                    nst = pick(a, 0, a - b, prio);
                } else if (st == ST_IX) {  /* candidates of Ix(i, j) at (i - 1, j), relative to X + e */
                    const int co = j == nB ? eo - ee : io - ie;
                    nst = pick(a + co, 0, a - b + co, prio);
                } else {                   /* candidates of Iy(i, j) at (i, j - 1), relative to Y + e */
                    const int ro = i == nA ? eo - ee : io - ie;
                    nst = pick(b + ro, b - a + ro, 0, prio);
                }
            }
            if (!first) {
                if (st == ST_M) {
                    score += x[i - 1] == y[j - 1] ? ma : mi;
                } else if (st == ST_IX) {
                    const int end = (j == nB || j == 0);
                    score += (nst == ST_IX) ? (end ? ee : ie) : (end ? eo : io);
                } else {
                    const int end = (i == nA || i == 0);
                    score += (nst == ST_IY) ? (end ? ee : ie) : (end ? eo : io);
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
    free(D1); free(D2); free(t1); free(t2); free(B); free(X);
    return best;
}

int proto_align(const char* x, int nA, const char* y, int nB, int* out, int* stats, int wrap) {
    return proto_align_sc(x, nA, y, nB, out, stats, wrap, 0);
}
