/*
 * C restatement of the TaxI2 versusAll / versusReference hot path.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py -- never by the product (taxi2_amd).  It is the
 * checker for the HIP kernels and the timed CPU baseline ("kind": "port").
 *
 * What it restates (the reference's own arithmetic lives in third-party packages
 * that are absent from /root/reference; their call sites are cited):
 *   - align:   src/itaxotools/taxi2/align.py:72-157 -> Biopython 1.85
 *              PairwiseAligner(**Scores).align(x, y)[0]; global Gotoh (NW when every
 *              open == extend), first path = end state M>Ix>Iy, each backward step takes
 *              the first predecessor in priority M>Ix>Iy (NW: H>V>D).
 *   - metrics: src/itaxotools/taxi2/distances.py:319-348 -> itaxotools.calculate_distances
 *              0.1.1 seq_distances_{p,p_gaps,jukes_cantor,kimura2p}.
 * It is pinned against the reference's vectors through oracle/restatement.py, which
 * reproduces tests/test_align.py:49-163 and tests/test_distances/metrics.tsv, and which
 * the tests compare this file against on random inputs (explicit traceback == carried
 * counters).
 *
 * Forward-carried counters: the traceback from (i, j, state) is a deterministic
 * function of that cell, so the (valid, ts, tv, gap) counters of the path it
 * reaches can be propagated forward: C(cell) = C(first tied predecessor) +
 * column contribution.  The (y, x) orientation is the same fill with the Ix/Iy
 * priority exchanged, so one fill yields both ordered pairs.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t valid, ts, tv, gap;
} t2o_counts;

typedef struct {
    int32_t match, mismatch, open, extend, end_open, end_extend;
} t2o_scores;

enum { T2O_P = 0, T2O_PGAPS = 1, T2O_JC = 2, T2O_K2P = 3 };

static const int32_t NEG = -(1 << 29);

/* base code: 0..3 for ACGT/acgt, -1 otherwise */
static inline int base_of(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return -1;
    }
}

static void nuc_span(const char* s, int n, int* f, int* l) {
    int a = n + 1, b = -1;
    for (int k = 0; k < n; k++)
        if (base_of((unsigned char)s[k]) >= 0) { a = k; break; }
    for (int k = n - 1; k >= 0; k--)
        if (base_of((unsigned char)s[k]) >= 0) { b = k; break; }
    *f = a;
    *l = b;
}

/* ---------------------------------------------------------------- pre-aligned (A8) */
void t2o_prealigned_counts(const char* x, int nx, const char* y, int ny, t2o_counts* out) {
    int fx, lx, fy, ly;
    nuc_span(x, nx, &fx, &lx);
    nuc_span(y, ny, &fy, &ly);
    int lo = fx > fy ? fx : fy;
    int hi = lx < ly ? lx : ly;
    t2o_counts c = {0, 0, 0, 0};
    for (int k = lo; k <= hi; k++) {
        int a = base_of((unsigned char)x[k]), b = base_of((unsigned char)y[k]);
        if (a >= 0 && b >= 0) {
            c.valid++;
            int d = a ^ b;
            if (d == 2) c.ts++;
            else if (d) c.tv++;
        } else if ((x[k] == '-' && b >= 0) || (y[k] == '-' && a >= 0)) {
            c.gap++;
        }
    }
    *out = c;
}

/* ---------------------------------------------------------------- metrics (A8) */
static double safe_log(double v) { return log(v); /* log(0) = -inf, log(<0) = NaN */ }

double t2o_metric(int code, const t2o_counts* c) {
    double valid = c->valid, mism = c->ts + c->tv;
    switch (code) {
        case T2O_P:
            return c->valid ? mism / valid : NAN;
        case T2O_PGAPS:
            return (c->valid + c->gap) ? (mism + c->gap) / (valid + c->gap) : NAN;
        case T2O_JC: {
            if (!c->valid) return NAN;
            double p = mism / valid;
            return -0.75 * safe_log(1.0 - (4.0 / 3.0) * p);
        }
        case T2O_K2P: {
            if (!c->valid) return NAN;
            double P = c->ts / valid, Q = c->tv / valid;
            return -0.5 * safe_log(1.0 - 2.0 * P - Q) - 0.25 * safe_log(1.0 - 2.0 * Q);
        }
    }
    return NAN;
}

/* ---------------------------------------------------------------- alignment (A5-A7) */
typedef struct {
    int32_t v[4]; /* valid, ts, tv, gap */
} cnt4;

static inline cnt4 cadd(cnt4 a, int dv, int dts, int dtv, int dg) {
    a.v[0] += dv;
    a.v[1] += dts;
    a.v[2] += dtv;
    a.v[3] += dg;
    return a;
}

/* contribution of a diagonal move consuming x[i-1], y[j-1] */
static inline void diag_contrib(unsigned char a, unsigned char b, int* dv, int* dts, int* dtv) {
    int ba = base_of(a), bb = base_of(b);
    *dv = *dts = *dtv = 0;
    if (ba >= 0 && bb >= 0) {
        *dv = 1;
        int d = ba ^ bb;
        if (d == 2) *dts = 1;
        else if (d) *dtv = 1;
    }
}

typedef struct {
    int32_t s[3];   /* M, Ix, Iy scores */
    cnt4 c[2][3];   /* [orientation][state] */
} gcell;

/* Gotoh (affine).  Returns score. */
static int32_t gotoh_counts(const char* x, int nA, const char* y, int nB, const t2o_scores* sc,
                            cnt4* outA, cnt4* outB) {
    int fx, lx, fy, ly;
    nuc_span(x, nA, &fx, &lx);
    nuc_span(y, nB, &fy, &ly);
    gcell* prev = (gcell*)calloc((size_t)nB + 1, sizeof(gcell));
    gcell* cur = (gcell*)calloc((size_t)nB + 1, sizeof(gcell));
    /* row 0 */
    prev[0].s[0] = 0;
    prev[0].s[1] = NEG;
    prev[0].s[2] = NEG;
    for (int j = 1; j <= nB; j++) {
        prev[j].s[0] = NEG;
        prev[j].s[1] = NEG;
        prev[j].s[2] = sc->end_open + sc->end_extend * (j - 1);
    }
    /* priority orders: A = M, Ix, Iy ; B = M, Iy, Ix */
    static const int ord[2][3] = {{0, 1, 2}, {0, 2, 1}};
    for (int i = 1; i <= nA; i++) {
        memset(&cur[0], 0, sizeof(gcell));
        cur[0].s[0] = NEG;
        cur[0].s[1] = sc->end_open + sc->end_extend * (i - 1);
        cur[0].s[2] = NEG;
        unsigned char a = (unsigned char)x[i - 1];
        int anuc = base_of(a) >= 0;
        int row_iy = (i - 1 >= fx) && (i <= lx); /* x side of an x-gap column in range */
        int oy = (i == nA) ? sc->end_open : sc->open;
        int ey = (i == nA) ? sc->end_extend : sc->extend;
        for (int j = 1; j <= nB; j++) {
            unsigned char b = (unsigned char)y[j - 1];
            const gcell* d = &prev[j - 1];
            const gcell* u = &prev[j];
            const gcell* l = &cur[j - 1];
            gcell* o = &cur[j];
            /* M */
            int32_t cand[3];
            cand[0] = d->s[0];
            cand[1] = d->s[1];
            cand[2] = d->s[2];
            int32_t best = cand[0] > cand[1] ? cand[0] : cand[1];
            best = best > cand[2] ? best : cand[2];
            o->s[0] = best + (a == b ? sc->match : sc->mismatch);
            int dv, dts, dtv;
            diag_contrib(a, b, &dv, &dts, &dtv);
            for (int r = 0; r < 2; r++) {
                int p = 0;
                for (int q = 0; q < 3; q++)
                    if (cand[ord[r][q]] == best) { p = ord[r][q]; break; }
                o->c[r][0] = cadd(d->c[r][p], dv, dts, dtv, 0);
            }
            /* Ix: consume x[i-1] against a gap, from the cell above */
            int ox = (j == nB) ? sc->end_open : sc->open;
            int ex = (j == nB) ? sc->end_extend : sc->extend;
            cand[0] = u->s[0] + ox;
            cand[1] = u->s[1] + ex;
            cand[2] = u->s[2] + ox;
            best = cand[0] > cand[1] ? cand[0] : cand[1];
            best = best > cand[2] ? best : cand[2];
            o->s[1] = best;
            int gx = anuc && (j - 1 >= fy) && (j <= ly);
            for (int r = 0; r < 2; r++) {
                int p = 0;
                for (int q = 0; q < 3; q++)
                    if (cand[ord[r][q]] == best) { p = ord[r][q]; break; }
                o->c[r][1] = cadd(u->c[r][p], 0, 0, 0, gx);
            }
            /* Iy: consume y[j-1] against a gap, from the cell to the left */
            cand[0] = l->s[0] + oy;
            cand[1] = l->s[1] + oy;
            cand[2] = l->s[2] + ey;
            best = cand[0] > cand[1] ? cand[0] : cand[1];
            best = best > cand[2] ? best : cand[2];
            o->s[2] = best;
            int gy = (base_of(b) >= 0) && row_iy;
            for (int r = 0; r < 2; r++) {
                int p = 0;
                for (int q = 0; q < 3; q++)
                    if (cand[ord[r][q]] == best) { p = ord[r][q]; break; }
                o->c[r][2] = cadd(l->c[r][p], 0, 0, 0, gy);
            }
        }
        gcell* t = prev;
        prev = cur;
        cur = t;
    }
    const gcell* e = &prev[nB];
    int32_t best = e->s[0] > e->s[1] ? e->s[0] : e->s[1];
    best = best > e->s[2] ? best : e->s[2];
    for (int r = 0; r < 2; r++) {
        int p = 0;
        for (int q = 0; q < 3; q++)
            if (e->s[ord[r][q]] == best) { p = ord[r][q]; break; }
        (r == 0 ? outA : outB)[0] = e->c[r][p];
    }
    free(prev);
    free(cur);
    return best;
}

typedef struct {
    int32_t s;
    cnt4 c[2];
} ncell;

/* Needleman-Wunsch (linear gaps): single matrix, traceback priority H>V>D (B: V>H>D). */
static int32_t nw_counts(const char* x, int nA, const char* y, int nB, const t2o_scores* sc,
                         cnt4* outA, cnt4* outB) {
    int fx, lx, fy, ly;
    nuc_span(x, nA, &fx, &lx);
    nuc_span(y, nB, &fy, &ly);
    ncell* prev = (ncell*)calloc((size_t)nB + 1, sizeof(ncell));
    ncell* cur = (ncell*)calloc((size_t)nB + 1, sizeof(ncell));
    for (int j = 0; j <= nB; j++) prev[j].s = j * sc->end_extend;
    /* move codes: 0 = D, 1 = V (from above, consumes x), 2 = H (from left, consumes y) */
    static const int ord[2][3] = {{2, 1, 0}, {1, 2, 0}};
    for (int i = 1; i <= nA; i++) {
        memset(&cur[0], 0, sizeof(ncell));
        cur[0].s = i * sc->end_extend;
        unsigned char a = (unsigned char)x[i - 1];
        int anuc = base_of(a) >= 0;
        int row_iy = (i - 1 >= fx) && (i <= lx);
        int hgap = (i == nA) ? sc->end_extend : sc->extend;
        for (int j = 1; j <= nB; j++) {
            unsigned char b = (unsigned char)y[j - 1];
            int vgap = (j == nB) ? sc->end_extend : sc->extend;
            int32_t cand[3];
            cand[0] = prev[j - 1].s + (a == b ? sc->match : sc->mismatch);
            cand[1] = prev[j].s + vgap;
            cand[2] = cur[j - 1].s + hgap;
            int32_t best = cand[0] > cand[1] ? cand[0] : cand[1];
            best = best > cand[2] ? best : cand[2];
            cur[j].s = best;
            int dv, dts, dtv;
            diag_contrib(a, b, &dv, &dts, &dtv);
            int gx = anuc && (j - 1 >= fy) && (j <= ly);
            int gy = (base_of(b) >= 0) && row_iy;
            for (int r = 0; r < 2; r++) {
                int mv = 0;
                for (int q = 0; q < 3; q++)
                    if (cand[ord[r][q]] == best) { mv = ord[r][q]; break; }
                if (mv == 0) cur[j].c[r] = cadd(prev[j - 1].c[r], dv, dts, dtv, 0);
                else if (mv == 1) cur[j].c[r] = cadd(prev[j].c[r], 0, 0, 0, gx);
                else cur[j].c[r] = cadd(cur[j - 1].c[r], 0, 0, 0, gy);
            }
        }
        ncell* t = prev;
        prev = cur;
        cur = t;
    }
    *outA = prev[nB].c[0];
    *outB = prev[nB].c[1];
    int32_t s = prev[nB].s;
    free(prev);
    free(cur);
    return s;
}

static int is_linear(const t2o_scores* sc) {
    return sc->open == sc->extend && sc->end_open == sc->end_extend;
}

/* Aligned counters of (x, y) and (y, x) from one fill; x, y must already be normalized. */
int32_t t2o_align_counts(const char* x, int nA, const char* y, int nB, const t2o_scores* sc,
                         t2o_counts* ab, t2o_counts* ba) {
    cnt4 a, b;
    int32_t s = is_linear(sc) ? nw_counts(x, nA, y, nB, sc, &a, &b)
                              : gotoh_counts(x, nA, y, nB, sc, &a, &b);
    ab->valid = a.v[0]; ab->ts = a.v[1]; ab->tv = a.v[2]; ab->gap = a.v[3];
    ba->valid = b.v[0]; ba->ts = b.v[1]; ba->tv = b.v[2]; ba->gap = b.v[3];
    return s;
}

/* ---------------------------------------------------------------- threaded batch */
typedef struct {
    const char* bytes;
    const int64_t* offs;
    const int64_t* pa;
    const int64_t* pb;
    int64_t npairs;
    int align;
    const t2o_scores* sc;
    const int* codes;
    int ncodes;
    double* out;
    int32_t* scores;
    int64_t next;
    pthread_mutex_t mu;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* J = (batch_job*)arg;
    const int64_t CH = 16;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        int64_t k0 = J->next;
        J->next += CH;
        pthread_mutex_unlock(&J->mu);
        if (k0 >= J->npairs) break;
        int64_t k1 = k0 + CH < J->npairs ? k0 + CH : J->npairs;
        for (int64_t k = k0; k < k1; k++) {
            int64_t a = J->pa[k], b = J->pb[k];
            const char* x = J->bytes + J->offs[a];
            const char* y = J->bytes + J->offs[b];
            int nx = (int)(J->offs[a + 1] - J->offs[a]);
            int ny = (int)(J->offs[b + 1] - J->offs[b]);
            t2o_counts ab, ba;
            int32_t s = 0;
            if (J->align) {
                s = t2o_align_counts(x, nx, y, ny, J->sc, &ab, &ba);
            } else {
                t2o_prealigned_counts(x, nx, y, ny, &ab);
                ba = ab;
            }
            if (J->scores) J->scores[k] = s;
            double* o = J->out + k * 2 * J->ncodes;
            for (int m = 0; m < J->ncodes; m++) {
                o[m] = t2o_metric(J->codes[m], &ab);
                o[J->ncodes + m] = t2o_metric(J->codes[m], &ba);
            }
        }
    }
    return NULL;
}

/* out: [npairs][2 orientations][ncodes] f64 (NaN = None); scores: [npairs] (nullable). */
int t2o_batch(const char* bytes, const int64_t* offs, const int64_t* pa, const int64_t* pb,
              int64_t npairs, int align, const t2o_scores* sc, const int* codes, int ncodes,
              double* out, int32_t* scores, int nthreads) {
    batch_job J;
    memset(&J, 0, sizeof J);
    J.bytes = bytes; J.offs = offs; J.pa = pa; J.pb = pb; J.npairs = npairs; J.align = align;
    J.sc = sc; J.codes = codes; J.ncodes = ncodes; J.out = out; J.scores = scores;
    pthread_mutex_init(&J.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads == 1) {
        batch_worker(&J);
    } else {
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &J);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
        free(th);
    }
    pthread_mutex_destroy(&J.mu);
    return 0;
}
