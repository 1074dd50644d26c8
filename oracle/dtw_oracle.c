/* dtw_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A full-size form of or_dtw (sonar_oracle.c) for the BASELINE C3 DTW (51,676 x 51,676, 12-dim
 * chroma), whose (N+1)(M+1) float64 matrix (21.4 GB) the plain restatement cannot hold:
 *
 *   DTWAlignment.Align / fillCostMatrix / backtrack / findPreviousStep
 *   (algorithms/stats/dtw.go:55-103, 106-135, 165-188, 191-217), EuclideanDistanceFunc
 *   (algorithms/stats/distance.go:29-36), default step pattern "symmetric2" (dtw.go:138-162).
 *
 * Same arithmetic as or_dtw, cell for cell (unfused float64, -ffp-contract=off; Go's math.Min
 * NaN / -Inf / -0 rules; the backtrack's strict '<' over up, left, diag), so every value equals
 * or_dtw's. Only the storage and the schedule differ:
 *   pass 1: rows are cut into stripes of SR rows and columns into blocks of CB; stripe s works
 *           on column block b once stripe s-1 has finished b (a wavefront over threads).  A cell
 *           keeps only its 2-bit backtrack code (findPreviousStep's choice, 668 MB at C3) and
 *           the stripe's last row goes to a hand-off row for the stripe below.
 *   backtrack from (N, M) over the codes (i == 0 -> left, j == 0 -> up as dtw.go:196-201).
 *   pass 2: the same sweep again; a path cell (i, j) takes C[i][j] - C[i-1][j-1] (dtw.go:172-176)
 *           when its row comes by.
 * Distance = C[N][M] / len(path) (dtw.go:91).
 */
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static double go_min(double x, double y) {             /* math.Min */
    if (isinf(x) && x < 0) return x;
    if (isinf(y) && y < 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? x : y;
    return x < y ? x : y;
}

enum { SR = 64, CB = 2048 };

typedef struct {
    const double *q, *r;
    int64_t nq, nr;
    int dim, band, nthreads, pass;
    uint8_t* codes;               /* pass 1: [nq][rowbytes], 2 bits per cell */
    int64_t rowbytes;
    double* handoff;              /* [nstripes][nr + 1]: row (s+1)*SR of C, i.e. the stripe's last */
    _Atomic int64_t* progress;    /* [nstripes]: column blocks finished */
    int64_t nstripes, nblocks;
    double final_c;               /* C[nq][nr] */
    /* pass 2 */
    const int64_t* row_first;     /* [nq + 2]: path entries of row i (1-based) are [row_first[i], row_first[i+1]) */
    const int32_t* pr;            /* path columns (0-based j-1), ascending path order */
    double* pc;
} Job;

typedef struct { Job* job; int tid; } Arg;

static void stripe(Job* J, int64_t s) {
    const int64_t i0 = s * SR + 1, i1 = (i0 + SR <= J->nq + 1) ? i0 + SR : J->nq + 1;   /* rows [i0, i1) */
    const int64_t nr = J->nr;
    const int dim = J->dim;
    double* above = s > 0 ? J->handoff + (s - 1) * (nr + 1) : NULL;
    double* mine = J->handoff + s * (nr + 1);
    double rows[2][CB + 1];
    double left[SR];               /* C[i][c0 - 1] for the stripe's rows */
    for (int k = 0; k < SR; k++) left[k] = INFINITY;   /* C[i][0] = +Inf, i >= 1 */
    for (int64_t b = 0; b < J->nblocks; b++) {
        const int64_t c0 = b * CB + 1, c1 = (c0 + CB <= nr + 1) ? c0 + CB : nr + 1;   /* columns [c0, c1) */
        if (s > 0)
            while (atomic_load_explicit(&J->progress[s - 1], memory_order_acquire) <= b) sched_yield();
        /* the row above the stripe, columns [c0-1, c1) */
        double* prev = rows[0];
        for (int64_t j = c0 - 1; j < c1; j++) {
            double v;
            if (s == 0) v = (j == 0) ? 0.0 : INFINITY;  /* C[0][0] = 0, C[0][j] = +Inf */
            else v = above[j];
            prev[j - (c0 - 1)] = v;
        }
        int cur_i = 1;
        for (int64_t i = i0; i < i1; i++) {
            double* cur = rows[cur_i];
            cur[0] = left[i - i0];
            const double* a = J->q + (i - 1) * dim;
            uint8_t* crow = J->codes ? J->codes + (i - 1) * J->rowbytes : NULL;
            int64_t pk = 0, pk1 = 0;
            if (J->pass == 2) { pk = J->row_first[i]; pk1 = J->row_first[i + 1]; }
            for (int64_t j = c0; j < c1; j++) {
                const int64_t x = j - (c0 - 1);
                double c;
                if (J->band > 0 && fabs((double)(i - j)) > (double)J->band) {
                    c = INFINITY;           /* skipped: stays +Inf (dtw.go:115-119) */
                } else {
                    const double* bb = J->r + (j - 1) * dim;
                    double sum = 0.0;
                    for (int d = 0; d < dim; d++) { double df = a[d] - bb[d]; sum += df * df; }
                    const double ld = sqrt(sum);
                    c = ld + go_min(go_min(prev[x], cur[x - 1]), prev[x - 1]);
                }
                cur[x] = c;
                if (crow) {                 /* findPreviousStep (dtw.go:203-216), strict '<' */
                    const double cv = prev[x], ch = cur[x - 1], cd = prev[x - 1];
                    int mi = 0; double best = cv;
                    if (ch < best) { mi = 1; best = ch; }
                    if (cd < best) mi = 2;
                    const int64_t jj = j - 1;
                    crow[jj >> 2] |= (uint8_t)(mi << (2 * (jj & 3)));
                }
            }
            if (J->pass == 2)               /* path cells of row i in this column block */
                for (int64_t k = pk; k < pk1; k++) {
                    const int64_t j = (int64_t)J->pr[k] + 1;
                    if (j >= c0 && j < c1 && j >= 1) J->pc[k] = cur[j - (c0 - 1)] - prev[j - 1 - (c0 - 1)];
                }
            left[i - i0] = cur[c1 - 1 - (c0 - 1)];
            if (i == i1 - 1) memcpy(mine + c0, cur + 1, sizeof(double) * (size_t)(c1 - c0));
            if (i == J->nq && c1 == nr + 1) J->final_c = cur[c1 - 1 - (c0 - 1)];
            cur_i ^= 1;
            prev = cur;
        }
        atomic_store_explicit(&J->progress[s], b + 1, memory_order_release);
    }
}

static void* worker(void* p) {
    Arg* A = (Arg*)p;
    Job* J = A->job;
    for (int64_t s = A->tid; s < J->nstripes; s += J->nthreads) stripe(J, s);
    return NULL;
}

static int run(Job* J) {
    J->nstripes = (J->nq + SR - 1) / SR;
    J->nblocks = (J->nr + CB - 1) / CB;
    J->handoff = malloc(sizeof(double) * (size_t)J->nstripes * (size_t)(J->nr + 1));
    J->progress = calloc((size_t)J->nstripes, sizeof(_Atomic int64_t));
    if (!J->handoff || !J->progress) { free(J->handoff); free((void*)J->progress); return -3; }
    for (int64_t s = 0; s < J->nstripes; s++) J->handoff[s * (J->nr + 1)] = INFINITY;
    int T = J->nthreads < 1 ? 1 : J->nthreads;
    if (T > J->nstripes) T = (int)J->nstripes;
    J->nthreads = T;
    pthread_t th[256];
    Arg args[256];
    if (T > 256) T = J->nthreads = 256;
    for (int t = 0; t < T; t++) { args[t].job = J; args[t].tid = t; pthread_create(&th[t], NULL, worker, &args[t]); }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    free(J->handoff); free((void*)J->progress);
    return 0;
}

/* or_dtw_stripes: path (pq, pr, pc: capacity nq + nr + 1), plen, dist as or_dtw; no cost matrix. */
int or_dtw_stripes(const double* q, int64_t nq, const double* r, int64_t nr, int dim, int band, int nthreads,
                   int32_t* pq, int32_t* pr, double* pc, int64_t* plen, double* dist) {
    if (nq == 0 || nr == 0) return -1;                   /* "empty sequences provided" */
    Job J;
    memset(&J, 0, sizeof J);
    J.q = q; J.r = r; J.nq = nq; J.nr = nr; J.dim = dim; J.band = band; J.nthreads = nthreads; J.pass = 1;
    J.rowbytes = (nr + 3) / 4;
    J.codes = calloc((size_t)nq, (size_t)J.rowbytes);
    if (!J.codes) return -3;
    int rc = run(&J);
    if (rc) { free(J.codes); return rc; }
    const double cnm = J.final_c;
    /* backtrack (dtw.go:165-188), collected in reverse */
    int64_t i = nq, j = nr, P = 0;
    while (i > 0 || j > 0) {
        pq[P] = (int32_t)(i - 1); pr[P] = (int32_t)(j - 1); pc[P] = 0.0; P++;
        if (i == 0) { j--; continue; }
        if (j == 0) { i--; continue; }
        const int mi = (J.codes[(i - 1) * J.rowbytes + ((j - 1) >> 2)] >> (2 * ((j - 1) & 3))) & 3;
        if (mi == 0) i--; else if (mi == 1) j--; else { i--; j--; }
    }
    free(J.codes);
    for (int64_t k = 0; k < P / 2; k++) {
        int32_t t = pq[k]; pq[k] = pq[P - 1 - k]; pq[P - 1 - k] = t;
        t = pr[k]; pr[k] = pr[P - 1 - k]; pr[P - 1 - k] = t;
    }
    /* pass 2: the point costs of the path cells with i, j >= 1 */
    int64_t* row_first = malloc(sizeof(int64_t) * (size_t)(nq + 2));
    if (!row_first) return -3;
    int64_t k = 0;
    for (int64_t ii = 0; ii <= nq + 1; ii++) {
        while (k < P && (int64_t)pq[k] + 1 < ii) k++;
        row_first[ii] = k;
    }
    memset(&J, 0, sizeof J);
    J.q = q; J.r = r; J.nq = nq; J.nr = nr; J.dim = dim; J.band = band; J.nthreads = nthreads; J.pass = 2;
    J.row_first = row_first; J.pr = pr; J.pc = pc;
    rc = run(&J);
    free(row_first);
    if (rc) return rc;
    *plen = P;
    *dist = cnm / (double)P;
    return 0;
}
