/*
 * cpu_cgs2.c — the "optimised CPU" comparison line of bench.py ("A second CPU
 * variant (OpenMP block CGS2)").  TEST / BASELINE INFRASTRUCTURE ONLY, like nekstab_oracle.c:
 * loaded only by tests/ and bench.py's cpu_baseline leg.
 *
 * Same inputs and H-column semantics as orc_update_hessenberg (krylov_decomposition.f90:103-189:
 * H(i,k) = pass-1 + pass-2 coefficient, H(k+1,k) = ||f||_W, f normalised), but classical
 * Gram–Schmidt with one re-orthogonalisation, blocked for the cache: per row block every column's
 * partial dot is accumulated while the block of f stays in L1/L2 (the basis is streamed once per
 * pass), per-thread partial sums are reduced once.  FMA contraction and AVX2 are allowed here
 * (this file is timed, not used as a parity oracle; -mavx2 -mfma run on any current x86 host).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int64_t nv;
    int64_t np;
    int32_t nwf;
    int32_t time_in_dot;
} orc_layout;

enum { RB = 2048 };   /* rows per block: 16 KB of f, k x 16 KB of Q streamed past it */

/* h[c] = <Q_c, f>_W (weighted fields only) [+ time term], c < k */
static void blk_dot(const orc_layout* L, const double* w, const double* Q, int64_t ld, int k,
                    const double* f, double* h) {
    const int64_t nb_f = (L->nv + RB - 1) / RB, nb = nb_f * L->nwf;
    memset(h, 0, sizeof(double) * (size_t)k);
#pragma omp parallel
    {
        double* hp = (double*)calloc((size_t)k, sizeof(double));
#pragma omp for schedule(static)
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t fld = b / nb_f, r0 = (b % nb_f) * RB;
            const int64_t r1 = r0 + RB < L->nv ? r0 + RB : L->nv;
            const int64_t off = fld * L->nv;
            double wf[RB];
            for (int64_t r = r0; r < r1; ++r) wf[r - r0] = w[r] * f[off + r];
            for (int c = 0; c < k; ++c) {
                const double* q = Q + (int64_t)c * ld + off;
                double s = 0.0;
#pragma omp simd reduction(+ : s)
                for (int64_t r = r0; r < r1; ++r) s += q[r] * wf[r - r0];
                hp[c] += s;
            }
        }
#pragma omp critical
        for (int c = 0; c < k; ++c) h[c] += hp[c];
        free(hp);
    }
    if (L->time_in_dot) {
        const int64_t t = (int64_t)L->nwf * L->nv + L->np;
        for (int c = 0; c < k; ++c) h[c] += Q[(int64_t)c * ld + t] * f[t];
    }
}

/* f -= Q h over every stored entry (fields, pressure, time: k_sub2 semantics) */
static void blk_update(const orc_layout* L, const double* Q, int64_t ld, int k, const double* h, double* f) {
    const int64_t n = (int64_t)L->nwf * L->nv + L->np + 1, nb = (n + RB - 1) / RB;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t r0 = b * RB, r1 = r0 + RB < n ? r0 + RB : n;
        for (int c = 0; c < k; ++c) {
            const double* q = Q + (int64_t)c * ld;
            const double hc = h[c];
#pragma omp simd
            for (int64_t r = r0; r < r1; ++r) f[r] -= q[r] * hc;
        }
    }
}

void cpu_cgs2_set_threads(int n) {
#ifdef _OPENMP
    omp_set_num_threads(n < 1 ? 1 : n);
#else
    (void)n;
#endif
}

/* Q: k vectors at stride nwf*nv + np + 1; Hcol: k+1 entries; wrk: >= k doubles */
void cpu_cgs2_update_hessenberg(const orc_layout* L, const double* w, double* Hcol, double* f, const double* Q,
                                int k, double* wrk) {
    const int64_t ld = (int64_t)L->nwf * L->nv + L->np + 1;
    blk_dot(L, w, Q, ld, k, f, Hcol);
    blk_update(L, Q, ld, k, Hcol, f);
    blk_dot(L, w, Q, ld, k, f, wrk);
    blk_update(L, Q, ld, k, wrk, f);
    for (int c = 0; c < k; ++c) Hcol[c] += wrk[c];
    double nrm2;
    blk_dot(L, w, f, ld, 1, f, &nrm2);
    const double beta = sqrt(nrm2), inv = 1.0 / beta;
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < ld; ++r) f[r] *= inv;
    Hcol[k] = beta;
}
