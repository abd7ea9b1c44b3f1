/*
 * arnoldi_c.c — a plain-C host driving the drop-in C ABI (include/nekkrylov.h) with no Python:
 * the shape of what a Fortran bind(C) host does on each MPI rank.
 *
 *   build:  make -C examples/c_host   (gcc, the HIP runtime API and libnekkrylov.so)
 *
 *   run:    examples/c_host/arnoldi_c [E] [m]
 *
 * 3-D lx1=8 layout with one scalar (E elements), diagonal synthetic operator, seed from
 * nkv_fill_hash, m DCGS2 Arnoldi steps (single rank: the all-reduces of INTEGRATION.md §2b are the
 * identity), the closing re-orthogonalisation, then checks of W-orthonormality of the basis and of
 * the Arnoldi relation A Q_m = Q_{m+1} H through the same ABI; then the same factorisation as ONE
 * call of the native driver nkv_arnoldi_dcgs2 (the operator as a callback), which must reproduce
 * Q and H bit for bit.  Last, the breakdown protocol of include/nekkrylov.h on a rank-3 operator:
 * nkv_arnoldi_dcgs2 with NKV_CHECK_BREAKDOWN returns NKV_EBREAKDOWN, the host restores the seed
 * column and redoes the factorisation with nkv_arnoldi_factorization(NKV_MGS2) (the reference's
 * order), whose basis must be W-orthonormal.  Then ts_gmres's inner loop as one call
 * (nkv_gmres_dcgs2) on the diagonal operator: the host solves the small least-squares problem (here
 * by Givens + back substitution; a Fortran host calls its lstsq/dgels), forms x = Q y with
 * nkv_combine and checks that ||b - A x||_W equals the last reported residual.  Exit status 0 on
 * success.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nekkrylov.h"

#define CK(x)                                                                             \
    do {                                                                                  \
        int rc_ = (x);                                                                    \
        if (rc_ != NKV_OK) {                                                              \
            fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, nkv_last_error());          \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)
#define HK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

static int64_t roundup(int64_t n, int64_t m) { return (n + m - 1) / m * m; }

/* the operator as a callback of nkv_arnoldi_dcgs2 (a Fortran host passes c_funloc of a bind(C)
   procedure wrapping its time-stepper) */
typedef struct {
    const nkv_layout* L;
    const double* d;
} diag_op;

static int diag_matvec(void* user, const double* x, double* y, void* stream) {
    const diag_op* op = (const diag_op*)user;
    return nkv_op_diag(op->L, op->d, x, y, 0.0, stream);
}

int main(int argc, char** argv) {
    const int E = argc > 1 ? atoi(argv[1]) : 512;
    const int m = argc > 2 ? atoi(argv[2]) : 24;
    const int ldim = 3, lx1 = 8, lx2 = 6, nsc = 1;
    nkv_layout L;
    L.n_v = (int64_t)lx1 * lx1 * lx1 * E;
    L.n_p = (int64_t)lx2 * lx2 * lx2 * E;
    L.n_wf = ldim + nsc;
    L.sv = roundup(L.n_v, NKV_TILE);
    L.sp = roundup(L.n_p, NKV_TILE);
    L.ld = roundup((int64_t)L.n_wf * L.sv + L.sp + 1, NKV_TILE);
    L.rank0 = 1;
    const int64_t rows = (int64_t)L.n_wf * L.sv + L.sp;

    if (nkv_abi_version() != NKV_ABI_VERSION) {
        fprintf(stderr, "ABI mismatch\n");
        return 1;
    }
    hipStream_t st;
    HK(hipStreamCreate(&st));
    double *Q, *f, *w, *d, *Hd, *hd, *coef, *nrm, *hcol, *ws;
    const size_t vbytes = (size_t)L.ld * sizeof(double);
    HK(hipMalloc((void**)&Q, (size_t)(m + 1) * vbytes));
    HK(hipMalloc((void**)&f, vbytes));
    HK(hipMalloc((void**)&d, vbytes));
    HK(hipMalloc((void**)&w, (size_t)L.sv * sizeof(double)));
    HK(hipMalloc((void**)&Hd, (size_t)m * (m + 1) * sizeof(double)));
    HK(hipMalloc((void**)&hd, (size_t)2 * (m + 1) * sizeof(double)));
    HK(hipMalloc((void**)&coef, (size_t)(3 * m + 8) * sizeof(double)));
    HK(hipMalloc((void**)&nrm, 8 * sizeof(double)));
    HK(hipMalloc((void**)&hcol, (size_t)(m + 2) * sizeof(double)));
    const size_t wsb = nkv_workspace_bytes(&L, m + 1);
    HK(hipMalloc((void**)&ws, wsb));
    HK(hipMemsetAsync(ws, 0, wsb, st));
    HK(hipMemsetAsync(Q, 0, (size_t)(m + 1) * vbytes, st));
    HK(hipMemsetAsync(Hd, 0, (size_t)m * (m + 1) * sizeof(double), st));

    /* weights: 1 on live points, 0 in the padding; operator: d_i in (0.05, 1) from the hash */
    double* hw = (double*)calloc((size_t)L.sv, sizeof(double));
    for (int64_t i = 0; i < L.n_v; ++i) hw[i] = 1.0;
    HK(hipMemcpyAsync(w, hw, (size_t)L.sv * sizeof(double), hipMemcpyHostToDevice, st));
    CK(nkv_fill_hash(&L, d, 99, 0, 0, st));
    double* hdg = (double*)malloc(vbytes);
    HK(hipMemcpyAsync(hdg, d, vbytes, hipMemcpyDeviceToHost, st));
    HK(hipStreamSynchronize(st));
    for (int64_t i = 0; i < L.ld; ++i) hdg[i] = 0.525 + 0.475 * hdg[i];   /* [-1,1] -> [0.05, 1] */
    HK(hipMemcpyAsync(d, hdg, vbytes, hipMemcpyHostToDevice, st));

    /* q_1 = seed / ||seed||_W */
    CK(nkv_fill_hash(&L, Q, 11, 0, 0, st));
    CK(nkv_dot(&L, w, Q, Q, nrm, ws, 0, st));
    CK(nkv_normalize_dev(&L, Q, nrm, NULL, 0, st));

    /* m DCGS2 steps (a multi-rank host all-reduces hd after block_dot2:
       beta^2 of the provisional column is the dot's own entry hd[j-1]) */
    for (int j = 1; j <= m; ++j) {
        double* u = Q + (int64_t)(j - 1) * L.ld;
        CK(nkv_op_diag(&L, d, u, f, 0.0, st));
        CK(nkv_block_dot2(&L, w, Q, j, u, f, hd, ws, NKV_X_IS_LAST, st));
        CK(nkv_dcgs2_coef(j - 1, hd, hd + j, j == 1 ? NULL : hd + (j - 1), Hd, m + 1, coef, ws, st));
        CK(nkv_dcgs2_update(&L, w, Q, j - 1, coef, u, f, Q + (int64_t)j * L.ld, NULL, ws, NKV_TIME, st));
    }
    double* um = Q + (int64_t)m * L.ld;
    CK(nkv_block_dot(&L, w, Q, m + 1, um, hd, ws, 0, st));
    CK(nkv_dcgs2_coef(m, hd, NULL, hd + m, Hd, m + 1, coef, ws, st));
    CK(nkv_block_update(&L, w, Q, m, hd, um, NULL, ws, NKV_TIME, st));
    CK(nkv_normalize_dev(&L, um, coef + 2 * m + 3, NULL, 0, st));
    CK(nkv_check_status(ws, st));

    double* H = (double*)malloc((size_t)m * (m + 1) * sizeof(double));
    HK(hipMemcpyAsync(H, Hd, (size_t)m * (m + 1) * sizeof(double), hipMemcpyDeviceToHost, st));
    HK(hipStreamSynchronize(st));

    /* checks through the ABI: G = Q^T W Q (column by column), and ||A q_c - Q H(:,c)||_W */
    double orth = 0.0, arn = 0.0, hmax = 0.0;
    double* g = (double*)malloc((size_t)(m + 1) * sizeof(double));
    for (int c = 0; c <= m; ++c) {
        CK(nkv_block_dot(&L, w, Q, m + 1, Q + (int64_t)c * L.ld, hd, ws, 0, st));
        HK(hipMemcpyAsync(g, hd, (size_t)(m + 1) * sizeof(double), hipMemcpyDeviceToHost, st));
        HK(hipStreamSynchronize(st));
        for (int r = 0; r <= m; ++r) {
            const double e = fabs(g[r] - (r == c ? 1.0 : 0.0));
            if (e > orth) orth = e;
        }
    }
    for (int i = 0; i < m * (m + 1); ++i) hmax = fmax(hmax, fabs(H[i]));
    for (int c = 0; c < m; c += (m > 4 ? m / 4 : 1)) {
        CK(nkv_op_diag(&L, d, Q + (int64_t)c * L.ld, f, 0.0, st));
        HK(hipMemcpyAsync(hcol, H + (int64_t)c * (m + 1), (size_t)(c + 2) * sizeof(double), hipMemcpyHostToDevice, st));
        CK(nkv_block_update(&L, w, Q, c + 2, hcol, f, nrm, ws, NKV_NORM2, st));
        double r2;
        HK(hipMemcpyAsync(&r2, nrm, sizeof(double), hipMemcpyDeviceToHost, st));
        HK(hipStreamSynchronize(st));
        arn = fmax(arn, sqrt(fabs(r2)));
    }
    printf("arnoldi_c: N=%lld m=%d  max|Q^T W Q - I| = %.3e  max ||A q - Q h|| / max|H| = %.3e  H(m+1,m) = %.6e\n",
           (long long)(L.n_wf * L.n_v + L.n_p), m, orth, arn / hmax, H[(int64_t)(m - 1) * (m + 1) + m]);

    /* the same factorisation as ONE call of the native driver (operator as a callback, no
       all-reduce on one rank): Q and H must equal the step-by-step loop's bit for bit */
    double *Q2, *Hd2, *scr;
    HK(hipMalloc((void**)&Q2, (size_t)(m + 1) * vbytes));
    HK(hipMalloc((void**)&Hd2, (size_t)m * (m + 1) * sizeof(double)));
    HK(hipMalloc((void**)&scr, nkv_arnoldi_scratch_doubles(m) * sizeof(double)));
    HK(hipMemsetAsync(Q2, 0, (size_t)(m + 1) * vbytes, st));
    HK(hipMemsetAsync(Hd2, 0, (size_t)m * (m + 1) * sizeof(double), st));
    CK(nkv_fill_hash(&L, Q2, 11, 0, 0, st));
    CK(nkv_dot(&L, w, Q2, Q2, nrm, ws, 0, st));
    CK(nkv_normalize_dev(&L, Q2, nrm, NULL, 0, st));
    diag_op op = {&L, d};
    CK(nkv_arnoldi_dcgs2(&L, w, Q2, 1, m, Hd2, m + 1, f, scr, ws, diag_matvec, &op, NULL, NULL, 0, st));
    double* H2 = (double*)malloc((size_t)m * (m + 1) * sizeof(double));
    double *qa = (double*)malloc(vbytes), *qb = (double*)malloc(vbytes);
    HK(hipMemcpyAsync(H2, Hd2, (size_t)m * (m + 1) * sizeof(double), hipMemcpyDeviceToHost, st));
    HK(hipStreamSynchronize(st));
    int same = memcmp(H, H2, (size_t)m * (m + 1) * sizeof(double)) == 0;
    for (int c = 0; c <= m && same; ++c) {
        HK(hipMemcpy(qa, Q + (int64_t)c * L.ld, vbytes, hipMemcpyDeviceToHost));
        HK(hipMemcpy(qb, Q2 + (int64_t)c * L.ld, vbytes, hipMemcpyDeviceToHost));
        same = memcmp(qa, qb, vbytes) == 0;
    }
    printf("arnoldi_c: nkv_arnoldi_dcgs2 (one call) %s the step-by-step loop\n",
           same ? "equals bit for bit" : "DIFFERS from");

    /* breakdown: d = diag(0.95, 0.85, 0.75) on three points, 0 elsewhere (the Krylov space of the
       seed closes after 4 steps: the seed and the three eigen-directions).  DCGS2 with the check -> NKV_EBREAKDOWN; restore and redo in MGS2 order. */
    for (int64_t i = 0; i < L.ld; ++i) hdg[i] = 0.0;
    hdg[7] = 0.95, hdg[14] = 0.85, hdg[21] = 0.75;
    HK(hipMemcpyAsync(d, hdg, vbytes, hipMemcpyHostToDevice, st));
    HK(hipMemcpyAsync(Q2, Q, vbytes, hipMemcpyDeviceToDevice, st));   /* the normalised seed */
    HK(hipMemsetAsync(Hd2, 0, (size_t)m * (m + 1) * sizeof(double), st));
    const int rb = nkv_arnoldi_dcgs2(&L, w, Q2, 1, m, Hd2, m + 1, f, scr, ws, diag_matvec, &op, NULL, NULL,
                                     NKV_CHECK_BREAKDOWN, st);
    printf("arnoldi_c: rank-3 operator, nkv_arnoldi_dcgs2 + NKV_CHECK_BREAKDOWN -> %d (%s)\n", rb,
           rb == NKV_OK ? "" : nkv_last_error());
    HK(hipMemcpyAsync(Q2, Q, vbytes, hipMemcpyDeviceToDevice, st));   /* restore Q(mstart) and H */
    HK(hipMemsetAsync(Hd2, 0, (size_t)m * (m + 1) * sizeof(double), st));
    CK(nkv_arnoldi_factorization(&L, w, Q2, 1, m, Hd2, m + 1, f, scr, ws, diag_matvec, &op, NULL, NULL, NKV_MGS2, st));
    CK(nkv_check_status(ws, st));
    double orth2 = 0.0;
    for (int c = 0; c <= m; ++c) {
        CK(nkv_block_dot(&L, w, Q2, m + 1, Q2 + (int64_t)c * L.ld, hd, ws, 0, st));
        HK(hipMemcpyAsync(g, hd, (size_t)(m + 1) * sizeof(double), hipMemcpyDeviceToHost, st));
        HK(hipStreamSynchronize(st));
        for (int r = 0; r <= m; ++r) orth2 = fmax(orth2, fabs(g[r] - (r == c ? 1.0 : 0.0)));
    }
    HK(hipMemcpy(H2, Hd2, (size_t)m * (m + 1) * sizeof(double), hipMemcpyDeviceToHost));
    printf("arnoldi_c: MGS2 fallback: H(5,4) = %.3e (span{q1, A q1, ...} invariant after 4 steps), max|Q^T W Q - I| = %.3e\n",
           H2[3 * (m + 1) + 4], orth2);
    const double h54 = H2[3 * (m + 1) + 4];
    /* ts_gmres inner loop as ONE call: A x = b with the well-conditioned diagonal of the first part
       (d in (0.05, 1)); Q column 0 = b / ||b||_W */
    HK(hipMemcpyAsync(d, hdg, vbytes, hipMemcpyHostToDevice, st));   /* hdg holds the rank-3 diagonal now: */
    CK(nkv_fill_hash(&L, d, 99, 0, 0, st));                           /* rebuild d in (0.05, 1)            */
    HK(hipMemcpyAsync(hdg, d, vbytes, hipMemcpyDeviceToHost, st));
    HK(hipStreamSynchronize(st));
    for (int64_t i = 0; i < L.ld; ++i) hdg[i] = 0.525 + 0.475 * hdg[i];
    HK(hipMemcpyAsync(d, hdg, vbytes, hipMemcpyHostToDevice, st));
    double *b, *x;
    HK(hipMalloc((void**)&b, vbytes));
    HK(hipMalloc((void**)&x, vbytes));
    HK(hipMemsetAsync(b, 0, vbytes, st));
    CK(nkv_fill_hash(&L, b, 3, 0, 0, st));
    CK(nkv_dot(&L, w, b, b, nrm, ws, 0, st));
    double bb;
    HK(hipMemcpyAsync(&bb, nrm, sizeof(double), hipMemcpyDeviceToHost, st));
    HK(hipStreamSynchronize(st));
    const double beta = sqrt(bb);
    HK(hipMemsetAsync(Q2, 0, (size_t)(m + 1) * vbytes, st));
    HK(hipMemsetAsync(Hd2, 0, (size_t)m * (m + 1) * sizeof(double), st));
    HK(hipMemcpyAsync(Q2, b, vbytes, hipMemcpyDeviceToDevice, st));
    CK(nkv_normalize_dev(&L, Q2, nrm, NULL, 0, st));
    double* res = (double*)calloc((size_t)m, sizeof(double));
    int kk = 0;
    CK(nkv_gmres_dcgs2(&L, w, Q2, m, beta, 1e-24, Hd2, m + 1, f, scr, ws, diag_matvec, &op, NULL, NULL, res, &kk, 0, st));
    HK(hipMemcpyAsync(H2, Hd2, (size_t)m * (m + 1) * sizeof(double), hipMemcpyDeviceToHost, st));
    HK(hipStreamSynchronize(st));
    /* least squares min ||beta e1 - H y||: Givens (nkv_givens_column) then R y = g */
    double *cs = (double*)calloc((size_t)m + 2, sizeof(double)), *sn = (double*)calloc((size_t)m + 2, sizeof(double));
    double *gv = (double*)calloc((size_t)m + 2, sizeof(double)), *R = (double*)calloc((size_t)(m + 2) * m, sizeof(double));
    double* y = (double*)calloc((size_t)m, sizeof(double));
    gv[0] = beta;
    double lsres = 0.0;
    for (int c = 0; c < kk; ++c) {
        double* rc = R + (size_t)c * (m + 2);
        for (int r = 0; r <= c + 1; ++r) rc[r] = H2[(size_t)c * (m + 1) + r];
        lsres = nkv_givens_column(c, rc, cs, sn, gv);
    }
    for (int r = kk - 1; r >= 0; --r) {
        double v = gv[r];
        for (int c = r + 1; c < kk; ++c) v -= R[(size_t)c * (m + 2) + r] * y[c];
        y[r] = v / R[(size_t)r * (m + 2) + r];
    }
    double* yd;
    HK(hipMalloc((void**)&yd, (size_t)m * sizeof(double)));
    HK(hipMemcpyAsync(yd, y, (size_t)kk * sizeof(double), hipMemcpyHostToDevice, st));
    CK(nkv_combine(&L, Q2, kk, yd, x, 0, st));                      /* x = Q_k y */
    CK(nkv_op_diag(&L, d, x, f, 0.0, st));                          /* f = A x - b */
    CK(nkv_axpby(&L, f, 1.0, b, -1.0, 0, st));
    CK(nkv_dot(&L, w, f, f, nrm, ws, 0, st));
    double rr;
    HK(hipMemcpyAsync(&rr, nrm, sizeof(double), hipMemcpyDeviceToHost, st));
    HK(hipStreamSynchronize(st));
    const double true_res = sqrt(rr);
    printf("arnoldi_c: nkv_gmres_dcgs2: %d columns, reported residual %.3e, least-squares %.3e, ||b - A x||_W = %.3e "
           "(||b|| = %.3e)\n", kk, res[kk - 1], lsres, true_res, beta);
    const int gm_ok = kk == m && fabs(true_res - lsres) <= 1e-10 * beta && fabs(res[kk - 1] - lsres) <= 1e-12 * beta &&
                      lsres < 1e-3 * beta;
    const int ok = orth < 1e-12 && arn / hmax < 1e-12 && same && rb == NKV_EBREAKDOWN && orth2 < 1e-8 &&
                   fabs(h54) < 1e-12 && gm_ok;
    printf(ok ? "arnoldi_c: OK\n" : "arnoldi_c: FAILED\n");
    (void)rows;
    return ok ? 0 : 1;
}
