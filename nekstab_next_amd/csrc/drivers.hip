// drivers.hip — one-call factorisations for hosts without Python (arnoldi_factorization,
// krylov_decomposition.f90:2-99; ts_gmres's inner loop, newton_krylov.f90:250-276): the step sequences of
// nekstab_next_amd/arnoldi.py and gmres.py over the entry points of the other translation units, with
// the operator and the all-reduce as host callbacks.
#include "nkv_internal.h"

#include <vector>

extern "C" {

// ---- the whole DCGS2 factorisation, driven natively (arnoldi_factorization, krylov_decomposition.f90:
// 2-99: the loop :68-96 with update_hessenberg_matrix replaced by the DCGS2 entry points above).  The
// host-side orchestration of nekstab_next_amd/arnoldi.py (_dcgs2_step / _dcgs2_close) in C++, for hosts
// without Python: the caller supplies the operator and the all-reduce as callbacks.
// DCGS2 / GMRES: [hd 2(m+1) | coef 4m+16];  NKV_MGS_ICWY: [hd 2(m+1) | h1 m+1 | h2 m+1 | nrm, pad | G (m+1)^2]
static size_t icwy_scratch_doubles(int m) { return (size_t)(4 * (m + 1) + 2) + (size_t)(m + 1) * (size_t)(m + 1); }
size_t nkv_arnoldi_scratch_doubles(int m) {
    const size_t base = (size_t)(2 * (m + 1) + 4 * m + 16), icwy = icwy_scratch_doubles(m);
    return base > icwy ? base : icwy;
}

// NKV_CHECK_BREAKDOWN: after a one-call factorisation, synchronise and test the new H columns c0..c1-1
// (include/nekkrylov.h, "Breakdown").  The same rule as nekstab_next_amd.krylov_schur.breakdown_column.
static constexpr double kBreakdownTol = 1e-8;

static int check_breakdown(const double* H_dev, int64_t ldh, int c0, int c1, void* ws, void* stream) {
    if (c0 < 0) c0 = 0;
    if (c1 <= c0) return NKV_OK;
    hipStream_t st = S(stream);
    const size_t n = (size_t)ldh * (size_t)(c1 - c0);
    double* h = static_cast<double*>(malloc(n * sizeof(double)));
    if (!h) return fail(NKV_EINVAL, "breakdown check: host allocation of %zu doubles failed", n);
    int flag = 0;
    hipError_t e = hipMemcpyAsync(h, H_dev + (int64_t)c0 * ldh, n * sizeof(double), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&flag, nan_flag_of(ws), sizeof(int), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        free(h);
        return fail(NKV_EHIP, "breakdown check: %s", hipGetErrorString(e));
    }
    int bad = -1;
    double ratio = 0.0;
    for (int c = c0; c < c1 && bad < 0; ++c) {
        const double* col = h + (size_t)(c - c0) * (size_t)ldh;
        double s2 = 0.0;
        for (int i = 0; i <= c + 1; ++i) s2 += col[i] * col[i];
        const double nrm = sqrt(s2);
        ratio = nrm > 0.0 ? fabs(col[c + 1]) / nrm : 0.0;
        if (!std::isfinite(s2) || nrm == 0.0 || ratio < kBreakdownTol) bad = c;
    }
    free(h);
    if (flag) {
        NKV_HIP(hipMemsetAsync(nan_flag_of(ws), 0, sizeof(int), st));
        return fail(NKV_EBREAKDOWN, "breakdown: NaN in the factorisation (first suspect column %d)", bad);
    }
    if (bad >= 0)
        return fail(NKV_EBREAKDOWN, "breakdown at column %d: |H(c+1,c)|/||H(:,c)|| = %.3g (invariant subspace)",
                    bad, ratio);
    return NKV_OK;
}

int nkv_arnoldi_dcgs2(const nkv_layout* L, const double* w, double* Q, int mstart, int mend, double* H_dev,
                      int64_t ldh, double* f, double* scratch_dev, void* ws, nkv_matvec_fn matvec, void* mv_user,
                      nkv_allreduce_fn allreduce, void* ar_user, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(Q, "Q"));
    CHECK(check_ptr(f, "f"));
    if (!matvec) return fail(NKV_EINVAL, "matvec callback is NULL");
    if (!H_dev || !scratch_dev) return fail(NKV_EINVAL, "H/scratch is NULL");
    if (mstart < 1 || mend > NKV_MAX_COLS) return fail(NKV_EINVAL, "steps %d..%d outside 1..%d", mstart, mend, NKV_MAX_COLS);
    if (mend < mstart) return NKV_OK;
    if (ldh < mend + 1) return fail(NKV_EINVAL, "ldh=%lld < mend+1=%d", (long long)ldh, mend + 1);
    const unsigned tf = (flags & NKV_TIME_DOT) ? NKV_TIME : 0u;   // time products in the dots (k_dot :52-54)
    double* hd = scratch_dev;                  // [Q^T W u ; Q^T W A u], 2(mend+1)
    double* coef = scratch_dev + 2 * (mend + 1);
    auto col = [L, Q](int c) { return Q + (int64_t)c * L->ld; };
    for (int j = mstart; j <= mend; ++j) {     // step j: column j-1 holds u (normalised at the first step)
        const int m = j - 1;
        double* u = col(m);
        int rc = matvec(mv_user, u, f, stream);
        if (rc != 0) return fail(NKV_ECALLBACK, "matvec callback returned %d at step %d", rc, j);
        CHECK(nkv_block_dot2(L, w, Q, j, u, f, hd, ws, tf | NKV_X_IS_LAST, stream));
        if (allreduce && (rc = allreduce(ar_user, hd, 2 * j, stream)) != 0)
            return fail(NKV_ECALLBACK, "allreduce callback returned %d at step %d", rc, j);
        CHECK(nkv_dcgs2_coef(m, hd, hd + j, j == mstart ? nullptr : hd + m, H_dev, ldh, coef, ws, stream));
        CHECK(nkv_dcgs2_update(L, w, Q, m, coef, u, f, col(j), nullptr, ws, NKV_TIME, stream));
    }
    // closing re-orthogonalisation and normalisation of the provisional column mend
    const int m = mend;
    double* u = col(m);
    CHECK(nkv_block_dot(L, w, Q, m + 1, u, hd, ws, tf, stream));
    if (allreduce) {
        const int rc = allreduce(ar_user, hd, m + 1, stream);
        if (rc != 0) return fail(NKV_ECALLBACK, "allreduce callback returned %d (closing step)", rc);
    }
    CHECK(nkv_dcgs2_coef(m, hd, nullptr, hd + m, H_dev, ldh, coef, ws, stream));
    CHECK(nkv_block_update(L, w, Q, m, hd, u, nullptr, ws, NKV_TIME, stream));
    CHECK(nkv_normalize_dev(L, u, coef + 2 * m + 3, nullptr, 0, stream));
    return (flags & NKV_CHECK_BREAKDOWN) ? check_breakdown(H_dev, ldh, mstart - 1, mend, ws, stream) : NKV_OK;
}

// ts_gmres's inner loop (newton_krylov.f90:250-276) as one call: one continuous DCGS2 factorisation with
// the norm of every new provisional vector fused into the update, the least-squares residual of each
// column from nkv_givens_column on the host, and the closing multi-dot that finalises H's last row
// (the orchestration of nekstab_next_amd/gmres.py dcgs2_cycle, same entry points in the same order).
int nkv_gmres_dcgs2(const nkv_layout* L, const double* w, double* Q, int kmax, double beta, double tol2,
                    double* H_dev, int64_t ldh, double* f, double* scratch_dev, void* ws, nkv_matvec_fn matvec,
                    void* mv_user, nkv_allreduce_fn allreduce, void* ar_user, double* res_hist, int* k_out,
                    unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(Q, "Q"));
    CHECK(check_ptr(f, "f"));
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(ws, "ws"));
    if (!matvec) return fail(NKV_EINVAL, "matvec callback is NULL");
    if (!H_dev || !scratch_dev || !res_hist || !k_out) return fail(NKV_EINVAL, "H/scratch/res_hist/k_out is NULL");
    if (kmax < 1 || kmax + 1 > NKV_MAX_COLS) return fail(NKV_EINVAL, "kmax=%d outside 1..%d", kmax, NKV_MAX_COLS - 1);
    if (ldh < kmax + 1) return fail(NKV_EINVAL, "ldh=%lld < kmax+1=%d", (long long)ldh, kmax + 1);
    hipStream_t st = S(stream);
    const unsigned tf = (flags & NKV_TIME_DOT) ? NKV_TIME : 0u;
    double* hd = scratch_dev;                                      // 2(kmax+1)
    double* coef = scratch_dev + 2 * (kmax + 1);                   // 3 kmax + 5
    double* nrm2 = scratch_dev + nkv_arnoldi_scratch_doubles(kmax) - 1;
    // pinned: the per-column H download is a direct DMA (no staging copy) before the residual test
    double* host = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&host), sizeof(double) * (size_t)(4 * (kmax + 2)),
                      hipHostMallocDefault) != hipSuccess || !host)
        return fail(NKV_EHIP, "gmres: pinned host allocation failed");
    double *h = host, *cs = host + (kmax + 2), *sn = cs + (kmax + 2), *g = sn + (kmax + 2);
    for (int i = 0; i < kmax + 2; ++i) g[i] = 0.0;
    g[0] = beta;
    auto col = [L, Q](int c) { return Q + (int64_t)c * L->ld; };
    auto reduce = [&](double* buf, int n, const char* what) -> int {
        if (!allreduce) return NKV_OK;
        const int rc = allreduce(ar_user, buf, n, stream);
        return rc == 0 ? NKV_OK : fail(NKV_ECALLBACK, "allreduce callback returned %d (%s)", rc, what);
    };
    int rc = NKV_OK, k_used = kmax;
    for (int k = 1; k <= kmax && rc == NKV_OK; ++k) {
        const int m = k - 1;
        double* u = col(m);
        const int mr = matvec(mv_user, u, f, stream);
        if (mr != 0) { rc = fail(NKV_ECALLBACK, "matvec callback returned %d at column %d", mr, k); break; }
        if ((rc = nkv_block_dot2(L, w, Q, k, u, f, hd, ws, tf | NKV_X_IS_LAST, stream)) != NKV_OK) break;
        if ((rc = reduce(hd, 2 * k, "multi-dot")) != NKV_OK) break;
        if ((rc = nkv_dcgs2_coef(m, hd, hd + k, k == 1 ? nullptr : nrm2, H_dev, ldh, coef, ws, stream)) != NKV_OK) break;
        if ((rc = nkv_dcgs2_update(L, w, Q, m, coef, u, f, col(k), nrm2, ws, NKV_TIME | (flags & NKV_TIME_DOT),
                                   stream)) != NKV_OK) break;
        if ((rc = reduce(nrm2, 1, "norm")) != NKV_OK) break;
        // H(0:k, k-1) (once-projected) and ||next u||^2 -> the residual test of column k
        hipError_t e = hipMemcpyAsync(h, H_dev + (int64_t)m * ldh, sizeof(double) * (size_t)k, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(h + k, nrm2, sizeof(double), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) { rc = fail(NKV_EHIP, "gmres: %s", hipGetErrorString(e)); break; }
        h[k] = sqrt(h[k]);
        const double res = nkv_givens_column(m, h, cs, sn, g);
        res_hist[m] = res;
        k_used = k;
        if (res * res < tol2) break;
    }
    (void)hipHostFree(host);
    if (rc != NKV_OK) return rc;
    *k_out = k_used;
    // close: Q column k_used against Q[0:k_used+1] -> H row k_used corrected, H(k_used, k_used-1) final
    const int m = k_used;
    CHECK(nkv_block_dot(L, w, Q, m + 1, col(m), hd, ws, tf, stream));
    CHECK(reduce(hd, m + 1, "closing multi-dot"));
    return nkv_dcgs2_coef(m, hd, nullptr, nrm2, H_dev, ldh, coef, ws, stream);
}

// update_hessenberg_matrix (krylov_decomposition.f90:103-189) as one call: the fused 3-pass CGS2
// sequence of nekstab_next_amd/arnoldi.py (orthonormalize, mode "cgs2") with the all-reduce as a
// callback — q_out = f/||f|| after two projections, H column in hcol_dev[0:j+1].
int nkv_update_hessenberg(const nkv_layout* L, const double* w, const double* Q, int j, double* f, double* q_out,
                          double* hcol_dev, double* scratch_dev, void* ws, nkv_allreduce_fn allreduce, void* ar_user,
                          unsigned flags, void* stream) {
    CHECK(check_layout(L));
    if (!hcol_dev || !scratch_dev) return fail(NKV_EINVAL, "hcol/scratch is NULL");
    if (j < 0 || j > NKV_MAX_COLS) return fail(NKV_EINVAL, "j=%d outside 0..%d", j, NKV_MAX_COLS);
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(f, "f"));
    CHECK(check_ptr(q_out, "q_out"));
    CHECK(check_ptr(ws, "ws"));
    if (j > 0) CHECK(check_ptr(Q, "Q"));
    const unsigned tf = (flags & NKV_TIME_DOT) ? NKV_TIME : 0u;
    double* h1 = scratch_dev;
    double* h2 = scratch_dev + (j + 1);
    double* nrm = scratch_dev + 2 * (j + 1);
    auto reduce = [&](double* buf, int n, const char* what) -> int {
        if (!allreduce) return NKV_OK;
        const int rc = allreduce(ar_user, buf, n, stream);
        return rc == 0 ? NKV_OK : fail(NKV_ECALLBACK, "allreduce callback returned %d (%s)", rc, what);
    };
    if (j == 0) {   // only normalise (the seed)
        CHECK(nkv_dot(L, w, f, f, nrm, ws, tf, stream));
        CHECK(reduce(nrm, 1, "norm"));
        return nkv_arnoldi_finish(L, f, nrm, q_out, 0, h1, nullptr, hcol_dev, 0, stream);
    }
    if (flags & NKV_MGS2) {   // :155-186 in the reference's order; H(i,k) = alpha1 + alpha2 in finish
        // alpha_0 by a dot, then per column ONE fused pass: f -= alpha_i q_i and the next coefficient
        // (alpha_{i+1}, the second pass's alpha_0, or finally ||f||^2) from the same read of f
        CHECK(nkv_dot(L, w, f, Q, h1, ws, tf, stream));
        CHECK(reduce(h1, 1, "first MGS pass"));
        for (int pass = 0; pass < 2; ++pass) {
            double* h = pass == 0 ? h1 : h2;
            for (int i = 0; i < j; ++i) {
                const double* qi = Q + (int64_t)i * L->ld;
                const bool last = i + 1 == j;
                const double* qn = !last ? qi + L->ld : (pass == 0 ? Q : nullptr);   // nullptr: ||f||^2
                double* out = !last ? h + i + 1 : (pass == 0 ? h2 : nrm);
                CHECK(nkv_axpy_dot(L, w, f, h + i, qi, qn, out, ws, NKV_TIME | (tf ? NKV_TIME_DOT : 0u), stream));
                CHECK(reduce(out, 1, last ? (pass == 0 ? "second MGS pass" : "norm") : (pass == 0 ? "first MGS pass" : "second MGS pass")));
            }
        }
        return nkv_arnoldi_finish(L, f, nrm, q_out, j, h1, h2, hcol_dev, 0, stream);
    }
    CHECK(nkv_block_dot(L, w, Q, j, f, h1, ws, tf, stream));
    CHECK(reduce(h1, j, "first projection"));
    CHECK(nkv_block_update_dot(L, w, Q, j, h1, f, h2, ws, NKV_TIME | (tf ? NKV_TIME_DOT : 0u), stream));
    CHECK(reduce(h2, j, "second projection"));
    CHECK(nkv_block_update(L, w, Q, j, h2, f, nrm, ws, NKV_TIME | NKV_NORM2 | (tf ? NKV_TIME_DOT : 0u), stream));
    CHECK(reduce(nrm, 1, "norm"));
    return nkv_arnoldi_finish(L, f, nrm, q_out, j, h1, h2, hcol_dev, 0, stream);
}

// ---- "mgs2-lagged" host algebra (nekstab_next_amd/arnoldi.py, lagged_coefficients): MGS2's
// coefficients for any basis (alpha = (I + L)^-1 Q^T W f, L the strictly lower part of the Gram matrix
// G) with the second pass of a column lagged into the next step's two-vector multi-dot, as DCGS2 does.
// Host-only (no device work); the Python mode and the one-call driver below both run it, so the two
// are bit-identical.  G: row-major, ldg >= c+1, symmetric (both triangles kept); H: column-major,
// ldh >= c+1.  stage 1 (first step of a factorisation, Q[c] final): hv = [Q[0:c+1]^T W q_c ;
// Q[0:c+1]^T W A q_c]; G row c <- hv[0:c+1], alpha = (I+L)^-1 hv[c+1:2c+2].  stage 0 (Q[c] holds u,
// the previous first-pass result): hv = [p ; u.u ; t ; u.A u] with p = Q[0:c]^T W u, t = Q[0:c]^T W A u;
// beta = (I+L)^-1 p, r^2 = u.u - 2 beta.p + beta^T G beta (NKV_ENAN unless > 0), H(0:c, c-1) += beta,
// H(c, c-1) = r, G row c = (p - G beta)/r (diagonal 1), alpha = (I+L)^-1 ([t ; (u.A u - beta.t)/r] -
// G H beta)/r with H = H(0:c+1, 0:c).  Both: H(0:c+1, c) = alpha and coef (3c+5, the layout of
// nkv_dcgs2_update) = [x = z[0:c] | 0 (c+1) | 1/r, z[c], 0, 1 | beta], z = H beta / r + alpha (stage 1:
// z = alpha, r = 1, beta = 0).  stage 2 (closing pass of the last column c): hv = Q[0:c]^T W u; coef[0:c]
// = beta = (I+L)^-1 hv, H(0:c, c-1) += beta.
static void unit_lower_solve(const double* G, int64_t ldg, int n, const double* rhs, double* x) {
    for (int i = 0; i < n; ++i) {
        double s = rhs[i];
        for (int l = 0; l < i; ++l) s -= G[(int64_t)i * ldg + l] * x[l];
        x[i] = s;
    }
}

int nkv_lagged_coef(int c, int stage, const double* hv, double* G, int64_t ldg, double* H, int64_t ldh,
                    double* coef) {
    if (c < 0 || c + 1 > NKV_MAX_COLS + 1 || stage < 0 || stage > 2 || (stage != 1 && c == 0))
        return fail(NKV_EINVAL, "lagged coefficients: c=%d, stage=%d", c, stage);
    if (!hv || !G || !H || !coef) return fail(NKV_EINVAL, "lagged coefficients: a NULL array");
    if (ldg < c + 1 || ldh < c + 1) return fail(NKV_EINVAL, "lagged coefficients: ldg=%lld, ldh=%lld < %d",
                                                (long long)ldg, (long long)ldh, c + 1);
    const int j = c + 1;
    auto g = [G, ldg](int i, int l) -> double& { return G[(int64_t)i * ldg + l]; };
    auto h = [H, ldh](int i, int col) -> double& { return H[(int64_t)col * ldh + i]; };
    std::vector<double> beta(c > 0 ? c : 1), alpha(j), z(j), Gb(c > 0 ? c : 1), Hb(j), b(j);
    if (stage == 2) {
        unit_lower_solve(G, ldg, c, hv, beta.data());
        for (int i = 0; i < c; ++i) {
            h(i, c - 1) += beta[i];
            coef[i] = beta[i];
        }
        return NKV_OK;
    }
    for (int k = 0; k < 3 * c + 5; ++k) coef[k] = 0.0;
    double rinv = 1.0;
    if (stage == 1) {
        for (int i = 0; i < j; ++i) g(c, i) = g(i, c) = hv[i];
        unit_lower_solve(G, ldg, j, hv + j, alpha.data());
        for (int i = 0; i < j; ++i) z[i] = alpha[i];
    } else {
        const double* p = hv;
        const double pu = hv[c];
        const double* t = hv + j;
        const double tu = hv[j + c];
        unit_lower_solve(G, ldg, c, p, beta.data());
        double bp = 0.0, bgb = 0.0, bt = 0.0;
        for (int i = 0; i < c; ++i) {
            double s = 0.0;
            for (int l = 0; l < c; ++l) s += g(i, l) * beta[l];
            Gb[i] = s;
        }
        for (int i = 0; i < c; ++i) {
            bp += beta[i] * p[i];
            bgb += beta[i] * Gb[i];
            bt += beta[i] * t[i];
        }
        const double r2 = pu - 2.0 * bp + bgb;
        if (!(std::isfinite(r2) && r2 > 0.0))
            return fail(NKV_ENAN, "mgs2-lagged: column %d has no new direction (r^2 = %.6g)", c, r2);
        const double r = sqrt(r2);
        for (int i = 0; i < c; ++i) h(i, c - 1) += beta[i];
        h(c, c - 1) = r;
        for (int i = 0; i < c; ++i) g(c, i) = g(i, c) = (p[i] - Gb[i]) / r;
        g(c, c) = 1.0;
        for (int i = 0; i < j; ++i) {
            double s = 0.0;
            for (int l = 0; l < c; ++l) s += h(i, l) * beta[l];
            Hb[i] = s;
        }
        for (int i = 0; i < j; ++i) {
            double s = 0.0;
            for (int l = 0; l < j; ++l) s += g(i, l) * Hb[l];
            const double bq = i < c ? t[i] : (tu - bt) / r;
            b[i] = (bq - s) / r;
        }
        unit_lower_solve(G, ldg, j, b.data(), alpha.data());
        for (int i = 0; i < j; ++i) z[i] = Hb[i] / r + alpha[i];
        for (int i = 0; i < c; ++i) coef[2 * c + 5 + i] = beta[i];
        rinv = 1.0 / r;
    }
    for (int i = 0; i < j; ++i) h(i, c) = alpha[i];
    for (int i = 0; i < c; ++i) coef[i] = z[i];
    coef[2 * c + 1] = rinv;
    coef[2 * c + 2] = z[c];
    coef[2 * c + 4] = 1.0;
    return NKV_OK;
}

// arnoldi_factorization (krylov_decomposition.f90:68-96) with the per-column update above: every
// column final when its step ends (the cgs2 / mgs2 modes of nekstab_next_amd/arnoldi.py as one call).
int nkv_arnoldi_factorization(const nkv_layout* L, const double* w, double* Q, int mstart, int mend, double* H_dev,
                              int64_t ldh, double* f, double* scratch_dev, void* ws, nkv_matvec_fn matvec,
                              void* mv_user, nkv_allreduce_fn allreduce, void* ar_user, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(Q, "Q"));
    CHECK(check_ptr(f, "f"));
    if (!matvec) return fail(NKV_EINVAL, "matvec callback is NULL");
    if (!H_dev || !scratch_dev) return fail(NKV_EINVAL, "H/scratch is NULL");
    if (mstart < 1 || mend > NKV_MAX_COLS) return fail(NKV_EINVAL, "steps %d..%d outside 1..%d", mstart, mend, NKV_MAX_COLS);
    if (mend < mstart) return NKV_OK;
    if (ldh < mend + 1) return fail(NKV_EINVAL, "ldh=%lld < mend+1=%d", (long long)ldh, mend + 1);
    if (flags & NKV_MGS_LAGGED) {   // the "mgs2-lagged" sequence of nekstab_next_amd/arnoldi.py (_lagged_*)
        if (flags & (NKV_MGS2 | NKV_MGS_ICWY)) return fail(NKV_EINVAL, "NKV_MGS_LAGGED excludes NKV_MGS2 / NKV_MGS_ICWY");
        CHECK(check_ptr(w, "w"));
        CHECK(check_ptr(ws, "ws"));
        hipStream_t st = S(stream);
        const unsigned tf = (flags & NKV_TIME_DOT) ? NKV_TIME : 0u;
        const unsigned dotf = NKV_TIME | (tf ? NKV_TIME_DOT : 0u);
        const int64_t ldg = mend + 1;
        double* hd = scratch_dev;                  // 2(mend+1)
        double* coef = hd + 2 * ldg;               // 3 mend + 5
        double* nrm = coef + 3 * mend + 6;         // + 2: within nkv_arnoldi_scratch_doubles(mend)
        double* bet = nrm + 1;
        auto col = [L, Q](int c) { return Q + (int64_t)c * L->ld; };
        auto reduce = [&](double* buf, int n, const char* what) -> int {
            if (!allreduce) return NKV_OK;
            const int rc = allreduce(ar_user, buf, n, stream);
            return rc == 0 ? NKV_OK : fail(NKV_ECALLBACK, "allreduce callback returned %d (%s)", rc, what);
        };
        auto d2h = [&](double* dst, const double* src, size_t n) -> int {   // stream-ordered, then waited for
            hipError_t e = hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            return e == hipSuccess ? NKV_OK : fail(NKV_EHIP, "mgs2-lagged: %s", hipGetErrorString(e));
        };
        std::vector<double> Gh((size_t)ldg * (size_t)ldg, 0.0), Hh((size_t)ldh * (size_t)mend), hv(2 * ldg),
            ch(3 * (size_t)mend + 5);
        CHECK(d2h(Hh.data(), H_dev, Hh.size()));
        for (int i = 0; i + 1 < mstart; ++i) {   // Gram rows of the columns before mstart (row mstart-1: step mstart)
            CHECK(nkv_block_dot(L, w, Q, i + 1, col(i), hd, ws, tf, stream));
            CHECK(reduce(hd, i + 1, "Gram row"));
            CHECK(d2h(hv.data(), hd, (size_t)(i + 1)));
            for (int l = 0; l <= i; ++l) Gh[(size_t)i * ldg + l] = Gh[(size_t)l * ldg + i] = hv[l];
        }
        for (int j = mstart; j <= mend; ++j) {
            const int c = j - 1;
            const int rc = matvec(mv_user, col(c), f, stream);
            if (rc != 0) return fail(NKV_ECALLBACK, "matvec callback returned %d at step %d", rc, j);
            CHECK(nkv_block_dot2(L, w, Q, j, col(c), f, hd, ws, tf | NKV_X_IS_LAST, stream));
            CHECK(reduce(hd, 2 * j, "multi-dot"));
            CHECK(d2h(hv.data(), hd, (size_t)(2 * j)));
            CHECK(nkv_lagged_coef(c, j == mstart ? 1 : 0, hv.data(), Gh.data(), ldg, Hh.data(), ldh, ch.data()));
            NKV_HIP(hipMemcpyAsync(coef, ch.data(), (3 * (size_t)c + 5) * sizeof(double), hipMemcpyHostToDevice, st));
            CHECK(nkv_dcgs2_update(L, w, Q, c, coef, col(c), f, col(j), nullptr, ws, dotf, stream));
        }
        const int m = mend;   // closing pass: finish the provisional column mend
        CHECK(nkv_block_dot(L, w, Q, m + 1, col(m), hd, ws, tf, stream));
        CHECK(reduce(hd, m + 1, "closing multi-dot"));
        CHECK(d2h(hv.data(), hd, (size_t)(m + 1)));
        CHECK(nkv_lagged_coef(m, 2, hv.data(), Gh.data(), ldg, Hh.data(), ldh, ch.data()));
        NKV_HIP(hipMemcpyAsync(coef, ch.data(), (size_t)m * sizeof(double), hipMemcpyHostToDevice, st));
        CHECK(nkv_block_update(L, w, Q, m, coef, col(m), nrm, ws, NKV_NORM2 | dotf, stream));
        CHECK(reduce(nrm, 1, "norm"));
        CHECK(nkv_normalize_dev(L, col(m), nrm, bet, 0, stream));
        CHECK(d2h(hv.data(), bet, 1));
        if (!(std::isfinite(hv[0]) && hv[0] > 0.0))
            return fail(NKV_ENAN, "mgs2-lagged: the last column has no new direction (||u|| = %.6g)", hv[0]);
        Hh[(size_t)(m - 1) * ldh + m] = hv[0];
        NKV_HIP(hipMemcpyAsync(H_dev, Hh.data(), Hh.size() * sizeof(double), hipMemcpyHostToDevice, st));
        NKV_HIP(hipStreamSynchronize(st));   // the host copies above must outlive the transfer
        return (flags & NKV_CHECK_BREAKDOWN) ? check_breakdown(H_dev, ldh, mstart - 1, mend, ws, stream) : NKV_OK;
    }
    if (flags & NKV_MGS_ICWY) {   // the "mgs2-icwy" sequence of nekstab_next_amd/arnoldi.py (_icwy_step)
        if (flags & NKV_MGS2) return fail(NKV_EINVAL, "NKV_MGS2 and NKV_MGS_ICWY are exclusive");
        CHECK(check_ptr(w, "w"));
        CHECK(check_ptr(ws, "ws"));
        const unsigned tf = (flags & NKV_TIME_DOT) ? NKV_TIME : 0u;
        const unsigned dotf = NKV_TIME | (tf ? NKV_TIME_DOT : 0u);
        const int64_t ldg = mend + 1;
        double* hd = scratch_dev;
        double* h1 = hd + 2 * ldg;
        double* h2 = h1 + ldg;
        double* nrm = h2 + ldg;
        double* G = nrm + 2;   // 16-byte aligned (the scratch is)
        auto col = [L, Q](int c) { return Q + (int64_t)c * L->ld; };
        auto reduce = [&](double* buf, int n, const char* what) -> int {
            if (!allreduce) return NKV_OK;
            const int rc = allreduce(ar_user, buf, n, stream);
            return rc == 0 ? NKV_OK : fail(NKV_ECALLBACK, "allreduce callback returned %d (%s)", rc, what);
        };
        for (int i = 1; i + 1 < mstart; ++i) {   // Gram rows of the columns before mstart (row mstart-1: step mstart)
            CHECK(nkv_block_dot(L, w, Q, i, col(i), G + i * ldg, ws, tf, stream));
            CHECK(reduce(G + i * ldg, i, "Gram row"));
        }
        for (int j = mstart; j <= mend; ++j) {
            const int rc = matvec(mv_user, col(j - 1), f, stream);
            if (rc != 0) return fail(NKV_ECALLBACK, "matvec callback returned %d at step %d", rc, j);
            CHECK(nkv_block_dot2(L, w, Q, j, col(j - 1), f, hd, ws, tf | NKV_X_IS_LAST, stream));
            CHECK(reduce(hd, 2 * j, "Gram row and first MGS pass"));
            CHECK(nkv_mgs_icwy_solve(j, G, ldg, hd, hd + j, h1, stream));
            CHECK(nkv_block_update_dot(L, w, Q, j, h1, f, h2, ws, dotf, stream));
            CHECK(reduce(h2, j, "second MGS pass"));
            CHECK(nkv_mgs_icwy_solve(j, G, ldg, nullptr, h2, h2, stream));
            CHECK(nkv_block_update(L, w, Q, j, h2, f, nrm, ws, NKV_NORM2 | dotf, stream));
            CHECK(reduce(nrm, 1, "norm"));
            CHECK(nkv_arnoldi_finish(L, f, nrm, col(j), j, h1, h2, H_dev + (int64_t)(j - 1) * ldh, 0, stream));
        }
        return (flags & NKV_CHECK_BREAKDOWN) ? check_breakdown(H_dev, ldh, mstart - 1, mend, ws, stream) : NKV_OK;
    }
    const unsigned uf = flags & (NKV_TIME_DOT | NKV_MGS2);
    for (int j = mstart; j <= mend; ++j) {   // f = A Q(j); orthonormalise against Q(1..j); Q(j+1) = f (:75-81)
        double* x = Q + (int64_t)(j - 1) * L->ld;
        const int rc = matvec(mv_user, x, f, stream);
        if (rc != 0) return fail(NKV_ECALLBACK, "matvec callback returned %d at step %d", rc, j);
        CHECK(nkv_update_hessenberg(L, w, Q, j, f, Q + (int64_t)j * L->ld, H_dev + (int64_t)(j - 1) * ldh, scratch_dev,
                                    ws, allreduce, ar_user, uf, stream));
    }
    return (flags & NKV_CHECK_BREAKDOWN) ? check_breakdown(H_dev, ldh, mstart - 1, mend, ws, stream) : NKV_OK;
}

// Host function (no device work): one column of the GMRES least-squares residual update
// (newton_krylov.f90:255-258 without solving for y).  h = H(0:k+1, k) of column k (0-based), cs/sn the
// k rotations stored so far (rotation k is appended), g the rotated right-hand side (g[k], g[k+1]
// updated; g[0] = beta on the first call).  Returns |g[k+1]| = ||beta e_1 - H y|| of the (k+2) x (k+1)
// least-squares problem; h is overwritten with the triangularised column.
double nkv_givens_column(int k, double* h, double* cs, double* sn, double* g) {
    if (k < 0 || !h || !cs || !sn || !g) {   // no status channel: a NaN residual never passes a test
        fail(NKV_EINVAL, "givens: k=%d or a NULL array", k);
        return std::nan("");
    }
    for (int i = 0; i < k; ++i) {
        const double t = cs[i] * h[i] + sn[i] * h[i + 1];
        h[i + 1] = -sn[i] * h[i] + cs[i] * h[i + 1];
        h[i] = t;
    }
    const double a = h[k], b = h[k + 1];
    const double r = std::hypot(a, b);
    const double c = r == 0.0 ? 1.0 : a / r, s = r == 0.0 ? 0.0 : b / r;
    cs[k] = c;
    sn[k] = s;
    h[k] = r;
    h[k + 1] = 0.0;
    g[k + 1] = -s * g[k];
    g[k] = c * g[k];
    return std::fabs(g[k + 1]);
}

}  // extern "C"
