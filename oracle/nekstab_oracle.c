/*
 * nekstab_oracle.c — CPU restatement of nekStab's Krylov hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline — never as the thing measured or shipped.
 * Parity status: the reference (Fortran compiled into Nek5000) cannot be built here without
 * stand-ins for Nek5000's SIZE/TOTAL headers and routines, so this restatement is checked against
 * closed-form known answers (tests/test_oracle_*.py) — "parity unpinned" against reference
 * outputs, see DESIGN.md §3.
 *
 * Layout (the reference's own, unpadded): one vector = [vx | vy | (vz) | t_1..t_s | pr | time],
 * each weighted field nv doubles, pressure np doubles, `time` the last double
 * (type krylov_vector, core/krylov_subspace.f90:12-17).  Weighted fields share the weights
 * bm1s (nv doubles).
 *
 * Operation order follows the reference line by line, compiled without FP contraction, so with
 * one thread every sum is the reference's sequential sum.  orc_set_threads(n > 1) parallelises
 * the loops with OpenMP (the CPU-baseline timing mode); sums are then regrouped.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int64_t nv;      /* points per weighted field (lx1*ly1*lz1*nelv)            */
    int64_t np;      /* pressure points (lx2*ly2*lz2*nelv)                      */
    int32_t nwf;     /* weighted fields: 2|3 velocities + active scalars        */
    int32_t time_in_dot; /* k_dot includes p%time*q%time iff uparam(1)==2.1 (:52-54) */
} orc_layout;

static int g_threads = 1;

void orc_set_threads(int n) {
    g_threads = n < 1 ? 1 : n;
#ifdef _OPENMP
    omp_set_num_threads(g_threads);
#endif
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

static inline int64_t n_all(const orc_layout* L) { return (int64_t)L->nwf * L->nv + L->np; }
static inline int64_t t_off(const orc_layout* L) { return n_all(L); }
int64_t orc_vector_len(const orc_layout* L) { return n_all(L) + 1; }

/* glsc3(a, b, mult, n) = sum_i a(i)*b(i)*mult(i) then gop('+')  [Nek5000, external]: the local
 * loop, left-to-right product. Single process: the all-reduce is the identity. */
double orc_glsc3(const double* a, const double* b, const double* mult, int64_t n) {
    double tmp = 0.0;
    if (g_threads > 1) {
#pragma omp parallel for reduction(+ : tmp) schedule(static) num_threads(g_threads)
        for (int64_t i = 0; i < n; ++i) tmp += a[i] * b[i] * mult[i];
    } else {
        for (int64_t i = 0; i < n; ++i) tmp = tmp + a[i] * b[i] * mult[i];
    }
    return tmp;
}

/* k_dot (krylov_subspace.f90:26-60): alpha = glsc3(p%vx,bm1s,q%vx) + glsc3(p%vy,..) [+ vz] [+ t..]
 * [+ p%time*q%time]; NaN -> returns NaN (the reference calls nek_end). */
double orc_k_dot(const orc_layout* L, const double* w, const double* p, const double* q) {
    double alpha = orc_glsc3(p, w, q, L->nv) + orc_glsc3(p + L->nv, w, q + L->nv, L->nv);
    for (int f = 2; f < L->nwf; ++f) alpha = alpha + orc_glsc3(p + f * L->nv, w, q + f * L->nv, L->nv);
    if (L->time_in_dot) alpha = alpha + p[t_off(L)] * q[t_off(L)];
    return alpha;
}

/* real_dot (nek_vectors.f90:80-114): the same fields, time ALWAYS included (:106). */
double orc_real_dot(const orc_layout* L, const double* w, const double* p, const double* q) {
    orc_layout l2 = *L;
    l2.time_in_dot = 1;
    return orc_k_dot(&l2, w, p, q);
}

/* Elementwise family over every stored field (nop* helpers, nek_vectors.f90:209-362) + time. */
void orc_k_cmult(const orc_layout* L, double* p, double c) {
    const int64_t n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) p[i] = p[i] * c;
    p[n] = p[n] * c;
}

void orc_k_add2(const orc_layout* L, double* p, const double* q) {
    const int64_t n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) p[i] = p[i] + q[i];
    p[n] = p[n] + q[n];
}

void orc_k_sub2(const orc_layout* L, double* p, const double* q) {
    const int64_t n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) p[i] = p[i] - q[i];
    p[n] = p[n] - q[n];
}

void orc_k_sub3(const orc_layout* L, double* p, const double* q, const double* r) {
    const int64_t n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) p[i] = q[i] - r[i];
    p[n] = q[n] - r[n];
}

void orc_k_zero(const orc_layout* L, double* p) {
    const int64_t n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) p[i] = 0.0;
    p[n] = 0.0;
}

void orc_k_copy(const orc_layout* L, double* p, const double* q) {
    const int64_t n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) p[i] = q[i];
    p[n] = q[n];
}

/* real_axpby (nek_vectors.f90:127-139 -> axpby :250-256): x(i) = x(i)*alpha + y(i)*beta over the
 * fields incl. pressure; time NOT updated. */
void orc_real_axpby(const orc_layout* L, double* x, double alpha, const double* y, double beta) {
    const int64_t n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) x[i] = x[i] * alpha + y[i] * beta;
}

/* update_hessenberg_matrix (krylov_decomposition.f90:103-189), MGS + full re-orthogonalisation.
 * Q: k vectors at stride orc_vector_len(L).  Hcol: k+1 entries (column k of H).  wrk: one vector. */
void orc_update_hessenberg(const orc_layout* L, const double* w, double* Hcol, double* f, const double* Q,
                           int k, double* wrk) {
    const int64_t ld = orc_vector_len(L);
    double alpha, beta;
    for (int i = 0; i < k; ++i) Hcol[i] = 0.0; /* rzero(h_vec) */
    beta = sqrt(orc_k_dot(L, w, f, f));         /* k_norm(beta, f) — result unused (:152) */
    (void)beta;
    for (int i = 0; i < k; ++i) { /* :155-168 */
        orc_k_copy(L, wrk, Q + (int64_t)i * ld);
        alpha = orc_k_dot(L, w, f, wrk);
        orc_k_cmult(L, wrk, alpha);
        orc_k_sub2(L, f, wrk);
        Hcol[i] = alpha;
    }
    for (int i = 0; i < k; ++i) { /* :171-180 */
        orc_k_copy(L, wrk, Q + (int64_t)i * ld);
        alpha = orc_k_dot(L, w, f, wrk);
        orc_k_cmult(L, wrk, alpha);
        orc_k_sub2(L, f, wrk);
        Hcol[i] = Hcol[i] + alpha;
    }
    alpha = sqrt(orc_k_dot(L, w, f, f)); /* k_normalize(f, alpha) :183 */
    orc_k_cmult(L, f, 1.0 / alpha);
    Hcol[k] = alpha;
}

/* k_matmul (krylov_subspace.f90:163-209): dq = sum_i y_i Q(i) field-wise (Fortran matmul order:
 * for each row, sum over i ascending), time = dot_product(times, y). */
void orc_k_matmul(const orc_layout* L, double* dq, const double* Q, const double* y, int k) {
    const int64_t ld = orc_vector_len(L), n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t r = 0; r < n; ++r) {
        double s = 0.0;
        for (int i = 0; i < k; ++i) s = s + Q[(int64_t)i * ld + r] * y[i];
        dq[r] = s;
    }
    double t = 0.0;
    for (int i = 0; i < k; ++i) t = t + Q[(int64_t)i * ld + n] * y[i];
    dq[n] = t;
}

/* schur_condensation basis update (eigensolvers.f90:421-442): Q(:,1:k) <- Q(:,1:k) V, fields only
 * (vx..t, pr), time untouched.  V is k x k column-major. */
void orc_rotate(const orc_layout* L, double* Q, int k, const double* V) {
    const int64_t ld = orc_vector_len(L), n = n_all(L);
#pragma omp parallel num_threads(g_threads) if (g_threads > 1)
    {
        double* row = (double*)malloc(sizeof(double) * (size_t)k);
#pragma omp for schedule(static)
        for (int64_t r = 0; r < n; ++r) {
            for (int i = 0; i < k; ++i) row[i] = Q[(int64_t)i * ld + r];
            for (int c = 0; c < k; ++c) {
                double s = 0.0;
                for (int i = 0; i < k; ++i) s = s + row[i] * V[(int64_t)c * k + i];
                Q[(int64_t)c * ld + r] = s;
            }
        }
        free(row);
    }
}

/* ---- synthetic operators ------------------------------------------------ */
void orc_op_diag(const orc_layout* L, const double* d, const double* x, double* y, double time_scale) {
    const int64_t n = n_all(L);
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) y[i] = d[i] * x[i];
    y[n] = time_scale * x[n];
}

/* ---- shard-independent generator (same bits as the device generator) -------------------- */
static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_fill_hash(const orc_layout* L, double* x, uint64_t seed, int64_t voff, int64_t poff) {
    const uint64_t key0 = seed * 0xD1342543DE82EF95ull;
    /* every element is a pure function of its index: threads change nothing but the speed */
    for (int f = 0; f < L->nwf; ++f)
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
        for (int64_t i = 0; i < L->nv; ++i) {
            const uint64_t z = mix64(key0 + (uint64_t)f * 0x9E3779B97F4A7C15ull + (uint64_t)(voff + i));
            x[(int64_t)f * L->nv + i] = 2.0 * ((double)(z >> 11) * 0x1.0p-53) - 1.0;
        }
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < L->np; ++i) {
        const uint64_t z = mix64(key0 + 31ull * 0x9E3779B97F4A7C15ull + (uint64_t)(poff + i));
        x[(int64_t)L->nwf * L->nv + i] = 2.0 * ((double)(z >> 11) * 0x1.0p-53) - 1.0;
    }
    x[n_all(L)] = 0.0;
}

/* ---- ordering rules of the restart (independent C transliteration of the Fortran) --------- */

/* quicksort2 (core/utils.f90:29-138), 1-based in the original; arr and idx (1-based values)
 * modified in place.  NOTE: transliterated as written, including its partition step. */
void orc_quicksort2(int n, double* arr1, int* idx1) {
    double* arr = arr1 - 1; /* 1-based views */
    int* idx = idx1 - 1;
    const int m = 7, nstack = 50;
    int istack[51];
    int i, ir, j, jstack = 0, k, l = 1, b, ti;
    double a, t;
    ir = n;
    for (;;) {
        if (ir - l < m) {
            for (j = l + 1; j <= ir; ++j) {
                a = arr[j];
                b = idx[j];
                i = j - 1;
                while (i >= l && arr[i] > a) {
                    arr[i + 1] = arr[i];
                    idx[i + 1] = idx[i];
                    i = i - 1;
                }
                arr[i + 1] = a;
                idx[i + 1] = b;
            }
            if (jstack == 0) return;
            ir = istack[jstack];
            l = istack[jstack - 1];
            jstack = jstack - 2;
        } else {
            k = (l + ir) / 2;
            t = arr[k]; arr[k] = arr[l + 1]; arr[l + 1] = t;
            ti = idx[k]; idx[k] = idx[l + 1]; idx[l + 1] = ti;
            if (arr[l] > arr[ir]) { t = arr[l]; arr[l] = arr[ir]; arr[ir] = t; ti = idx[l]; idx[l] = idx[ir]; idx[ir] = ti; }
            if (arr[l + 1] > arr[ir]) { t = arr[l + 1]; arr[l + 1] = arr[ir]; arr[ir] = t; ti = idx[l + 1]; idx[l + 1] = idx[ir]; idx[ir] = ti; }
            if (arr[l] > arr[l + 1]) { t = arr[l]; arr[l] = arr[l + 1]; arr[l + 1] = t; ti = idx[l]; idx[l] = idx[l + 1]; idx[l + 1] = ti; }
            i = l + 1;
            j = ir;
            a = arr[l + 1];
            b = idx[l + 1];
            for (;;) {
                while (arr[i] < a) i = i + 1;
                while (arr[j] > a) j = j - 1;
                if (i >= j) break;
                t = arr[i]; arr[i] = arr[j]; arr[j] = t;
                ti = idx[i]; idx[i] = idx[j]; idx[j] = ti;
                i = i + 1;
                j = j - 1;
            }
            arr[l + 1] = arr[j];
            arr[j] = a;
            idx[l + 1] = idx[j];
            idx[j] = b;
            jstack = jstack + 2;
            if (jstack > nstack) return; /* "NSTACK too small" */
            if (ir - i + 1 >= j - l) {
                istack[jstack] = ir;
                istack[jstack - 1] = i;
                ir = j - 1;
            } else {
                istack[jstack] = j - 1;
                istack[jstack - 1] = l;
                l = i;
            }
        }
    }
}

/* select_eigenvalues (eigensolvers.f90:688-754).  re/im: n eigenvalues (Schur order).
 * selected: n ints (0/1).  Returns cnt. */
int orc_select_eigenvalues(int n, const double* re, const double* im, double delta, int nev, int* selected) {
    int* idx = (int*)malloc(sizeof(int) * (size_t)n);
    double* mod = (double*)malloc(sizeof(double) * (size_t)n);
    for (int i = 0; i < n; ++i) {
        idx[i] = i + 1;
        mod[i] = hypot(re[i], im[i]); /* abs(complex) */
    }
    double* arr = (double*)malloc(sizeof(double) * (size_t)n);
    memcpy(arr, mod, sizeof(double) * (size_t)n);
    orc_quicksort2(n, arr, idx);
    /* k_dim < nev+4 would index idx(0) and below (out of bounds in the reference too): refused,
     * as the product does; at k_dim == nev+4 the conjugate check has no idx(0) to look at. */
    if (n - (nev + 4) < 0) {
        free(idx);
        free(mod);
        free(arr);
        return -1;
    }
    for (int i = 0; i < n; ++i) selected[i] = mod[i] >= (1.0 - delta);
    for (int p = n - (nev + 3); p <= n; ++p) selected[idx[p - 1] - 1] = 1; /* idx(n-(nev+3):n) */
    if (n - (nev + 4) >= 1) {
        const int a = idx[n - (nev + 3) - 1] - 1, b = idx[n - (nev + 4) - 1] - 1;
        if (im[a] == -im[b]) selected[b] = 1;
    }
    int cnt = 0;
    for (int i = 0; i < n; ++i) cnt += selected[i] ? 1 : 0;
    free(idx);
    free(mod);
    free(arr);
    return cnt;
}

/* sort_eigendecomp (lapack_wrapper.f90:181-228): exchange sort on sqrt(re^2+im^2), strict <.
 * vecs_re/vecs_im: n x n column-major. */
void orc_sort_eigendecomp(int n, double* re, double* im, double* vre, double* vim) {
    double* nrm = (double*)malloc(sizeof(double) * (size_t)n);
    for (int i = 0; i < n; ++i) nrm[i] = sqrt(re[i] * re[i] + im[i] * im[i]);
    for (int k = 0; k < n - 1; ++k)
        for (int l = k + 1; l < n; ++l)
            if (nrm[k] < nrm[l]) {
                double t = nrm[k]; nrm[k] = nrm[l]; nrm[l] = t;
                t = re[k]; re[k] = re[l]; re[l] = t;
                t = im[k]; im[k] = im[l]; im[l] = t;
                for (int r = 0; r < n; ++r) {
                    t = vre[(int64_t)k * n + r]; vre[(int64_t)k * n + r] = vre[(int64_t)l * n + r]; vre[(int64_t)l * n + r] = t;
                    t = vim[(int64_t)k * n + r]; vim[(int64_t)k * n + r] = vim[(int64_t)l * n + r]; vim[(int64_t)l * n + r] = t;
                }
            }
    free(nrm);
}
