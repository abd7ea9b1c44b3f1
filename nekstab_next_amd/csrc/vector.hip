// vector.hip — BLAS-1 over the (vx, vy, [vz], t.., pr, time) layout, weighted dots and multi-dots
// (k_dot / real_dot / glsc3), normalisation, the reference-order MGS column step (krylov_subspace.f90,
// nek_vectors.f90, krylov_decomposition.f90:155-186).
#include "nkv_internal.h"

namespace {

// ------------------------------------------------------------------------------------------
// block weighted multi-dot:  partials[c][b] = sum over this block's tiles of q_c . (w f)
// grid = (bx, n_wf): blockIdx.y is the weighted field, so the weight index is the row within
// the field (no per-element division).  Each thread keeps its 8 rows of w.f in registers and
// streams the j basis columns past them, kColUnroll columns in flight.
// ------------------------------------------------------------------------------------------
template <int kPairs>
__global__ __launch_bounds__(kThreads) void k_block_dot(const double* __restrict__ Q, int64_t ld,
                                                        int j, const double* __restrict__ f,
                                                        const double* __restrict__ w, int64_t sv,
                                                        int tiles_per_field,
                                                        double* __restrict__ partials, int B) {
    constexpr int kTile = kThreads * kPairs * 2;
    extern __shared__ double red[];  // [4 waves][j]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int c = threadIdx.x; c < 4 * j; c += kThreads) red[c] = 0.0;
    __syncthreads();

    const int64_t fb = (int64_t)blockIdx.y * sv;
    for (int t = blockIdx.x; t < tiles_per_field; t += gridDim.x) {
        const int64_t r0 = (int64_t)t * kTile + 2 * threadIdx.x;
        double2 wf[kPairs];
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            const double2 wv = ld2(w + r0 + k * 2 * kThreads);
            const double2 fv = ld2(f + fb + r0 + k * 2 * kThreads);
            wf[k].x = wv.x * fv.x;
            wf[k].y = wv.y * fv.y;
        }
        const double* qb = Q + fb + r0;
        int c = 0;
        for (; c + kColUnroll <= j; c += kColUnroll) {
            double2 q[kColUnroll][kPairs];
#pragma unroll
            for (int u = 0; u < kColUnroll; ++u)
#pragma unroll
                for (int k = 0; k < kPairs; ++k) q[u][k] = ldq(qb + (int64_t)(c + u) * ld + k * 2 * kThreads);
            double s[kColUnroll];
#pragma unroll
            for (int u = 0; u < kColUnroll; ++u) {
                double a = 0.0;
#pragma unroll
                for (int k = 0; k < kPairs; ++k) {
                    a = fma(q[u][k].x, wf[k].x, a);
                    a = fma(q[u][k].y, wf[k].y, a);
                }
                s[u] = a;
            }
#if NKV_D2_RED && NKV_COLU == 4   // four columns = four sums
            const double v = wave_sum4(s[0], s[1], s[2], s[3], lane);
            if ((lane & 15) == 0) red[wave * j + c + (lane >> 4)] += v;
#else
#pragma unroll
            for (int off = 32; off > 0; off >>= 1)
#pragma unroll
                for (int u = 0; u < kColUnroll; ++u) s[u] += __shfl_xor(s[u], off, 64);
            if (lane == 0) {
#pragma unroll
                for (int u = 0; u < kColUnroll; ++u) red[wave * j + c + u] += s[u];
            }
#endif
        }
        for (; c < j; ++c) {
            double a = 0.0;
#pragma unroll
            for (int k = 0; k < kPairs; ++k) {
                const double2 q = ldq(qb + (int64_t)c * ld + k * 2 * kThreads);
                a = fma(q.x, wf[k].x, a);
                a = fma(q.y, wf[k].y, a);
            }
            a = wave_sum(a);
            if (lane == 0) red[wave * j + c] += a;
        }
    }
    __syncthreads();
    const int b = blockIdx.y * gridDim.x + blockIdx.x;
    for (int c = threadIdx.x; c < j; c += kThreads)
        partials[(int64_t)c * B + b] = (red[c] + red[j + c]) + (red[2 * j + c] + red[3 * j + c]);
}

// Second stage: out[c] = sum_b partials[c][b] in a fixed order (+ replicated time term).
// Columns c >= jc are a second right-hand side (two-vector multi-dot): their time term uses tb2
// and basis column c - jc.
__global__ __launch_bounds__(kThreads) void k_reduce_cols(const double* __restrict__ partials, int B,
                                                          double* __restrict__ out,
                                                          const double* __restrict__ ta, int64_t lda,
                                                          const double* __restrict__ tb,
                                                          const double* __restrict__ tb2, int jc,
                                                          int* __restrict__ nan_flag) {
    __shared__ double lds4[4];
    const int c = blockIdx.x;
    double s = 0.0;
    for (int b = threadIdx.x; b < B; b += kThreads) s += partials[(int64_t)c * B + b];
    s = block_sum(s, lds4);
    if (threadIdx.x == 0) {
        if (ta) s += (c < jc) ? ta[(int64_t)c * lda] * tb[0] : ta[(int64_t)(c - jc) * lda] * tb2[0];
        if (s != s) atomicOr(nan_flag, 1);
        out[c] = s;
    }
}

// ------------------------------------------------------------------------------------------
// Fused MGS column step (the reference's order, one pass instead of an axpy and a dot):
//   f <- f - alpha qa   (all stored rows; NKV_TIME: the time slot too)
//   partials[b] = sum over this block's weighted rows of w f_new qb   (qb = nullptr: w f_new f_new)
// The next column's projection coefficient (or, after the last column, the next pass's first one
// or ||f||^2) comes out of the same read of f.
// ------------------------------------------------------------------------------------------
template <int kPairs>
__global__ __launch_bounds__(kThreads) void k_axpy_dot(const double* __restrict__ qa,
                                                       const double* __restrict__ alpha,
                                                       double* __restrict__ f,
                                                       const double* __restrict__ qb,
                                                       const double* __restrict__ w, int64_t sv,
                                                       int tiles_per_field, int tiles_w, int tiles_total,
                                                       int64_t time_off, int do_time,
                                                       double* __restrict__ partials, int t_lo, int acc_part) {
    constexpr int kTile = kThreads * kPairs * 2;
    __shared__ double lds4[4];
    const double a = -alpha[0];
    if (do_time && blockIdx.x == 0 && threadIdx.x == 0) f[time_off] = fma(a, qa[time_off], f[time_off]);
    double s = 0.0;
    for (int t = t_lo + blockIdx.x; t < tiles_total; t += gridDim.x) {
        const int64_t r0 = (int64_t)t * kTile + 2 * threadIdx.x;
        double2 fn[kPairs];
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            const double2 fv = ld2(f + r0 + k * 2 * kThreads);
            const double2 qv = ldq(qa + r0 + k * 2 * kThreads);
            fn[k] = make_double2(fma(a, qv.x, fv.x), fma(a, qv.y, fv.y));
        }
        if (t < tiles_w) {
            const int64_t wr = r0 - (int64_t)(t / tiles_per_field) * sv;
#pragma unroll
            for (int k = 0; k < kPairs; ++k) {
                const double2 wv = ld2(w + wr + k * 2 * kThreads);
                const double2 bv = qb ? ldq(qb + r0 + k * 2 * kThreads) : fn[k];
                s = fma(wv.x * fn[k].x, bv.x, s);
                s = fma(wv.y * fn[k].y, bv.y, s);
            }
        }
#pragma unroll
        for (int k = 0; k < kPairs; ++k) st2(f + r0 + k * 2 * kThreads, fn[k]);
    }
    s = block_sum(s, lds4);   // a row band after the first adds to the block's partial (fixed order)
    if (threadIdx.x == 0) partials[blockIdx.x] = acc_part ? partials[blockIdx.x] + s : s;
}

// ------------------------------------------------------------------------------------------
// Arnoldi finish / normalise:  q = f / sqrt(nrm2)  (all rows + time), H column on the device.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_finish(const double* f,  // may alias q (in-place)
                                                     const double* __restrict__ nrm2,
                                                     double* q, int64_t rows,
                                                     int64_t time_off, int j,
                                                     const double* __restrict__ h1,
                                                     const double* __restrict__ h2,
                                                     double* __restrict__ hcol,
                                                     double* __restrict__ beta_out) {
    const double beta = sqrt(nrm2[0]);
    const double inv = 1.0 / beta;  // k_normalize: inv_alpha = 1/alpha; k_cmult (krylov_subspace.f90:87-90)
    // rows is a multiple of NKV_TILE, so whole chunks of kStreamUnr double2 per thread; all loads
    // of a chunk are issued before its stores (f may alias q)
    const int64_t chunks = rows / (2 * kThreads * kStreamUnr);
    for (int64_t ci = blockIdx.x; ci < chunks; ci += gridDim.x) {
        const int64_t p0 = ci * kThreads * kStreamUnr + threadIdx.x;
        double2 v[kStreamUnr];
#pragma unroll
        for (int u = 0; u < kStreamUnr; ++u) v[u] = ld2(f + 2 * (p0 + u * kThreads));
#pragma unroll
        for (int u = 0; u < kStreamUnr; ++u) {
            v[u].x *= inv;
            v[u].y *= inv;
            st2s(q + 2 * (p0 + u * kThreads), v[u]);
        }
    }
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            q[time_off] = f[time_off] * inv;
            if (beta_out) beta_out[0] = beta;
        }
        if (hcol) {
            for (int i = threadIdx.x; i < j; i += kThreads) hcol[i] = h1[i] + (h2 ? h2[i] : 0.0);
            if (threadIdx.x == 0) hcol[j] = beta;
        }
    }
}

// ------------------------------------------------------------------------------------------
// BLAS-1 family (one kernel, op selected per launch):  rows [0, rows) as double2 + time slot.
// ------------------------------------------------------------------------------------------
enum Op : int { OP_ZERO = 0, OP_COPY, OP_SCAL, OP_AXPBY, OP_SUB3, OP_AXPY_DEV };

template <int OP>
__global__ __launch_bounds__(kThreads) void k_blas1(double* x, const double* y,  // may alias
                                                    const double* z, double a, double b,
                                                    const double* __restrict__ a_dev, int64_t rows,
                                                    int64_t time_off, int do_time) {
    if (OP == OP_AXPY_DEV) a = b * a_dev[0];
    // rows is a multiple of NKV_TILE: whole chunks of kStreamUnr double2 per thread, every load of
    // a chunk issued before its stores (x may alias y / z)
    const int64_t chunks = rows / (2 * kThreads * kStreamUnr);
    for (int64_t ci = blockIdx.x; ci < chunks; ci += gridDim.x) {
        const int64_t p0 = ci * kThreads * kStreamUnr + threadIdx.x;
        double2 xv[kStreamUnr], yv[kStreamUnr], zv[kStreamUnr];
#pragma unroll
        for (int u = 0; u < kStreamUnr; ++u) {
            const int64_t i = 2 * (p0 + u * kThreads);
            if (OP == OP_SCAL || OP == OP_AXPBY || OP == OP_AXPY_DEV) xv[u] = ld2(x + i);
            if (OP != OP_ZERO && OP != OP_SCAL) yv[u] = ld2(y + i);
            if (OP == OP_SUB3) zv[u] = ld2(z + i);
        }
#pragma unroll
        for (int u = 0; u < kStreamUnr; ++u) {
            double2 r = make_double2(0.0, 0.0);
            if (OP == OP_COPY) r = yv[u];
            if (OP == OP_SCAL) r = make_double2(xv[u].x * a, xv[u].y * a);
            if (OP == OP_AXPBY)  // nek axpby: x(i) = x(i)*alpha + y(i)*beta (nek_vectors.f90:250-256)
                r = make_double2(xv[u].x * a + yv[u].x * b, xv[u].y * a + yv[u].y * b);
            if (OP == OP_SUB3) r = make_double2(yv[u].x - zv[u].x, yv[u].y - zv[u].y);
            if (OP == OP_AXPY_DEV) r = make_double2(fma(a, yv[u].x, xv[u].x), fma(a, yv[u].y, xv[u].y));
            st2(x + 2 * (p0 + u * kThreads), r);
        }
    }
    if (do_time && blockIdx.x == 0 && threadIdx.x == 0) {  // scalar time component
        const int64_t i = time_off;
        if (OP == OP_ZERO) x[i] = 0.0;
        if (OP == OP_COPY) x[i] = y[i];
        if (OP == OP_SCAL) x[i] = x[i] * a;
        if (OP == OP_AXPBY) x[i] = x[i] * a + y[i] * b;
        if (OP == OP_SUB3) x[i] = y[i] - z[i];
        if (OP == OP_AXPY_DEV) x[i] = fma(a, y[i], x[i]);
    }
}

__global__ void k_accumulate(double* __restrict__ dst, const double* __restrict__ src) {
    if (threadIdx.x == 0) dst[0] += src[0];
}

template <int P>
int launch_block_dot_p(const nkv_layout* L, const double* w, const double* Q, int64_t ld, int j,
                       const double* f, double* out, void* ws, unsigned flags, hipStream_t st) {
    constexpr int kTile = kThreads * P * 2;
    const int tpf = (int)(L->sv / kTile);
    const int bmax = (P == NKV_PAIRS_SMALL && P != NKV_PAIRS && NKV_DOT_SMALL_B < kMaxBlocks) ? NKV_DOT_SMALL_B : kMaxBlocks;
    int bx = bmax / L->n_wf;
    if (bx > tpf) bx = tpf;
    if (bx < 1) bx = 1;
    const int B = bx * L->n_wf;
    double* part = partials_of(ws);
    if (tpf > 0) {
        hipLaunchKernelGGL(k_block_dot<P>, dim3(bx, L->n_wf), dim3(kThreads), 4 * j * sizeof(double), st,
                           Q, ld, j, f, w, L->sv, tpf, part, B);
        NKV_LAUNCHED();
    }
    const int64_t T = rows_of(L);
    const bool tdot = (flags & NKV_TIME) && L->rank0;
    hipLaunchKernelGGL(k_reduce_cols, dim3(j), dim3(kThreads), 0, st, part, tpf > 0 ? B : 0, out,
                       tdot ? Q + T : nullptr, ld, tdot ? f + T : nullptr, nullptr, 1 << 30, nan_flag_of(ws));
    NKV_LAUNCHED();
    return NKV_OK;
}

}  // namespace

namespace nkvi {

// Shared launcher for block dots (nkv_dot is the j = 1 case).
int launch_block_dot(const nkv_layout* L, const double* w, const double* Q, int64_t ld, int j,
                     const double* f, double* out, void* ws, unsigned flags, hipStream_t st) {
    return use_large_tiles(L) ? launch_block_dot_p<NKV_PAIRS>(L, w, Q, ld, j, f, out, ws, flags, st)
                              : launch_block_dot_p<NKV_PAIRS_SMALL>(L, w, Q, ld, j, f, out, ws, flags, st);
}

int launch_reduce_cols(int ncols, const double* partials, int B, double* out, const double* ta, int64_t lda,
                       const double* tb, const double* tb2, int jc, int* nan_flag, hipStream_t st) {
    hipLaunchKernelGGL(k_reduce_cols, dim3(ncols), dim3(kThreads), 0, st, partials, B, out, ta, lda, tb, tb2, jc,
                       nan_flag);
    NKV_LAUNCHED();
    return NKV_OK;
}

}  // namespace nkvi

extern "C" {

static int blas1(const nkv_layout* L, int op, double* x, const double* y, const double* z, double a,
                 double b, const double* a_dev, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(x, "x"));
    const int64_t rows = rows_of(L);
    const int g = grid_for(rows / 2 + 1);
    const int dt = (flags & NKV_TIME) ? 1 : 0;
    hipStream_t st = S(stream);
    switch (op) {
        case OP_ZERO: hipLaunchKernelGGL(k_blas1<OP_ZERO>, dim3(g), dim3(kThreads), 0, st, x, y, z, a, b, a_dev, rows, rows, dt); break;
        case OP_COPY: hipLaunchKernelGGL(k_blas1<OP_COPY>, dim3(g), dim3(kThreads), 0, st, x, y, z, a, b, a_dev, rows, rows, dt); break;
        case OP_SCAL: hipLaunchKernelGGL(k_blas1<OP_SCAL>, dim3(g), dim3(kThreads), 0, st, x, y, z, a, b, a_dev, rows, rows, dt); break;
        case OP_AXPBY: hipLaunchKernelGGL(k_blas1<OP_AXPBY>, dim3(g), dim3(kThreads), 0, st, x, y, z, a, b, a_dev, rows, rows, dt); break;
        case OP_SUB3: hipLaunchKernelGGL(k_blas1<OP_SUB3>, dim3(g), dim3(kThreads), 0, st, x, y, z, a, b, a_dev, rows, rows, dt); break;
        case OP_AXPY_DEV: hipLaunchKernelGGL(k_blas1<OP_AXPY_DEV>, dim3(g), dim3(kThreads), 0, st, x, y, z, a, b, a_dev, rows, rows, dt); break;
        default: return fail(NKV_EINVAL, "bad op");
    }
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_zero(const nkv_layout* L, double* x, unsigned flags, void* stream) {
    return blas1(L, OP_ZERO, x, nullptr, nullptr, 0, 0, nullptr, flags, stream);
}
int nkv_copy(const nkv_layout* L, double* dst, const double* src, unsigned flags, void* stream) {
    CHECK(check_ptr(src, "src"));
    return blas1(L, OP_COPY, dst, src, nullptr, 0, 0, nullptr, flags, stream);
}
int nkv_scal(const nkv_layout* L, double* x, double alpha, unsigned flags, void* stream) {
    return blas1(L, OP_SCAL, x, nullptr, nullptr, alpha, 0, nullptr, flags, stream);
}
int nkv_axpby(const nkv_layout* L, double* x, double alpha, const double* y, double beta,
              unsigned flags, void* stream) {
    CHECK(check_ptr(y, "y"));
    return blas1(L, OP_AXPBY, x, y, nullptr, alpha, beta, nullptr, flags, stream);
}
int nkv_sub3(const nkv_layout* L, double* p, const double* q, const double* r, unsigned flags,
             void* stream) {
    CHECK(check_ptr(q, "q"));
    CHECK(check_ptr(r, "r"));
    return blas1(L, OP_SUB3, p, q, r, 0, 0, nullptr, flags, stream);
}
int nkv_axpy_dev(const nkv_layout* L, double* x, const double* alpha_dev, double sign,
                 const double* y, unsigned flags, void* stream) {
    CHECK(check_ptr(y, "y"));
    if (!alpha_dev) return fail(NKV_EINVAL, "alpha_dev is NULL");
    return blas1(L, OP_AXPY_DEV, x, y, nullptr, 0, sign, alpha_dev, flags, stream);
}

int nkv_normalize_dev(const nkv_layout* L, double* x, const double* nrm2_dev, double* beta_dev,
                      unsigned flags, void* stream) {
    (void)flags;
    CHECK(check_layout(L));
    CHECK(check_ptr(x, "x"));
    if (!nrm2_dev) return fail(NKV_EINVAL, "nrm2_dev is NULL");
    const int64_t rows = rows_of(L);
    hipLaunchKernelGGL(k_finish, dim3(grid_for(rows / 2)), dim3(kThreads), 0, S(stream), x, nrm2_dev,
                       x, rows, rows, 0, nullptr, nullptr, nullptr, beta_dev);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_dot(const nkv_layout* L, const double* w, const double* a, const double* b, double* out_dev,
            void* ws, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(a, "a"));
    CHECK(check_ptr(b, "b"));
    CHECK(check_ptr(ws, "ws"));
    if (!out_dev) return fail(NKV_EINVAL, "out_dev is NULL");
    return launch_block_dot(L, w, a, L->ld, 1, b, out_dev, ws, flags, S(stream));
}

int nkv_block_dot(const nkv_layout* L, const double* w, const double* Q, int j, const double* f,
                  double* h_dev, void* ws, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(Q, "Q"));
    CHECK(check_ptr(f, "f"));
    CHECK(check_ptr(ws, "ws"));
    if (!h_dev) return fail(NKV_EINVAL, "h_dev is NULL");
    if (j < 1 || j > NKV_MAX_COLS) return fail(NKV_EINVAL, "j=%d outside 1..%d", j, NKV_MAX_COLS);
    return launch_block_dot(L, w, Q, L->ld, j, f, h_dev, ws, flags, S(stream));
}

int nkv_arnoldi_finish(const nkv_layout* L, const double* f, const double* nrm2_dev, double* q_out,
                       int j, const double* h1_dev, const double* h2_dev, double* hcol_dev,
                       unsigned flags, void* stream) {
    (void)flags;
    CHECK(check_layout(L));
    CHECK(check_ptr(f, "f"));
    CHECK(check_ptr(q_out, "q_out"));
    if (!nrm2_dev) return fail(NKV_EINVAL, "nrm2_dev is NULL");
    if (hcol_dev && (!h1_dev || j < 0)) return fail(NKV_EINVAL, "hcol needs h1 and j >= 0");
    const int64_t rows = rows_of(L);
    hipLaunchKernelGGL(k_finish, dim3(grid_for(rows / 2)), dim3(kThreads), 0, S(stream), f, nrm2_dev,
                       q_out, rows, rows, j, h1_dev, h2_dev, hcol_dev, nullptr);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_normalize_store(const nkv_layout* L, const double* f, const double* nrm2_dev, double* q_next,
                        double* beta_dev, unsigned flags, void* stream) {
    (void)flags;
    CHECK(check_layout(L));
    CHECK(check_ptr(f, "f"));
    CHECK(check_ptr(q_next, "q_next"));
    if (!nrm2_dev) return fail(NKV_EINVAL, "nrm2_dev is NULL");
    const int64_t rows = rows_of(L);
    hipLaunchKernelGGL(k_finish, dim3(grid_for(rows / 2)), dim3(kThreads), 0, S(stream), f, nrm2_dev, q_next, rows,
                       rows, 0, nullptr, nullptr, nullptr, beta_dev);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_axpy_dot(const nkv_layout* L, const double* w, double* f, const double* alpha_dev, const double* qa,
                 const double* qb, double* out_dev, void* ws, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(f, "f"));
    CHECK(check_ptr(qa, "qa"));
    CHECK(check_ptr(ws, "ws"));
    if (!alpha_dev || !out_dev) return fail(NKV_EINVAL, "alpha_dev/out_dev is NULL");
    if (qb) CHECK(check_ptr(qb, "qb"));
    // 4 double2 per thread at every size: +5 % over the 8 of the wide kernels at N=1e8 for this
    // four-stream shape (profiles/r02bl_tune_fewcol.log)
    constexpr int P = NKV_PAIRS_SMALL;
    const int kTile = kThreads * P * 2;
    const int tpf = (int)(L->sv / kTile);
    const int tiles_w = tpf * L->n_wf;
    const int tiles_total = (int)(rows_of(L) / kTile);
    int g = tiles_total < kMaxBlocks ? tiles_total : kMaxBlocks;
    if (g < 1) g = 1;
    const int64_t T = rows_of(L);
    const int dt = (flags & NKV_TIME) ? 1 : 0;
    double* part = partials_of(ws);
    hipStream_t st = S(stream);
    auto kern = k_axpy_dot<P>;
    // NKV_AXD_ROUNDS > 0: one launch per row band of that many grid-stride rounds (first band: whole grid)
    const int64_t b = (int64_t)NKV_AXD_ROUNDS * g;
    const int band = (NKV_AXD_ROUNDS <= 0 || b >= tiles_total || tiles_total < 2 * b) ? (tiles_total > 0 ? tiles_total : 1)
                                                                                        : (int)b;
    for (int lo = 0; lo == 0 || lo < tiles_total; lo += band) {
        const int hi = lo + band < tiles_total ? lo + band : tiles_total;
        const int gb = lo == 0 ? g : (g < hi - lo ? g : hi - lo);
        hipLaunchKernelGGL(kern, dim3(gb), dim3(kThreads), 0, st, qa, alpha_dev, f, qb, w, L->sv, tpf, tiles_w, hi, T,
                           lo == 0 ? dt : 0, part, lo, lo == 0 ? 0 : 1);
        NKV_LAUNCHED();
    }
    const bool tdot = (flags & NKV_TIME_DOT) && L->rank0;   // the replicated time product, once
    const double* tq = qb ? qb : f;
    hipLaunchKernelGGL(k_reduce_cols, dim3(1), dim3(kThreads), 0, st, part, tiles_total > 0 ? g : 0, out_dev,
                       tdot ? tq + T : nullptr, (int64_t)0, tdot ? f + T : nullptr, nullptr, 1 << 30, nan_flag_of(ws));
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_mgs2_step(const nkv_layout* L, const double* w, const double* Q, int j, double* f, double* q_out,
                  double* hcol_dev, void* ws, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(f, "f"));
    CHECK(check_ptr(q_out, "q_out"));
    CHECK(check_ptr(ws, "ws"));
    if (!hcol_dev) return fail(NKV_EINVAL, "hcol_dev is NULL");
    if (j < 0 || j > NKV_MAX_COLS) return fail(NKV_EINVAL, "j=%d outside 0..%d", j, NKV_MAX_COLS);
    if (j > 0) CHECK(check_ptr(Q, "Q"));
    const unsigned tdot = (flags & NKV_TIME_DOT) ? NKV_TIME : 0u;
    double* tmp = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + 128);   // control-area scratch
    hipStream_t st = S(stream);
    // krylov_decomposition.f90:155-168, then :171-180: alpha_0 by a dot, then per column one fused
    // pass (f -= alpha_i q_i, next coefficient from the same read; the second pass's alphas
    // alternate between tmp[0] and tmp[2], ||f||^2 lands in tmp[1])
    if (j > 0) CHECK(nkv_dot(L, w, f, Q, hcol_dev, ws, tdot, st));
    for (int pass = 0; pass < 2; ++pass) {
        for (int i = 0; i < j; ++i) {
            const double* qi = Q + (int64_t)i * L->ld;
            double* h = pass == 0 ? hcol_dev + i : tmp + 2 * (i & 1);
            const bool last = i + 1 == j;
            const double* qn = !last ? qi + L->ld : (pass == 0 ? Q : nullptr);
            double* out = !last ? (pass == 0 ? hcol_dev + i + 1 : tmp + 2 * ((i + 1) & 1)) : (pass == 0 ? tmp : tmp + 1);
            if (pass == 1) {
                hipLaunchKernelGGL(k_accumulate, dim3(1), dim3(64), 0, st, hcol_dev + i, h);   // H(i,k) += alpha2
                NKV_LAUNCHED();
            }
            CHECK(nkv_axpy_dot(L, w, f, h, qi, qn, out, ws, NKV_TIME | (tdot ? NKV_TIME_DOT : 0u), st));
        }
    }
    if (j == 0) CHECK(nkv_dot(L, w, f, f, tmp + 1, ws, tdot, st));          // ||f||^2
    const int64_t rows = rows_of(L);                                          // q_out = f/||f||, H(k+1,k)
    hipLaunchKernelGGL(k_finish, dim3(grid_for(rows / 2)), dim3(kThreads), 0, st, f, tmp + 1, q_out, rows, rows, 0,
                       nullptr, nullptr, nullptr, hcol_dev + j);
    NKV_LAUNCHED();
    return NKV_OK;
}

}  // extern "C"
