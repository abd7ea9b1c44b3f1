// operators.hip — synthetic operators behind the matvec boundary (linear_operators.f90:17-23) and the
// shard-independent hashed vectors the tests and the bench fill.
#include "nkv_internal.h"

namespace {

// ------------------------------------------------------------------------------------------
// synthetic operators and data
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_op_diag(const double* __restrict__ d,
                                                      const double* __restrict__ x,
                                                      double* __restrict__ y, int64_t time_off, double ts,
                                                      int64_t c_lo, int64_t c_hi) {
    for (int64_t ci = c_lo + blockIdx.x; ci < c_hi; ci += gridDim.x) {   // this launch's row band
        const int64_t p0 = ci * kThreads * kStreamUnr + threadIdx.x;
        double2 dv[kStreamUnr], xv[kStreamUnr];
#pragma unroll
        for (int u = 0; u < kStreamUnr; ++u) {
            dv[u] = ld2(d + 2 * (p0 + u * kThreads));
            xv[u] = ld2(x + 2 * (p0 + u * kThreads));
        }
#pragma unroll
        for (int u = 0; u < kStreamUnr; ++u)
            st2p(y, 2 * (p0 + u * kThreads), make_double2(dv[u].x * xv[u].x, dv[u].y * xv[u].y));
    }
    if (c_lo == 0 && blockIdx.x == 0 && threadIdx.x == 0) y[time_off] = ts * x[time_off];
}

__global__ __launch_bounds__(kThreads) void k_op_rot2(const double* __restrict__ cs,
                                                      const double* __restrict__ sn,
                                                      const double* __restrict__ dr,
                                                      const double* __restrict__ x,
                                                      double* __restrict__ y, int64_t sv,
                                                      int64_t rows, int64_t time_off, double sgn) {
    const int64_t pairs = rows / 2;
    const int64_t pv = sv / 2;
    for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < pairs;
         p += (int64_t)gridDim.x * kThreads) {
        if (p < pv) {  // (u, v) = (field 0, field 1) at the same point
            const double2 c = ld2(cs + 2 * p), s = ld2(sn + 2 * p);
            const double2 u = ld2(x + 2 * p), v = ld2(x + sv + 2 * p);
            st2(y + 2 * p, make_double2(c.x * u.x - sgn * s.x * v.x, c.y * u.y - sgn * s.y * v.y));
            st2(y + sv + 2 * p, make_double2(sgn * s.x * u.x + c.x * v.x, sgn * s.y * u.y + c.y * v.y));
        } else if (p >= 2 * pv) {
            const double2 xv = ld2(x + 2 * p);
            const double2 dv = dr ? ld2(dr + 2 * p) : make_double2(0.0, 0.0);
            st2(y + 2 * p, make_double2(dv.x * xv.x, dv.y * xv.y));
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) y[time_off] = 0.0;
}

// Complex diagonal operator on a re/im pair vector (nekstab_next_amd.layout.PairLayout): in each
// segment (weighted field f: rows [f sv, f sv + n_v); pressure: [n_wf sv, n_wf sv + n_p)) the first
// half holds re, the second im.  y = c x (conj: y = conj(c) x), c = cr + i ci read at the re rows.
// grid (bx, n_wf + 1): blockIdx.y = segment (n_wf = pressure).
__global__ __launch_bounds__(kThreads) void k_op_cdiag(const double* __restrict__ cr,
                                                       const double* __restrict__ ci,
                                                       const double* __restrict__ x, double* __restrict__ y,
                                                       int64_t sv, int64_t n_v, int64_t n_p, int n_wf,
                                                       int64_t time_off, double sg) {
    const int seg = blockIdx.y;
    const int64_t base = (int64_t)seg * sv;
    const int64_t half = (seg < n_wf ? n_v : n_p) / 2;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < half; i += (int64_t)gridDim.x * kThreads) {
        const int64_t r = base + i, m = r + half;
        const double a = cr[r], b = sg * ci[r], xr = x[r], xi = x[m];
        y[r] = a * xr - b * xi;
        y[m] = b * xr + a * xi;
    }
    if (seg == 0 && blockIdx.x == 0 && threadIdx.x == 0) y[time_off] = 0.0;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void k_fill_hash(double* __restrict__ x, uint64_t seed,
                                                        int n_wf, int64_t n_v, int64_t sv,
                                                        int64_t n_p, int64_t rows,
                                                        int64_t time_off, int64_t voff,
                                                        int64_t poff) {
    const uint64_t key0 = seed * 0xD1342543DE82EF95ull;
    for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < rows;
         r += (int64_t)gridDim.x * kThreads) {
        int64_t field = r / sv, i = r - field * sv;
        bool live;
        uint64_t gp, fid;
        if (field < n_wf) {
            live = i < n_v;
            gp = (uint64_t)(voff + i);
            fid = (uint64_t)field;
        } else {
            i = r - (int64_t)n_wf * sv;
            live = i < n_p;
            gp = (uint64_t)(poff + i);
            fid = 31ull;
        }
        double v = 0.0;
        if (live) {
            const uint64_t z = mix64(key0 + fid * 0x9E3779B97F4A7C15ull + gp);
            const double u = (double)(z >> 11) * 0x1.0p-53;
            v = 2.0 * u - 1.0;
        }
        x[r] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) x[time_off] = 0.0;
}

}  // namespace

extern "C" {

int nkv_op_diag(const nkv_layout* L, const double* d, const double* x, double* y, double time_scale,
                void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(d, "d"));
    CHECK(check_ptr(x, "x"));
    CHECK(check_ptr(y, "y"));
    const int64_t rows = rows_of(L);
    // one launch per NKV_STREAM_ROUNDS grid-stride rounds (a row band): +5-7 % at N=1e8
    // (profiles/r02h_tune_bands_update_opdiag.log), as for the DCGS2 updates
    const int g = grid_for(rows / 2);
    const int64_t chunks = rows / (2 * kThreads * kStreamUnr);
    const int64_t band = NKV_STREAM_ROUNDS > 0 && chunks >= 2 * (int64_t)NKV_STREAM_ROUNDS * g
                             ? (int64_t)NKV_STREAM_ROUNDS * g : (chunks > 0 ? chunks : 1);
    for (int64_t lo = 0; lo == 0 || lo < chunks; lo += band) {
        const int64_t hi = lo + band < chunks ? lo + band : chunks;
        hipLaunchKernelGGL(k_op_diag, dim3(g), dim3(kThreads), 0, S(stream), d, x, y, rows, time_scale, lo, hi);
        NKV_LAUNCHED();
    }
    return NKV_OK;
}

int nkv_op_rot2(const nkv_layout* L, const double* c, const double* s, const double* d_rest,
                const double* x, double* y, int transpose, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(c, "c"));
    CHECK(check_ptr(s, "s"));
    CHECK(check_ptr(x, "x"));
    CHECK(check_ptr(y, "y"));
    if (d_rest) CHECK(check_ptr(d_rest, "d_rest"));
    if (L->n_wf < 2) return fail(NKV_EINVAL, "rot2 needs two velocity fields");
    if (x == y) return fail(NKV_EINVAL, "rot2 cannot run in place");
    const int64_t rows = rows_of(L);
    hipLaunchKernelGGL(k_op_rot2, dim3(grid_for(rows / 2)), dim3(kThreads), 0, S(stream), c, s, d_rest, x,
                       y, L->sv, rows, rows, transpose ? -1.0 : 1.0);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_op_cdiag(const nkv_layout* L, const double* cr, const double* ci, const double* x, double* y, int conj,
                 void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(cr, "cr"));
    CHECK(check_ptr(ci, "ci"));
    CHECK(check_ptr(x, "x"));
    CHECK(check_ptr(y, "y"));
    if (x == y) return fail(NKV_EINVAL, "cdiag cannot run in place");
    if ((L->n_v % 2) || (L->n_p % 2)) return fail(NKV_ESHAPE, "cdiag: not a re/im pair layout (odd n_v / n_p)");
    const int64_t half = (L->n_v > L->n_p ? L->n_v : L->n_p) / 2;
    int bx = grid_for(half, 1024);
    hipLaunchKernelGGL(k_op_cdiag, dim3(bx, L->n_wf + 1), dim3(kThreads), 0, S(stream), cr, ci, x, y, L->sv, L->n_v,
                       L->n_p, L->n_wf, rows_of(L), conj ? -1.0 : 1.0);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_fill_hash(const nkv_layout* L, double* x, uint64_t seed, int64_t v_offset, int64_t p_offset,
                  void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(x, "x"));
    const int64_t rows = rows_of(L);
    hipLaunchKernelGGL(k_fill_hash, dim3(grid_for(rows)), dim3(kThreads), 0, S(stream), x, seed, L->n_wf,
                       L->n_v, L->sv, L->n_p, rows, rows, v_offset, p_offset);
    NKV_LAUNCHED();
    return NKV_OK;
}

}  // extern "C"
