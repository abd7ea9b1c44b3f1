// sensitivity.hip — seeds and post-processing on the device: the seed noise of op_add_noise / mth_rand
// (utils.f90:258-418), add_symmetric_seed (:361-406), wave_maker (sensitivity.f90:3-77), gradm1 and the
// base-flow sensitivity terms (sensitivity.f90:81-269).
#include "nkv_internal.h"

namespace {

// wave_maker's pointwise product (sensitivity.f90:69-71):
//   out[i] = sqrt(vx_dRe^2 + vx_dIm^2 + vy_dRe^2 + ...) * sqrt(vx_aRe^2 + vx_aIm^2 + ...)
// over NC velocity components, summed left to right in the reference's order with no contraction
// (bit-identical to a plain restatement).  Pure HBM streaming: 4 NC reads and one write per point.
template <int NC>
__global__ __launch_bounds__(kThreads) void k_wavemaker(const double* __restrict__ dRe, const double* __restrict__ dIm,
                                                        const double* __restrict__ aRe, const double* __restrict__ aIm,
                                                        double* __restrict__ out, int64_t sv, int64_t pairs) {
#pragma clang fp contract(off)
    for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < pairs; p += (int64_t)gridDim.x * kThreads) {
        double2 dr[NC], di[NC], ar[NC], ai[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            dr[c] = ldq(dRe + c * sv + 2 * p);
            di[c] = ldq(dIm + c * sv + 2 * p);
            ar[c] = ldq(aRe + c * sv + 2 * p);
            ai[c] = ldq(aIm + c * sv + 2 * p);
        }
        double2 sd = make_double2(dr[0].x * dr[0].x + di[0].x * di[0].x, dr[0].y * dr[0].y + di[0].y * di[0].y);
        double2 sa = make_double2(ar[0].x * ar[0].x + ai[0].x * ai[0].x, ar[0].y * ar[0].y + ai[0].y * ai[0].y);
#pragma unroll
        for (int c = 1; c < NC; ++c) {
            sd.x = sd.x + dr[c].x * dr[c].x;
            sd.x = sd.x + di[c].x * di[c].x;
            sd.y = sd.y + dr[c].y * dr[c].y;
            sd.y = sd.y + di[c].y * di[c].y;
            sa.x = sa.x + ar[c].x * ar[c].x;
            sa.x = sa.x + ai[c].x * ai[c].x;
            sa.y = sa.y + ar[c].y * ar[c].y;
            sa.y = sa.y + ai[c].y * ai[c].y;
        }
        st2s(out + 2 * p, make_double2(sqrt(sd.x) * sqrt(sa.x), sqrt(sd.y) * sqrt(sa.y)));
    }
}

}  // namespace

// ---- bf_sensitivity (sensitivity.f90:81-269): gradm1 and the pointwise sensitivity terms -------------
//
// gradm1 (Nek5000 navier5.f; not in the reference tree) with the geometric factors of Nek5000's
// glmapm1 / xyzrst (coef.f) computed on the fly from the GLL coordinates: for every point
//   xr = sum_m D(i,m) x(m,j,k),  xs = sum_m D(j,m) x(i,m,k),  xt = sum_m D(k,m) x(i,j,m)   (mxm order)
//   2-D: jac = xr ys - xs yr;  rx = ys, ry = -xs, sx = -yr, sy = xr
//   3-D: jac = xr ys zt + xt yr zs + xs yt zr - xr yt zs - xs yr zt - xt ys zr (addcol4 / subcol4),
//        rx = ys zt - yt zs, ry = xt zs - xs zt, rz = xs yt - xt ys, sx = yt zr - yr zt, ...  (ascol5)
//   ux = (1/jac) (ur rx + us sx [+ ut tx]),  uy, uz likewise
// One workgroup holds `epb` whole elements in LDS; each thread owns one point, keeps its rows of D
// and its geometric factors in registers and differentiates NFLD fields (field f at u + f u_stride)
// against them, so the coordinates are read and the factors formed once per launch, not per field.
// NX (= lx1) is a template parameter; the line sums are unrolled by 2 (full unrolling hoists every
// LDS read into registers: 228 VGPRs at lx1=8 in 3-D, 2 waves per SIMD and 1.6x slower; by 1 or 4
// within 2-7 %, profiles/r03bh_gradm1_variants.log).  No contraction (the reference's operand order).
// Element-local: it shards with the elements.
template <int LDIM, int NX>
constexpr int gradm1_threads() {   // whole elements per workgroup, whole waves
    return (LDIM == 3 ? NX * NX * NX : NX * NX) >= 256 ? ((LDIM == 3 ? NX * NX * NX : NX * NX) + 63) / 64 * 64 : 256;
}

template <int LDIM, int NX>
__global__ __launch_bounds__((gradm1_threads<LDIM, NX>())) void k_gradm1(int64_t nel, int epb, int nfld, const double* __restrict__ Dg,
                                                 const double* __restrict__ xm, const double* __restrict__ ym,
                                                 const double* __restrict__ zm, const double* __restrict__ u,
                                                 int64_t u_stride, double* __restrict__ grad, int64_t g_stride) {
#pragma clang fp contract(off)
    extern __shared__ double lds[];
    constexpr int pts = LDIM == 3 ? NX * NX * NX : NX * NX;
    constexpr int sj = NX, sk = NX * NX;     // strides of s and t inside an element
    const int nt = epb * pts;
    double* D = lds;                         // D(i, m) at D[i*NX + m]
    double* X = D + NX * NX;
    double* Y = X + nt;
    double* Z = Y + nt;                      // 3-D only
    double* U = LDIM == 3 ? Z + nt : Z;
    const int tid = threadIdx.x;
    for (int t = tid; t < NX * NX; t += blockDim.x) D[t] = Dg[t];
    const int le = tid / pts, r = tid - le * pts;
    const int i = r % NX, j = (r / NX) % NX, k = LDIM == 3 ? r / (NX * NX) : 0;
    const int base = (tid < nt ? le : 0) * pts;   // lanes past the last whole element read element 0
    const int ri = base + j * sj + k * sk;   // line along r through (., j, k)
    const int si = base + i + k * sk;        // line along s through (i, ., k)
    const int ti = base + i + j * sj;        // line along t through (i, j, .)
    const double* Di = D + i * NX;           // this point's rows of D (LDS)
    const double* Dj = D + j * NX;
    const double* Dk = D + k * NX;
    for (int64_t e0 = (int64_t)blockIdx.x * epb; e0 < nel; e0 += (int64_t)gridDim.x * epb) {
        const int64_t p = e0 * pts + tid;
        const bool live = tid < nt && e0 + le < nel;
        __syncthreads();   // the previous group's reads are done (and D is staged on the first pass)
        if (live) {
            X[tid] = xm[p];
            Y[tid] = ym[p];
            if (LDIM == 3) Z[tid] = zm[p];
        }
        __syncthreads();
        // geometric factors of this point (registers; dead lanes compute garbage they never store)
        double xr = Di[0] * X[ri], yr = Di[0] * Y[ri];
        double xs = X[si] * Dj[0], ys = Y[si] * Dj[0];
#pragma unroll 2
        for (int m = 1; m < NX; ++m) {
            xr = xr + Di[m] * X[ri + m];
            yr = yr + Di[m] * Y[ri + m];
            xs = xs + X[si + m * sj] * Dj[m];
            ys = ys + Y[si + m * sj] * Dj[m];
        }
        double g[3][3], jacmi;   // g[direction][reference coordinate r, s, t]
        if constexpr (LDIM == 2) {
            double jac = 0.0;
            jac = jac + xr * ys;
            jac = jac - xs * yr;
            g[0][0] = ys;
            g[1][0] = -xs;
            g[0][1] = -yr;
            g[1][1] = xr;
            jacmi = 1.0 / jac;
        } else {
            double zr = Di[0] * Z[ri], zs = Z[si] * Dj[0];
            double xt = X[ti] * Dk[0], yt = Y[ti] * Dk[0], zt = Z[ti] * Dk[0];
#pragma unroll 2
            for (int m = 1; m < NX; ++m) {
                zr = zr + Di[m] * Z[ri + m];
                zs = zs + Z[si + m * sj] * Dj[m];
                xt = xt + X[ti + m * sk] * Dk[m];
                yt = yt + Y[ti + m * sk] * Dk[m];
                zt = zt + Z[ti + m * sk] * Dk[m];
            }
            double jac = 0.0;
            jac = jac + xr * ys * zt;
            jac = jac + xt * yr * zs;
            jac = jac + xs * yt * zr;
            jac = jac - xr * yt * zs;
            jac = jac - xs * yr * zt;
            jac = jac - xt * ys * zr;
            g[0][0] = ys * zt - yt * zs;   // rx
            g[1][0] = xt * zs - xs * zt;   // ry
            g[2][0] = xs * yt - xt * ys;   // rz
            g[0][1] = yt * zr - yr * zt;   // sx
            g[1][1] = xr * zt - xt * zr;   // sy
            g[2][1] = xt * yr - xr * yt;   // sz
            g[0][2] = yr * zs - ys * zr;   // tx
            g[1][2] = xs * zr - xr * zs;   // ty
            g[2][2] = xr * ys - xs * yr;   // tz
            jacmi = 1.0 / jac;
        }
        for (int f = 0; f < nfld; ++f) {
            if (f > 0) __syncthreads();   // every lane is done reading the previous field
            if (live) U[tid] = u[f * u_stride + p];
            __syncthreads();
            if (live) {
                double ur = Di[0] * U[ri], us = U[si] * Dj[0], ut = 0.0;
#pragma unroll 2
                for (int m = 1; m < NX; ++m) {
                    ur = ur + Di[m] * U[ri + m];
                    us = us + U[si + m * sj] * Dj[m];
                }
                if constexpr (LDIM == 3) {
                    ut = U[ti] * Dk[0];
#pragma unroll 2
                    for (int m = 1; m < NX; ++m) ut = ut + U[ti + m * sk] * Dk[m];
                }
                double* out = grad + (int64_t)f * LDIM * g_stride + p;
#pragma unroll
                for (int d = 0; d < LDIM; ++d) {
                    const double acc = LDIM == 3 ? ur * g[d][0] + us * g[d][1] + ut * g[d][2]
                                                 : ur * g[d][0] + us * g[d][1];
                    out[d * g_stride] = jacmi * acc;
                }
            }
        }
    }
}

// The pointwise part of bf_sensitivity (sensitivity.f90:202-235, 258-259) after gradm1 + dsavg:
// tr, ti (direct-gradient terms), pr, pi (adjoint-gradient terms), then sr = tr + pr, si = ti + pi,
// each accumulated from zero in the reference's opaddcol3 order (a += b c, no contraction).  The
// reference's index slips are kept: its lines 204/207/213/216 multiply vy_a* by dwdz_d* (not dvdz_d*)
// in the z component.  In 2-D the reference's vz terms read arrays it never set (opcopy skips vz);
// here they are absent.  G: gradients [mode dRe,dIm,aRe,aIm][component u,v,w][direction x,y,z], each a
// field segment of sv doubles; out: [tr, ti, pr, pi, sr, si][component], segments of sv doubles.
template <int LDIM>
__global__ __launch_bounds__(kThreads) void k_bf_sensitivity(int64_t n, int64_t sv, const double* __restrict__ dRe,
                                                             const double* __restrict__ dIm,
                                                             const double* __restrict__ aRe,
                                                             const double* __restrict__ aIm,
                                                             const double* __restrict__ G, double* __restrict__ out) {
#pragma clang fp contract(off)
    enum { DR = 0, DI = 1, AR = 2, AI = 3 };
    for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < n; p += (int64_t)gridDim.x * kThreads) {
        // gradient d(comp)/d(dir) of mode md at this point; components/directions beyond 2-D read nothing
        auto g = [&](int md, int c, int d) -> double {
            return (c < LDIM && d < LDIM) ? G[((int64_t)(md * LDIM + c) * LDIM + d) * sv + p] : 0.0;
        };
        double v[4][3];
        const double* modes[4] = {dRe, dIm, aRe, aIm};
#pragma unroll
        for (int md = 0; md < 4; ++md)
#pragma unroll
            for (int c = 0; c < 3; ++c) v[md][c] = c < LDIM ? modes[md][c * sv + p] : 0.0;
        double tr[3] = {0.0, 0.0, 0.0}, ti[3] = {0.0, 0.0, 0.0}, pr[3] = {0.0, 0.0, 0.0}, pi[3] = {0.0, 0.0, 0.0};
        // opaddcol3(a1, a2, a3, b, b, b, c1, c2, c3): a_c = a_c + b c_c (a3 only in 3-D)
        auto add = [&](double* a, double b, double c1, double c2, double c3) {
            a[0] = a[0] + b * c1;
            a[1] = a[1] + b * c2;
            if (LDIM == 3) a[2] = a[2] + b * c3;
        };
        const int X = 0, Y = 1, Z = 2, U = 0, V = 1, W = 2;
        add(tr, -v[AR][U], g(DR, U, X), g(DR, U, Y), g(DR, U, Z));                    // :203
        add(tr, -v[AR][V], g(DR, V, X), g(DR, V, Y), g(DR, W, Z));                    // :204 (dwdz)
        if (LDIM == 3) add(tr, -v[AR][W], g(DR, W, X), g(DR, W, Y), g(DR, W, Z));     // :205
        add(tr, -v[AI][U], g(DI, U, X), g(DI, U, Y), g(DI, U, Z));                    // :206
        add(tr, -v[AI][V], g(DI, V, X), g(DI, V, Y), g(DI, W, Z));                    // :207 (dwdz)
        if (LDIM == 3) add(tr, -v[AI][W], g(DI, W, X), g(DI, W, Y), g(DI, W, Z));     // :208
        add(ti, v[AR][U], g(DI, U, X), g(DI, U, Y), g(DI, U, Z));                     // :212
        add(ti, v[AR][V], g(DI, V, X), g(DI, V, Y), g(DI, W, Z));                     // :213 (dwdz)
        if (LDIM == 3) add(ti, v[AR][W], g(DI, W, X), g(DI, W, Y), g(DI, W, Z));      // :214
        add(ti, -v[AI][U], g(DR, U, X), g(DR, U, Y), g(DR, U, Z));                    // :215
        add(ti, -v[AI][V], g(DR, V, X), g(DR, V, Y), g(DR, W, Z));                    // :216 (dwdz)
        if (LDIM == 3) add(ti, -v[AI][W], g(DR, W, X), g(DR, W, Y), g(DR, W, Z));     // :217
        add(pr, v[DR][U], g(AR, U, X), g(AR, V, X), g(AR, W, X));                     // :221
        add(pr, v[DR][V], g(AR, U, Y), g(AR, V, Y), g(AR, W, Y));                     // :222
        if (LDIM == 3) add(pr, v[DR][W], g(AR, U, Z), g(AR, V, Z), g(AR, W, Z));      // :223
        add(pr, v[DI][U], g(AI, U, X), g(AI, V, X), g(AI, W, X));                     // :224
        add(pr, v[DI][V], g(AI, U, Y), g(AI, V, Y), g(AI, W, Y));                     // :225
        if (LDIM == 3) add(pr, v[DI][W], g(AI, U, Z), g(AI, V, Z), g(AI, W, Z));      // :226
        add(pi, v[DR][U], g(AI, U, X), g(AI, V, X), g(AI, W, X));                     // :230
        add(pi, v[DR][V], g(AI, U, Y), g(AI, V, Y), g(AI, W, Y));                     // :231
        if (LDIM == 3) add(pi, v[DR][W], g(AI, U, Z), g(AI, V, Z), g(AI, W, Z));      // :232
        add(pi, -v[DI][U], g(AR, U, X), g(AR, V, X), g(AR, W, X));                    // :233
        add(pi, -v[DI][V], g(AR, U, Y), g(AR, V, Y), g(AR, W, Y));                    // :234
        if (LDIM == 3) add(pi, -v[DI][W], g(AR, U, Z), g(AR, V, Z), g(AR, W, Z));     // :235
#pragma unroll
        for (int c = 0; c < LDIM; ++c) {
            out[(0 * LDIM + c) * sv + p] = tr[c];
            out[(1 * LDIM + c) * sv + p] = ti[c];
            out[(2 * LDIM + c) * sv + p] = pr[c];
            out[(3 * LDIM + c) * sv + p] = pi[c];
            out[(4 * LDIM + c) * sv + p] = tr[c] + pr[c];   // opadd2, :258
            out[(5 * LDIM + c) * sv + p] = ti[c] + pi[c];   // :259
        }
    }
}

template <int LDIM, int NX>
static void launch_gradm1(int64_t nel, int nfld, const double* D, const double* xm, const double* ym, const double* zm,
                          const double* u, int64_t u_stride, double* grad, int64_t g_stride, void* stream) {
    constexpr int pts = LDIM == 3 ? NX * NX * NX : NX * NX;
    const int epb = pts >= 256 ? 1 : 256 / pts;             // whole elements per workgroup
    const int threads = gradm1_threads<LDIM, NX>();
    const size_t lds = sizeof(double) * ((size_t)NX * NX + (size_t)(LDIM + 1) * epb * pts);
    const int64_t groups = (nel + epb - 1) / epb;
    const int grid = (int)std::min<int64_t>(groups, 16384);
    hipLaunchKernelGGL((k_gradm1<LDIM, NX>), dim3(grid), dim3(threads), lds, S(stream), nel, epb, nfld, D, xm, ym, zm,
                       u, u_stride, grad, g_stride);
}

// ---- correctly rounded sin / cos (the seed hash only) ----------------------------------------
// mth_rand's cos(1e3 sin(1e3 sin r)) turns one unit in the last place of a sin into ~1e-3 of noise,
// so the device hash equals the reference's (gfortran + glibc libm, which rounds sin/cos correctly
// in all but rare cases) only if its sin/cos round correctly too: double-double range reduction
// by pi/2 in four parts (|k| < 2^53) and double-double Taylor series on |r| <= pi/4 (~2^-100
// relative), rounded once to double.  Not used on any solver path.
struct nkv_dd { double hi, lo; };
__device__ __forceinline__ nkv_dd dd_two_sum(double a, double b) {
#pragma clang fp contract(off)
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ nkv_dd dd_fast(double a, double b) {
#pragma clang fp contract(off)
    const double s = a + b;
    return {s, b - (s - a)};
}
__device__ __forceinline__ nkv_dd dd_add(nkv_dd a, nkv_dd b) {
#pragma clang fp contract(off)
    nkv_dd s = dd_two_sum(a.hi, b.hi);
    const nkv_dd t = dd_two_sum(a.lo, b.lo);
    s = dd_fast(s.hi, s.lo + t.hi);
    return dd_fast(s.hi, s.lo + t.lo);
}
__device__ __forceinline__ nkv_dd dd_mul(nkv_dd a, nkv_dd b) {
#pragma clang fp contract(off)
    const double p = a.hi * b.hi;
    const double e = fma(a.hi, b.hi, -p);
    return dd_fast(p, e + (a.hi * b.lo + a.lo * b.hi));
}
__device__ __forceinline__ nkv_dd dd_prod(double a, double b) {   // exact
    const double p = a * b;
    return {p, fma(a, b, -p)};
}
__device__ const double kNkvSinC[15][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.5555555555555p-3, -0x1.5555555555555p-57},
    {0x1.1111111111111p-7, 0x1.1111111111111p-63},
    {-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73},
    {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},
    {-0x1.ae64567f544e4p-26, 0x1.c062e06d1f209p-80},
    {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},
    {-0x1.ae7f3e733b81fp-41, -0x1.1d8656b0ee8cbp-97},
    {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},
    {-0x1.2f49b46814157p-57, -0x1.2650f61dbdcb4p-112},
    {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},
    {-0x1.761b41316381ap-75, 0x1.3423c7d91404fp-130},
    {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139},
    {-0x1.d1ab1c2dccea3p-94, -0x1.054d0c78aea14p-149},
    {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157},
};
__device__ const double kNkvCosC[16][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.0000000000000p-1, 0x0.0p+0},
    {0x1.5555555555555p-5, 0x1.5555555555555p-59},
    {-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65},
    {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},
    {-0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76},
    {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},
    {-0x1.93974a8c07c9dp-37, -0x1.05d6f8a2efd1fp-92},
    {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},
    {-0x1.6827863b97d97p-53, -0x1.eec01221a8b0bp-107},
    {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},
    {-0x1.0ce396db7f853p-70, 0x1.aebcdbd20331cp-124},
    {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135},
    {-0x1.88e85fc6a4e5ap-89, 0x1.71c37ebd16540p-143},
    {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153},
    {-0x1.3932c5047d60ep-108, -0x1.832b7b530a627p-162},
};

// quadrant k mod 4 and r = x - k pi/2 as a double-double
__device__ __forceinline__ int dd_reduce(double x, nkv_dd* r) {
#pragma clang fp contract(off)
    const double k = rint(x * 0x1.45f306dc9c883p-1);   // x * 2/pi
    nkv_dd t = dd_add({x, 0.0}, dd_prod(-k, 0x1.921fb54442d18p+0));
    t = dd_add(t, dd_prod(-k, 0x1.1a62633145c07p-54));
    t = dd_add(t, dd_prod(-k, -0x1.f1976b7ed8fbcp-110));
    t = dd_add(t, dd_prod(-k, 0x1.4cf98e804177dp-164));
    *r = t;
    return (int)(((int64_t)k) & 3);
}
__device__ __forceinline__ nkv_dd dd_sin_r(nkv_dd r) {   // |r| <= ~pi/4
    const nkv_dd z = dd_mul(r, r);
    nkv_dd p = {kNkvSinC[14][0], kNkvSinC[14][1]};
    for (int i = 13; i >= 0; --i) p = dd_add(dd_mul(p, z), {kNkvSinC[i][0], kNkvSinC[i][1]});
    return dd_mul(p, r);
}
__device__ __forceinline__ nkv_dd dd_cos_r(nkv_dd r) {
    const nkv_dd z = dd_mul(r, r);
    nkv_dd p = {kNkvCosC[15][0], kNkvCosC[15][1]};
    for (int i = 14; i >= 0; --i) p = dd_add(dd_mul(p, z), {kNkvCosC[i][0], kNkvCosC[i][1]});
    return p;
}
__device__ double cr_sin(double x) {
    if (!(fabs(x) < 0x1p50)) return sin(x);   // not reached by the hash (|x| < 1e10)
    nkv_dd r;
    const int q = dd_reduce(x, &r);
    const nkv_dd v = (q & 1) ? dd_cos_r(r) : dd_sin_r(r);
    const double s = v.hi + v.lo;
    return (q & 2) ? -s : s;
}
__device__ double cr_cos(double x) {
    if (!(fabs(x) < 0x1p50)) return cos(x);
    nkv_dd r;
    const int q = dd_reduce(x, &r);
    const nkv_dd v = (q & 1) ? dd_sin_r(r) : dd_cos_r(r);
    const double c = v.hi + v.lo;
    return ((q + 1) & 2) ? -c : c;
}

// Seed noise of op_add_noise / add_noise_scal (utils.f90:258-359): q[p] += mth_rand(il, jl, kl, ieg,
// xl, fc) (utils.f90:408-418) at every point p of one weighted field, in Nek's point order (il fastest)
// with ieg = e_first + e + 1 the global element number:
//   r = fc1 (ieg + x sin y) + fc2 il jl + fc3 il;   3-D: r = fc1 (ieg + z sin r) + fc2 kl il + fc3 kl
//   mth_rand = cos(1e3 sin(1e3 sin r))
// evaluated in the reference's operand order with no contraction, every sin / cos correctly rounded
// (cr_sin / cr_cos above).  The hash amplifies the last bit of every sin by ~1e6, so the result
// depends on the math library's rounding: it equals the formula with correctly rounded libm bit for
// bit, and glibc's (which misrounds ~0.1 % of near-midpoint cases) at >99 % of the points.
__global__ __launch_bounds__(kThreads) void k_mth_rand_add(int nx, int ny, int nz, int64_t n, int64_t e_first,
                                                           const double* __restrict__ xm,
                                                           const double* __restrict__ ym,
                                                           const double* __restrict__ zm, double fc1, double fc2,
                                                           double fc3, double* __restrict__ q) {
#pragma clang fp contract(off)
    const int64_t ppe = (int64_t)nx * ny * nz;
    for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < n; p += (int64_t)gridDim.x * kThreads) {
        const int64_t e = p / ppe;
        const int r = (int)(p - e * ppe);
        const double il = (double)(r % nx + 1), jl = (double)((r / nx) % ny + 1), kl = (double)(r / (nx * ny) + 1);
        const double ieg = (double)(e_first + e + 1);
        double m = fc1 * (ieg + xm[p] * cr_sin(ym[p])) + fc2 * il * jl + fc3 * il;
        if (zm) m = fc1 * (ieg + zm[p] * cr_sin(m)) + fc2 * kl * il + fc3 * kl;
        q[p] = q[p] + cr_cos(1.0e3 * cr_sin(1.0e3 * cr_sin(m)));
    }
}

// Direct-stiffness averaging on one rank (dssum then vmult, as op_add_noise applies to its noise,
// utils.f90:339-340): every point of a group of coincident GLL points (CSR: members[start[g] ..
// start[g+1])) gets the group's mean, summed in member order.  Singleton points keep their value.
__global__ __launch_bounds__(kThreads) void k_group_average(int64_t n_groups, const int64_t* __restrict__ start,
                                                            const int64_t* __restrict__ members,
                                                            double* __restrict__ q) {
#pragma clang fp contract(off)
    for (int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x; g < n_groups; g += (int64_t)gridDim.x * kThreads) {
        const int64_t a = start[g], b = start[g + 1];
        double s = 0.0;
        for (int64_t i = a; i < b; ++i) s = s + q[members[i]];
        const double v = s * (1.0 / (double)(b - a));
        for (int64_t i = a; i < b; ++i) q[members[i]] = v;
    }
}

// add_symmetric_seed's perturbation (utils.f90:361-406, before its amplitude scaling), pointwise:
//   qx = cos(alpha z) sin(2 pi y),  qz = -(2 pi)/alpha cos(alpha z) cos(2 pi y),  qt = cos(alpha z) cos(2 pi y)
// (qy is not written: the reference leaves it as it was).  No contraction, the reference's order.
__global__ __launch_bounds__(kThreads) void k_symmetric_seed(int64_t n, const double* __restrict__ ym,
                                                             const double* __restrict__ zm, double alpha,
                                                             double* __restrict__ qx, double* __restrict__ qz,
                                                             double* __restrict__ qt) {
#pragma clang fp contract(off)
    const double twopi = 2.0 * 3.14159265358979323846;
    for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < n; p += (int64_t)gridDim.x * kThreads) {
        const double y = ym[p], z = zm[p];
        qx[p] = cos(alpha * z) * sin(twopi * y);
        qz[p] = -twopi / alpha * cos(alpha * z) * cos(twopi * y);
        qt[p] = cos(alpha * z) * cos(twopi * y);
    }
}

extern "C" {

int nkv_symmetric_seed(const nkv_layout* L, const double* ym, const double* zm, double alpha, double* qx,
                       double* qz, double* qt, void* stream) {
    CHECK(check_layout(L));
    if (L->n_v == 0) return NKV_OK;   // an empty shard (more ranks than elements): nothing to touch
    CHECK(check_ptr(ym, "ym"));
    CHECK(check_ptr(zm, "zm"));
    CHECK(check_ptr(qx, "qx"));
    CHECK(check_ptr(qz, "qz"));
    CHECK(check_ptr(qt, "qt"));
    if (!(alpha != 0.0) || !std::isfinite(alpha)) return fail(NKV_EINVAL, "symmetric seed: alpha=%g", alpha);
    hipLaunchKernelGGL(k_symmetric_seed, dim3(grid_for(L->n_v)), dim3(kThreads), 0, S(stream), L->n_v, ym, zm, alpha,
                       qx, qz, qt);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_mth_rand_add(const nkv_layout* L, int lx1, int ly1, int lz1, int64_t e_first, const double* xm,
                     const double* ym, const double* zm, double fc1, double fc2, double fc3, double* q,
                     void* stream) {
    CHECK(check_layout(L));
    if (L->n_v == 0) return NKV_OK;   // an empty shard (more ranks than elements): nothing to touch
    if (lx1 < 1 || ly1 < 1 || lz1 < 1 || L->n_v % ((int64_t)lx1 * ly1 * lz1) != 0)
        return fail(NKV_EINVAL, "mth_rand: lx1*ly1*lz1=%d*%d*%d does not divide n_v=%lld", lx1, ly1, lz1,
                    (long long)L->n_v);
    if (e_first < 0) return fail(NKV_EINVAL, "mth_rand: e_first=%lld < 0", (long long)e_first);
    if ((lz1 > 1) != (zm != nullptr)) return fail(NKV_EINVAL, "mth_rand: zm must be given exactly when lz1 > 1");
    CHECK(check_ptr(xm, "xm"));
    CHECK(check_ptr(ym, "ym"));
    CHECK(check_ptr(q, "q"));
    hipLaunchKernelGGL(k_mth_rand_add, dim3(grid_for(L->n_v)), dim3(kThreads), 0, S(stream), lx1, ly1, lz1, L->n_v,
                       e_first, xm, ym, zm, fc1, fc2, fc3, q);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_group_average(int64_t n_groups, const int64_t* start, const int64_t* members, double* q, void* stream) {
    if (n_groups < 0) return fail(NKV_EINVAL, "group_average: n_groups=%lld < 0", (long long)n_groups);
    if (n_groups == 0) return NKV_OK;
    if (!start || !members || !q) return fail(NKV_EINVAL, "group_average: start/members/q is NULL");
    hipLaunchKernelGGL(k_group_average, dim3(grid_for(n_groups)), dim3(kThreads), 0, S(stream), n_groups, start,
                       members, q);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_wavemaker(const nkv_layout* L, const double* dRe, const double* dIm, const double* aRe, const double* aIm,
                  double* out, int ncomp, void* stream) {
    CHECK(check_layout(L));
    if (L->n_v == 0) return NKV_OK;   // an empty shard (more ranks than elements): nothing to touch
    CHECK(check_ptr(dRe, "dRe"));
    CHECK(check_ptr(dIm, "dIm"));
    CHECK(check_ptr(aRe, "aRe"));
    CHECK(check_ptr(aIm, "aIm"));
    CHECK(check_ptr(out, "out"));
    if (ncomp < 2 || ncomp > 3 || ncomp > L->n_wf)
        return fail(NKV_EINVAL, "wavemaker: ncomp=%d must be 2 or 3 and <= n_wf=%d", ncomp, L->n_wf);
    const int64_t pairs = L->sv / 2;
    auto kern = ncomp == 3 ? k_wavemaker<3> : k_wavemaker<2>;
    hipLaunchKernelGGL(kern, dim3(grid_for(pairs)), dim3(kThreads), 0, S(stream), dRe, dIm, aRe, aIm, out, L->sv, pairs);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_gradm1(const nkv_layout* L, int lx1, int ldim, const double* D, const double* xm, const double* ym,
               const double* zm, const double* u, int nfld, int64_t u_stride, double* grad, int64_t g_stride,
               void* stream) {
    CHECK(check_layout(L));
    if (L->n_v == 0) return NKV_OK;   // an empty shard (more ranks than elements): nothing to touch
    if (ldim != 2 && ldim != 3) return fail(NKV_EINVAL, "gradm1: ldim=%d must be 2 or 3", ldim);
    if (lx1 < 2 || lx1 > 10) return fail(NKV_EINVAL, "gradm1: lx1=%d outside 2..10", lx1);
    const int pts = ldim == 3 ? lx1 * lx1 * lx1 : lx1 * lx1;
    if (L->n_v % pts != 0)
        return fail(NKV_EINVAL, "gradm1: %d points per element do not divide n_v=%lld", pts, (long long)L->n_v);
    if ((ldim == 3) != (zm != nullptr)) return fail(NKV_EINVAL, "gradm1: zm must be given exactly in 3-D");
    if (nfld < 1) return fail(NKV_EINVAL, "gradm1: nfld=%d < 1", nfld);
    if ((nfld > 1 && u_stride < L->n_v) || g_stride < L->n_v)
        return fail(NKV_EINVAL, "gradm1: strides u=%lld g=%lld below n_v=%lld", (long long)u_stride,
                    (long long)g_stride, (long long)L->n_v);
    CHECK(check_ptr(D, "D"));
    CHECK(check_ptr(xm, "xm"));
    CHECK(check_ptr(ym, "ym"));
    CHECK(check_ptr(u, "u"));
    CHECK(check_ptr(grad, "grad"));
    const int64_t nel = L->n_v / pts;
#define NKV_GRADM1_CASE(NX)                                                                                   \
    case NX:                                                                                                  \
        if (ldim == 3) launch_gradm1<3, NX>(nel, nfld, D, xm, ym, zm, u, u_stride, grad, g_stride, stream);  \
        else launch_gradm1<2, NX>(nel, nfld, D, xm, ym, zm, u, u_stride, grad, g_stride, stream);            \
        break;
    switch (lx1) {
        NKV_GRADM1_CASE(2)
        NKV_GRADM1_CASE(3)
        NKV_GRADM1_CASE(4)
        NKV_GRADM1_CASE(5)
        NKV_GRADM1_CASE(6)
        NKV_GRADM1_CASE(7)
        NKV_GRADM1_CASE(8)
        NKV_GRADM1_CASE(9)
        NKV_GRADM1_CASE(10)
    }
#undef NKV_GRADM1_CASE
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_bf_sensitivity(const nkv_layout* L, const double* dRe, const double* dIm, const double* aRe,
                       const double* aIm, const double* grad, double* out, int ncomp, void* stream) {
    CHECK(check_layout(L));
    if (L->n_v == 0) return NKV_OK;   // an empty shard (more ranks than elements): nothing to touch
    CHECK(check_ptr(dRe, "dRe"));
    CHECK(check_ptr(dIm, "dIm"));
    CHECK(check_ptr(aRe, "aRe"));
    CHECK(check_ptr(aIm, "aIm"));
    CHECK(check_ptr(grad, "grad"));
    CHECK(check_ptr(out, "out"));
    if (ncomp < 2 || ncomp > 3 || ncomp > L->n_wf)
        return fail(NKV_EINVAL, "bf_sensitivity: ncomp=%d must be 2 or 3 and <= n_wf=%d", ncomp, L->n_wf);
    auto kern = ncomp == 3 ? k_bf_sensitivity<3> : k_bf_sensitivity<2>;
    hipLaunchKernelGGL(kern, dim3(grid_for(L->n_v)), dim3(kThreads), 0, S(stream), L->n_v, L->sv, dRe, dIm, aRe, aIm,
                       grad, out);
    NKV_LAUNCHED();
    return NKV_OK;
}

}  // extern "C"
