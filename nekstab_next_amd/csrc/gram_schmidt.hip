// gram_schmidt.hip — the Gram–Schmidt hot loop (update_hessenberg_matrix, krylov_decomposition.f90:103-189):
// block updates, the fused CGS2 middle pass, DCGS2 (two-vector multi-dot, device coefficients, dual
// update), Golub–Kahan–Lanczos coefficients (svds) and MGS in inverse compact WY form.
#include "nkv_internal.h"

namespace {

// ------------------------------------------------------------------------------------------
// block update:  f <- f - Q h  (or f <- Q h), optional fused ||f_new||_W^2 partial.
// 1-D grid-stride over all tiles of the vector; a tile never straddles fields (sv, sp are
// multiples of the tile), so the weight row is r - field*sv.
// ------------------------------------------------------------------------------------------
template <bool OVERWRITE, bool NORM, int kPairs>
__global__ __launch_bounds__(kThreads) void k_block_update(const double* __restrict__ Q, int64_t ld,
                                                           int j, const double* __restrict__ h,
                                                           double* __restrict__ f,
                                                           const double* __restrict__ w, int64_t sv,
                                                           int tiles_per_field, int tiles_w,
                                                           int tiles_total, int64_t time_off,
                                                           int do_time,
                                                           double* __restrict__ partials, int t_lo,
                                                           int acc_part) {
    constexpr int kTile = kThreads * kPairs * 2;
    __shared__ double lds4[4];
    // time slot (one double): wave 0 of block 0, lanes split the columns.
    if (do_time && blockIdx.x == 0 && threadIdx.x < 64) {
        double s = 0.0;
        for (int c = threadIdx.x; c < j; c += 64) s = fma(Q[time_off + (int64_t)c * ld], h[c], s);
        s = wave_sum(s);
        if (threadIdx.x == 0) f[time_off] = OVERWRITE ? s : f[time_off] - s;
    }
    double nrm = 0.0;
    for (int t = t_lo + blockIdx.x; t < tiles_total; t += gridDim.x) {   // tiles t_lo..tiles_total-1
        const int64_t r0 = (int64_t)t * kTile + 2 * threadIdx.x;
        double2 acc[kPairs];
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            if (OVERWRITE) acc[k] = make_double2(0.0, 0.0);
            else acc[k] = ld2(f + r0 + k * 2 * kThreads);
        }
        const double* qb = Q + r0;
        int c = 0;
        for (; c + 4 <= j; c += 4) {
            double2 q[4][kPairs];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int k = 0; k < kPairs; ++k) q[u][k] = ldq(qb + (int64_t)(c + u) * ld + k * 2 * kThreads);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double hc = OVERWRITE ? h[c + u] : -h[c + u];
#pragma unroll
                for (int k = 0; k < kPairs; ++k) {
                    acc[k].x = fma(hc, q[u][k].x, acc[k].x);
                    acc[k].y = fma(hc, q[u][k].y, acc[k].y);
                }
            }
        }
        for (; c < j; ++c) {
            const double hc = OVERWRITE ? h[c] : -h[c];
#pragma unroll
            for (int k = 0; k < kPairs; ++k) {
                const double2 q = ldq(qb + (int64_t)c * ld + k * 2 * kThreads);
                acc[k].x = fma(hc, q.x, acc[k].x);
                acc[k].y = fma(hc, q.y, acc[k].y);
            }
        }
#pragma unroll
        for (int k = 0; k < kPairs; ++k) st2(f + r0 + k * 2 * kThreads, acc[k]);
        if (NORM && t < tiles_w) {
            const int64_t wr = r0 - (int64_t)(t / tiles_per_field) * sv;
#pragma unroll
            for (int k = 0; k < kPairs; ++k) {
                const double2 wv = ld2(w + wr + k * 2 * kThreads);
                nrm = fma(wv.x * acc[k].x, acc[k].x, nrm);
                nrm = fma(wv.y * acc[k].y, acc[k].y, nrm);
            }
        }
    }
    if (NORM) {   // a row band after the first adds to the block's partial (fixed order: deterministic)
        nrm = block_sum(nrm, lds4);
        if (threadIdx.x == 0) partials[blockIdx.x] = acc_part ? partials[blockIdx.x] + nrm : nrm;
    }
}

// ------------------------------------------------------------------------------------------
// Fused CGS2 middle pass:  f <- f - Q h  AND  partials[c][b] = q_c . (w f_new)  in ONE read of Q.
// A 512-thread workgroup owns 128-row tiles (lane = 2 rows, double2); its 8 waves split the j
// columns (wave v holds columns v, v+8, ...: CPW double2 per lane in registers).  The per-wave
// partial sums of Q h meet in LDS, every wave forms f_new for its rows, and the same registers
// then feed the second projection, accumulated per lane across all tiles of the workgroup and
// reduced across lanes once at the end.
// ------------------------------------------------------------------------------------------
constexpr int kFuseRows = 128;

template <int NW, int CPW>
__global__ __launch_bounds__(NW * 64) void k_update_dot(const double* __restrict__ Q, int64_t ld, int j,
                                                         const double* __restrict__ h,
                                                         double* __restrict__ f,
                                                         const double* __restrict__ w, int64_t sv,
                                                         int64_t tiles_per_field, int64_t tiles_w,
                                                         int64_t tiles_total, int64_t time_off,
                                                         int do_time, double* __restrict__ partials,
                                                         int B, int64_t t_lo, int acc_part) {
    __shared__ double2 part[2][NW][64];  // double-buffered: one barrier per tile
    // wave index made provably uniform: column bases become scalar registers, the per-lane part of
    // every address is one 32-bit row offset
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (do_time && blockIdx.x == 0 && wv == 0) {  // scalar time component of f (k_sub2 keeps it)
        double s = 0.0;
        for (int c = lane; c < j; c += 64) s = fma(Q[time_off + (int64_t)c * ld], h[c], s);
        s = wave_sum(s);
        if (lane == 0) f[time_off] -= s;
    }
    const double* qcol[CPW];
    double hc[CPW];
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
        const int c = wv + NW * i;
        qcol[i] = Q + (int64_t)(c < j ? c : 0) * ld;
        hc[i] = c < j ? h[c] : 0.0;
    }
    double acc[CPW];
#pragma unroll
    for (int i = 0; i < CPW; ++i) acc[i] = 0.0;
    int buf = 0;
    auto load_tile = [&](double2 (&q)[CPW], int64_t t) {
        const uint32_t rb = ((uint32_t)(t * kFuseRows) + 2u * lane) * 8u;  // rows < 2^29 (checked)
#pragma unroll
        for (int i = 0; i < CPW - 1; ++i) q[i] = ldq(at_b(qcol[i], rb));
        // CPW = ceil(j/NW): only the last slot can lie past j (wave-uniform test, never fetched)
        q[CPW - 1] = (wv + NW * (CPW - 1) < j) ? ldq(at_b(qcol[CPW - 1], rb)) : make_double2(0.0, 0.0);
    };
    double2 q[CPW];
    for (int64_t t = t_lo + blockIdx.x; t < tiles_total; t += gridDim.x, buf ^= 1) {   // tiles t_lo..
        const uint32_t r = (uint32_t)(t * kFuseRows) + 2u * lane;
        load_tile(q, t);
        double2 s = make_double2(0.0, 0.0);
#pragma unroll
        for (int i = 0; i < CPW; ++i) {
            s.x = fma(hc[i], q[i].x, s.x);
            s.y = fma(hc[i], q[i].y, s.y);
        }
        const double2 fv = ld2(at_b(f, r * 8u));
        const bool weighted = t < tiles_w;
        // weights are loaded before any prefetch: vmcnt retires in order, so a load issued after
        // the prefetch would wait for it
        const double2 ww = weighted ? ld2(at_b(w, (r - (uint32_t)((t / tiles_per_field) * sv)) * 8u)) : make_double2(0.0, 0.0);
        part[buf][wv][lane] = s;
        __syncthreads();
        double2 tot = part[buf][0][lane];
#pragma unroll
        for (int k = 1; k < NW; ++k) {
            const double2 p = part[buf][k][lane];
            tot.x += p.x;
            tot.y += p.y;
        }
        const double2 f1 = make_double2(fv.x - tot.x, fv.y - tot.y);
        if (wv == 0) st2(const_cast<double*>(at_b(f, r * 8u)), f1);
        if (weighted) {
            const double a = ww.x * f1.x, b = ww.y * f1.y;
#pragma unroll
            for (int i = 0; i < CPW; ++i) acc[i] = fma(q[i].y, b, fma(q[i].x, a, acc[i]));
        }
        // no second barrier: the next tile writes the other buffer, and a wave can only reach the
        // barrier after it once every wave has passed this tile's barrier (and read this buffer)
    }
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
        const int c = wv + NW * i;
        const double v = wave_sum(acc[i]);
        if (lane == 0 && c < j)   // a row band after the first adds to the block's partials (fixed order)
            partials[(int64_t)c * B + blockIdx.x] = acc_part ? partials[(int64_t)c * B + blockIdx.x] + v : v;
    }
}

// ------------------------------------------------------------------------------------------
// DCGS2 (classical Gram–Schmidt with delayed re-orthogonalisation) — two reads of Q per step.
//
// Two-vector multi-dot: partials[c][b] = q_c . (w x), partials[j + c][b] = q_c . (w y) in ONE
// read of Q (x = the provisional q_j, y = A q_j).  Same grid and tiling as k_block_dot.
// ------------------------------------------------------------------------------------------
template <int kPairs>
__global__ __launch_bounds__(kThreads)
void k_block_dot2(const double* __restrict__ Q, int64_t ld,
                                                         int j, const double* __restrict__ x,
                                                         const double* __restrict__ y,
                                                         const double* __restrict__ w, int64_t sv,
                                                         int tiles_per_field, int n_fields, int x_last,
                                                         double* __restrict__ partials, int B) {
    // grid (bx, n_wf / n_fields): each block walks n_fields weighted fields per row tile, so with
    // n_fields = n_wf the weights of a tile are read from HBM once instead of once per field.
    // x_last: x IS column j-1 of Q, so that column is not streamed again — its two dots (x.Wx,
    // x.Wy) are formed from the registers that hold x and y.
    constexpr int kTile = kThreads * kPairs * 2;
    constexpr int U = NKV_D2_U;  // columns in flight (two right-hand sides double the registers per column)
    extern __shared__ double red[];  // [4 waves][2j]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int c = threadIdx.x; c < 8 * j; c += kThreads) red[c] = 0.0;
    __syncthreads();
    for (int t = blockIdx.x; t < tiles_per_field; t += gridDim.x) {
        const int64_t r0 = (int64_t)t * kTile + 2 * threadIdx.x;
        double2 wv[kPairs];
#pragma unroll
        for (int k = 0; k < kPairs; ++k) wv[k] = ld2(w + r0 + k * 2 * kThreads);
        for (int fi = 0; fi < n_fields; ++fi) {
            const int64_t fb = (int64_t)(blockIdx.y * n_fields + fi) * sv;
            double2 wx[kPairs], wy[kPairs];
            double sxx = 0.0, sxy = 0.0;
#pragma unroll
            for (int k = 0; k < kPairs; ++k) {
                const double2 xv = ld2(x + fb + r0 + k * 2 * kThreads);
                const double2 yv = ld2(y + fb + r0 + k * 2 * kThreads);
                wx[k] = make_double2(wv[k].x * xv.x, wv[k].y * xv.y);
                wy[k] = make_double2(wv[k].x * yv.x, wv[k].y * yv.y);
                if (x_last) {
                    sxx = fma(xv.x, wx[k].x, sxx);
                    sxx = fma(xv.y, wx[k].y, sxx);
                    sxy = fma(xv.x, wy[k].x, sxy);
                    sxy = fma(xv.y, wy[k].y, sxy);
                }
            }
            if (x_last) {
                sxx = wave_sum(sxx);
                sxy = wave_sum(sxy);
                if (lane == 0) {
                    red[wave * 2 * j + j - 1] += sxx;
                    red[wave * 2 * j + 2 * j - 1] += sxy;
                }
            }
            const int jl = x_last ? j - 1 : j;   // columns streamed from Q
            const double* qb = Q + fb + r0;
            for (int c = 0; c < jl; c += U) {
                double2 q[U][kPairs];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int k = 0; k < kPairs; ++k)
                        q[u][k] = (c + u < jl) ? ldq(qb + (int64_t)(c + u) * ld + k * 2 * kThreads)
                                               : make_double2(0.0, 0.0);
                double s[2 * U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    double a = 0.0, b = 0.0;
#pragma unroll
                    for (int k = 0; k < kPairs; ++k) {
                        a = fma(q[u][k].x, wx[k].x, a);
                        a = fma(q[u][k].y, wx[k].y, a);
                        b = fma(q[u][k].x, wy[k].x, b);
                        b = fma(q[u][k].y, wy[k].y, b);
                    }
                    s[u] = a;
                    s[U + u] = b;
                }
#if NKV_D2_RED && NKV_D2_U == 2   // two columns x two right-hand sides = four sums
                const double v = wave_sum4(s[0], s[1], s[2], s[3], lane);
                if ((lane & 15) == 0) {
                    const int q = lane >> 4;                 // 0: x.c  1: x.(c+1)  2: y.c  3: y.(c+1)
                    const int cc = c + (q & 1);
                    if (cc < jl) red[wave * 2 * j + (q >> 1) * j + cc] += v;
                }
#else
#pragma unroll
                for (int off = 32; off > 0; off >>= 1)
#pragma unroll
                    for (int u = 0; u < 2 * U; ++u) s[u] += __shfl_xor(s[u], off, 64);
                if (lane == 0) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (c + u < jl) {
                            red[wave * 2 * j + c + u] += s[u];
                            red[wave * 2 * j + j + c + u] += s[U + u];
                        }
                    }
                }
#endif
            }
        }
    }
    __syncthreads();
    const int b = blockIdx.y * gridDim.x + blockIdx.x;
    for (int c = threadIdx.x; c < 2 * j; c += kThreads)
        partials[(int64_t)c * B + b] =
            (red[c] + red[2 * j + c]) + (red[4 * j + c] + red[6 * j + c]);
}

// DCGS2 small dense step (one workgroup).  Columns 0..m-1 of Q are final; column m holds
// u = beta q_j, the provisional (once-orthogonalised) vector NOT yet divided by its norm beta
// (nrm_prev = beta^2 from the previous step's all-reduce; NULL: u = q_j is normalised, beta = 1).
// hq = [Q_m^T W u ; u^T W u], hw = [Q_m^T W A u ; u^T W A u] (raw); scaled by 1/beta, 1/beta^2
// they give a, alpha, b, b_j of q_j.  With r = sqrt(alpha - a.a) the final vector is
// qbar = (q_j - Q_m a)/r, so
//   * H(m, m-1) = beta (the pending subdiagonal of the previous column) and H row m is corrected
//     in place (delayed re-orthogonalisation): H(0:m, c) += a H(m, c), H(m, c) *= r, c < m
//     (then A Q_m = [Q_m qbar] Hbar holds);
//   * g = Hbar a  (from the old H: g_i = (H a)_i + a_i t, g_m = r t, t = H(m,:) a);
//   * the CGS coefficients of A qbar = (A q_j - [Q_m qbar] g)/r, written to H column m:
//       c_i = (b_i - g_i)/r,  c_m = ((b_j - a.b)/r - g_m)/r;
//   * the update f = A qbar - [Q_m qbar] c = (A u) s/r - Q_m x - qbar y, s = 1/beta, with
//       x = g/r + c (first m),  y = g_m/r + c_m.
// coef layout: [x (m) | c (m+1) | rinv, y, (beta r)^2, s | a (m)].  Without hw only the pending
// subdiagonal, the H correction, r and a are produced (closing re-orthogonalisation of the last
// vector: q = (u - Q_m (beta a)) / (beta r)).

// out[i] = sum_{c in [lo(i), hi(i))} A(i, c) v[c] for i < m, by the whole block: row i is split
// over P = min(8, kThreads / m) threads (strided columns, four independent accumulators, so the
// loads of one thread are in flight together), the P partials summed in a fixed order (the result
// does not depend on timing).  v may live in LDS or global memory; part holds max(kThreads, m)
// doubles of LDS.  Every thread of the block must call it (it synchronises).
template <class FA, class FLo, class FHi>
__device__ __forceinline__ void block_matvec(int m, FA A, FLo lo, FHi hi, const double* v, double* part,
                                             double* out) {
    int P = m > 0 ? kThreads / m : 1;
    P = P < 1 ? 1 : (P > 8 ? 8 : P);
    for (int w = threadIdx.x; w < P * m; w += kThreads) {
        const int i = w % m, q = w / m;
        const int c1 = hi(i);
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        int c = lo(i) + q;
        for (; c + 3 * P < c1; c += 4 * P) {
            a0 = fma(A(i, c), v[c], a0);
            a1 = fma(A(i, c + P), v[c + P], a1);
            a2 = fma(A(i, c + 2 * P), v[c + 2 * P], a2);
            a3 = fma(A(i, c + 3 * P), v[c + 3 * P], a3);
        }
        for (; c < c1; c += P) a0 = fma(A(i, c), v[c], a0);
        part[q * m + i] = (a0 + a1) + (a2 + a3);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += kThreads) {
        double s = 0.0;
        for (int q = 0; q < P; ++q) s += part[q * m + i];
        out[i] = s;
    }
    __syncthreads();
}

// dynamic LDS of k_dcgs2_coef (doubles): sa m | srow m | sg m | part max(kThreads, m)
inline size_t dcgs2_coef_lds(int m) {
    return (size_t)(3 * m + (m > kThreads ? m : kThreads)) * sizeof(double);
}

__global__ __launch_bounds__(kThreads) void k_dcgs2_coef(int m, const double* __restrict__ hq,
                                                         const double* __restrict__ hw,
                                                         const double* __restrict__ nrm_prev,
                                                         double* __restrict__ H, int64_t ldh,
                                                         double* __restrict__ coef,
                                                         int* __restrict__ nan_flag) {
    __shared__ double lds4[4];
    __shared__ double sc[4];
    extern __shared__ double dyn[];
    double* sa = dyn;                 // a
    double* srow = sa + m;            // H(m, c) with the pending subdiagonal filled in
    double* sg = srow + m;            // mat-vec results
    double* part = sg + m;            // mat-vec partials
    auto all = [](int) { return 0; };
    auto to_m = [m](int) { return m; };
    const bool pend = nrm_prev != nullptr && m > 0;
    const double beta = nrm_prev ? sqrt(nrm_prev[0]) : 1.0;
    const double s1 = 1.0 / beta, s2 = s1 * s1;
    double* ca = coef + 2 * m + 5;
    double s = 0.0, p = 0.0, tt = 0.0;
    for (int i = threadIdx.x; i < m; i += kThreads) {
        const double ai = hq[i] * s1;
        const double hr = (pend && i == m - 1) ? beta : H[(int64_t)i * ldh + m];
        sa[i] = ai;
        ca[i] = ai;
        srow[i] = hr;
        s = fma(ai, ai, s);
        tt = fma(hr, ai, tt);   // t = H(m, :) a
        if (hw) p = fma(ai, hw[i] * s1, p);
    }
    s = block_sum(s, lds4);
    __syncthreads();
    if (threadIdx.x == 0) sc[0] = s;
    __syncthreads();
    p = block_sum(p, lds4);
    __syncthreads();
    if (threadIdx.x == 0) sc[1] = p;
    __syncthreads();
    tt = block_sum(tt, lds4);
    __syncthreads();
    if (threadIdx.x == 0) sc[2] = tt;
    __syncthreads();
    const double r2 = hq[m] * s2 - sc[0];
    const double r = sqrt(r2), rinv = 1.0 / r;
    const double t = sc[2];
    if (hw) {
        block_matvec(m, [H, ldh](int i, int c) { return H[(int64_t)c * ldh + i]; }, all, to_m, sa, part, sg);
        double* hm = H + (int64_t)m * ldh;   // column m (new, provisional)
        for (int i = threadIdx.x; i < m; i += kThreads) {
            const double gi = fma(sa[i], t, sg[i]);
            const double ci = (hw[i] * s1 - gi) * rinv;
            coef[m + i] = ci;               // c_i
            coef[i] = fma(gi, rinv, ci);    // x_i
            hm[i] = ci;
        }
        if (threadIdx.x == 0) {
            const double gm = r * t;
            const double cm = ((hw[m] * s2 - sc[1]) * rinv - gm) * rinv;
            coef[2 * m] = cm;
            coef[2 * m + 2] = fma(gm, rinv, cm);  // y
            hm[m] = cm;
        }
    }
    __syncthreads();  // every read of the old H is done before it is corrected
    // H(0:m, c) += a H(m, c): only the columns with H(m, c) != 0 (one in a plain Arnoldi run, the
    // restart row's columns after a Krylov–Schur condensation); the block sweeps a column at a time
    for (int c = 0; c < m; ++c) {
        const double hr = srow[c];
        if (hr != 0.0) {
            double* hc = H + (int64_t)c * ldh;
            for (int i = threadIdx.x; i < m; i += kThreads) hc[i] = fma(sa[i], hr, hc[i]);
        }
    }
    for (int c = threadIdx.x; c < m; c += kThreads) H[(int64_t)c * ldh + m] = srow[c] * r;
    if (threadIdx.x == 0) {
        coef[2 * m + 1] = rinv;
        coef[2 * m + 3] = r2 * beta * beta;
        coef[2 * m + 4] = s1;
        if (!(r2 > 0.0)) atomicOr(nan_flag, 1);   // breakdown: q_j in span(Q_m)
    }
}

// Golub–Kahan–Lanczos bidiagonalisation with delayed re-orthogonalisation (svds, nekStab's
// transient_growth_analysis / resolvent_analysis, linear_stab.f90:112,153): two interleaved DCGS2
// sequences.  The U side's "operator output" is A applied to V's PROVISIONAL vector, the V side's
// is A^T applied to U's provisional vector; each side's pass finishes its own provisional vector
// (re-orthogonalisation folded into the next pass over that basis) and projects the other side's
// output once.  Projection coefficients are corrected one step later, when the provisional vector
// they were formed from is finished.  One workgroup; side 0 = U (matrix M = C, A V = U C), side 1 =
// V (M = D, A^T U = V D).  At pass m of a side (its basis holds m final columns and the provisional
// one, column m):
//   a = hq[0:m], r = sqrt(hq[m] - a.a)  (the provisional column's re-orthogonalisation)
//   with hw (the other side's raw output f): raw coefficients b = hw[0:m],
//     b_m = (hw[m] - a.b)/r into M column p+1 (p = m - side), and the dual-update coefficients
//     coef = [x = b/r | c | rinv, y = b_m/r, r^2, s = 1 | a]  (f_out = f/r - Q_m x - qbar y);
//   M column p finalised (p >= 0) from the other side's (a_o, r_o) at index p and this side's
//     previous r (rho; 1 at m = 0):  M[0:m, p] = (M[0:m, p] - M[0:m, 0:p] a_o + rho a)/r_o,
//     M[m, p] = rho r / r_o.
// A_self / r_self receive (a, r) at index m (column m of A_self, leading dimension lda).
__global__ __launch_bounds__(kThreads) void k_gkl_coef(int side, int m, const double* __restrict__ hq,
                                                       const double* __restrict__ hw, double* __restrict__ M,
                                                       int64_t ldm, double* __restrict__ As, double* __restrict__ rs,
                                                       const double* __restrict__ Ao, const double* __restrict__ ro,
                                                       int64_t lda, double* __restrict__ coef,
                                                       int* __restrict__ nan_flag) {
    __shared__ double lds4[4];
    __shared__ double sc[2];
    extern __shared__ double dyn[];
    double* part = dyn;                                   // block_matvec partials: max(kThreads, m)
    double* sg = part + (m > kThreads ? m : kThreads);    // M[0:m, 0:p] a_o
    double* ca = coef + 2 * m + 5;
    double s = 0.0, pab = 0.0;
    for (int i = threadIdx.x; i < m; i += kThreads) {
        const double ai = hq[i];
        As[(int64_t)m * lda + i] = ai;
        ca[i] = ai;
        s = fma(ai, ai, s);
        if (hw) pab = fma(ai, hw[i], pab);
    }
    s = block_sum(s, lds4);
    __syncthreads();
    if (threadIdx.x == 0) sc[0] = s;
    __syncthreads();
    pab = block_sum(pab, lds4);
    __syncthreads();
    if (threadIdx.x == 0) sc[1] = pab;
    __syncthreads();
    const double r2 = hq[m] - sc[0];
    const double r = sqrt(r2), rinv = 1.0 / r;
    const int p = m - side;
    if (hw) {
        double* Mq = M + (int64_t)(p + 1) * ldm;
        for (int i = threadIdx.x; i < m; i += kThreads) {
            const double bi = hw[i];
            Mq[i] = bi;
            coef[m + i] = bi;
            coef[i] = bi * rinv;
        }
        if (threadIdx.x == 0) {
            const double bm = (hw[m] - sc[1]) * rinv;
            Mq[m] = bm;
            coef[2 * m] = bm;
            coef[2 * m + 2] = bm * rinv;
        }
    }
    if (p >= 0) {
        const double* ao = Ao + (int64_t)p * lda;
        auto all = [](int) { return 0; };
        auto to_p = [p](int) { return p; };
        block_matvec(m, [M, ldm](int i, int c) { return M[(int64_t)c * ldm + i]; }, all, to_p, ao, part, sg);
        const double rho = m > 0 ? rs[m - 1] : 1.0;
        const double roi = 1.0 / ro[p];
        double* Mp = M + (int64_t)p * ldm;
        for (int i = threadIdx.x; i < m; i += kThreads) Mp[i] = fma(rho, hq[i], Mp[i] - sg[i]) * roi;
        if (threadIdx.x == 0) Mp[m] = rho * r * roi;
    }
    if (threadIdx.x == 0) {
        rs[m] = r;
        coef[2 * m + 1] = rinv;
        coef[2 * m + 3] = r2;
        coef[2 * m + 4] = 1.0;
        if (!(r2 > 0.0)) atomicOr(nan_flag, 1);   // breakdown: the provisional vector in span(Q_m)
    }
}

// DCGS2 update, one read of Q_m (m columns):  qbar = (u s - Q_m a) * rinv  -> column m (in place),
// f = (A u) s rinv - Q_m x - qbar * yc  -> fout (the next column: normalised one step later),
// ||f||_W^2 partial.  One row tile (kTile rows at r0): returns f in af.
template <int kPairs>
__device__ __forceinline__ void dcgs2_tile(const double* __restrict__ Q, int64_t ld, int m,
                                           const double* __restrict__ a, const double* __restrict__ x,
                                           double rinv, double yc, double sc, double* __restrict__ qj,
                                           const double* __restrict__ win, double* __restrict__ f,
                                           int64_t r0, double2 (&af)[kPairs]) {
    double2 aq[kPairs];
    const double wsc = sc * rinv;
#pragma unroll
    for (int k = 0; k < kPairs; ++k) {
        const double2 uv = ld2(qj + r0 + k * 2 * kThreads);
        aq[k] = make_double2(uv.x * sc, uv.y * sc);
        const double2 fv = ld2(win + r0 + k * 2 * kThreads);
        af[k] = make_double2(fv.x * wsc, fv.y * wsc);
    }
    const double* qb = Q + r0;
    constexpr int U = NKV_DC_U;
    int c = 0;
    for (; c + U <= m; c += U) {
        double2 q[U][kPairs];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < kPairs; ++k) q[u][k] = ldq(qb + (int64_t)(c + u) * ld + k * 2 * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double ac = -a[c + u], xc = -x[c + u];
#pragma unroll
            for (int k = 0; k < kPairs; ++k) {
                aq[k].x = fma(ac, q[u][k].x, aq[k].x);
                aq[k].y = fma(ac, q[u][k].y, aq[k].y);
                af[k].x = fma(xc, q[u][k].x, af[k].x);
                af[k].y = fma(xc, q[u][k].y, af[k].y);
            }
        }
    }
    for (; c < m; ++c) {
        const double ac = -a[c], xc = -x[c];
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            const double2 q = ldq(qb + (int64_t)c * ld + k * 2 * kThreads);
            aq[k].x = fma(ac, q.x, aq[k].x);
            aq[k].y = fma(ac, q.y, aq[k].y);
            af[k].x = fma(xc, q.x, af[k].x);
            af[k].y = fma(xc, q.y, af[k].y);
        }
    }
#pragma unroll
    for (int k = 0; k < kPairs; ++k) {
        const double2 qbv = make_double2(aq[k].x * rinv, aq[k].y * rinv);
        af[k].x = fma(-yc, qbv.x, af[k].x);
        af[k].y = fma(-yc, qbv.y, af[k].y);
        st2p(qj, r0 + k * 2 * kThreads, qbv);
        st2p(f, r0 + k * 2 * kThreads, af[k]);
    }
}

// kNrm = false: no ||f||_W^2 partial (the next step's dot of u with itself supplies beta^2, see
// nkv_dcgs2_coef), so the weights are not read and no partials are written.
template <int kPairs, bool kNrm>
__global__ __launch_bounds__(kThreads)
void k_dcgs2_update(const double* __restrict__ Q, int64_t ld, int m,
                                                           const double* __restrict__ coef,
                                                           double* __restrict__ qj, const double* __restrict__ win,
                                                           double* __restrict__ f,
                                                           const double* __restrict__ w, int64_t sv,
                                                           int tiles_per_field, int tiles_w, int tiles_total,
                                                           int64_t time_off, int do_time,
                                                           double* __restrict__ partials, int t_lo, int t_hi) {
    constexpr int kTile = kThreads * kPairs * 2;
    __shared__ double lds4[4];
    const double* x = coef;
    const double* a = coef + 2 * m + 5;
    const double rinv = coef[2 * m + 1], yc = coef[2 * m + 2], sc = coef[2 * m + 4];
    if (do_time && blockIdx.x == 0 && threadIdx.x < 64) {
        double s1 = 0.0, s2 = 0.0;
        for (int c = threadIdx.x; c < m; c += 64) {
            const double qt = Q[time_off + (int64_t)c * ld];
            s1 = fma(qt, a[c], s1);
            s2 = fma(qt, x[c], s2);
        }
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        if (threadIdx.x == 0) {
            const double qb = (qj[time_off] * sc - s1) * rinv;
            qj[time_off] = qb;
            f[time_off] = win[time_off] * (sc * rinv) - s2 - qb * yc;
        }
    }
    double2 af[kPairs];
    if constexpr (!kNrm) {
        for (int t = t_lo + blockIdx.x; t < t_hi; t += gridDim.x)   // this launch's row band
            dcgs2_tile<kPairs>(Q, ld, m, a, x, rinv, yc, sc, qj, win, f, (int64_t)t * kTile + 2 * threadIdx.x, af);
        return;
    }
    double nrm = 0.0;
    if (tiles_per_field < (int)gridDim.x && m >= 8) {
        // small problems: fewer row tiles per field than blocks — one tile per work unit so every
        // block has work (the weights of a row tile are re-read per field; they stay cache-resident).
        // +3-8 % at N=2e6 and at the 8-GPU shard for m >= 16; below m = 8 the weight re-reads cost
        // more than the balance gains (profiles/r03ai_tune_dcgs2_norm_units.log)
        for (int t = blockIdx.x; t < tiles_total; t += gridDim.x) {
            const int64_t r0 = (int64_t)t * kTile + 2 * threadIdx.x;
            dcgs2_tile<kPairs>(Q, ld, m, a, x, rinv, yc, sc, qj, win, f, r0, af);
            if (t < tiles_w) {
                const int64_t wr = r0 - (int64_t)(t / tiles_per_field) * sv;
#pragma unroll
                for (int k = 0; k < kPairs; ++k) {
                    const double2 wv = ld2(w + wr + k * 2 * kThreads);
                    nrm = fma(wv.x * af[k].x, af[k].x, nrm);
                    nrm = fma(wv.y * af[k].y, af[k].y, nrm);
                }
            }
        }
        nrm = block_sum(nrm, lds4);
        if (threadIdx.x == 0) partials[blockIdx.x] = nrm;
        return;
    }
    // work unit = one row tile of EVERY weighted field (the norm's weights are read once per unit,
    // not once per field), then the pressure tiles one by one
    const int n_wf = tiles_per_field > 0 ? tiles_w / tiles_per_field : 0;
    const int n_units = tiles_per_field + (tiles_total - tiles_w);
    for (int u = blockIdx.x; u < n_units; u += gridDim.x) {
        if (u < tiles_per_field) {
            double2 wv[kPairs];
#pragma unroll
            for (int k = 0; k < kPairs; ++k) wv[k] = ld2(w + (int64_t)u * kTile + 2 * threadIdx.x + k * 2 * kThreads);
            for (int fi = 0; fi < n_wf; ++fi) {
                dcgs2_tile<kPairs>(Q, ld, m, a, x, rinv, yc, sc, qj, win, f,
                                   (int64_t)(fi * tiles_per_field + u) * kTile + 2 * threadIdx.x, af);
#pragma unroll
                for (int k = 0; k < kPairs; ++k) {
                    nrm = fma(wv[k].x * af[k].x, af[k].x, nrm);
                    nrm = fma(wv[k].y * af[k].y, af[k].y, nrm);
                }
            }
        } else {
            dcgs2_tile<kPairs>(Q, ld, m, a, x, rinv, yc, sc, qj, win, f,
                               (int64_t)(tiles_w + u - tiles_per_field) * kTile + 2 * threadIdx.x, af);
        }
    }
    nrm = block_sum(nrm, lds4);
    if (threadIdx.x == 0) partials[blockIdx.x] = nrm;
}

template <int P>
int launch_block_update_p(const nkv_layout* L, const double* w, const double* Q, int j, const double* h_dev,
                          double* f, double* part, unsigned flags, hipStream_t st, int* g_out) {
    constexpr int kTile = kThreads * P * 2;
    const bool over = (flags & NKV_OVERWRITE) != 0;
    const bool norm = (flags & NKV_NORM2) != 0;
    const int tpf = (int)(L->sv / kTile);
    const int tiles_w = tpf * L->n_wf;
    const int tiles_total = (int)(rows_of(L) / kTile);
    // few columns: a 4x larger grid (the norm partials still fit: the workspace holds at least
    // 4 * kMaxBlocks slots, nkv_workspace_bytes with max_cols >= 1)
    const int gmax = j <= NKV_UPD_SMALL_J ? 4 * kMaxBlocks : kMaxBlocks;
    int g = tiles_total < gmax ? tiles_total : gmax;
    if (g < 1) g = 1;
    *g_out = g;
    const int64_t T = rows_of(L);
    const int dt = (flags & NKV_TIME) ? 1 : 0;
    auto kern = over ? (norm ? k_block_update<true, true, P> : k_block_update<true, false, P>)
                     : (norm ? k_block_update<false, true, P> : k_block_update<false, false, P>);
    // NKV_UPD_ROUNDS > 0: one launch per row band of that many grid-stride rounds, as the DCGS2
    // updates (the first band launches the whole grid, so every block's partial slot is written)
    const int64_t b = (int64_t)NKV_UPD_ROUNDS * g;
    const int band = (NKV_UPD_ROUNDS <= 0 || b >= tiles_total || tiles_total < 2 * b) ? (tiles_total > 0 ? tiles_total : 1)
                                                                                        : (int)b;
    for (int lo = 0; lo == 0 || lo < tiles_total; lo += band) {
        const int hi = lo + band < tiles_total ? lo + band : tiles_total;
        const int gb = lo == 0 ? g : (g < hi - lo ? g : hi - lo);
        hipLaunchKernelGGL(kern, dim3(gb), dim3(kThreads), 0, st, Q, L->ld, j, h_dev, f, w, L->sv, tpf, tiles_w, hi, T,
                           lo == 0 ? dt : 0, part, lo, lo == 0 ? 0 : 1);
        NKV_LAUNCHED();
    }
    return NKV_OK;
}

// Tiles per launch of a banded update (NKV_DC_ROUNDS grid-stride rounds of a g-block grid); all
// tiles in one launch when banding is off or the vector is shorter than two bands.
inline int band_tiles(int tiles_total, int g) {
    if (NKV_DC_ROUNDS <= 0) return tiles_total > 0 ? tiles_total : 1;
    const int64_t b = (int64_t)NKV_DC_ROUNDS * g;
    return (b >= tiles_total || tiles_total < 2 * b) ? (tiles_total > 0 ? tiles_total : 1) : (int)b;
}

// MGS pass coefficients in inverse compact WY form: see nkv_mgs_icwy_solve.
// MGS pass coefficients in inverse compact WY form (nkv_mgs_icwy_solve): x = (I + L)^{-1} b by
// column sweeps, L the strictly lower part of the row-major Gram matrix G.  One workgroup; x lives
// in LDS; sweep k subtracts G(i,k) x_k from every x_i, i > k (one barrier per column), so x_i
// accumulates its terms in the order k = 0, 1, ... (fixed: the result does not depend on timing).
// Row j-1 is taken from grow when given (and stored into G for the next steps).
__global__ __launch_bounds__(kThreads) void k_mgs_icwy_solve(int j, double* __restrict__ G, int64_t ldg,
                                                             const double* __restrict__ grow,
                                                             const double* b, double* x) {
    extern __shared__ double xs[];
    for (int i = threadIdx.x; i < j; i += kThreads) xs[i] = b[i];
    if (grow)
        for (int k = threadIdx.x; k < j - 1; k += kThreads) G[(int64_t)(j - 1) * ldg + k] = grow[k];
    for (int k = 0; k + 1 < j; ++k) {
        __syncthreads();
        const double xk = xs[k];
        for (int i = k + 1 + threadIdx.x; i < j; i += kThreads) {
            const double g = (grow && i == j - 1) ? grow[k] : G[(int64_t)i * ldg + k];
            xs[i] = xs[i] - g * xk;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < j; i += kThreads) x[i] = xs[i];
}

}  // namespace

extern "C" {

int nkv_block_update(const nkv_layout* L, const double* w, const double* Q, int j, const double* h_dev,
                     double* f, double* nrm2_dev, void* ws, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(Q, "Q"));
    CHECK(check_ptr(f, "f"));
    if (!h_dev) return fail(NKV_EINVAL, "h_dev is NULL");
    if (j < 0) return fail(NKV_EINVAL, "j=%d < 0", j);
    const bool norm = (flags & NKV_NORM2) != 0;
    if (norm) {
        CHECK(check_ptr(w, "w"));
        CHECK(check_ptr(ws, "ws"));
        if (!nrm2_dev) return fail(NKV_EINVAL, "nrm2_dev is NULL");
    }
    double* part = ws ? partials_of(ws) : nullptr;
    hipStream_t st = S(stream);
    int g = 1;
    const int64_t T = rows_of(L);
    if (use_large_tiles(L)) CHECK(launch_block_update_p<NKV_PAIRS>(L, w, Q, j, h_dev, f, part, flags, st, &g));
    else CHECK(launch_block_update_p<NKV_PAIRS_SMALL>(L, w, Q, j, h_dev, f, part, flags, st, &g));
    if (norm) {
        // ||f||^2 time term (NKV_TIME_DOT: uparam(1)==2.1 / real_dot) only on the rank owning the
        // replicated scalar.  NKV_TIME alone updates the slot but keeps it out of the norm (k_norm
        // without the time product, krylov_subspace.f90:52-54).
        const bool tdot = (flags & NKV_TIME_DOT) && L->rank0;
        CHECK(launch_reduce_cols(1, part, g, nrm2_dev, tdot ? f + T : nullptr, (int64_t)0, tdot ? f + T : nullptr, nullptr, 1 << 30, nan_flag_of(ws), st));
    }
    return NKV_OK;
}

int nkv_block_update_dot(const nkv_layout* L, const double* w, const double* Q, int j, const double* h_dev,
                         double* f, double* hout_dev, void* ws, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(Q, "Q"));
    CHECK(check_ptr(f, "f"));
    CHECK(check_ptr(ws, "ws"));
    if (!h_dev || !hout_dev) return fail(NKV_EINVAL, "h_dev/hout_dev is NULL");
    if (j < 1 || j > NKV_MAX_COLS) return fail(NKV_EINVAL, "j=%d outside 1..%d", j, NKV_MAX_COLS);
    const unsigned upd_flags = (flags & NKV_TIME) ? NKV_TIME : 0u;
    const unsigned dot_flags = (flags & NKV_TIME_DOT) ? NKV_TIME : 0u;
    if (j > 256 || rows_of(L) >= (int64_t)1 << 29) {  // tile does not fit registers / 32-bit offsets
        CHECK(nkv_block_update(L, w, Q, j, h_dev, f, nullptr, ws, upd_flags, stream));
        return launch_block_dot(L, w, Q, L->ld, j, f, hout_dev, ws, dot_flags, S(stream));
    }
    const int64_t rows = rows_of(L);
    const int64_t tiles_total = rows / kFuseRows;
    const int64_t tpf = L->sv / kFuseRows;
    const int64_t tiles_w = tpf * L->n_wf;
    // mid-size column counts run the fused pass on a smaller grid (NKV_FUSE_G_MID workgroups for
    // NKV_FUSE_MID_LO <= j <= NKV_FUSE_MID_HI)
    const int64_t gcap = (j >= NKV_FUSE_MID_LO && j <= NKV_FUSE_MID_HI) ? NKV_FUSE_G_MID : NKV_FUSE_G;
    int64_t g = tiles_total < gcap ? tiles_total : gcap;
    if (g < 1) g = 1;
    const int B = (int)g;
    const int64_t T = rows;
    const int dt = (flags & NKV_TIME) ? 1 : 0;
    double* part = partials_of(ws);
    hipStream_t st = S(stream);
    // NKV_FUSE_ROUNDS > 0: one launch per row band of that many grid-stride rounds (the first band
    // launches the whole grid, so every partial slot is written before later bands add to it)
    const int64_t fb = (int64_t)NKV_FUSE_ROUNDS * g;
    const int64_t fband = (NKV_FUSE_ROUNDS <= 0 || fb >= tiles_total || tiles_total < 2 * fb)
                              ? (tiles_total > 0 ? tiles_total : 1) : fb;   // >= 1: an empty shard launches once
#define NKV_FUSE(NW, CPW)                                                                                        \
    for (int64_t lo = 0; lo == 0 || lo < tiles_total; lo += fband) {                                             \
        const int64_t hi = lo + fband < tiles_total ? lo + fband : tiles_total;                                  \
        const int64_t gb = lo == 0 ? g : (g < hi - lo ? g : hi - lo);                                            \
        hipLaunchKernelGGL((k_update_dot<NW, CPW>), dim3((unsigned)gb), dim3(NW * 64), 0, st, Q, L->ld, j, h_dev, f, \
                           w, L->sv, tpf, tiles_w, hi, T, lo == 0 ? dt : 0, part, B, lo, lo == 0 ? 0 : 1);        \
    }
    constexpr int NW = NKV_FUSE_NW;
    const int cpw = j <= NW * 16 ? (j + NW - 1) / NW : (j + 15) / 16;
    if (j <= NKV_FUSE_SMALL_J) {   // few columns: 4 waves per workgroup (+4 % at j = 8, +28 % at j = 2)
        switch ((j + 3) / 4) {
            case 1: NKV_FUSE(4, 1); break;
            case 2: NKV_FUSE(4, 2); break;
            case 3: NKV_FUSE(4, 3); break;
            default: NKV_FUSE(4, 4); break;
        }
    } else if (j <= NW * 16) {
        switch (cpw) {
            case 1: NKV_FUSE(NW, 1); break;
            case 2: NKV_FUSE(NW, 2); break;
            case 3: NKV_FUSE(NW, 3); break;
            case 4: NKV_FUSE(NW, 4); break;
            case 5: NKV_FUSE(NW, 5); break;
            case 6: NKV_FUSE(NW, 6); break;
            case 7: NKV_FUSE(NW, 7); break;
            case 8: NKV_FUSE(NW, 8); break;
            case 9: NKV_FUSE(NW, 9); break;
            case 10: NKV_FUSE(NW, 10); break;
            case 11: NKV_FUSE(NW, 11); break;
            case 12: NKV_FUSE(NW, 12); break;
            case 13: NKV_FUSE(NW, 13); break;
            case 14: NKV_FUSE(NW, 14); break;
            case 15: NKV_FUSE(NW, 15); break;
            default: NKV_FUSE(NW, 16); break;
        }
    } else {  // 16 waves, up to 16 columns each (j <= 256)
        switch (cpw) {
            case 9: NKV_FUSE(16, 9); break;
            case 10: NKV_FUSE(16, 10); break;
            case 11: NKV_FUSE(16, 11); break;
            case 12: NKV_FUSE(16, 12); break;
            case 13: NKV_FUSE(16, 13); break;
            case 14: NKV_FUSE(16, 14); break;
            case 15: NKV_FUSE(16, 15); break;
            default: NKV_FUSE(16, 16); break;
        }
    }
#undef NKV_FUSE
    NKV_LAUNCHED();
    const bool tdot = (flags & NKV_TIME_DOT) && L->rank0;
    CHECK(launch_reduce_cols(j, part, B, hout_dev, tdot ? Q + T : nullptr, L->ld, tdot ? f + T : nullptr, nullptr, 1 << 30, nan_flag_of(ws), st));
    return NKV_OK;
}

int nkv_block_dot2(const nkv_layout* L, const double* w, const double* Q, int j, const double* x,
                   const double* y, double* h_dev, void* ws, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(Q, "Q"));
    CHECK(check_ptr(x, "x"));
    CHECK(check_ptr(y, "y"));
    CHECK(check_ptr(ws, "ws"));
    if (!h_dev) return fail(NKV_EINVAL, "h_dev is NULL");
    if (j < 1 || j > NKV_MAX_COLS) return fail(NKV_EINVAL, "j=%d outside 1..%d", j, NKV_MAX_COLS);
    if ((flags & NKV_X_IS_LAST) && x != Q + (int64_t)(j - 1) * L->ld)
        return fail(NKV_EINVAL, "NKV_X_IS_LAST: x is not column j-1 of Q");
    hipStream_t st = S(stream);
    const bool large = use_large_tiles(L);
    const int P = large ? NKV_D2_PAIRS : NKV_PAIRS_SMALL;
    const int kTile = kThreads * P * 2;
    const int tpf = (int)(L->sv / kTile);
    // large problems: one block row walks every field of its tiles (weights read once per tile)
    const int nf = (large && NKV_D2_FIELDLOOP) ? L->n_wf : 1;
    const int gy = L->n_wf / nf;
    // one workgroup per CU for large problems (8 rows/thread keep enough loads in flight); two per
    // CU for small problems (4 rows/thread), each walking a few tiles
    const int bmax = large ? NKV_D2_MAXB : NKV_D2_SMALL_B;
    int bx = (bmax < kMaxBlocks ? bmax : kMaxBlocks) / gy;
    if (bx > tpf) bx = tpf;
    if (bx < 1) bx = 1;
    const int B = bx * gy;
    double* part = partials_of(ws);
    if (tpf > 0) {
        const int xl = (flags & NKV_X_IS_LAST) ? 1 : 0;
        if (large)
            hipLaunchKernelGGL(k_block_dot2<NKV_D2_PAIRS>, dim3(bx, gy), dim3(kThreads), 8 * j * sizeof(double), st,
                               Q, L->ld, j, x, y, w, L->sv, tpf, nf, xl, part, B);
        else
            hipLaunchKernelGGL(k_block_dot2<NKV_PAIRS_SMALL>, dim3(bx, gy), dim3(kThreads), 8 * j * sizeof(double),
                               st, Q, L->ld, j, x, y, w, L->sv, tpf, nf, xl, part, B);
        NKV_LAUNCHED();
    }
    const int64_t T = rows_of(L);
    const bool tdot = (flags & NKV_TIME) && L->rank0;
    CHECK(launch_reduce_cols(2 * j, part, tpf > 0 ? B : 0, h_dev, tdot ? Q + T : nullptr, L->ld, tdot ? x + T : nullptr, tdot ? y + T : nullptr, j, nan_flag_of(ws), st));
    return NKV_OK;
}

int nkv_mgs_icwy_solve(int j, double* G, int64_t ldg, const double* grow, const double* b, double* x,
                       void* stream) {
    if (j < 1 || j > NKV_MAX_COLS) return fail(NKV_EINVAL, "icwy: j=%d outside 1..%d", j, NKV_MAX_COLS);
    if (!G || !b || !x) return fail(NKV_EINVAL, "icwy: G/b/x is NULL");
    if (ldg < j) return fail(NKV_EINVAL, "icwy: ldg=%lld < j=%d", (long long)ldg, j);
    hipLaunchKernelGGL(k_mgs_icwy_solve, dim3(1), dim3(kThreads), j * sizeof(double), S(stream), j, G, ldg, grow,
                       b, x);
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_dcgs2_coef(int m, const double* hq_dev, const double* hw_dev, const double* nrm_prev_dev, double* H_dev,
                   int64_t ldh, double* coef_dev, void* ws, void* stream) {
    if (m < 0 || m > NKV_MAX_COLS) return fail(NKV_EINVAL, "m=%d outside 0..%d", m, NKV_MAX_COLS);
    if (!hq_dev || !H_dev || !coef_dev) return fail(NKV_EINVAL, "hq/H/coef is NULL");
    if (ldh < m + 1) return fail(NKV_EINVAL, "ldh=%lld < m+1=%d", (long long)ldh, m + 1);
    CHECK(check_ptr(ws, "ws"));
    hipLaunchKernelGGL(k_dcgs2_coef, dim3(1), dim3(kThreads), dcgs2_coef_lds(m), S(stream), m, hq_dev, hw_dev,
                       nrm_prev_dev, H_dev, ldh, coef_dev, nan_flag_of(ws));
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_gkl_coef(int side, int m, const double* hq_dev, const double* hw_dev, double* M_dev, int64_t ldm,
                 double* A_self, double* r_self, const double* A_other, const double* r_other, int64_t lda,
                 double* coef_dev, void* ws, void* stream) {
    if (side != 0 && side != 1) return fail(NKV_EINVAL, "side=%d must be 0 (U) or 1 (V)", side);
    if (m < 0 || m > NKV_MAX_COLS) return fail(NKV_EINVAL, "m=%d outside 0..%d", m, NKV_MAX_COLS);
    if (!hq_dev || !M_dev || !A_self || !r_self || !coef_dev) return fail(NKV_EINVAL, "hq/M/A_self/r_self/coef is NULL");
    if (m - side >= 0 && (!A_other || !r_other)) return fail(NKV_EINVAL, "A_other/r_other is NULL");
    if (ldm < m + 1 || lda < m + 1) return fail(NKV_EINVAL, "ldm=%lld / lda=%lld < m+1=%d", (long long)ldm,
                                                (long long)lda, m + 1);
    CHECK(check_ptr(ws, "ws"));
    const size_t lds = (size_t)((m > kThreads ? m : kThreads) + (m > 0 ? m : 1)) * sizeof(double);
    hipLaunchKernelGGL(k_gkl_coef, dim3(1), dim3(kThreads), lds, S(stream), side, m, hq_dev, hw_dev, M_dev, ldm,
                       A_self, r_self, A_other, r_other, lda, coef_dev, nan_flag_of(ws));
    NKV_LAUNCHED();
    return NKV_OK;
}

int nkv_dcgs2_update(const nkv_layout* L, const double* w, const double* Q, int m, const double* coef_dev,
                     double* qj, const double* win, double* fout, double* nrm2_dev, void* ws, unsigned flags,
                     void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(w, "w"));
    CHECK(check_ptr(Q, "Q"));
    CHECK(check_ptr(qj, "qj"));
    CHECK(check_ptr(win, "win"));
    CHECK(check_ptr(fout, "fout"));
    CHECK(check_ptr(ws, "ws"));
    if (m < 0) return fail(NKV_EINVAL, "m=%d < 0", m);
    if (!coef_dev) return fail(NKV_EINVAL, "coef is NULL");
    hipStream_t st = S(stream);
    const bool large = use_large_tiles(L);
    const int P = large ? NKV_DC_PAIRS : NKV_PAIRS_SMALL;
    const int kTile = kThreads * P * 2;
    const int tpf = (int)(L->sv / kTile);
    const int tiles_w = tpf * L->n_wf;
    const int tiles_total = (int)(rows_of(L) / kTile);
    const int gmax = NKV_DC_G < kMaxBlocks ? NKV_DC_G : kMaxBlocks;
    int g = tiles_total < gmax ? tiles_total : gmax;
    if (g < 1) g = 1;
    const int64_t T = rows_of(L);
    const int dt = (flags & NKV_TIME) ? 1 : 0;
    double* part = partials_of(ws);
    auto kern = large ? (nrm2_dev ? k_dcgs2_update<NKV_DC_PAIRS, true> : k_dcgs2_update<NKV_DC_PAIRS, false>)
                      : (nrm2_dev ? k_dcgs2_update<NKV_PAIRS_SMALL, true> : k_dcgs2_update<NKV_PAIRS_SMALL, false>);
    if (!nrm2_dev) {
        // one launch per row band of NKV_DC_ROUNDS grid-stride rounds: every launch boundary is a
        // grid-wide point where all loads and stores of the band have retired (no in-kernel barrier)
        const int band = band_tiles(tiles_total, g);
        for (int lo = 0; lo == 0 || lo < tiles_total; lo += band) {   // >= 1 launch: also the time slot
            const int hi = lo + band < tiles_total ? lo + band : tiles_total;
            const int gb = g < hi - lo ? g : (hi - lo > 0 ? hi - lo : 1);
            hipLaunchKernelGGL(kern, dim3(gb), dim3(kThreads), 0, st, Q, L->ld, m, coef_dev, qj, win, fout, w, L->sv,
                               tpf, tiles_w, tiles_total, T, lo == 0 ? dt : 0, part, lo, hi);
            NKV_LAUNCHED();
        }
        return NKV_OK;
    }
    // with the fused norm every block leaves one partial: a single launch over all tiles
    hipLaunchKernelGGL(kern, dim3(g), dim3(kThreads), 0, st, Q, L->ld, m, coef_dev, qj, win, fout, w, L->sv, tpf,
                       tiles_w, tiles_total, T, dt, part, 0, tiles_total);
    NKV_LAUNCHED();
    const bool tdot = (flags & NKV_TIME_DOT) && L->rank0;
    CHECK(launch_reduce_cols(1, part, g, nrm2_dev, tdot ? fout + T : nullptr, (int64_t)0, tdot ? fout + T : nullptr, nullptr, 1 << 30, nan_flag_of(ws), st));
    return NKV_OK;
}

int nkv_combine(const nkv_layout* L, const double* Q, int k, const double* y_dev, double* out, unsigned flags,
                void* stream) {
    return nkv_block_update(L, nullptr, Q, k, y_dev, out, nullptr, nullptr,
                            (flags & ~(unsigned)NKV_NORM2) | NKV_OVERWRITE, stream);
}

}  // extern "C"
