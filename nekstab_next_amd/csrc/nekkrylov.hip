// nekkrylov.hip — gfx950 (MI355X / CDNA4) kernels + C ABI for nekStab's Krylov hot path.
//
// Layout, flags and the reference functions each entry point replaces: include/nekkrylov.h.
// Design notes (roofline, bytes per launch): DESIGN.md.
//
// Every kernel here is HBM-bound fp64 streaming (BLAS-1/2): 16-B (double2) coalesced loads,
// 256-thread workgroups (4 wave64s), wave reductions by cross-lane shuffles, LDS for the
// per-workgroup partials, and a deterministic two-stage reduction (fixed block->tile map,
// fixed-order second stage; no floating-point atomics) so results do not depend on timing.
// The one near-ridge kernel (restart rotation Q <- Q V) is LDS-tiled with 4x4 register blocks.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "nekkrylov.h"

namespace {

// Tuning knobs (compile-time; tools/tune_kernels.py builds variants and times them on MI355X):
#ifndef NKV_PAIRS
#define NKV_PAIRS 8  // double2 per thread per tile in the dot/update kernels (large problems)
#endif
#ifndef NKV_PAIRS_SMALL
#define NKV_PAIRS_SMALL 4  // ... when the vector has fewer than NKV_SMALL_TILES large tiles (4: +9-13 % on the
                           // multi-dot at N=2e6 over 2, profiles/r01m_tune_small.log)
#endif
#ifndef NKV_SMALL_TILES
#define NKV_SMALL_TILES 2048
#endif
#ifndef NKV_COLU
#define NKV_COLU 4  // basis columns in flight per thread in the multi-dot
#endif
#ifndef NKV_NT
#define NKV_NT 1  // non-temporal loads for the streamed basis columns
#endif
#ifndef NKV_MAXB
#define NKV_MAXB 1024  // workgroups (= reduction partials per column) of the dot/update kernels
#endif
#ifndef NKV_FUSE_NW
#define NKV_FUSE_NW 8  // waves per workgroup of the fused update+dot for j <= 16*NKV_FUSE_NW
#endif
#ifndef NKV_FUSE_G
#define NKV_FUSE_G 1024  // workgroups of the fused update+dot
#endif
#ifndef NKV_FUSE_G_MID
#define NKV_FUSE_G_MID 512  // ... for NKV_FUSE_MID_LO <= j <= NKV_FUSE_MID_HI: +5-8 % at N = 1.25e7,
#endif                      // 5e7 and 1e8 (profiles/r02ao_tune_fmid.log)
#ifndef NKV_FUSE_MID_LO
#define NKV_FUSE_MID_LO 16
#endif
#ifndef NKV_FUSE_MID_HI
#define NKV_FUSE_MID_HI 32
#endif
#ifndef NKV_DC_PAIRS
#define NKV_DC_PAIRS 8  // double2 per thread per tile in the DCGS2 kernels (large problems)
#endif
#ifndef NKV_DC_U
#define NKV_DC_U 2  // basis columns in flight in the DCGS2 dual update
#endif
#ifndef NKV_NT_ST
#define NKV_NT_ST 1  // non-temporal stores of streamed vectors (DCGS2 update, finish, synthetic matvec)
#endif
#ifndef NKV_STREAM_UNR
#define NKV_STREAM_UNR 4  // double2 per thread in flight in the streaming vector kernels
#endif
#ifndef NKV_DC_G
#define NKV_DC_G 768  // workgroups of the DCGS2 dual update: 3 per CU (122 VGPRs allow 4) is 1-6 %
                      // faster than 4 per CU at N=1e8 and at the 8-GPU shard; non-multiples of the
                      // 256 CUs lose 5-10 % (profiles/r01k_tune_update_grid.log)
#endif
#ifndef NKV_UPD_ROUNDS
#define NKV_UPD_ROUNDS 2  // block update (CGS2 passes, DCGS2 close): row-band launches of this many rounds
#endif                    // (+2 % on update+norm at N=1e8, profiles/r02bh_tune_upd_bands.log)
#ifndef NKV_AXD_ROUNDS
#define NKV_AXD_ROUNDS 0  // fused MGS column step (nkv_axpy_dot): row-band launches of this many rounds
#endif
#ifndef NKV_UPD_SMALL_J
#define NKV_UPD_SMALL_J 2   // block update: 4x the workgroups up to this many columns (+5-9 % at j <= 2,
                            // neutral to -4 % from j = 4 on: profiles/r02br_tune_upd_small*.log)
#endif
#ifndef NKV_FUSE_SMALL_J
#define NKV_FUSE_SMALL_J 12  // fused CGS2 middle pass: 4-wave workgroups up to this many columns
#endif                       // (profiles/r02bn_tune_fuse_small*.log); 0 disables
static_assert(NKV_FUSE_SMALL_J >= 0 && NKV_FUSE_SMALL_J <= 16,
              "the 4-wave fused pass instantiates at most 16 columns (NKV_FUSE(4, 4))");
#ifndef NKV_FUSE_ROUNDS
#define NKV_FUSE_ROUNDS 0  // fused CGS2 middle pass: row-band launches of this many rounds (0: one launch)
#endif
#ifndef NKV_DC_ROUNDS
#define NKV_DC_ROUNDS 2  // DCGS2 updates: one launch per this many grid-stride rounds of row tiles (a
                         // "row band"); the launch boundaries keep the grid's loads and stores in one
                         // band: +9-19 % at N=1e8, +0-1 % at the 8-GPU shard (profiles/r02f_tune_*)
#endif
#ifndef NKV_STREAM_ROUNDS
#define NKV_STREAM_ROUNDS 2  // synthetic diagonal matvec: one launch per this many grid-stride rounds
#endif
#ifndef NKV_D2_MAXB
#define NKV_D2_MAXB 256  // workgroups of the two-vector multi-dot: one per CU (+1 % over 1024 at
                          // N=1e8 and at the 8-GPU shard; 384 = 1.5 per CU loses 6-10 %)
#endif
#ifndef NKV_D2_SMALL_B
#define NKV_D2_SMALL_B 512  // ... and for small problems (2-row tiles, no field loop): two per CU; the
                            // kMaxBlocks grid (one tile per block) loses 10-27 % at N=2e6
                            // (profiles/r03aa_tune_d2_small_grid.log)
#endif
#ifndef NKV_DOT_SMALL_B
#define NKV_DOT_SMALL_B 512  // workgroups of the one-vector multi-dot / dot on small problems: as the
                            // two-vector one, +6-12 % at N=2e6, j >= 4 (profiles/r03ac_tune_dot_small_grid.log)
#endif
#ifndef NKV_D2_FIELDLOOP
#define NKV_D2_FIELDLOOP 1  // two-vector multi-dot: one block walks all weighted fields of a tile
#endif
#ifndef NKV_D2_U
#define NKV_D2_U 2  // basis columns in flight in the two-vector multi-dot
#endif
// The round-1 timing experiments (store skipping, grid-wide soft barriers, tile-interleaved and
// field-major sweeps, XCD tile maps, buffer-store cache policies, register-budget schedules;
// DESIGN.md §6 "What did not help") are not part of this file.  The knobs above change speed only.
#if defined(NKV_DC_EXPERIMENT) || defined(NKV_DC_SYNC) || defined(NKV_QTILE_EXP) || defined(NKV_D2_FIELDMAJOR) || \
    defined(NKV_DC_SCHED) || defined(NKV_D2_SCHED) || defined(NKV_ST_AUX) || defined(NKV_XCD_MAP) ||           \
    defined(NKV_DC_FIELDLOOP) || defined(NKV_FUSE_PF) || defined(NKV_LD_ALIGN)
#error "round-1 experiment switches were removed from the product kernel"
#endif

constexpr int kThreads = 256;                       // 4 waves of 64
constexpr int kStreamUnr = NKV_STREAM_UNR;
static_assert(NKV_TILE % (2 * kThreads * NKV_STREAM_UNR) == 0, "stream chunk must divide the padding");
static_assert(NKV_TILE % (kThreads * NKV_PAIRS * 2) == 0, "kernel tile must divide the padding");
static_assert(NKV_TILE % (kThreads * NKV_PAIRS_SMALL * 2) == 0, "kernel tile must divide the padding");
constexpr int kMaxBlocks = NKV_MAXB;                 // reduction partial slots per column
constexpr int kColUnroll = NKV_COLU;                 // columns in flight per thread (block dot)
constexpr size_t kCtrlBytes = 256;                   // control words at the head of the workspace
constexpr int kRotMaxK = NKV_ROT_MAX_K;               // rotation: 64-row tiles up to k=256, 32-row beyond

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define NKV_HIP(call)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(NKV_EHIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__,  \
                        __LINE__);                                                           \
    } while (0)

#define NKV_LAUNCHED()                                                                       \
    do {                                                                                     \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ != hipSuccess)                                                                \
            return fail(NKV_EHIP, "kernel launch: %s (%s:%d)", hipGetErrorString(e_),        \
                        __FILE__, __LINE__);                                                 \
    } while (0)

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Rows that every BLAS-1 op streams (weighted fields + pressure, padded); the time slot sits at
// this offset.
inline int64_t rows_of(const nkv_layout* L) { return (int64_t)L->n_wf * L->sv + L->sp; }

// Compute units of the current device (cached per device id; 256 on MI355X).
int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        cus[dev] = (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                       ? n : 256;
    }
    return cus[dev];
}

int check_layout(const nkv_layout* L) {
    if (!L) return fail(NKV_EINVAL, "layout is NULL");
    if (L->n_wf < 1 || L->n_v < 0 || L->n_p < 0)
        return fail(NKV_EINVAL, "bad layout: n_wf=%d n_v=%lld n_p=%lld", L->n_wf,
                    (long long)L->n_v, (long long)L->n_p);
    if (L->sv < L->n_v || L->sp < L->n_p || L->sv % NKV_TILE || L->sp % NKV_TILE || L->ld % NKV_TILE)
        return fail(NKV_ESHAPE, "layout not padded to NKV_TILE: sv=%lld sp=%lld ld=%lld",
                    (long long)L->sv, (long long)L->sp, (long long)L->ld);
    if (L->ld < rows_of(L) + 1)
        return fail(NKV_ESHAPE, "ld=%lld too small for %lld rows + time", (long long)L->ld,
                    (long long)rows_of(L));
    return NKV_OK;
}

int check_ptr(const void* p, const char* what) {
    if (!p) return fail(NKV_EINVAL, "%s is NULL", what);
    if (reinterpret_cast<uintptr_t>(p) % 16) return fail(NKV_ESHAPE, "%s not 16-byte aligned", what);
    return NKV_OK;
}

#define CHECK(x)                   \
    do {                           \
        int rc_ = (x);             \
        if (rc_ != NKV_OK) return rc_; \
    } while (0)

// ------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

#ifndef NKV_D2_RED
#define NKV_D2_RED 1  // transposed wave reduction in the multi-dots (DPP within rows): +4-10 % on
                      // the two-vector dot at N=2e6, +0.3 % at N=1e8 (profiles/r01m_tune_d2red.log)
#endif

// One DPP move of a double (two 32-bit halves), every lane reading its source lane.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(__double_as_longlong(v) & 0xffffffffll), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(__double_as_longlong(v) >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Sums of FOUR per-lane values over the 64 lanes in 7 exchanges instead of 24: the xor-32 and
// xor-16 steps each hand half of the values to the partner (so every lane keeps one value from
// there on), the in-row steps run on DPP (quad xor 1, quad xor 2, half-row mirror, row mirror).
// Value v lands in lane 16 v (v = 0..3).  Deterministic (a fixed exchange pattern).
__device__ __forceinline__ double wave_sum4(double s0, double s1, double s2, double s3, int lane) {
    const bool up = (lane & 32) != 0;
    const double k0 = (up ? s2 : s0) + __shfl_xor(up ? s0 : s2, 32, 64);
    const double k1 = (up ? s3 : s1) + __shfl_xor(up ? s1 : s3, 32, 64);
    const bool b4 = (lane & 16) != 0;
    double v = (b4 ? k1 : k0) + __shfl_xor(b4 ? k0 : k1, 16, 64);
    v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_d<0x141>(v);   // row_half_mirror
    v += dpp_d<0x140>(v);   // row_mirror
    return v;
}

// Block-wide sum of one double (256 threads); result valid in thread 0.
__device__ __forceinline__ double block_sum(double v, double* lds4) {
    v = wave_sum(v);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) lds4[wave] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) r = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    return r;
}

__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
// uniform base + 32-bit byte offset: lets the compiler use the SGPR-base/VGPR-offset load form
// instead of a 64-bit VGPR address per column (fewer VGPRs in the register-resident kernels)
__device__ __forceinline__ const double* at_b(const double* base, uint32_t byte_off) {
    return reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + byte_off);
}

typedef double v2d __attribute__((ext_vector_type(2)));
// Loads of streamed basis columns: each byte is read once per pass and, at the sizes that matter,
// the basis is far larger than L2 + Infinity Cache, so the loads are non-temporal (NKV_NT).
__device__ __forceinline__ double2 ldq(const double* p) {
#if NKV_NT
    const v2d v = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(p));
    return make_double2(v.x, v.y);
#else
    return ld2(p);
#endif
}
__device__ __forceinline__ void st2(double* p, double2 v) { *reinterpret_cast<double2*>(p) = v; }
// Stores of whole streamed vectors (800 MB at N=1e8, never re-read from cache): non-temporal (NKV_NT_ST)
__device__ __forceinline__ void st2s(double* p, double2 v) {
#if NKV_NT_ST
    __builtin_nontemporal_store(v2d{v.x, v.y}, reinterpret_cast<v2d*>(p));
#else
    st2(p, v);
#endif
}
// Store of one double2 at element offset `off` of a streamed vector `base`.
__device__ __forceinline__ void st2p(double* base, int64_t off, double2 v) { st2s(base + off, v); }

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
//
// Lazy basis (T != NULL): the stored columns S_0..S_{m-1} are the raw provisional vectors and the
// orthonormal basis is Q_m = S T_m (T upper triangular, column i at T + i ldt).  The raw dots are
// mapped first (hq <- T_m^T hq, hw <- T_m^T hw; the u entries stay), the algebra above is
// unchanged, and instead of writing qbar the kernel appends T's column m,
//   qbar = S_{0..m} t,  t = [-T_m a / r ; s / r],
// and the update's coefficients z = [T_m x + t_{0:m} y ; t_m y] (coef + 3m + 5, m + 1 entries):
// f = (A u) s/r - S_{0..m} z, one output vector.  Closing call (hw NULL): z = beta T_m a (for
// u <- u - S_{0:m} z, then u / (beta r)) and T's column m = e_m (the closed column is final).
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

// dynamic LDS of k_dcgs2_coef (doubles): tq 2(m+1) | sa m | srow m | sg m | part max(kThreads, m)
inline size_t dcgs2_coef_lds(int m) {
    return (size_t)(2 * (m + 1) + 3 * m + (m > kThreads ? m : kThreads)) * sizeof(double);
}

__global__ __launch_bounds__(kThreads) void k_dcgs2_coef(int m, const double* __restrict__ hq_raw,
                                                         const double* __restrict__ hw_raw,
                                                         const double* __restrict__ nrm_prev,
                                                         double* __restrict__ H, int64_t ldh,
                                                         double* __restrict__ coef,
                                                         double* __restrict__ T, int64_t ldt,
                                                         int* __restrict__ nan_flag) {
    __shared__ double lds4[4];
    __shared__ double sc[4];
    extern __shared__ double dyn[];
    double* tq = dyn;                 // lazy: [T^T hq (m+1) | T^T hw (m+1)]; later T x
    double* sa = tq + 2 * (m + 1);    // a
    double* srow = sa + m;            // H(m, c) with the pending subdiagonal filled in; later x
    double* sg = srow + m;            // mat-vec results
    double* part = sg + m;            // mat-vec partials
    const double* hq = hq_raw;
    const double* hw = hw_raw;
    auto all = [](int) { return 0; };
    auto to_m = [m](int) { return m; };
    if (T) {   // hq <- T_m^T hq: (T^T h)_i = sum_{l <= i} T(l, i) h_l, column i of T contiguous
        auto Tt = [T, ldt](int i, int l) { return T[(int64_t)i * ldt + l]; };
        auto upto = [](int i) { return i + 1; };
        block_matvec(m, Tt, all, upto, hq_raw, part, tq);
        if (hw_raw) block_matvec(m, Tt, all, upto, hw_raw, part, tq + (m + 1));
        if (threadIdx.x == 0) {
            tq[m] = hq_raw[m];
            if (hw_raw) tq[2 * m + 1] = hw_raw[m];
        }
        __syncthreads();
        hq = tq;
        hw = hw_raw ? tq + (m + 1) : nullptr;
    }
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
    if (T) {   // lazy basis: T's column m and the single-output update coefficients z
        __syncthreads();   // x (coef[0:m]) and y are written; srow is free
        for (int i = threadIdx.x; i < m; i += kThreads) srow[i] = hw ? coef[i] : 0.0;
        __syncthreads();
        // (T v)_l = sum_{i >= l} T(l, i) v_i
        auto Tl = [T, ldt](int l, int i) { return T[(int64_t)i * ldt + l]; };
        auto from = [](int l) { return l; };
        block_matvec(m, Tl, from, to_m, sa, part, sg);              // T a
        if (hw) block_matvec(m, Tl, from, to_m, srow, part, tq);    // T x (tq is free)
        double* tm = T + (int64_t)m * ldt;
        double* z = coef + 3 * m + 5;
        const double yv = hw ? coef[2 * m + 2] : 0.0;
        const double tmm = s1 * rinv;
        for (int l = threadIdx.x; l < m; l += kThreads) {
            if (hw) {
                const double tl = -sg[l] * rinv;
                tm[l] = tl;
                z[l] = fma(tl, yv, tq[l]);
            } else {
                tm[l] = 0.0;
                z[l] = beta * sg[l];
            }
        }
        if (threadIdx.x == 0) {
            tm[m] = hw ? tmm : 1.0;
            z[m] = hw ? tmm * yv : 0.0;
        }
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

// Lazy-basis DCGS2 update (see k_dcgs2_coef): f = (A u) s/r - S_{0..m} z in one read of the m+1
// stored columns (u included), ONE output vector; the finished qbar is never written (it is
// column m of S T).  Same tiling and streaming as the dual update.
#ifndef NKV_DL_U
#define NKV_DL_U 2  // columns in flight in the lazy update
#endif
template <int kPairs>
__global__ __launch_bounds__(kThreads) void k_dcgs2_lazy_update(const double* __restrict__ S, int64_t ld, int m,
                                                                const double* __restrict__ coef,
                                                                const double* __restrict__ win,
                                                                double* __restrict__ f, int t_lo, int t_hi,
                                                                int64_t time_off, int do_time) {
    constexpr int kTile = kThreads * kPairs * 2;
    constexpr int U = NKV_DL_U;
    const double* z = coef + 3 * m + 5;
    const double c0 = coef[2 * m + 1] * coef[2 * m + 4];   // s / r
    const int n = m + 1;
    if (do_time && blockIdx.x == 0 && threadIdx.x < 64) {
        double s = 0.0;
        for (int c = threadIdx.x; c < n; c += 64) s = fma(S[time_off + (int64_t)c * ld], z[c], s);
        s = wave_sum(s);
        if (threadIdx.x == 0) f[time_off] = win[time_off] * c0 - s;
    }
    for (int t = t_lo + blockIdx.x; t < t_hi; t += gridDim.x) {
        const int64_t r0 = (int64_t)t * kTile + 2 * threadIdx.x;
        double2 af[kPairs];
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            const double2 fv = ld2(win + r0 + k * 2 * kThreads);
            af[k] = make_double2(fv.x * c0, fv.y * c0);
        }
        const double* qb = S + r0;
        int c = 0;
        for (; c + U <= n; c += U) {
            double2 q[U][kPairs];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int k = 0; k < kPairs; ++k) q[u][k] = ldq(qb + (int64_t)(c + u) * ld + k * 2 * kThreads);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double zc = -z[c + u];
#pragma unroll
                for (int k = 0; k < kPairs; ++k) {
                    af[k].x = fma(zc, q[u][k].x, af[k].x);
                    af[k].y = fma(zc, q[u][k].y, af[k].y);
                }
            }
        }
        for (; c < n; ++c) {
            const double zc = -z[c];
#pragma unroll
            for (int k = 0; k < kPairs; ++k) {
                const double2 q = ldq(qb + (int64_t)c * ld + k * 2 * kThreads);
                af[k].x = fma(zc, q.x, af[k].x);
                af[k].y = fma(zc, q.y, af[k].y);
            }
        }
#pragma unroll
        for (int k = 0; k < kPairs; ++k) st2s(f + r0 + k * 2 * kThreads, af[k]);
    }
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

// ------------------------------------------------------------------------------------------
// Restart rotation, in place:  Q[:, 0:k] <- Q[:, 0:k] V.   One workgroup owns R rows: the
// R x k input tile is staged in LDS (so outputs can overwrite those rows), V streams through LDS
// in 16 x CC chunks, each thread accumulates a 4 x 4 register block.  R = 64 up to k = 256,
// R = 32 up to k = 576 (the tile must fit the 160 KiB LDS).
// ------------------------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(kThreads) void k_rotate(double* __restrict__ Q, int64_t ld, int k,
                                                     const double* __restrict__ V, int ldv,
                                                     int64_t n_tiles) {
    constexpr int RG = R / 4;          // row groups of 4
    constexpr int CG = kThreads / RG;  // column groups of 4
    constexpr int CC = 4 * CG;         // columns per chunk
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* A = sm;            // [k][R]
    double* Vs = sm + k * R;   // [16][CC]
    const int tr = threadIdx.x % RG;  // rows 4*tr .. 4*tr+3
    const int tc = threadIdx.x / RG;  // cols 4*tc .. 4*tc+3 of the current chunk
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t row0 = tile * R;
        __syncthreads();
        for (int idx = threadIdx.x; idx < k * (R / 2); idx += kThreads) {
            const int c = idx / (R / 2), r2 = idx % (R / 2);
            st2(A + c * R + 2 * r2, ld2(Q + (int64_t)c * ld + row0 + 2 * r2));
        }
        __syncthreads();
        for (int cc = 0; cc < k; cc += CC) {
            double acc[4][4];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
            for (int ii = 0; ii < k; ii += 16) {
                for (int e = threadIdx.x; e < 16 * CC; e += kThreads) {
                    const int i = e / CC, c = e % CC;
                    const int gi = ii + i, gc = cc + c;
                    Vs[e] = (gi < k && gc < k) ? V[gi + (int64_t)gc * ldv] : 0.0;
                }
                __syncthreads();
                const int imax = min(16, k - ii);
                for (int i = 0; i < imax; ++i) {
                    const double2 a01 = ld2(A + (ii + i) * R + 4 * tr);
                    const double2 a23 = ld2(A + (ii + i) * R + 4 * tr + 2);
                    const double2 v01 = ld2(Vs + i * CC + 4 * tc);
                    const double2 v23 = ld2(Vs + i * CC + 4 * tc + 2);
                    const double av[4] = {a01.x, a01.y, a23.x, a23.y};
                    const double vv[4] = {v01.x, v01.y, v23.x, v23.y};
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int b = 0; b < 4; ++b) acc[a][b] = fma(av[a], vv[b], acc[a][b]);
                }
                __syncthreads();
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int gc = cc + 4 * tc + b;
                if (gc < k) {
                    double* dst = Q + (int64_t)gc * ld + row0 + 4 * tr;
                    st2(dst, make_double2(acc[0][b], acc[1][b]));
                    st2(dst + 2, make_double2(acc[2][b], acc[3][b]));
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Restart rotation on the f64 matrix cores:  Q[:, 0:n_out] <- Q[:, 0:k] V[:, 0:n_out].
// Computed as the transpose, D = V^T Q^T, so that D's fast (lane & 15) index runs along the
// points: every 16-lane group stores 128 contiguous bytes of one column.  One workgroup owns R
// rows; its R x k input tile is staged in LDS before any output is written (in place is safe).
// Waves: WR = R/16 row blocks x WC = 4/WR column groups; each wave keeps MB 16x16 accumulators
// (v_mfma_f64_16x16x4_f64: A[l&15][l>>4], B[l>>4][l&15], D[(l>>4)+4r][l&15]).  V streams through
// LDS KB rows at a time, stored column-major with an odd stride (KB + 1); the Q tile is
// XOR-swizzled (column ^ 16 on odd rows): both ds_read_b64 operand reads are conflict-free.
// ------------------------------------------------------------------------------------------
typedef double nkv_f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int rot_swz(int row, int col) { return col ^ ((row & 1) << 4); }

template <int R, int CC, int KB>
__global__ __launch_bounds__(kThreads) void k_rotate_mfma(double* __restrict__ Q, int64_t ld, int k,
                                                          const double* __restrict__ V, int ldv, int n_out,
                                                          int64_t n_tiles) {
    constexpr int WR = R / 16, WC = 4 / WR, MB = CC / 16 / WC;
    static_assert(WR * WC == 4 && MB >= 1, "tile shape");
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int kpad = (k + 3) & ~3;
    double* A = sm;                 // [kpad][R]
    double* Vs = sm + kpad * R;     // [CC][KB + 1]: odd stride, conflict-free column reads
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = wave % WR, wc = wave / WR;
    const int lr = lane & 15, lk = lane >> 4;
    for (int idx = k * R + threadIdx.x; idx < kpad * R; idx += kThreads) A[idx] = 0.0;  // k..kpad rows
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t row0 = tile * R;
        __syncthreads();
        for (int idx = threadIdx.x; idx < k * (R / 2); idx += kThreads) {
            const int c = idx / (R / 2), r = 2 * (idx % (R / 2));
            st2(A + c * R + rot_swz(c, r), ld2(Q + (int64_t)c * ld + row0 + r));
        }
        for (int cc = 0; cc < n_out; cc += CC) {
            nkv_f64x4 acc[MB];
#pragma unroll
            for (int m = 0; m < MB; ++m) acc[m] = nkv_f64x4{0.0, 0.0, 0.0, 0.0};
            const int nact = (min(CC, n_out - cc) + 15) / 16;   // active 16-column blocks in the chunk
            for (int ii = 0; ii < k; ii += KB) {
                __syncthreads();
                for (int e = threadIdx.x; e < KB * CC; e += kThreads) {
                    const int i = e % KB, c = e / KB;   // i fastest: coalesced reads of column-major V
                    const int gi = ii + i, gc = cc + c;
                    Vs[c * (KB + 1) + i] = (gi < k && gc < n_out) ? V[gi + (int64_t)gc * ldv] : 0.0;
                }
                __syncthreads();
                const int kmax = min(KB, kpad - ii);
                for (int kk = 0; kk < kmax; kk += 4) {
                    const int ia = ii + kk + lk, iv = kk + lk;
                    const double b = A[ia * R + rot_swz(ia, wr * 16 + lr)];
#pragma unroll
                    for (int m = 0; m < MB; ++m) {
                        const int blk = wc + WC * m;
                        if (blk < nact) {
                            const double a = Vs[(blk * 16 + lr) * (KB + 1) + iv];
                            acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[m], 0, 0, 0);
                        }
                    }
                }
            }
#pragma unroll
            for (int m = 0; m < MB; ++m) {
                const int blk = wc + WC * m;
                if (blk < nact) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int gc = cc + blk * 16 + lk + 4 * r;
                        if (gc < n_out) Q[(int64_t)gc * ld + row0 + wr * 16 + lr] = acc[m][r];
                    }
                }
            }
        }
    }
}

// streaming rotation: U k-steps of 4 loaded per batch, the next batch's loads issued before this
// batch's MFMAs (NKV_ROT_PIPE): +13 % at k = 128 with 64-128 kept columns (fewer registers, two
// workgroups per CU), within 2-4 % elsewhere (profiles/r02az_tune_rot_pipe*.log)
#ifndef NKV_ROT_U
#define NKV_ROT_U 4
#endif
#ifndef NKV_ROT_PIPE
#define NKV_ROT_PIPE 1
#endif

// ------------------------------------------------------------------------------------------
// Restart rotation, streaming form (n_out <= 16*MB and V[:, 0:n_out] fits LDS): V is staged in
// LDS once per workgroup; afterwards every wave streams its own NB x 16-row slabs of Q straight
// from HBM into the MFMA B operand, with no barrier and no LDS round trip for Q.  All k inputs
// of a slab are consumed before any of its n_out outputs is stored, and no other wave touches
// those rows, so in place is safe.  A workgroup's waves cover one contiguous WAVES*NB*16-row
// tile, so each column is read in WAVES*NB*128-byte runs.  LDS: Vs[c * kp + i], kp = 2 (mod 32)
// doubles: the two 16-lane k-rows of a ds_read_b64 land on disjoint bank pairs.
// ------------------------------------------------------------------------------------------
template <int NB, int MB, int WAVES, int U>
__global__ __launch_bounds__(WAVES * 64) void k_rotate_stream(double* __restrict__ Q, int64_t ld, int k,
                                                              const double* __restrict__ V, int ldv, int n_out,
                                                              int kp, int64_t n_tiles) {
    extern __shared__ __attribute__((aligned(16))) double Vs[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    // Vs[c][i] for c < 16*MB, i < kp (zero beyond n_out / k: the last 4U-step batch needs no guard)
    for (int e = threadIdx.x; e < MB * 16 * kp; e += WAVES * 64) {
        const int c = e / kp, i = e % kp;
        Vs[e] = (i < k && c < n_out) ? V[i + (int64_t)c * ldv] : 0.0;
    }
    __syncthreads();
    const double* vs = Vs + lr * kp + lk;
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t row0 = (tile * WAVES + wave) * (NB * 16);
        const double* q = Q + row0 + lr;
        nkv_f64x4 acc[NB][MB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int m = 0; m < MB; ++m) acc[nb][m] = nkv_f64x4{0.0, 0.0, 0.0, 0.0};
        auto load = [&](double (&b)[U][NB], int i0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + 4 * u + lk;
                const double* qi = q + (int64_t)(i < k ? i : 0) * ld;
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) b[u][nb] = i < k ? qi[nb * 16] : 0.0;
            }
        };
        auto mma = [&](const double (&b)[U][NB], int i0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int m = 0; m < MB; ++m) {
                    const double a = vs[m * 16 * kp + i0 + 4 * u];
#pragma unroll
                    for (int nb = 0; nb < NB; ++nb)
                        acc[nb][m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[u][nb], acc[nb][m], 0, 0, 0);
                }
            }
        };
        if (NKV_ROT_PIPE) {   // the next batch's loads in flight while this batch's MFMAs issue
            double b0[U][NB], b1[U][NB];   // two batches per trip: no register copies
            load(b0, 0);
            for (int i0 = 0;; i0 += 8 * U) {   // b0 holds the batch at i0 < k (wave-uniform branches)
                const bool more1 = i0 + 4 * U < k;
                if (more1) load(b1, i0 + 4 * U);
                mma(b0, i0);
                if (!more1) break;
                const bool more2 = i0 + 8 * U < k;
                if (more2) load(b0, i0 + 8 * U);
                mma(b1, i0 + 4 * U);
                if (!more2) break;
            }
        } else {
            for (int i0 = 0; i0 < k; i0 += 4 * U) {
                double b[U][NB];
                load(b, i0);
                mma(b, i0);
            }
        }
#pragma unroll
        for (int m = 0; m < MB; ++m) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gc = m * 16 + lk + 4 * r;
                if (gc < n_out) {
#pragma unroll
                    for (int nb = 0; nb < NB; ++nb) Q[(int64_t)gc * ld + row0 + nb * 16 + lr] = acc[nb][m][r];
                }
            }
        }
    }
}

#ifndef NKV_ROT_CHUNK_SB
#define NKV_ROT_CHUNK_SB 1
#endif
#ifndef NKV_ROT_CHUNK_W8_MAX
#define NKV_ROT_CHUNK_W8_MAX 8   // chunked rotation: 8 waves up to this many 16-column blocks (+12 % at
                                 // 8 blocks over 4 waves, profiles/r02bf_tune_rot_w8.log), 4 above
#endif

// ------------------------------------------------------------------------------------------
// Restart rotation, V streamed through LDS in k-chunks (n_out <= 16*MB <= 256 when V[:, 0:n_out]
// does not fit LDS whole: k > 128 with many kept columns, where the staged tile kernel above keeps
// one workgroup per CU and exposes every load).  As k_rotate_stream, every wave owns one 16-row
// slab and holds all of its n_out outputs in registers until its k inputs are consumed (in place
// is safe); V moves through two LDS buffers of KC k-rows (next chunk's V and Q loads in flight
// while this chunk's MFMAs issue, one barrier per chunk).  LDS: Vs[buf][c][i], stride KP = 2
// (mod 32) doubles as in k_rotate_stream.
// ------------------------------------------------------------------------------------------
template <int MB, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_rotate_chunked(double* __restrict__ Q, int64_t ld, int k,
                                                               const double* __restrict__ V, int ldv, int n_out,
                                                               int64_t n_tiles) {
    constexpr int KC = MB > 8 ? 16 : 32, KP = 34, U = KC / 4;
    constexpr int VN = MB * 16 * KC, NT = WAVES * 64, PER = (VN + NT - 1) / NT;
    constexpr int BUF = MB * 16 * KP;
    extern __shared__ __attribute__((aligned(16))) double Vs[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    const int nchunks = (k + KC - 1) / KC;
    auto vload = [&](double (&r)[PER], int kc) {
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int e = threadIdx.x + p * NT, c = e / KC, gi = kc + e % KC;
            r[p] = (e < VN && gi < k && c < n_out) ? V[gi + (int64_t)c * ldv] : 0.0;
        }
    };
    auto vstore = [&](const double (&r)[PER], int buf) {
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int e = threadIdx.x + p * NT;
            if (e < VN) Vs[buf * BUF + (e / KC) * KP + e % KC] = r[p];
        }
    };
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t row0 = (tile * WAVES + wave) * 16;
        const double* q = Q + row0 + lr;
        auto bload = [&](double (&b)[U], int kc) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = kc + 4 * u + lk;
                b[u] = i < k ? q[(int64_t)i * ld] : 0.0;
            }
        };
        nkv_f64x4 acc[MB];
#pragma unroll
        for (int m = 0; m < MB; ++m) acc[m] = nkv_f64x4{0.0, 0.0, 0.0, 0.0};
        double vr[PER], b[U];
        vload(vr, 0);
        bload(b, 0);
        vstore(vr, 0);
        __syncthreads();
        for (int ch = 0; ch < nchunks; ++ch) {
            const int cur = ch & 1;
            const bool more = ch + 1 < nchunks;
            double bn[U];
            if (more) {
                vload(vr, (ch + 1) * KC);
                bload(bn, (ch + 1) * KC);
            }
            const double* vs = Vs + cur * BUF + lr * KP + lk;
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int m = 0; m < MB; ++m)
                    acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(vs[m * 16 * KP + 4 * u], b[u], acc[m], 0, 0, 0);
                // 8 waves (256 registers each): keep the next k-step's MB operand reads from being
                // hoisted here — MB x 4 accumulators plus one k-step of A operands fit, all U k-steps
                // at once do not.  4 waves (512 registers): NKV_ROT_CHUNK_SB chooses.
                if (WAVES > 4 || NKV_ROT_CHUNK_SB) __builtin_amdgcn_sched_barrier(0);
            }
            if (more) {
                vstore(vr, cur ^ 1);   // that buffer's readers passed the previous chunk's barrier
#pragma unroll
                for (int u = 0; u < U; ++u) b[u] = bn[u];
            }
            __syncthreads();
        }
#pragma unroll
        for (int m = 0; m < MB; ++m) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gc = m * 16 + lk + 4 * r;
                if (gc < n_out) Q[(int64_t)gc * ld + row0 + lr] = acc[m][r];
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Restart rotation for a few kept columns (n_out = NO <= NKV_ROTF_MAX, the Krylov–Schur case:
// mstart-1 selected Schur vectors out of k): the multi-dot's streaming shape — every thread owns
// P row pairs of a tile, walks the k columns U at a time with 16-byte non-temporal loads (1 KiB
// per wave instruction, each column read in kThreads*P*16-byte runs), and keeps NO accumulators
// per row; V[c, 0:NO] is wave-uniform (scalar loads).  2 N k NO flop against 8 N (k + NO) bytes:
// at NO <= 16 this is HBM-bound on the VALU, where the MFMA tile would waste 16-NO of its 16
// output columns and read Q in 128-byte pieces.  All k inputs of a row are consumed before its NO
// outputs are stored and no other thread touches that row, so in place is safe.
// ------------------------------------------------------------------------------------------
#ifndef NKV_ROTF_MAX
#define NKV_ROTF_MAX 16   // 0: never use the few-column rotation
#endif
#ifndef NKV_ROTF_P
#define NKV_ROTF_P 4
#endif
#ifndef NKV_ROTF_U
#define NKV_ROTF_U 4
#endif
#ifndef NKV_ROTF_G
#define NKV_ROTF_G 768   // workgroups of the few-column rotation
#endif
#ifndef NKV_ROTF_ROUNDS
#define NKV_ROTF_ROUNDS 1   // few-column rotation: one launch per this many grid-stride rounds (0: one launch)
#endif
static_assert(NKV_TILE % (kThreads * NKV_ROTF_P * 2) == 0, "rotate-few tile must divide the padding");
static_assert(NKV_TILE % (kThreads * 2 * 2) == 0, "rotate-few tile (9-16 kept columns) must divide the padding");
template <int NO, int P, int U>
__global__ __launch_bounds__(kThreads) void k_rotate_few(double* __restrict__ Q, int64_t ld, int k,
                                                         const double* __restrict__ V, int ldv, int64_t t_lo,
                                                         int64_t t_hi) {
    constexpr int kTile = kThreads * P * 2;
    for (int64_t t = t_lo + blockIdx.x; t < t_hi; t += gridDim.x) {   // this launch's row band
        const int64_t r0 = t * kTile + 2 * threadIdx.x;
        const double* qb = Q + r0;
        double2 acc[NO][P];
#pragma unroll
        for (int o = 0; o < NO; ++o)
#pragma unroll
            for (int p = 0; p < P; ++p) acc[o][p] = make_double2(0.0, 0.0);
        int c = 0;
        for (; c + U <= k; c += U) {
            double2 q[U][P];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int p = 0; p < P; ++p) q[u][p] = ldq(qb + (int64_t)(c + u) * ld + p * 2 * kThreads);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int o = 0; o < NO; ++o) {
                    const double v = V[c + u + (int64_t)o * ldv];
#pragma unroll
                    for (int p = 0; p < P; ++p) {
                        acc[o][p].x = fma(q[u][p].x, v, acc[o][p].x);
                        acc[o][p].y = fma(q[u][p].y, v, acc[o][p].y);
                    }
                }
        }
        for (; c < k; ++c) {
            double2 q[P];
#pragma unroll
            for (int p = 0; p < P; ++p) q[p] = ldq(qb + (int64_t)c * ld + p * 2 * kThreads);
#pragma unroll
            for (int o = 0; o < NO; ++o) {
                const double v = V[c + (int64_t)o * ldv];
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    acc[o][p].x = fma(q[p].x, v, acc[o][p].x);
                    acc[o][p].y = fma(q[p].y, v, acc[o][p].y);
                }
            }
        }
#pragma unroll
        for (int o = 0; o < NO; ++o)
#pragma unroll
            for (int p = 0; p < P; ++p) st2s(Q + (int64_t)o * ld + r0 + p * 2 * kThreads, acc[o][p]);
    }
}

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

#ifndef NKV_STREAM_G
#define NKV_STREAM_G 4096  // workgroup cap of the streaming kernels (op_diag, finish, BLAS-1)
#endif
int grid_for(int64_t work_items, int cap = NKV_STREAM_G) {
    int64_t g = (work_items + kThreads - 1) / kThreads;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

struct Ctrl {
    int nan_flag;
};

inline int* nan_flag_of(void* ws) { return &reinterpret_cast<Ctrl*>(ws)->nan_flag; }
inline double* partials_of(void* ws) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + kCtrlBytes);
}

// Rows per thread: NKV_PAIRS*2 when the vector has enough large tiles to fill the chip, else fewer.
inline bool use_large_tiles(const nkv_layout* L) {
    return rows_of(L) / (kThreads * NKV_PAIRS * 2) >= NKV_SMALL_TILES;
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

// Shared launcher for block dots (nkv_dot is the j = 1 case).
int launch_block_dot(const nkv_layout* L, const double* w, const double* Q, int64_t ld, int j,
                     const double* f, double* out, void* ws, unsigned flags, hipStream_t st) {
    return use_large_tiles(L) ? launch_block_dot_p<NKV_PAIRS>(L, w, Q, ld, j, f, out, ws, flags, st)
                              : launch_block_dot_p<NKV_PAIRS_SMALL>(L, w, Q, ld, j, f, out, ws, flags, st);
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

}  // namespace

// ==========================================================================================
// C ABI
// ==========================================================================================
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

extern "C" {

int nkv_abi_version(void) { return NKV_ABI_VERSION; }

const char* nkv_last_error(void) { return g_err; }

int nkv_device_info(int* device, int* cu_count, int64_t* hbm_bytes, char* name, int name_len) {
    int dev = 0;
    NKV_HIP(hipGetDevice(&dev));
    hipDeviceProp_t p;
    NKV_HIP(hipGetDeviceProperties(&p, dev));
    if (device) *device = dev;
    if (cu_count) *cu_count = p.multiProcessorCount;
    if (hbm_bytes) *hbm_bytes = (int64_t)p.totalGlobalMem;
    if (name && name_len > 0) {
        snprintf(name, name_len, "%s", p.gcnArchName);
    }
    return NKV_OK;
}

size_t nkv_workspace_bytes(const nkv_layout* L, int max_cols) {
    (void)L;
    if (max_cols < 1) max_cols = 1;
    return kCtrlBytes + (size_t)kMaxBlocks * (size_t)(2 * max_cols + 2) * sizeof(double);  // 2 RHS (DCGS2)
}

int nkv_check_status(void* ws, void* stream) {
    CHECK(check_ptr(ws, "ws"));
    int flag = 0;
    NKV_HIP(hipMemcpyAsync(&flag, nan_flag_of(ws), sizeof(int), hipMemcpyDeviceToHost, S(stream)));
    NKV_HIP(hipStreamSynchronize(S(stream)));
    if (flag) {
        NKV_HIP(hipMemsetAsync(nan_flag_of(ws), 0, sizeof(int), S(stream)));
        return fail(NKV_ENAN, "NaN detected in dot product");  // nek_vectors.f90:108-111
    }
    return NKV_OK;
}

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
        hipLaunchKernelGGL(k_reduce_cols, dim3(1), dim3(kThreads), 0, st, part, g, nrm2_dev,
                           tdot ? f + T : nullptr, (int64_t)0, tdot ? f + T : nullptr, nullptr, 1 << 30, nan_flag_of(ws));
        NKV_LAUNCHED();
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
    hipLaunchKernelGGL(k_reduce_cols, dim3(j), dim3(kThreads), 0, st, part, B, hout_dev, tdot ? Q + T : nullptr,
                       L->ld, tdot ? f + T : nullptr, nullptr, 1 << 30, nan_flag_of(ws));
    NKV_LAUNCHED();
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
    const int P = large ? NKV_DC_PAIRS : NKV_PAIRS_SMALL;
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
            hipLaunchKernelGGL(k_block_dot2<NKV_DC_PAIRS>, dim3(bx, gy), dim3(kThreads), 8 * j * sizeof(double), st,
                               Q, L->ld, j, x, y, w, L->sv, tpf, nf, xl, part, B);
        else
            hipLaunchKernelGGL(k_block_dot2<NKV_PAIRS_SMALL>, dim3(bx, gy), dim3(kThreads), 8 * j * sizeof(double),
                               st, Q, L->ld, j, x, y, w, L->sv, tpf, nf, xl, part, B);
        NKV_LAUNCHED();
    }
    const int64_t T = rows_of(L);
    const bool tdot = (flags & NKV_TIME) && L->rank0;
    hipLaunchKernelGGL(k_reduce_cols, dim3(2 * j), dim3(kThreads), 0, st, part, tpf > 0 ? B : 0, h_dev,
                       tdot ? Q + T : nullptr, L->ld, tdot ? x + T : nullptr, tdot ? y + T : nullptr, j,
                       nan_flag_of(ws));
    NKV_LAUNCHED();
    return NKV_OK;
}

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
    return nkv_dcgs2_coef_lazy(m, hq_dev, hw_dev, nrm_prev_dev, H_dev, ldh, coef_dev, nullptr, 0, ws, stream);
}

int nkv_dcgs2_coef_lazy(int m, const double* hq_dev, const double* hw_dev, const double* nrm_prev_dev,
                        double* H_dev, int64_t ldh, double* coef_dev, double* T_dev, int64_t ldt, void* ws,
                        void* stream) {
    if (m < 0 || m > NKV_MAX_COLS) return fail(NKV_EINVAL, "m=%d outside 0..%d", m, NKV_MAX_COLS);
    if (!hq_dev || !H_dev || !coef_dev) return fail(NKV_EINVAL, "hq/H/coef is NULL");
    if (ldh < m + 1) return fail(NKV_EINVAL, "ldh=%lld < m+1=%d", (long long)ldh, m + 1);
    if (T_dev && ldt < m + 1) return fail(NKV_EINVAL, "ldt=%lld < m+1=%d", (long long)ldt, m + 1);
    CHECK(check_ptr(ws, "ws"));
    hipLaunchKernelGGL(k_dcgs2_coef, dim3(1), dim3(kThreads), dcgs2_coef_lds(m), S(stream), m, hq_dev, hw_dev,
                       nrm_prev_dev, H_dev,
                       ldh, coef_dev, T_dev, ldt, nan_flag_of(ws));
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

// Tiles per launch of a banded update (NKV_DC_ROUNDS grid-stride rounds of a g-block grid); all
// tiles in one launch when banding is off or the vector is shorter than two bands.
inline int band_tiles(int tiles_total, int g) {
    if (NKV_DC_ROUNDS <= 0) return tiles_total > 0 ? tiles_total : 1;
    const int64_t b = (int64_t)NKV_DC_ROUNDS * g;
    return (b >= tiles_total || tiles_total < 2 * b) ? (tiles_total > 0 ? tiles_total : 1) : (int)b;
}

int nkv_dcgs2_update_lazy(const nkv_layout* L, const double* S_cols, int m, const double* coef_dev,
                          const double* win, double* fout, void* ws, unsigned flags, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(S_cols, "S"));
    CHECK(check_ptr(win, "win"));
    CHECK(check_ptr(fout, "fout"));
    if (m < 0 || m > NKV_MAX_COLS) return fail(NKV_EINVAL, "m=%d outside 0..%d", m, NKV_MAX_COLS);
    if (!coef_dev) return fail(NKV_EINVAL, "coef is NULL");
    (void)ws;
    hipStream_t st = S(stream);
    const bool large = use_large_tiles(L);
    const int P = large ? NKV_DC_PAIRS : NKV_PAIRS_SMALL;
    const int tiles_total = (int)(rows_of(L) / (kThreads * P * 2));
    const int gmax = NKV_DC_G < kMaxBlocks ? NKV_DC_G : kMaxBlocks;
    int g = tiles_total < gmax ? tiles_total : gmax;
    if (g < 1) g = 1;
    const int dt = (flags & NKV_TIME) ? 1 : 0;
    auto kern = large ? k_dcgs2_lazy_update<NKV_DC_PAIRS> : k_dcgs2_lazy_update<NKV_PAIRS_SMALL>;
    const int band = band_tiles(tiles_total, g);
    // one launch per row band (NKV_DC_ROUNDS); at least one, which also updates the time slot
    for (int lo = 0; lo == 0 || lo < tiles_total; lo += band) {
        const int hi = lo + band < tiles_total ? lo + band : tiles_total;
        const int gb = g < hi - lo ? g : (hi - lo > 0 ? hi - lo : 1);
        hipLaunchKernelGGL(kern, dim3(gb), dim3(kThreads), 0, st, S_cols, L->ld, m, coef_dev, win, fout, lo, hi,
                           rows_of(L), lo == 0 ? dt : 0);
        NKV_LAUNCHED();
    }
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
    hipLaunchKernelGGL(k_reduce_cols, dim3(1), dim3(kThreads), 0, st, part, g, nrm2_dev, tdot ? fout + T : nullptr,
                       (int64_t)0, tdot ? fout + T : nullptr, nullptr, 1 << 30, nan_flag_of(ws));
    NKV_LAUNCHED();
    return NKV_OK;
}

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

int nkv_combine(const nkv_layout* L, const double* Q, int k, const double* y_dev, double* out, unsigned flags,
                void* stream) {
    return nkv_block_update(L, nullptr, Q, k, y_dev, out, nullptr, nullptr,
                            (flags & ~(unsigned)NKV_NORM2) | NKV_OVERWRITE, stream);
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

__global__ void k_accumulate(double* __restrict__ dst, const double* __restrict__ src) {
    if (threadIdx.x == 0) dst[0] += src[0];
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

#ifndef NKV_ROT_VALU
#define NKV_ROT_VALU 0   // 1: the VALU (4x4 register block) rotation instead of the f64 MFMA one
#endif
#ifndef NKV_ROT_SMALLR
#define NKV_ROT_SMALLR 64   // MFMA rotation tile rows for k <= 256 (64 or 32)
#endif

extern "C++" template <int R, int CC, int KB>
static int launch_rotate_mfma(const nkv_layout* L, double* Q, int k, const double* V, int ldv, int n_out,
                              void* stream) {
    const int kpad = (k + 3) & ~3;
    const size_t lds = ((size_t)kpad * R + (size_t)(KB + 1) * CC) * sizeof(double);
    static bool attr_set = false;
    if (!attr_set) {
        NKV_HIP(hipFuncSetAttribute((const void*)k_rotate_mfma<R, CC, KB>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set = true;
    }
    if (lds > 160 * 1024) return fail(NKV_EINVAL, "rotate: k=%d needs %zu B of LDS", k, lds);
    const int64_t n_tiles = rows_of(L) / R;
    const int64_t g = n_tiles < 4096 ? n_tiles : 4096;
    if (g < 1) return NKV_OK;
    hipLaunchKernelGGL((k_rotate_mfma<R, CC, KB>), dim3((unsigned)g), dim3(kThreads), lds, S(stream), Q, L->ld, k,
                       V, ldv, n_out, n_tiles);
    NKV_LAUNCHED();
    return NKV_OK;
}

static int rotate_valu(const nkv_layout* L, double* Q, int k, const double* V_dev, int ldv, void* stream) {
    static bool attr_set = false;
    if (!attr_set) {
        NKV_HIP(hipFuncSetAttribute((const void*)k_rotate<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)((256 * 64 + 16 * 64) * sizeof(double))));
        NKV_HIP(hipFuncSetAttribute((const void*)k_rotate<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)((kRotMaxK * 32 + 16 * 128) * sizeof(double))));
        attr_set = true;
    }
    const bool big = k > 256;
    const int R = big ? 32 : 64;
    const size_t lds = ((size_t)k * R + 16 * (big ? 128 : 64)) * sizeof(double);
    const int64_t n_tiles = rows_of(L) / R;
    int64_t g = n_tiles < 4096 ? n_tiles : 4096;
    if (g < 1) return NKV_OK;
    if (big)
        hipLaunchKernelGGL(k_rotate<32>, dim3((unsigned)g), dim3(kThreads), lds, S(stream), Q, L->ld, k, V_dev, ldv, n_tiles);
    else
        hipLaunchKernelGGL(k_rotate<64>, dim3((unsigned)g), dim3(kThreads), lds, S(stream), Q, L->ld, k, V_dev, ldv, n_tiles);
    NKV_LAUNCHED();
    return NKV_OK;
}

#ifndef NKV_ROT_STREAM
#define NKV_ROT_STREAM 1   // 0: never use the streaming rotation
#endif
#ifndef NKV_ROT_WAVES
#define NKV_ROT_WAVES 16
#endif
#ifndef NKV_ROT_NB
#define NKV_ROT_NB 1
#endif


extern "C++" template <int MB>
static int launch_rotate_stream(const nkv_layout* L, double* Q, int k, const double* V, int ldv, int n_out,
                                int kp, size_t lds, void* stream) {
    // register budget: ~21*MB + 55 VGPRs (U = 8); 16 waves/WG allow 128 per lane, so wide column blocks
    // run with half the waves (256 VGPRs)
    constexpr int NB = NKV_ROT_NB, W = MB <= 3 ? NKV_ROT_WAVES : NKV_ROT_WAVES / 2, U = NKV_ROT_U;
    auto kern = k_rotate_stream<NB, MB, W, U>;
    static bool attr_set = false;
    if (!attr_set) {
        NKV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set = true;
    }
    const int64_t rows_tile = (int64_t)W * NB * 16;
    const int64_t n_tiles = rows_of(L) / rows_tile;
    if (n_tiles < 1) return NKV_OK;
    int per_cu = (int)((160 * 1024) / lds);
    per_cu = per_cu < 1 ? 1 : (per_cu > 32 / W ? 32 / W : per_cu);   // LDS and 32 waves per CU
    const int64_t g0 = (int64_t)device_cus() * per_cu;
    const int64_t g = n_tiles < g0 ? n_tiles : g0;
    hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(W * 64), lds, S(stream), Q, L->ld, k, V, ldv, n_out, kp,
                       n_tiles);
    NKV_LAUNCHED();
    return NKV_OK;
}

#ifndef NKV_ROT_CHUNKED
#define NKV_ROT_CHUNKED 1   // 0: the staged tile kernel where V does not fit LDS whole
#endif
#ifndef NKV_ROT_CHUNK_FROM
#define NKV_ROT_CHUNK_FROM 17   // 16-column blocks from which the chunked kernel replaces the streaming one
#endif

extern "C++" template <int MB>
static int launch_rotate_chunked(const nkv_layout* L, double* Q, int k, const double* V, int ldv, int n_out,
                                 void* stream) {
    // past NKV_ROT_CHUNK_W8_MAX 16-column blocks the 4 x MB accumulators need one wave per SIMD
    // (512 registers)
    constexpr int W = MB > NKV_ROT_CHUNK_W8_MAX ? 4 : 8;
    auto kern = k_rotate_chunked<MB, W>;
    const size_t lds = 2 * (size_t)MB * 16 * 34 * sizeof(double);
    static bool attr_set = false;
    if (!attr_set) {
        NKV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set = true;
    }
    const int64_t n_tiles = rows_of(L) / (W * 16);
    if (n_tiles < 1) return NKV_OK;
    int per_cu = (int)((160 * 1024) / lds);
    per_cu = per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu);
    const int64_t g0 = (int64_t)device_cus() * per_cu;
    const int64_t g = n_tiles < g0 ? n_tiles : g0;
    hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(W * 64), lds, S(stream), Q, L->ld, k, V, ldv, n_out, n_tiles);
    NKV_LAUNCHED();
    return NKV_OK;
}

extern "C++" template <int NO>
static int launch_rotate_few(const nkv_layout* L, double* Q, int k, const double* V, int ldv, void* stream) {
    // NO accumulators per row pair: past 8 kept columns fewer row pairs per thread keep the register
    // budget (9-12: 2 pairs x 2 columns in flight, 130 VGPRs at NO = 12; 13-16: 2 x 4) — +32 % at
    // NO = 12 and +10 % at NO = 16 over the MFMA streaming rotation (profiles/r02v_tune_rotf16_E44176.log)
    constexpr int P = NO <= 8 ? NKV_ROTF_P : 2, U = NO <= 8 ? NKV_ROTF_U : (NO <= 12 ? 2 : 4);
    const int64_t n_tiles = rows_of(L) / (kThreads * P * 2);
    if (n_tiles < 1) return NKV_OK;
    // one launch per row band of NKV_ROTF_ROUNDS grid-stride rounds of an NKV_ROTF_G grid, as the DCGS2
    // updates: +17-21 % at N=1e8 over one 1024-workgroup launch (profiles/r02s_tune_rotf*.log)
    const int64_t g = n_tiles < NKV_ROTF_G ? n_tiles : NKV_ROTF_G;
    const int64_t band = NKV_ROTF_ROUNDS > 0 ? (int64_t)NKV_ROTF_ROUNDS * g : n_tiles;
    for (int64_t lo = 0; lo < n_tiles; lo += band) {
        const int64_t hi = lo + band < n_tiles ? lo + band : n_tiles;
        hipLaunchKernelGGL((k_rotate_few<NO, P, U>), dim3((unsigned)(g < hi - lo ? g : hi - lo)), dim3(kThreads), 0,
                           S(stream), Q, L->ld, k, V, ldv, lo, hi);
        NKV_LAUNCHED();
    }
    return NKV_OK;
}

int nkv_rotate_cols(const nkv_layout* L, double* Q, int k, const double* V_dev, int ldv, int n_out, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(Q, "Q"));
    if (!V_dev) return fail(NKV_EINVAL, "V_dev is NULL");
    // the few-column streaming kernel holds no k-sized state: any k up to NKV_MAX_COLS
    const int kmax = (n_out >= 1 && n_out <= NKV_ROTF_MAX) ? NKV_MAX_COLS : kRotMaxK;
    if (k < 1 || k > kmax) return fail(NKV_EINVAL, "rotate: k=%d outside [1, %d] (n_out=%d)", k, kmax, n_out);
    if (ldv < k) return fail(NKV_EINVAL, "rotate: ldv=%d < k=%d", ldv, k);
    if (n_out < 1 || n_out > k) return fail(NKV_EINVAL, "rotate: n_out=%d outside [1, k=%d]", n_out, k);
    if (NKV_ROT_VALU && n_out == k) return rotate_valu(L, Q, k, V_dev, ldv, stream);
    if (n_out <= NKV_ROTF_MAX) {
        switch (n_out) {
            case 1: return launch_rotate_few<1>(L, Q, k, V_dev, ldv, stream);
            case 2: return launch_rotate_few<2>(L, Q, k, V_dev, ldv, stream);
            case 3: return launch_rotate_few<3>(L, Q, k, V_dev, ldv, stream);
            case 4: return launch_rotate_few<4>(L, Q, k, V_dev, ldv, stream);
            case 5: return launch_rotate_few<5>(L, Q, k, V_dev, ldv, stream);
            case 6: return launch_rotate_few<6>(L, Q, k, V_dev, ldv, stream);
            case 7: return launch_rotate_few<7>(L, Q, k, V_dev, ldv, stream);
            case 8: return launch_rotate_few<8>(L, Q, k, V_dev, ldv, stream);
            case 9: return launch_rotate_few<9>(L, Q, k, V_dev, ldv, stream);
            case 10: return launch_rotate_few<10>(L, Q, k, V_dev, ldv, stream);
            case 11: return launch_rotate_few<11>(L, Q, k, V_dev, ldv, stream);
            case 12: return launch_rotate_few<12>(L, Q, k, V_dev, ldv, stream);
            case 13: return launch_rotate_few<13>(L, Q, k, V_dev, ldv, stream);
            case 14: return launch_rotate_few<14>(L, Q, k, V_dev, ldv, stream);
            case 15: return launch_rotate_few<15>(L, Q, k, V_dev, ldv, stream);
            case 16: return launch_rotate_few<16>(L, Q, k, V_dev, ldv, stream);
            default: break;
        }
    }
    if (NKV_ROT_STREAM && (n_out + 15) / 16 < NKV_ROT_CHUNK_FROM &&
        rows_of(L) % ((int64_t)NKV_ROT_WAVES * NKV_ROT_NB * 16) == 0) {
        const int kp = ((k + 31) & ~31) + 2;
        const int nact = (n_out + 15) / 16;
        const size_t lds = (size_t)nact * 16 * kp * sizeof(double);
        if (lds <= 160 * 1024) {
            switch (nact) {
                case 1: return launch_rotate_stream<1>(L, Q, k, V_dev, ldv, n_out, kp, lds, stream);
                case 2: return launch_rotate_stream<2>(L, Q, k, V_dev, ldv, n_out, kp, lds, stream);
                case 3: return launch_rotate_stream<3>(L, Q, k, V_dev, ldv, n_out, kp, lds, stream);
                case 4: return launch_rotate_stream<4>(L, Q, k, V_dev, ldv, n_out, kp, lds, stream);
                case 5: return launch_rotate_stream<5>(L, Q, k, V_dev, ldv, n_out, kp, lds, stream);
                case 6: return launch_rotate_stream<6>(L, Q, k, V_dev, ldv, n_out, kp, lds, stream);
                case 7: return launch_rotate_stream<7>(L, Q, k, V_dev, ldv, n_out, kp, lds, stream);
                case 8: return launch_rotate_stream<8>(L, Q, k, V_dev, ldv, n_out, kp, lds, stream);
                default: break;
            }
        }
    }
    if (NKV_ROT_CHUNKED && rows_of(L) % (8 * 16) == 0) {   // V through LDS in k-chunks, n_out <= 256
        const int nact = (n_out + 15) / 16;
        if (nact <= 2) return launch_rotate_chunked<2>(L, Q, k, V_dev, ldv, n_out, stream);
        if (nact <= 4) return launch_rotate_chunked<4>(L, Q, k, V_dev, ldv, n_out, stream);
        if (nact <= 8) return launch_rotate_chunked<8>(L, Q, k, V_dev, ldv, n_out, stream);
        if (nact <= 12) return launch_rotate_chunked<12>(L, Q, k, V_dev, ldv, n_out, stream);
        if (nact <= 16) return launch_rotate_chunked<16>(L, Q, k, V_dev, ldv, n_out, stream);
    }
    if (k <= 256) {
        if (NKV_ROT_SMALLR == 32) return launch_rotate_mfma<32, 128, 16>(L, Q, k, V_dev, ldv, n_out, stream);
        return launch_rotate_mfma<64, 128, 16>(L, Q, k, V_dev, ldv, n_out, stream);
    }
    return launch_rotate_mfma<32, 128, 8>(L, Q, k, V_dev, ldv, n_out, stream);
}

int nkv_rotate(const nkv_layout* L, double* Q, int k, const double* V_dev, int ldv, void* stream) {
    return nkv_rotate_cols(L, Q, k, V_dev, ldv, k, stream);
}

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
