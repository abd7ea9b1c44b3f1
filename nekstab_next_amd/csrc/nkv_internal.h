// nkv_internal.h — shared by the translation units of libnekkrylov.so (not installed; the public
// C ABI is include/nekkrylov.h).  Tuning knobs, error plumbing, layout helpers and the CDNA4 device
// helpers every kernel family uses (wave64 reductions, 16-byte streaming loads/stores).
//
// Every kernel of the library is HBM-bound fp64 streaming (BLAS-1/2) except the restart rotation
// (f64 MFMA): 16-B (double2) coalesced loads, 256-thread workgroups (4 wave64s), wave reductions by
// cross-lane shuffles and DPP, LDS for the per-workgroup partials, and a deterministic two-stage
// reduction (fixed block->tile map, fixed-order second stage; no floating-point atomics) so results
// do not depend on timing.  Layout, flags and the reference functions each entry point replaces:
// include/nekkrylov.h.  Rooflines and bytes per launch: DESIGN.md §4.
//
// Translation units (one kernel family each, linked into one .so by __graft_entry__.build()):
//   core.hip          error state, device info, workspace, NaN status
//   vector.hip        BLAS-1, weighted dots / multi-dot, second-stage reduction, normalise, MGS column step
//   gram_schmidt.hip  block updates, fused CGS2 pass, DCGS2 multi-dot / coefficients / dual update,
//                     GKL coefficients, MGS in inverse compact WY form
//   rotate.hip        Krylov–Schur restart rotation Q <- Q V (VALU few-column, f64 MFMA stream/chunked)
//   drivers.hip       one-call factorisations (DCGS2, CGS2/MGS2, MGS2-ICWY), GMRES cycle, Givens column
//   operators.hip     synthetic operators and the hashed test vectors
//   sensitivity.hip   seed noise (mth_rand), symmetric seed, wave-maker, gradm1, base-flow sensitivity
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "nekkrylov.h"

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
#ifndef NKV_D2_PAIRS
#define NKV_D2_PAIRS NKV_DC_PAIRS  // double2 per thread per tile in the two-vector multi-dot (large problems)
#endif
// The round-1 timing experiments (store skipping, grid-wide soft barriers, tile-interleaved and
// field-major sweeps, XCD tile maps, buffer-store cache policies, register-budget schedules;
// CHANGELOG.md, "What did not help") are not part of this file.  The knobs above change speed only.
#if defined(NKV_DC_EXPERIMENT) || defined(NKV_DC_SYNC) || defined(NKV_QTILE_EXP) || defined(NKV_D2_FIELDMAJOR) || \
    defined(NKV_DC_SCHED) || defined(NKV_D2_SCHED) || defined(NKV_ST_AUX) || defined(NKV_XCD_MAP) ||           \
    defined(NKV_DC_FIELDLOOP) || defined(NKV_FUSE_PF) || defined(NKV_LD_ALIGN)
#error "round-1 experiment switches were removed from the product kernel"
#endif

// ---- cross-TU host helpers (hidden: not part of the exported ABI) -------------------------------
#pragma GCC visibility push(hidden)
namespace nkvi {
// Record an error message for nkv_last_error() and return `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
// Compute units of the current device (cached per device id; 256 on MI355X).
int device_cus();
int check_layout(const nkv_layout* L);
int check_ptr(const void* p, const char* what);
// Weighted multi-dot h = Q^T W f over j columns (+ the second stage), the j = 1 case is nkv_dot.
int launch_block_dot(const nkv_layout* L, const double* w, const double* Q, int64_t ld, int j, const double* f,
                     double* out, void* ws, unsigned flags, hipStream_t st);
// Second stage of every reduction: out[c] = sum_b partials[c][b] in a fixed order, c < ncols
// (+ the replicated time term ta[c] tb / ta[c - jc] tb2; NaN -> flag).
int launch_reduce_cols(int ncols, const double* partials, int B, double* out, const double* ta, int64_t lda,
                       const double* tb, const double* tb2, int jc, int* nan_flag, hipStream_t st);
}  // namespace nkvi
#pragma GCC visibility pop
using namespace nkvi;

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

#define CHECK(x)                   \
    do {                           \
        int rc_ = (x);             \
        if (rc_ != NKV_OK) return rc_; \
    } while (0)

namespace {

constexpr int kThreads = 256;                       // 4 waves of 64
constexpr int kStreamUnr = NKV_STREAM_UNR;
static_assert(NKV_TILE % (2 * kThreads * NKV_STREAM_UNR) == 0, "stream chunk must divide the padding");
static_assert(NKV_TILE % (kThreads * NKV_PAIRS * 2) == 0, "kernel tile must divide the padding");
static_assert(NKV_TILE % (kThreads * NKV_PAIRS_SMALL * 2) == 0, "kernel tile must divide the padding");
constexpr int kMaxBlocks = NKV_MAXB;                 // reduction partial slots per column
constexpr int kColUnroll = NKV_COLU;                 // columns in flight per thread (block dot)
constexpr size_t kCtrlBytes = 256;                   // control words at the head of the workspace

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Rows that every BLAS-1 op streams (weighted fields + pressure, padded); the time slot sits at
// this offset.
inline int64_t rows_of(const nkv_layout* L) { return (int64_t)L->n_wf * L->sv + L->sp; }

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

#ifndef NKV_STREAM_G
#define NKV_STREAM_G 4096  // workgroup cap of the streaming kernels (op_diag, finish, BLAS-1)
#endif
inline int grid_for(int64_t work_items, int cap = NKV_STREAM_G) {
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

}  // namespace
