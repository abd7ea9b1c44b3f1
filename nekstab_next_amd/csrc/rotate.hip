// rotate.hip — the Krylov–Schur restart rotation Q[:, 0:n_out] <- Q[:, 0:k] V (schur_condensation,
// eigensolvers.f90:421-442), in place: a VALU streaming kernel for <= 16 kept columns, the f64 MFMA
// streaming kernel when V fits LDS, the k-chunked MFMA kernel otherwise (n_out <= NKV_ROT_MAX_OUT).
#include "nkv_internal.h"

namespace {

typedef double nkv_f64x4 __attribute__((ext_vector_type(4)));

// streaming rotation: U k-steps of 4 loaded per batch, the next batch's loads issued before this
// batch's MFMAs (NKV_ROT_PIPE): +13 % at k = 128 with 64-128 kept columns (fewer registers, two
// workgroups per CU), within 2-4 % elsewhere (profiles/r02az_tune_rot_pipe*.log)
#ifndef NKV_ROT_U
#define NKV_ROT_U 4
#endif
#ifndef NKV_ROT_PIPE
#define NKV_ROT_PIPE 1
#endif
#ifndef NKV_ROT_PIPE3_FROM
#define NKV_ROT_PIPE3_FROM 5   // 16-column blocks from which two batches are kept ahead
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
        auto load_all = [&](double (&b)[U][NB], int i0) {   // a batch whose k-rows are all < k
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double* qi = q + (int64_t)(i0 + 4 * u + lk) * ld;
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) b[u][nb] = qi[nb * 16];
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
        if (NKV_ROT_PIPE && MB >= NKV_ROT_PIPE3_FROM) {   // two batches ahead (wide column blocks: one
            // wave per SIMD holds all of its MB accumulators, so its own loads must cover the latency)
            double b0[U][NB], b1[U][NB], b2[U][NB];   // three batches per trip: no register copies
            load(b0, 0);
            if (4 * U < k) load(b1, 4 * U);
            int i0 = 0;
            // steady trips: every k-row of the batches loaded here is < k, so the loads carry no
            // per-lane guard (a guarded load is an exec-masked branch, after which the compiler
            // waits with vmcnt(0), for every load in flight, instead of for the batch it needs)
            for (; i0 + 20 * U <= k; i0 += 12 * U) {   // b0, b1: batches i0, i0+4U; i0+8U..i0+16U whole
                load_all(b2, i0 + 8 * U);
                mma(b0, i0);
                load_all(b0, i0 + 12 * U);
                mma(b1, i0 + 4 * U);
                load_all(b1, i0 + 16 * U);
                mma(b2, i0 + 8 * U);
            }
            // b0 holds the batch at i0 < k, b1 the one at i0+4U when it exists: the rest, guarded
            for (;; i0 += 8 * U) {   // wave-uniform branches
                mma(b0, i0);
                if (i0 + 4 * U >= k) break;
                const bool more2 = i0 + 8 * U < k;
                if (more2) load(b0, i0 + 8 * U);
                mma(b1, i0 + 4 * U);
                if (!more2) break;
                if (i0 + 12 * U < k) load(b1, i0 + 12 * U);
            }
        } else if (NKV_ROT_PIPE) {   // the next batch's loads in flight while this batch's MFMAs issue
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

// ------------------------------------------------------------------------------------------
// Restart rotation, wide-load streaming form (17 .. 16*NKV_ROTW_MAX_MB kept columns, V in LDS whole):
// as k_rotate_stream, but every lane loads 16 B (rows 2r, 2r+1 of one column), so a wave
// instruction reads 4 columns x 256 contiguous bytes and feeds TWO MFMAs per V operand (the even
// and the odd rows of a 32-row slab: two 16x16 output tiles).  The k-rows past k are clamped to
// column k-1 (V is zero there in LDS), so no load carries a per-lane guard and the compiler can
// wait for exactly the batch an MFMA group consumes (a guarded load is an exec-masked branch, after
// which it waits for every load in flight).  Three batches rotate through registers, two ahead of
// the MFMAs; the next tile's first two batches are issued before this tile's stores.  V sits in
// LDS k-major, Vs[i * cp + c] with cp = 16 (mod 32) doubles: the 16 lanes of one k-row read 128
// contiguous bytes and the next k-row lands on the other half of the banks (no conflicts for
// ds_read_b64, nor for the ds_read2_b64 the compiler forms from two column blocks).
// In place is safe as in k_rotate_stream: a wave consumes all k inputs of its 32 rows before it
// stores any of their n_out outputs, and no other wave touches those rows.
// ------------------------------------------------------------------------------------------
template <int MB, int WAVES, int U>
__global__ __launch_bounds__(WAVES * 64) void k_rotate_wide(double* __restrict__ Q, int64_t ld, int k,
                                                            const double* __restrict__ V, int ldv, int n_out,
                                                            int cp, int64_t t_lo, int64_t t_hi) {
    extern __shared__ __attribute__((aligned(16))) double Vs[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    const int nb = (k + 4 * U - 1) / (4 * U);   // batches of U k-steps of 4
    const int kpad = nb * 4 * U;
    // Vs[i][c] for i < kpad, c < cp (zero beyond k / n_out); V is read column by column (coalesced)
    for (int e = threadIdx.x; e < kpad * 16 * MB; e += WAVES * 64) {
        const int c = e / kpad, i = e % kpad;
        Vs[i * cp + c] = (i < k && c < n_out) ? V[i + (int64_t)c * ldv] : 0.0;
    }
    __syncthreads();
    const double* vs = Vs + lk * cp + lr;
    const int kl = k - 1, nf = k / (4 * U);   // nf: batches whose k-rows are all < k
    // a lane's byte offset from its wave's (uniform) row base: SGPR base + 32-bit VGPR offset per
    // load, with no per-lane 64-bit address arithmetic (lk * ld * 8 < 4 GB: ld < 2^27 doubles)
    const uint32_t lane_off = (uint32_t)(((int64_t)lk * ld + 2 * lr) * (int64_t)sizeof(double));
    typedef double2 Batch[U];
    int64_t tile = t_lo + blockIdx.x;   // this launch's row band: tiles [t_lo, t_hi)
    if (tile >= t_hi) return;
    auto wbase = [&](int64_t t) { return Q + (t * WAVES + wave) * 32; };
    const double* qw = wbase(tile);
    auto load_full = [&](Batch& b, const double* qq, int t) {   // batch t < nf
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ldq(at_b(qq + (int64_t)(t * 4 * U + 4 * u) * ld, lane_off));
    };
    auto load = [&](Batch& b, const double* qq, int t) {   // any batch t < nb: the k-rows past k are clamped
        if (t < nf) {
            load_full(b, qq, t);
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = t * 4 * U + 4 * u + lk;
                b[u] = ldq(qq + (int64_t)(i < kl ? i : kl) * ld + 2 * lr);
            }
        }
    };
    nkv_f64x4 acc[2][MB];
    auto mma = [&](const Batch& b, int t) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int m = 0; m < MB; ++m) {
                const double a = vs[(t * 4 * U + 4 * u) * cp + m * 16];
                acc[0][m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[u].x, acc[0][m], 0, 0, 0);
                acc[1][m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[u].y, acc[1][m], 0, 0, 0);
            }
        }
    };
    // the issue order is the pipeline: keep the scheduler from moving loads across MFMA groups
#define NKV_ROTW_FENCE __builtin_amdgcn_sched_barrier(0)
    // prologue and next-tile loads are unconditional (batch 1 of a one-batch k is clamped, the tile
    // after the last one re-reads the last): every path into the loop has the same loads in flight,
    // so the compiler's wait counts stay exact
    Batch b0, b1, b2;
    load(b0, qw, 0);
    load(b1, qw, 1);
    for (;;) {
#pragma unroll
        for (int m = 0; m < MB; ++m) {
            acc[0][m] = nkv_f64x4{0.0, 0.0, 0.0, 0.0};
            acc[1][m] = nkv_f64x4{0.0, 0.0, 0.0, 0.0};
        }
        int t = 0;
        // steady trips: the three batches loaded here (t+2, t+3, t+4) are whole: no branch between a
        // load and the MFMAs that wait for it
        for (; t + 4 < nf; t += 3) {
            NKV_ROTW_FENCE;
            load_full(b2, qw, t + 2);
            NKV_ROTW_FENCE;
            mma(b0, t);
            NKV_ROTW_FENCE;
            load_full(b0, qw, t + 3);
            NKV_ROTW_FENCE;
            mma(b1, t + 1);
            NKV_ROTW_FENCE;
            load_full(b1, qw, t + 4);
            NKV_ROTW_FENCE;
            mma(b2, t + 2);
        }
        NKV_ROTW_FENCE;
        // b0 holds batch t < nb, b1 batch t+1 when it exists: the rest (wave-uniform branches)
        for (;; t += 2) {
            mma(b0, t);
            if (t + 1 >= nb) break;
            const bool more2 = t + 2 < nb;
            if (more2) load(b0, qw, t + 2);
            mma(b1, t + 1);
            if (!more2) break;
            if (t + 3 < nb) load(b1, qw, t + 3);
        }
        NKV_ROTW_FENCE;
#undef NKV_ROTW_FENCE
        // the next tile's first two batches go out before this tile's stores (other rows)
        const int64_t next = tile + gridDim.x;
        double* qo = const_cast<double*>(qw) + 2 * lr;
        qw = wbase(next < t_hi ? next : tile);
        load(b0, qw, 0);
        load(b1, qw, 1);
#pragma unroll
        for (int m = 0; m < MB; ++m) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gc = m * 16 + lk + 4 * r;
                if (gc < n_out) st2s(qo + (int64_t)gc * ld, make_double2(acc[0][m][r], acc[1][m][r]));
            }
        }
        if (next >= t_hi) break;
        tile = next;
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
// does not fit LDS whole: k > 128 with many kept columns).  As k_rotate_stream, every wave owns one 16-row
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

#ifndef NKV_ROT_STREAM
#define NKV_ROT_STREAM 1   // 0: never use the streaming rotation
#endif
#ifndef NKV_ROT_WAVES
#define NKV_ROT_WAVES 16
#endif
#ifndef NKV_ROT_NB
#define NKV_ROT_NB 1
#endif
#ifndef NKV_ROT_CHUNK_FROM
#define NKV_ROT_CHUNK_FROM 17   // 16-column blocks from which the chunked kernel replaces the streaming one
#endif
static_assert(NKV_TILE % (4 * 16) == 0 && NKV_TILE % (8 * 16) == 0, "a 16-row slab per wave must tile the padding");

template <int MB>
int launch_rotate_stream(const nkv_layout* L, double* Q, int k, const double* V, int ldv, int n_out,
                                int kp, size_t lds, void* stream) {
    // register budget (gfx950, U = 4, measured with -Rpass-analysis=kernel-resource-usage in round 6):
    // MB = 1/2/3 at 16 waves per workgroup 52/74/96 VGPRs; MB = 4..8 at 8 waves 118/146/168/235/245 (the
    // three-batch path from MB = 5), no spills; 16 waves/WG allow 128 per lane, so wide column blocks run
    // with half the waves (256 VGPRs)
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

#ifndef NKV_ROTW
#define NKV_ROTW 1   // 0: never use the wide-load rotation (the k_rotate_stream / k_rotate_chunked path)
#endif
#ifndef NKV_ROTW_MAX_MB
#define NKV_ROTW_MAX_MB 4   // wide-load rotation up to this many 16-column blocks (64 kept columns)
#endif
#ifndef NKV_ROTW_W
#define NKV_ROTW_W 8   // waves per workgroup of the wide-load rotation
#endif
#ifndef NKV_ROTW_U
#define NKV_ROTW_U 4   // k-steps of 4 per batch of the wide-load rotation
#endif
#ifndef NKV_ROTW_ROUNDS
#define NKV_ROTW_ROUNDS 0   // wide-load rotation: one launch per this many grid-stride rounds (0: one launch; bands
                            // lose here: 2 rounds -10 %, 8 rounds -2 %, profiles/r06d_tune_rotw_bands.log)
#endif
static_assert(NKV_TILE % (NKV_ROTW_W * 32) == 0, "a 32-row slab per wave must tile the padding");

// LDS of the wide-load rotation: V k-major, kpad rows of cp doubles (cp = 16 mod 32)
inline int rotw_cp(int nact) { return ((16 * nact + 31) / 32) * 32 + 16; }
inline int rotw_kpad(int k) { return ((k + 4 * NKV_ROTW_U - 1) / (4 * NKV_ROTW_U)) * 4 * NKV_ROTW_U; }

template <int MB>
int launch_rotate_wide(const nkv_layout* L, double* Q, int k, const double* V, int ldv, int n_out, void* stream) {
    constexpr int W = NKV_ROTW_W, U = NKV_ROTW_U;
    auto kern = k_rotate_wide<MB, W, U>;
    const int cp = rotw_cp(MB);
    const size_t lds = (size_t)rotw_kpad(k) * cp * sizeof(double);
    static bool attr_set = false;
    if (!attr_set) {
        NKV_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set = true;
    }
    const int64_t n_tiles = rows_of(L) / ((int64_t)W * 32);
    if (n_tiles < 1) return NKV_OK;
    // persistent grid: as many workgroups as are resident at once (registers, LDS and waves per CU)
    int per_cu = 0;
    NKV_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, W * 64, lds));
    if (per_cu < 1) per_cu = 1;
    const int64_t g0 = (int64_t)device_cus() * per_cu;
    const int64_t g = n_tiles < g0 ? n_tiles : g0;
    // one launch per row band of NKV_ROTW_ROUNDS grid-stride rounds, as the few-column rotation and
    // the DCGS2 updates: the workgroups stay on one compact window of rows, reading each column in
    // step, instead of drifting apart over the whole vector (0: one persistent launch)
    const int64_t band = NKV_ROTW_ROUNDS > 0 ? (int64_t)NKV_ROTW_ROUNDS * g : n_tiles;
    for (int64_t lo = 0; lo < n_tiles; lo += band) {
        const int64_t hi = lo + band < n_tiles ? lo + band : n_tiles;
        hipLaunchKernelGGL(kern, dim3((unsigned)(g < hi - lo ? g : hi - lo)), dim3(W * 64), lds, S(stream), Q, L->ld,
                           k, V, ldv, n_out, cp, lo, hi);
        NKV_LAUNCHED();
    }
    return NKV_OK;
}

template <int MB>
int launch_rotate_chunked(const nkv_layout* L, double* Q, int k, const double* V, int ldv, int n_out,
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

template <int NO>
int launch_rotate_few(const nkv_layout* L, double* Q, int k, const double* V, int ldv, void* stream) {
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

}  // namespace

extern "C" {

int nkv_rotate_cols(const nkv_layout* L, double* Q, int k, const double* V_dev, int ldv, int n_out, void* stream) {
    CHECK(check_layout(L));
    CHECK(check_ptr(Q, "Q"));
    if (!V_dev) return fail(NKV_EINVAL, "V_dev is NULL");
    // no kernel holds k-sized state (V streams through LDS in k-chunks where it does not fit whole):
    // any k up to NKV_MAX_COLS; every output column lives in registers, so at most NKV_ROT_MAX_OUT
    if (k < 1 || k > NKV_MAX_COLS) return fail(NKV_EINVAL, "rotate: k=%d outside [1, %d]", k, NKV_MAX_COLS);
    if (ldv < k) return fail(NKV_EINVAL, "rotate: ldv=%d < k=%d", ldv, k);
    if (n_out < 1 || n_out > k) return fail(NKV_EINVAL, "rotate: n_out=%d outside [1, k=%d]", n_out, k);
    if (n_out > NKV_ROT_MAX_OUT)
        return fail(NKV_ESHAPE, "rotate: n_out=%d kept columns > NKV_ROT_MAX_OUT=%d", n_out, NKV_ROT_MAX_OUT);
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
    if (NKV_ROTW && (n_out + 15) / 16 <= NKV_ROTW_MAX_MB && rows_of(L) % ((int64_t)NKV_ROTW_W * 32) == 0) {
        const int nact = (n_out + 15) / 16;
        if ((size_t)rotw_kpad(k) * rotw_cp(nact) * sizeof(double) <= 160 * 1024) {
            switch (nact) {
                case 1: return launch_rotate_wide<1>(L, Q, k, V_dev, ldv, n_out, stream);
                case 2: return launch_rotate_wide<2>(L, Q, k, V_dev, ldv, n_out, stream);
                case 3: return launch_rotate_wide<3>(L, Q, k, V_dev, ldv, n_out, stream);
                case 4: return launch_rotate_wide<4>(L, Q, k, V_dev, ldv, n_out, stream);
#if NKV_ROTW_MAX_MB > 4
                case 5: return launch_rotate_wide<5>(L, Q, k, V_dev, ldv, n_out, stream);
                case 6: return launch_rotate_wide<6>(L, Q, k, V_dev, ldv, n_out, stream);
                case 7: return launch_rotate_wide<7>(L, Q, k, V_dev, ldv, n_out, stream);
                case 8: return launch_rotate_wide<8>(L, Q, k, V_dev, ldv, n_out, stream);
#endif
                default: break;
            }
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
    // V through LDS in k-chunks: 17..NKV_ROT_MAX_OUT kept columns where V[:, 0:n_out] does not fit
    // LDS whole (rows are whole NKV_TILE tiles, so every 16-row slab of 8 waves is full)
    const int nact = (n_out + 15) / 16;
    if (nact <= 2) return launch_rotate_chunked<2>(L, Q, k, V_dev, ldv, n_out, stream);
    if (nact <= 4) return launch_rotate_chunked<4>(L, Q, k, V_dev, ldv, n_out, stream);
    if (nact <= 8) return launch_rotate_chunked<8>(L, Q, k, V_dev, ldv, n_out, stream);
    if (nact <= 12) return launch_rotate_chunked<12>(L, Q, k, V_dev, ldv, n_out, stream);
    return launch_rotate_chunked<16>(L, Q, k, V_dev, ldv, n_out, stream);
}

int nkv_rotate(const nkv_layout* L, double* Q, int k, const double* V_dev, int ldv, void* stream) {
    return nkv_rotate_cols(L, Q, k, V_dev, ldv, k, stream);
}

}  // extern "C"
