/*
 * nekkrylov.h — C ABI of the MI355X (gfx950) Krylov hot path for nekStab.
 *
 * This is the drop-in boundary.  Everything below takes plain device pointers,
 * sizes and a HIP stream (as `void*`), returns an `int` status, and never
 * synchronises the host except where stated.  The reference interfaces each
 * entry point replaces are cited as `file:line` into nekStab_next
 * (reference @ 2025-02-27); see INTEGRATION.md for the Fortran `bind(C)`
 * interface block a nekStab maintainer would add.
 *
 * ---------------------------------------------------------------------------
 * State-vector layout (one nekStab `krylov_vector` / `real_nek_vector`,
 * core/krylov_subspace.f90:12-17, core/nek_vectors.f90:20-31), fp64 in HBM:
 *
 *   [ wf_0 | wf_1 | ... | wf_{n_wf-1} | pr | time | pad ]
 *     each wf_f is `sv` doubles: n_v live points + zero padding
 *     pr is `sp` doubles: n_p live points + zero padding
 *     time is one double at offset  nkv_time_offset(L) = n_wf*sv + sp
 *
 * Weighted fields are vx, vy, [vz], [t_1 .. t_s] — exactly the fields that
 * enter `glsc3(.., bm1s, .., n)` in k_dot / real_dot
 * (krylov_subspace.f90:40-50, nek_vectors.f90:94-104).  Pressure is stored
 * and is touched by every BLAS-1 op (nopaxpby/nopcmult/..., nek_vectors.f90:
 * 229-362) but never enters a dot.  `time` is the scalar component of the
 * vector (krylov_subspace.f90:16).
 *
 * sv and sp are multiples of NKV_TILE (padding rows are zero and their
 * weight is zero), so every kernel streams whole tiles without masking.
 * A Krylov basis is (k+1) vectors at stride `ld` doubles (ld >= time offset+1,
 * multiple of NKV_TILE): Q[c] = Q + c*ld.
 *
 * The weight vector `w` (bm1s, core/NEKSTAB:86-89; zeroed inside a sponge by
 * core/forcing.f90:101-104) has `sv` doubles, shared by every weighted field.
 *
 * Multi-GPU: each rank holds an element-contiguous shard (same layout, local
 * n_v/n_p).  Every reduction entry point writes the LOCAL partial sum to a
 * device buffer; the caller all-reduces it (RCCL) before the consuming entry
 * point runs on the same stream — the MI355X replacement of the per-field
 * MPI_Allreduce hidden in Nek5000's glsc3.
 * ------------------------------------------------------------------------- */
#ifndef NEKKRYLOV_H
#define NEKKRYLOV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NKV_ABI_VERSION 3   /* 3 (round 6): nkv_layout_init added (refuses nelt != nelv); 2 (round 5): the opt-in
                               deferred-basis DCGS2 entry points removed; rotation limited by kept columns */

/* Rows per tile: fields are padded to a multiple of this many doubles. */
#define NKV_TILE 4096
/* Most basis columns one multi-dot (nkv_block_dot / nkv_block_dot2) takes: its per-column partials
 * live in LDS (64 B per column for the two-vector dot).  The reference's k_dim defaults to 100
 * (main.f90:9); GMRES on the cylinder uses 200 (1cyl.usr:14). */
#define NKV_MAX_COLS 1024
/* Most output columns of one basis rotation (nkv_rotate / nkv_rotate_cols): every output column is
 * held in registers while the k input columns stream past (no k-sized state, so any k up to
 * NKV_MAX_COLS).  A Krylov–Schur restart keeps mstart-1 < k_dim columns; the reference's k_dim is
 * at most 200 (1cyl.usr:14), so 256 covers every restart of k_dim <= 257. */
#define NKV_ROT_MAX_OUT 256

/* Status codes (every entry point). */
#define NKV_OK 0
#define NKV_EINVAL 1 /* bad argument / shape                          */
#define NKV_EHIP 2   /* HIP runtime error (see nkv_last_error)        */
#define NKV_ENAN 3   /* NaN detected in a reduction (k_dot :57 guard)  */
#define NKV_ESHAPE 4 /* layout not padded/aligned as documented above  */
#define NKV_ECALLBACK 5 /* a host callback (operator, all-reduce) of a one-call driver failed */
#define NKV_EBREAKDOWN 6 /* NKV_CHECK_BREAKDOWN: the Krylov space became invariant (nkv_arnoldi_factorization) */

/* Flags. */
#define NKV_TIME 0x1u      /* include the `time` slot (dot: add p.time*q.time; BLAS-1: update it) */
#define NKV_ACCUMULATE 0x2u /* block_update: f <- f - Q h   (default)                             */
#define NKV_OVERWRITE 0x4u  /* block_update: f <- + Q h     (k_matmul, krylov_subspace.f90:163)    */
#define NKV_NORM2 0x8u      /* block_update: also write the local ||f||_W^2 partial               */
#define NKV_TIME_DOT 0x10u  /* block_update_dot / block_update+NORM2: time product in the dot/norm */
#define NKV_X_IS_LAST 0x20u /* block_dot2: x is column j-1 of Q (its two dots come from registers)  */
#define NKV_MGS2 0x40u      /* update_hessenberg / arnoldi_factorization: the reference's MGS2 order */
#define NKV_CHECK_BREAKDOWN 0x80u /* one-call factorisations: check the new H columns on return      */
#define NKV_MGS_ICWY 0x100u /* arnoldi_factorization: both MGS passes in inverse compact WY form (3 reads) */
#define NKV_MGS_LAGGED 0x200u /* arnoldi_factorization: MGS2 coefficients, second pass lagged (2 reads) */

typedef struct nkv_layout {
    int64_t n_v;  /* live points per weighted field on this rank (lx1*ly1*lz1*nelv)  */
    int64_t n_p;  /* live pressure points on this rank (lx2*ly2*lz2*nelv; 0: no pr)  */
    int64_t sv;   /* padded stride of one weighted field (multiple of NKV_TILE)     */
    int64_t sp;   /* padded length of the pressure segment (multiple of NKV_TILE)   */
    int64_t ld;   /* stride between basis vectors, doubles (multiple of NKV_TILE)   */
    int32_t n_wf; /* number of weighted fields: 2 or 3 velocities + active scalars  */
    int32_t rank0;/* 1 on the rank that owns the replicated `time` term of a dot    */
} nkv_layout;

/* ---- runtime ---------------------------------------------------------- */
int nkv_abi_version(void);
/* Fill *L for one rank's shard from nekStab's SIZE/TOTAL facts (core/nek_vectors.f90:16-31):
 * ldim (2/3, if3d), lx1, lx2 (pressure points per direction; ignored when !ifpo), nelv and nelt (this
 * rank's velocity and temperature/scalar elements), n_scalars (dotted scalars: ifto + ifpsco(:)),
 * ifpo (pressure stored), rank0 (owns the replicated `time` term).  Pads sv, sp, ld to NKV_TILE.
 * NKV_ESHAPE when n_scalars > 0 and nelt != nelv: k_dot / real_dot dot a scalar over nelt elements
 * with the nelv-element weights bm1s (krylov_subspace.f90:36-44, nek_vectors.f90:88-99, NEKSTAB:86),
 * i.e. past the end of bm1s, so conjugate heat transfer layouts have no reference result and are
 * refused.  NKV_EINVAL on bad parameters. */
int nkv_layout_init(nkv_layout* L, int ldim, int lx1, int lx2, int64_t nelv, int64_t nelt, int n_scalars,
                    int ifpo, int rank0);
const char* nkv_last_error(void);
/* Device properties of the current HIP device (host sync-free). */
int nkv_device_info(int* device, int* cu_count, int64_t* hbm_bytes, char* name, int name_len);
/* Bytes of device scratch the reduction entry points need for up to `max_cols` columns. */
size_t nkv_workspace_bytes(const nkv_layout* L, int max_cols);
/* Reads (with a stream sync) and clears the NaN flag kept in the workspace. */
int nkv_check_status(void* ws, void* stream);

/* ---- BLAS-1 over all stored fields (a5/a6) ----------------------------------------------
 * k_zero/real_zero        krylov_subspace.f90:141-150, nek_vectors.f90:70-78
 * k_copy                  krylov_subspace.f90:152-161
 * k_cmult/real_scal       krylov_subspace.f90:94-104,  nek_vectors.f90:116-125
 * real_axpby (time NOT updated unless NKV_TIME)           nek_vectors.f90:127-139,257-277
 * k_add2/k_sub2 = axpby(1,±1), k_sub3                     krylov_subspace.f90:106-139 */
int nkv_zero(const nkv_layout* L, double* x, unsigned flags, void* stream);
int nkv_copy(const nkv_layout* L, double* dst, const double* src, unsigned flags, void* stream);
int nkv_scal(const nkv_layout* L, double* x, double alpha, unsigned flags, void* stream);
int nkv_axpby(const nkv_layout* L, double* x, double alpha, const double* y, double beta,
              unsigned flags, void* stream);
int nkv_sub3(const nkv_layout* L, double* p, const double* q, const double* r, unsigned flags,
             void* stream);
/* x <- x + sign * (*alpha_dev) * y, the scalar read on the device (MGS step, stream-ordered). */
int nkv_axpy_dev(const nkv_layout* L, double* x, const double* alpha_dev, double sign, const double* y,
                 unsigned flags, void* stream);
/* x <- x / sqrt(*nrm2_dev)   (k_normalize, krylov_subspace.f90:75-92); writes sqrt to beta_dev. */
/* Every stored row is scaled, the time slot included (flags reserved, pass 0); eigensolvers.f90's
 * own normalize (nopcmult, :78-116) keeps time — its host restores the slot. */
int nkv_normalize_dev(const nkv_layout* L, double* x, const double* nrm2_dev, double* beta_dev,
                      unsigned flags, void* stream);

/* ---- weighted inner product (a1-a3) -------------------------------------------------------
 * out_dev[0] = sum_fields sum_i a_i*w_i*b_i (+ a.time*b.time if NKV_TIME and rank0)
 * k_dot krylov_subspace.f90:26-60 (time only when uparam(1)==2.1), real_dot nek_vectors.f90:80-114
 * (time always), inner_product eigensolvers.f90:3-56, glsc3 [Nek5000].  LOCAL partial. */
int nkv_dot(const nkv_layout* L, const double* w, const double* a, const double* b, double* out_dev,
            void* ws, unsigned flags, void* stream);

/* ---- block Gram–Schmidt (a7, update_hessenberg_matrix krylov_decomposition.f90:103-189) ----
 * block_dot:    h_dev[0:j] = Q[:,0:j]^T W f  (LOCAL partials, deterministic 2-stage reduction)
 * block_update: f <- f - Q[:,0:j] h           (NKV_ACCUMULATE, default)
 *               f <- Q[:,0:j] h               (NKV_OVERWRITE: k_matmul / mode reconstruction)
 *               with NKV_NORM2 also nrm2_dev[0] = ||f_new||_W^2 local partial (+ f.time^2 with
 *               NKV_TIME_DOT on rank0; NKV_TIME alone updates the slot, not the norm)
 * arnoldi_finish: q_out = f/beta, beta = sqrt(nrm2_dev[0]); H column k written on the device:
 *               hcol[i] = h1[i] + h2[i] (i<j; h2 may be NULL), hcol[j] = beta (H(k+1,k), :183-186) */
int nkv_block_dot(const nkv_layout* L, const double* w, const double* Q, int j, const double* f,
                  double* h_dev, void* ws, unsigned flags, void* stream);
int nkv_block_update(const nkv_layout* L, const double* w, const double* Q, int j, const double* h_dev,
                     double* f, double* nrm2_dev, void* ws, unsigned flags, void* stream);
/* Fused CGS2 middle pass (one read of Q): f <- f - Q[:,0:j] h, then hout_dev[0:j] = Q^T W f_new
 * (LOCAL partials).  NKV_TIME updates f.time, NKV_TIME_DOT adds the time product to hout (rank0). */
int nkv_block_update_dot(const nkv_layout* L, const double* w, const double* Q, int j, const double* h_dev,
                         double* f, double* hout_dev, void* ws, unsigned flags, void* stream);
int nkv_arnoldi_finish(const nkv_layout* L, const double* f, const double* nrm2_dev, double* q_out,
                       int j, const double* h1_dev, const double* h2_dev, double* hcol_dev,
                       unsigned flags, void* stream);

/* The remaining block entry points SURVEY.md §8(b) names:
 * nkv_combine:          out <- Q[:,0:k] y  (k_matmul krylov_subspace.f90:163-209, mode
 *                       reconstruction eigensolvers.f90:565-585; = nkv_block_update NKV_OVERWRITE)
 * nkv_normalize_store:  q_next <- f / sqrt(*nrm2_dev), *beta_dev = sqrt(*nrm2_dev) (the reduced
 *                       ||f||_W^2; update_hessenberg_matrix's last lines :183-186 with Q(k+1) = f, :81)
 * nkv_mgs2_step:        the reference's whole update_hessenberg_matrix in ITS operation order
 *                       (:155-186: two MGS passes, one weighted dot + axpy per column, H(i,k) =
 *                       alpha1 + alpha2, H(k+1,k) = ||f||, q_out = f/||f||), device-side with no
 *                       host sync.  SINGLE PROCESS: its dots are not all-reduced — a sharded host
 *                       runs nkv_dot + all-reduce + nkv_axpy_dev per column (the mgs2 mode of
 *                       nekstab_next_amd.arnoldi).  hcol_dev: j+1 doubles.  NKV_TIME_DOT adds the
 *                       time products to the dots (uparam(1)==2.1, rank0); f.time follows the axpys. */
int nkv_combine(const nkv_layout* L, const double* Q, int k, const double* y_dev, double* out, unsigned flags,
                void* stream);
int nkv_normalize_store(const nkv_layout* L, const double* f, const double* nrm2_dev, double* q_next,
                        double* beta_dev, unsigned flags, void* stream);
int nkv_mgs2_step(const nkv_layout* L, const double* w, const double* Q, int j, double* f, double* q_out,
                  double* hcol_dev, void* ws, unsigned flags, void* stream);
/* One column of an MGS pass fused with the next one's projection (update_hessenberg_matrix's
 * k_cmult + k_sub2 then k_dot, krylov_decomposition.f90:157-166 / :173-180, in that order):
 *   f <- f - (*alpha_dev) qa                 (NKV_TIME: the time slot too, as k_sub2)
 *   *out_dev = <f_new, qb>_W  LOCAL partial  (qb = NULL: <f_new, f_new>, the closing k_normalize);
 * NKV_TIME_DOT adds the time product (rank0).  One read of f for the pair of operations; the MGS2
 * sequences of nkv_update_hessenberg(NKV_MGS2) and nkv_mgs2_step are built from it. */
int nkv_axpy_dot(const nkv_layout* L, const double* w, double* f, const double* alpha_dev, const double* qa,
                 const double* qb, double* out_dev, void* ws, unsigned flags, void* stream);

/* ---- DCGS2: classical Gram–Schmidt with delayed re-orthogonalisation (two reads of Q per step,
 * ONE all-reduce per step, no separate normalisation pass).  Same replacement target as the CGS2
 * entry points above (update_hessenberg_matrix, krylov_decomposition.f90:103-189); the
 * re-orthogonalisation AND the normalisation of q_j are folded into step j+1, the previous H
 * column corrected on the device.  Step j (m = j-1 final columns; Q column m holds u = beta q_j;
 * f = A u):
 *   nkv_block_dot2(Q, j, x=u, y=f) -> h[0:j] = Q^T W u, h[j:2j] = Q^T W f          (all-reduce 2j)
 *   nkv_dcgs2_coef(m, h, h+j, nrm, H, ldh, coef)   H(m,m-1) = beta, row m corrected, column m = c;
 *                                                  coef = [x | c | rinv, y, (beta r)^2, s | a]
 *   nkv_dcgs2_update(Q, m, coef, u, f, Q col j, NULL) -> column m final, column j = the next u
 * nrm points at beta^2: h + m (= u^T W u, the dot's last entry) -- or NULL at the first step
 * (u normalised, beta = 1), or a separately reduced ||u||_W^2 (nkv_dcgs2_update with a non-NULL
 * nrm2 computes it, fused, from the f it writes: one more all-reduce per step).
 * After the last step (m = mend): nkv_block_dot(Q, m+1, u) -> h, nkv_dcgs2_coef(m, h, NULL, h+m, ...),
 * nkv_block_update(Q, m, h, u), nkv_normalize_dev(u, coef+2m+3).
 * H is column-major with leading dimension ldh (>= m+1) in device memory. */
int nkv_block_dot2(const nkv_layout* L, const double* w, const double* Q, int j, const double* x,
                   const double* y, double* h_dev, void* ws, unsigned flags, void* stream);
int nkv_dcgs2_coef(int m, const double* hq_dev, const double* hw_dev, const double* nrm_prev_dev, double* H_dev,
                   int64_t ldh, double* coef_dev, void* ws, void* stream);
int nkv_dcgs2_update(const nkv_layout* L, const double* w, const double* Q, int m, const double* coef_dev,
                     double* qj, const double* win, double* fout, double* nrm2_dev, void* ws, unsigned flags,
                     void* stream);

/* ---- MGS2 in inverse compact WY form (mode "mgs2-icwy"; Swirydowicz et al. 2020) -----------
 * One modified Gram–Schmidt pass of update_hessenberg_matrix (krylov_decomposition.f90:155-168,
 * repeated at :171-180) over q_0..q_{j-1}: alpha_i = <f_i, q_i>_W with f_i = f - sum_{k<i} alpha_k q_k.
 * In exact arithmetic alpha_i = b_i - sum_{k<i} G(i,k) alpha_k with b = Q^T W f (classical dots) and
 * G(i,k) = <q_k, q_i>_W, whether or not the basis is orthonormal (it is not after the reference's
 * unnormalised noise/load seed, eigensolvers.f90:192-223, or a restart with time in k_dot), so
 * alpha = (I + L)^{-1} b, L the strictly lower part of G: the pass becomes one multi-dot, this
 * O(j^2) solve (one workgroup, no host sync) and one block update — three reads of Q per step for
 * both passes instead of the reference order's per-column stream of f.
 * G: row-major, row i at G + i*ldg (ldg >= j); columns k < i are read.  grow (may be NULL): the
 * row G(j-1, 0:j-1) of the newest column, stored into G first (nkv_block_dot2's first j-1 entries
 * with x = q_{j-1}).  x may alias b.  Step j of the factorisation:
 *   nkv_block_dot2(Q, j, x=q_{j-1}, y=f, NKV_X_IS_LAST) -> h; all-reduce 2j
 *   nkv_mgs_icwy_solve(j, G, ldg, h, h+j, h1)                  (pass-1 coefficients)
 *   nkv_block_update_dot(Q, j, h1, f, h2); all-reduce j      (f -= Q h1; h2 = Q^T W f)
 *   nkv_mgs_icwy_solve(j, G, ldg, NULL, h2, h2)              (pass-2 coefficients)
 *   nkv_block_update(Q, j, h2, f, nrm, NKV_NORM2); all-reduce 1; nkv_arnoldi_finish(f, nrm, ...) */
int nkv_mgs_icwy_solve(int j, double* G, int64_t ldg, const double* grow, const double* b, double* x,
                       void* stream);

/* ---- svds: Golub–Kahan–Lanczos with delayed re-orthogonalisation (f1; LightKrylov svds as called by
 * transient_growth_analysis / resolvent_analysis, linear_stab.f90:112,153).  Two bases U, V, each
 * read twice per step (a two-vector multi-dot and a dual update) instead of three times (CGS2).
 * Step j (1-based; V col j-1 and U col j-2 provisional; C = projections of A V on U, D of A^T U on V):
 *   f = A V[j-1];  j = 1: U[0] = f;  else
 *     nkv_block_dot2(U, j-1, x=U[j-2], y=f, NKV_X_IS_LAST) -> h (all-reduce 2(j-1))
 *     nkv_gkl_coef(0, j-2, h, h+(j-1), C, ...)  ->  coef;  C column j-3... finalised
 *     nkv_dcgs2_update(U, j-2, coef, U[j-2], f, U[j-1], NULL)
 *   f = A^T U[j-1];
 *     nkv_block_dot2(V, j, x=V[j-1], y=f, NKV_X_IS_LAST) -> h (all-reduce 2j)
 *     nkv_gkl_coef(1, j-1, h, h+j, D, ...);  nkv_dcgs2_update(V, j-1, coef, V[j-1], f, V[j], NULL)
 * After step k each basis closes its provisional column: nkv_block_dot(Q, m+1, Q[m]) -> h,
 * nkv_gkl_coef(side, m, h, NULL, ...), nkv_block_update(Q, m, coef+2m+5, Q[m]), nkv_normalize_dev(Q[m],
 * coef+2m+3) with m = k-1 (U) and k (V).  Then A V_k = U_k C (k x k upper triangular) and
 * A^T U_k = V_{k+1} D, both bases W-orthonormal.  The coefficient algebra (one workgroup):
 *   a = hq[0:m], r = sqrt(hq[m] - a.a); with hw: M column p+1 (p = m - side) = [hw[0:m] ;
 *   (hw[m] - a.hw[0:m])/r] (raw), coef = [hw[0:m]/r | . | 1/r, M(m,p+1)/r, r^2, 1 | a]; M column p
 *   finalised (p >= 0): M[0:m,p] = (M[0:m,p] - M[0:m,0:p] A_other[:,p] + rho a)/r_other[p],
 *   M[m,p] = rho r / r_other[p], rho = r_self[m-1] (1 at m = 0); A_self[:,m] = a, r_self[m] = r.
 * M, A_self, A_other: device, column-major (ldm, lda >= m+1); r^2 <= 0 raises the NaN flag. */
int nkv_gkl_coef(int side, int m, const double* hq_dev, const double* hw_dev, double* M_dev, int64_t ldm,
                 double* A_self, double* r_self, const double* A_other, const double* r_other, int64_t lda,
                 double* coef_dev, void* ws, void* stream);

/* ---- the whole factorisation natively (a8: arnoldi_factorization, krylov_decomposition.f90:2-99 —
 * the loop :68-96 calling matvec then update_hessenberg_matrix) as ONE call: the DCGS2 sequence
 * above for mstep = mstart..mend, then the closing re-orthogonalisation, orchestrated in C++ (the
 * same entry points in the same order as nekstab_next_amd/arnoldi.py, so the results are identical
 * bit for bit).  For a Fortran/C host that replaces `call arnoldi_factorization(Q, H, mstart, mend,
 * ksize)` without a Python layer.
 *   On entry columns 0..mstart-1 of Q are final and W-orthonormal (column mstart-1: the normalised
 *   seed, or Q(k+1) moved to Q(mstart) by a Krylov–Schur restart) and H columns 0..mstart-2 hold the
 *   factorisation so far (row mstart-1 the restart row).  On return Q columns 0..mend and H columns
 *   0..mend-1 form an Arnoldi factorisation A Q_mend = Q_{mend+1} H.
 *   H_dev: device, column-major, leading dimension ldh >= mend+1.  f: one device vector (scratch).
 *   scratch_dev: nkv_arnoldi_scratch_doubles(mend) doubles of device memory; ws: at least
 *   nkv_workspace_bytes(L, mend + 1) bytes (the multi-dots' partials for up to mend+1 columns).
 *   matvec(mv_user, x, y, stream): y = A x for device vectors x, y, enqueued on `stream`; returns 0.
 *   allreduce(ar_user, buf, n, stream): in-place SUM of n device doubles over the ranks, ordered on
 *   `stream` (ncclAllReduce on it, or a stream sync + MPI_Allreduce); NULL on a single rank.
 *   flags: NKV_TIME_DOT includes the time products in the dots (uparam(1)==2.1, k_dot :52-54);
 *   NKV_CHECK_BREAKDOWN: see "Breakdown" under nkv_arnoldi_factorization below.
 *   A callback's non-zero return stops the factorisation with NKV_ECALLBACK (see nkv_last_error). */
typedef int (*nkv_matvec_fn)(void* user, const double* x, double* y, void* stream);
typedef int (*nkv_allreduce_fn)(void* user, double* buf, int n, void* stream);
size_t nkv_arnoldi_scratch_doubles(int m);
int nkv_arnoldi_dcgs2(const nkv_layout* L, const double* w, double* Q, int mstart, int mend, double* H_dev,
                      int64_t ldh, double* f, double* scratch_dev, void* ws, nkv_matvec_fn matvec, void* mv_user,
                      nkv_allreduce_fn allreduce, void* ar_user, unsigned flags, void* stream);

/* ts_gmres's inner loop (a17: newton_krylov.f90:250-276, each column arnoldi_factorization(Q,H,k,k)
 * then lstsq and norm2(e - H y)) as ONE call on a continuous DCGS2 factorisation: per column k the
 * DCGS2 step of nkv_arnoldi_dcgs2 with the norm of the next provisional vector fused into the update
 * (one more all-reduce), the least-squares residual from nkv_givens_column on H(0:k+1, k-1) with
 * H(k, k-1) = that norm (the column's once-projected coefficients: its O(eps) re-orthogonalisation
 * correction arrives with the next column, so the test needs no lag and no extra matvec), stored in
 * res_hist[k-1]; stop when res^2 < tol2 (the reference's beta**2 < tol, or max(tol, 1e-8) for its
 * iffindiff exit) or at kmax.  Then one closing multi-dot finalises H's last row.
 *   On entry Q column 0 = r0 / beta (W-normalised), beta = ||r0||_W.  On return *k_out = k columns,
 *   H_dev (column-major, ldh >= kmax+1) holds the (k+1) x k Hessenberg matrix of A Q_k = Q_{k+1} H;
 *   Q columns 0..k-1 are final (column k is left unfinished: the solution update does not read it).
 *   The host then solves y = lstsq(H, beta e_1) (dgels, lapack_wrapper.f90:248-300, as the reference)
 *   and forms sol += Q_k y (nkv_combine).  res_hist: kmax host doubles.  scratch_dev:
 *   nkv_arnoldi_scratch_doubles(kmax) doubles; ws: nkv_workspace_bytes(L, kmax + 1).  Callbacks and
 *   flags (NKV_TIME_DOT) as nkv_arnoldi_dcgs2. */
int nkv_gmres_dcgs2(const nkv_layout* L, const double* w, double* Q, int kmax, double beta, double tol2,
                    double* H_dev, int64_t ldh, double* f, double* scratch_dev, void* ws, nkv_matvec_fn matvec,
                    void* mv_user, nkv_allreduce_fn allreduce, void* ar_user, double* res_hist, int* k_out,
                    unsigned flags, void* stream);

/* update_hessenberg_matrix(H, f, Q, k) itself as one call (krylov_decomposition.f90:103-189): the
 * fused 3-pass CGS2 sequence of the block Gram–Schmidt section above (block_dot, all-reduce,
 * block_update_dot, all-reduce, block_update + norm, all-reduce, arnoldi_finish) with the
 * all-reduce as the callback of nkv_arnoldi_dcgs2 (NULL on one rank).  f is orthogonalised twice
 * against Q[:,0:j] (W inner product), q_out = f/||f||_W, hcol_dev[0:j+1] = H(1:k+1, k).  j = 0
 * only normalises.  scratch_dev: nkv_arnoldi_scratch_doubles(j) doubles; ws: nkv_workspace_bytes(L, j)
 * bytes at least.  flags: NKV_TIME_DOT
 * (time products in the dots); NKV_MGS2: the reference's own order instead (:155-186, two MGS passes,
 * one dot + all-reduce + axpy per column; 2j+3 scratch doubles, covered by nkv_arnoldi_scratch_doubles(j)).
 * For per-column consumers (GMRES: newton_krylov.f90:252) and
 * checkpointing Arnoldi, where each column must be final when its step returns. */
int nkv_update_hessenberg(const nkv_layout* L, const double* w, const double* Q, int j, double* f, double* q_out,
                          double* hcol_dev, double* scratch_dev, void* ws, nkv_allreduce_fn allreduce, void* ar_user,
                          unsigned flags, void* stream);

/* arnoldi_factorization (krylov_decomposition.f90:2-99) with per-column orthogonalisation: for
 * mstep = mstart..mend, matvec(Q col mstep-1 -> f), then nkv_update_hessenberg(Q, mstep, f,
 * q_out = Q col mstep, hcol = H col mstep-1).  Same arguments as nkv_arnoldi_dcgs2; every column is
 * final when its step ends and columns < mstart are never written.  flags: NKV_TIME_DOT,
 * NKV_MGS2 (the reference's operation order, its dots all-reduced one at a time through the
 * callback: the sharded form of nkv_mgs2_step), NKV_MGS_ICWY (the same two MGS passes in inverse
 * compact WY form, three reads of Q per step — see nkv_mgs_icwy_solve — for the non-orthonormal bases
 * of the reference's default noise seed; the Gram rows of columns 1..mstart-2 are rebuilt first;
 * scratch: nkv_arnoldi_scratch_doubles(mend), which covers its (mend+1)^2 Gram matrix),
 * NKV_MGS_LAGGED (the same MGS2 coefficients with the second pass lagged into the next step's
 * multi-dot: two reads of Q per step, nkv_lagged_coef on the host between the multi-dot and the
 * dual update, so each step synchronises the stream once; the Gram rows of columns 0..mstart-2 are
 * rebuilt first and H columns 0..mend-1 are downloaded, updated on the host and written back; it
 * uses the Arnoldi relation of the columns before mstart, which the reference's restart breaks in
 * the time slot, so not with NKV_TIME_DOT after a restart), NKV_CHECK_BREAKDOWN.
 *
 * Breakdown (both one-call factorisations).  When the operator's Krylov space closes before mend
 * (A restricted to span(Q) is invariant: a rank-deficient operator), each later f is rounding noise.
 * The reference's MGS2 normalises the noise and carries on; the classical forms cannot: DCGS2's
 * norm sqrt(||u||^2 - ||Q^T W u||^2) cancels to a negative (NaN) and CGS2 leaves O(eps/ratio)
 * components in span(Q).  With NKV_CHECK_BREAKDOWN the driver synchronises the stream on return,
 * and returns NKV_EBREAKDOWN (message: the column and its ratio) if the NaN flag is set (it is
 * cleared) or any new column c has a non-finite entry or |H(c+1,c)| < 1e-8 ||H(0:c+2,c)||.  Normal
 * runs sit at ratios >= 0.1.  nkv_arnoldi_dcgs2 has by then rewritten Q column mstart-1 and H row
 * mstart-1 (the delayed re-orthogonalisation of the seed column): the caller restores both from its
 * own copies and redoes the factorisation with nkv_arnoldi_factorization(..., NKV_MGS2, ...), as
 * nekstab_next_amd.krylov_schur does.  H is replicated, so every rank reaches the same ratio test;
 * the NaN flag is per rank, so a sharded host all-reduces its breakdown decision before branching. */
int nkv_arnoldi_factorization(const nkv_layout* L, const double* w, double* Q, int mstart, int mend, double* H_dev,
                              int64_t ldh, double* f, double* scratch_dev, void* ws, nkv_matvec_fn matvec,
                              void* mv_user, nkv_allreduce_fn allreduce, void* ar_user, unsigned flags, void* stream);

/* ---- Krylov–Schur restart (a10, schur_condensation eigensolvers.f90:421-442) --------------
 * In place: Q[:,0:k] <- Q[:,0:k] * V, V k-by-k column-major (leading dim ldv) in device memory.
 * The time slot is not rotated (the reference copies vx..t only, :421-432).  k <= NKV_ROT_MAX_OUT
 * (NKV_ESHAPE beyond). */
int nkv_rotate(const nkv_layout* L, double* Q, int k, const double* V_dev, int ldv, void* stream);

/* Partial restart rotation, in place: Q[:,0:n_out] <- Q[:,0:k] * V[:,0:n_out], 1 <= n_out <= k.
 * Columns n_out..k-1 are left as they were.  schur_condensation only keeps the mstart selected
 * Schur vectors (eigensolvers.f90:416-459: Q(mstart+1..k) are overwritten by the next
 * factorisation before being read), so the restart calls this with n_out = mstart.
 * k <= NKV_MAX_COLS, n_out <= NKV_ROT_MAX_OUT (NKV_ESHAPE beyond). */
int nkv_rotate_cols(const nkv_layout* L, double* Q, int k, const double* V_dev, int ldv, int n_out,
                    void* stream);

/* ---- synthetic operators (the matvec boundary, linear_operators.f90:17-23) ----------------
 * op_diag: y = d .* x over every stored row; y.time = time_scale * x.time.
 * op_rot2: per weighted point i, (u,v) = (wf_0[i], wf_1[i]):
 *          y = [[c_i, -s_i],[s_i, c_i]] (u,v)   (transpose: s -> -s), other weighted fields and
 *          pressure multiplied by d_rest[row] (may be NULL → 0), y.time = 0. */
int nkv_op_diag(const nkv_layout* L, const double* d, const double* x, double* y, double time_scale,
                void* stream);
int nkv_op_rot2(const nkv_layout* L, const double* c, const double* s, const double* d_rest,
                const double* x, double* y, int transpose, void* stream);
/* op_cdiag: complex diagonal y = c x (conj: conj(c) x) on a re/im pair vector (the complex
 * cmplx_nek_vector{re, im} of nek_vectors.f90:33-42 stored as one real vector: in every segment the
 * re half first, then the im half; c = cr + i ci read at the re rows); y.time = 0.  The synthetic
 * resolvent (i omega - L)^-1 of resolvent_analysis (linear_stab.f90:120-163). */
int nkv_op_cdiag(const nkv_layout* L, const double* cr, const double* ci, const double* x, double* y, int conj,
                 void* stream);

/* ---- sensitivity post-processing (sensitivity.f90) ---------------------------------------
 * These entry points and the two seed kernels below work on field segments only (no time slot):
 * on an empty shard (n_v = 0, a rank without elements) they return NKV_OK without reading any
 * pointer, since its segment arrays are empty (NULL).
 *
 * wave_maker's pointwise product (sensitivity.f90:69-71), after biorthogonalize (:63-66):
 *   out[i] = sqrt(sum_c dRe_c[i]^2 + dIm_c[i]^2) * sqrt(sum_c aRe_c[i]^2 + aIm_c[i]^2),
 * c over the first ncomp (2 or 3, <= n_wf) weighted fields — the velocity components — summed in
 * the reference's left-to-right order without contraction.  out: sv doubles (one field segment;
 * padding rows give 0).  The reference's 2-D case adds its uninitialised vz arrays; here ncomp = 2
 * has no vz terms. */
int nkv_wavemaker(const nkv_layout* L, const double* dRe, const double* dIm, const double* aRe, const double* aIm,
                  double* out, int ncomp, void* stream);
/* bf_sensitivity (sensitivity.f90:81-269), the base-flow sensitivity of Marquet et al.:
 * nkv_gradm1: Nek5000's gradm1 (the calls at sensitivity.f90:170-199; navier5.f, with glmapm1 /
 * xyzrst's geometric factors from the GLL coordinates xm, ym, [zm]) of nfld fields (field f: n_v
 * points at u + f*u_stride, Nek point order, lx1^ldim per element, lx1 <= 10) into
 * grad + (f*ldim + d)*g_stride for direction d = x, y, [z]; the geometric factors are formed once
 * for all nfld fields.  D is the lx1 x lx1 GLL derivative matrix (row-major D[i*lx1+m] = l_m'(z_i),
 * device).  Element-local.  zm exactly when ldim = 3.
 * nkv_bf_sensitivity: the pointwise terms (:202-235) and their sums (:258-259) after gradm1 + dsavg:
 * grad = 4*ncomp*ncomp field segments [dRe, dIm, aRe, aIm][u, v, w][x, y, z] (sv doubles each),
 * out = 6*ncomp segments [tr, ti, pr, pi, sr, si][component].  The reference's dwdz-for-dvdz slips
 * (:204, 207, 213, 216) are kept; its 2-D reads of never-set vz arrays are absent. */
int nkv_gradm1(const nkv_layout* L, int lx1, int ldim, const double* D, const double* xm, const double* ym,
               const double* zm, const double* u, int nfld, int64_t u_stride, double* grad, int64_t g_stride,
               void* stream);
int nkv_bf_sensitivity(const nkv_layout* L, const double* dRe, const double* dIm, const double* aRe,
                       const double* aIm, const double* grad, double* out, int ncomp, void* stream);

/* ---- seeds (utils.f90:258-418; the noise seed is the reference's default, main.f90:29) ---------
 * nkv_mth_rand_add: one weighted field q (n_v points, Nek point order) += mth_rand(il, jl, kl, ieg,
 * xl, fc) (utils.f90:408-418), the pointwise part of op_add_noise (fc per velocity component,
 * :321-331) and add_noise_scal (:258-295); xm/ym/zm are this rank's GLL coordinates (n_v each; zm
 * exactly when lz1 > 1), e_first the 0-based global number of its first element (ieg = e_first+e+1).
 * nkv_group_average: q[m] <- mean of q over m's group, for CSR groups of coincident points
 * (start: n_groups+1 offsets, members: point indices; device arrays) — dssum followed by vmult on
 * one rank (:339-340). */
int nkv_mth_rand_add(const nkv_layout* L, int lx1, int ly1, int lz1, int64_t e_first, const double* xm,
                     const double* ym, const double* zm, double fc1, double fc2, double fc3, double* q,
                     void* stream);
int nkv_group_average(int64_t n_groups, const int64_t* start, const int64_t* members, double* q, void* stream);
/* add_symmetric_seed's perturbation (utils.f90:361-406, 3-D): qx = cos(alpha z) sin(2 pi y),
 * qz = -(2 pi)/alpha cos(alpha z) cos(2 pi y), qt = cos(alpha z) cos(2 pi y) on n_v points (qy is
 * left alone, as the reference does); alpha = 2 pi / (zmax - zmin).  The amplitude scaling
 * 1e-6 / (0.5 sum glsc3(q, bm1, q)) is the host's (two dots and a scal). */
int nkv_symmetric_seed(const nkv_layout* L, const double* ym, const double* zm, double alpha, double* qx,
                       double* qz, double* qt, void* stream);

/* ---- ts_gmres host helper (a17, newton_krylov.f90:250-269) -------------------------------
 * The least-squares residual ||beta e_1 - H(1:k+2, 1:k+1) y|| after one more Hessenberg column, in
 * O(k) host work (Givens rotations; no device work, no stream).  h: H(0:k+1, k) (0-based column k,
 * overwritten with its triangularised form), cs/sn: the k rotations so far (the new one appended at
 * index k), g: k+2 doubles, g[0] = beta before the first column.  The reference solves the whole
 * system with dgels at every column for this number (:255-258); y itself still comes from dgels on
 * the final system.  k < 0 or a NULL array: returns NaN (message in nkv_last_error). */
double nkv_givens_column(int k, double* h, double* cs, double* sn, double* g);

/* ---- "mgs2-lagged" host algebra (a7 for non-orthonormal bases: the noise / load seed's unnormalised
 * Q(1), eigensolvers.f90:192-223; update_hessenberg_matrix's two MGS passes, krylov_decomposition.f90:
 * 155-186) -------------------------------------------------------------------------------------
 * MGS2's coefficients alpha = (I + L)^-1 Q^T W f for ANY basis (L the strictly lower part of the Gram
 * matrix G), with the second pass of a column lagged into the next step's two-vector multi-dot as
 * DCGS2 does: one multi-dot and one nkv_dcgs2_update per step.  Host-only, no device work.  G:
 * row-major (ldg >= c+1), symmetric; H: column-major (ldh >= c+1), both host memory, updated in place.
 * stage 1 (first step of a factorisation, Q[c] final), 0 (Q[c] holds the previous step's first-pass
 * result u; NKV_ENAN when u has no new direction), 2 (closing pass of the last column).  hv: the
 * step's all-reduced multi-dot (stage 0/1: nkv_block_dot2 with x = Q[c], NKV_X_IS_LAST; stage 2:
 * nkv_block_dot of Q[c] against Q[0:c+1]).  coef: 3c+5 doubles in nkv_dcgs2_update's layout
 * (stage 2: coef[0:c] = the second pass's coefficients, for nkv_block_update).  The algebra in full:
 * drivers.hip; nkv_arnoldi_factorization with NKV_MGS_LAGGED runs the whole sequence. */
int nkv_lagged_coef(int c, int stage, const double* hv, double* G, int64_t ldg, double* H, int64_t ldh,
                    double* coef);

/* ---- shard-independent synthetic data ----------------------------------------------------
 * x[row] = 2*u - 1, u = hash(seed, field, global point) in [0,1) with 53 exact bits, for live
 * rows; padding rows = 0; time = 0.  Global point of local point i in a weighted field is
 * v_offset + i, in pressure p_offset + i (element-contiguous shards).  Bit-identical to the
 * oracle's generator for every shard split. */
int nkv_fill_hash(const nkv_layout* L, double* x, uint64_t seed, int64_t v_offset, int64_t p_offset,
                  void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NEKKRYLOV_H */
