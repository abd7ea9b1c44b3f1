! arnoldi_f.f90 — a Fortran host (the reference's language) running DCGS2 Arnoldi through the C ABI:
! the replacement of arnoldi_factorization / update_hessenberg_matrix (krylov_decomposition.f90)
! by the loop of INTEGRATION.md §2b on one rank (gop = identity), then W-orthonormality and the
! Arnoldi relation A Q_m = Q_{m+1} H checked through the same calls; then ts_gmres
! (newton_krylov.f90:241-294) with its inner loop as ONE library call (nkv_gmres_dcgs2): restarts,
! the small least-squares problem on the host (Givens + back substitution here; the reference's
! lstsq/dgels in nekStab), x += Q y with nkv_combine; then an unnormalised Q(1) (the default noise
! seed) through nkv_arnoldi_factorization with NKV_MGS2, NKV_MGS_ICWY and NKV_MGS_LAGGED.   usage: arnoldi_f [E [m]]
module diag_callback
   ! the operator handed to nkv_arnoldi_dcgs2 as a callback: y = d .* x on the library's stream
   use iso_c_binding
   use nkv_bindings
   implicit none
   type(nkv_layout), save :: Lcb
   type(c_ptr), save :: dcb
contains
   integer(c_int) function diag_mv(user, x, y, stream) bind(C)
      type(c_ptr), value :: user, x, y, stream
      diag_mv = nkv_op_diag(Lcb, dcb, x, y, 0.0d0, stream)
   end function diag_mv
end module diag_callback

program arnoldi_f
   use iso_c_binding
   use nkv_bindings
   use diag_callback
   implicit none
   type(nkv_layout), target :: L
   type(c_ptr) :: Q, f, d, w, Hdev, hv, coef, nrm, hcol, ws, st, u, Q2, H2dev, scr
   real(c_double), allocatable, target :: H2(:, :), qa(:), qb(:)
   logical :: same
   integer :: E, m, j, c, r, nargs
   character(len=32) :: arg
   integer(c_size_t) :: vbytes, wsb
   real(c_double), allocatable, target :: hw(:), H(:, :), g(:), dh(:)
   real(c_double), target :: r2
   real(c_double) :: orth, arn, hmax
   logical :: gm_ok, mg_ok

   E = 512; m = 24
   nargs = command_argument_count()
   if (nargs >= 1) then; call get_command_argument(1, arg); read (arg, *) E; end if
   if (nargs >= 2) then; call get_command_argument(2, arg); read (arg, *) m; end if
   st = c_null_ptr                              ! the null (default) stream

   if (nkv_abi_version() /= 3) stop 'ABI mismatch'
   ! 3-D lx1=8 / lx2=6, one dotted scalar (nelt = nelv), pressure stored, this rank owns `time`
   call ck(nkv_layout_init(L, 3, 8, 6, int(E, c_int64_t), int(E, c_int64_t), 1, 1, 1), 'layout')

   vbytes = int(L%ld, c_size_t)*8
   call ck(hipMalloc(Q, (m + 1)*vbytes), 'hipMalloc Q')
   call ck(hipMalloc(f, vbytes), 'hipMalloc f')
   call ck(hipMalloc(d, vbytes), 'hipMalloc d')
   call ck(hipMalloc(w, int(L%sv, c_size_t)*8), 'hipMalloc w')
   call ck(hipMalloc(Hdev, int(m*(m + 1), c_size_t)*8), 'hipMalloc H')
   call ck(hipMalloc(hv, int(2*(m + 1), c_size_t)*8), 'hipMalloc h')
   call ck(hipMalloc(coef, int(3*m + 8, c_size_t)*8), 'hipMalloc coef')
   call ck(hipMalloc(nrm, 64_c_size_t), 'hipMalloc nrm')
   call ck(hipMalloc(hcol, int(m + 2, c_size_t)*8), 'hipMalloc hcol')
   wsb = nkv_workspace_bytes(L, m + 1)
   call ck(hipMalloc(ws, wsb), 'hipMalloc ws')
   call ck(hipMemset(ws, 0, wsb), 'memset ws')
   call ck(hipMemset(Q, 0, (m + 1)*vbytes), 'memset Q')
   call ck(hipMemset(Hdev, 0, int(m*(m + 1), c_size_t)*8), 'memset H')

   allocate (hw(L%sv), dh(L%ld), H(m + 1, m), g(m + 1))
   hw = 0.0d0; hw(1:L%n_v) = 1.0d0                          ! bm1s: 1 on live points
   call ck(hipMemcpy(w, c_loc(hw), int(L%sv, c_size_t)*8, hipMemcpyHostToDevice), 'w')
   call ck(nkv_fill_hash(L, d, 99_c_int64_t, 0_c_int64_t, 0_c_int64_t, st), 'hash d')
   call ck(hipMemcpy(c_loc(dh), d, vbytes, hipMemcpyDeviceToHost), 'd down')
   dh = 0.525d0 + 0.475d0*dh                                 ! diag in (0.05, 1)
   call ck(hipMemcpy(d, c_loc(dh), vbytes, hipMemcpyHostToDevice), 'd up')

   call ck(nkv_fill_hash(L, Q, 11_c_int64_t, 0_c_int64_t, 0_c_int64_t, st), 'seed')
   call ck(nkv_dot(L, w, Q, Q, nrm, ws, 0, st), 'seed norm')
   call ck(nkv_normalize_dev(L, Q, nrm, c_null_ptr, 0, st), 'normalise')

   do j = 1, m
      u = col(Q, j - 1, L%ld)
      call ck(nkv_op_diag(L, d, u, f, 0.0d0, st), 'matvec')
      call ck(nkv_block_dot2(L, w, Q, j, u, f, hv, ws, NKV_X_IS_LAST, st), 'block_dot2')
      if (j == 1) then
         call ck(nkv_dcgs2_coef(j - 1, hv, off(hv, j), c_null_ptr, Hdev, int(m + 1, c_int64_t), coef, ws, st), 'coef')
      else
         call ck(nkv_dcgs2_coef(j - 1, hv, off(hv, j), off(hv, j - 1), Hdev, int(m + 1, c_int64_t), coef, ws, st), 'coef')
      end if
      call ck(nkv_dcgs2_update(L, w, Q, j - 1, coef, u, f, col(Q, j, L%ld), c_null_ptr, ws, NKV_TIME, st), 'update')
   end do
   u = col(Q, m, L%ld)
   call ck(nkv_block_dot(L, w, Q, m + 1, u, hv, ws, 0, st), 'close dot')
   call ck(nkv_dcgs2_coef(m, hv, c_null_ptr, off(hv, m), Hdev, int(m + 1, c_int64_t), coef, ws, st), 'close coef')
   call ck(nkv_block_update(L, w, Q, m, hv, u, c_null_ptr, ws, NKV_TIME, st), 'close update')
   call ck(nkv_normalize_dev(L, u, off(coef, 2*m + 3), c_null_ptr, 0, st), 'close normalise')
   call ck(nkv_check_status(ws, st), 'NaN check')
   call ck(hipMemcpy(c_loc(H), Hdev, int(m*(m + 1), c_size_t)*8, hipMemcpyDeviceToHost), 'H down')

   orth = 0.0d0
   do c = 0, m
      call ck(nkv_block_dot(L, w, Q, m + 1, col(Q, c, L%ld), hv, ws, 0, st), 'gram')
      call ck(hipMemcpy(c_loc(g), hv, int(m + 1, c_size_t)*8, hipMemcpyDeviceToHost), 'g down')
      do r = 0, m
         if (r == c) then
            orth = max(orth, abs(g(r + 1) - 1.0d0))
         else
            orth = max(orth, abs(g(r + 1)))
         end if
      end do
   end do
   hmax = maxval(abs(H)); arn = 0.0d0
   do c = 0, m - 1, max(1, m/4)
      call ck(nkv_op_diag(L, d, col(Q, c, L%ld), f, 0.0d0, st), 'matvec')
      call ck(hipMemcpy(hcol, c_loc(H(1, c + 1)), int(c + 2, c_size_t)*8, hipMemcpyHostToDevice), 'hcol')
      call ck(nkv_block_update(L, w, Q, c + 2, hcol, f, nrm, ws, NKV_NORM2, st), 'residual')
      call ck(hipMemcpy(c_loc(r2), nrm, 8_c_size_t, hipMemcpyDeviceToHost), 'r2')
      arn = max(arn, sqrt(abs(r2)))
   end do
   print '(a,i0,a,i0,a,es10.3,a,es10.3,a,es14.6)', 'arnoldi_f: N=', L%n_wf*L%n_v + L%n_p, ' m=', m, &
      '  max|Q^T W Q - I| = ', orth, '  max||A q - Q h||/max|H| = ', arn/hmax, '  H(m+1,m) = ', H(m + 1, m)
   ! the same factorisation as ONE native call, the operator a Fortran callback: bit-identical
   call ck(hipMalloc(Q2, (m + 1)*vbytes), 'hipMalloc Q2')
   call ck(hipMalloc(H2dev, int(m*(m + 1), c_size_t)*8), 'hipMalloc H2')
   call ck(hipMalloc(scr, nkv_arnoldi_scratch_doubles(int(m, c_int))*8), 'hipMalloc scratch')
   call ck(hipMemset(Q2, 0, (m + 1)*vbytes), 'memset Q2')
   call ck(hipMemset(H2dev, 0, int(m*(m + 1), c_size_t)*8), 'memset H2')
   call ck(nkv_fill_hash(L, Q2, 11_c_int64_t, 0_c_int64_t, 0_c_int64_t, st), 'seed 2')
   call ck(nkv_dot(L, w, Q2, Q2, nrm, ws, 0, st), 'seed norm 2')
   call ck(nkv_normalize_dev(L, Q2, nrm, c_null_ptr, 0, st), 'normalise 2')
   Lcb = L; dcb = d
   call ck(nkv_arnoldi_dcgs2(L, w, Q2, 1, int(m, c_int), H2dev, int(m + 1, c_int64_t), f, scr, ws, &
                             c_funloc(diag_mv), c_null_ptr, c_null_funptr, c_null_ptr, 0, st), 'arnoldi_dcgs2')
   allocate (H2(m + 1, m), qa(L%ld), qb(L%ld))
   call ck(hipMemcpy(c_loc(H2), H2dev, int(m*(m + 1), c_size_t)*8, hipMemcpyDeviceToHost), 'H2 down')
   same = all(H2 == H)
   do c = 0, m
      call ck(hipMemcpy(c_loc(qa), col(Q, c, L%ld), vbytes, hipMemcpyDeviceToHost), 'q down')
      call ck(hipMemcpy(c_loc(qb), col(Q2, c, L%ld), vbytes, hipMemcpyDeviceToHost), 'q2 down')
      same = same .and. all(qa == qb)
   end do
   if (same) then
      print '(a)', 'arnoldi_f: nkv_arnoldi_dcgs2 (one call, Fortran callback) equals the step-by-step loop bit for bit'
   else
      print '(a)', 'arnoldi_f: nkv_arnoldi_dcgs2 DIFFERS from the step-by-step loop'
   end if
   call gmres_leg(gm_ok)
   call mgs_leg(mg_ok)
   if (orth < 1.0d-12 .and. arn/hmax < 1.0d-12 .and. same .and. gm_ok .and. mg_ok) then
      print '(a)', 'arnoldi_f: OK'
   else
      print '(a)', 'arnoldi_f: FAILED'
      stop 1
   end if
contains

   subroutine mgs_leg(ok)
      ! the in-tree solver's default noise seed leaves Q(1) unnormalised (eigensolvers.f90:192-203):
      ! only modified Gram-Schmidt reproduces the reference there.  nkv_arnoldi_factorization with
      ! NKV_MGS2 (the reference's per-column order), with NKV_MGS_ICWY (inverse compact WY form,
      ! three reads of Q per step) and with NKV_MGS_LAGGED (the second pass lagged into the next
      ! multi-dot, two reads) must agree to rounding.
      logical, intent(out) :: ok
      type(c_ptr) :: Qa, Qb, Qc, Ha, Hb, Hc, sc
      real(c_double), allocatable, target :: Hah(:, :), Hbh(:, :), Hch(:, :)
      real(c_double) :: dmax, dmaxl
      integer :: mm
      mm = min(m, 16)
      call ck(hipMalloc(Qa, (mm + 1)*vbytes), 'hipMalloc Qa')
      call ck(hipMalloc(Qb, (mm + 1)*vbytes), 'hipMalloc Qb')
      call ck(hipMalloc(Ha, int(mm*(mm + 1), c_size_t)*8), 'hipMalloc Ha')
      call ck(hipMalloc(Hb, int(mm*(mm + 1), c_size_t)*8), 'hipMalloc Hb')
      call ck(hipMalloc(Qc, (mm + 1)*vbytes), 'hipMalloc Qc')
      call ck(hipMalloc(Hc, int(mm*(mm + 1), c_size_t)*8), 'hipMalloc Hc')
      call ck(hipMemset(Hc, 0, int(mm*(mm + 1), c_size_t)*8), 'memset Hc')
      call ck(hipMalloc(sc, nkv_arnoldi_scratch_doubles(int(mm, c_int))*8), 'hipMalloc scratch')
      call ck(hipMemset(Ha, 0, int(mm*(mm + 1), c_size_t)*8), 'memset Ha')
      call ck(hipMemset(Hb, 0, int(mm*(mm + 1), c_size_t)*8), 'memset Hb')
      call ck(nkv_fill_hash(L, Qb, 7_c_int64_t, 0_c_int64_t, 0_c_int64_t, st), 'seed')
      call ck(nkv_dot(L, w, Qb, Qb, nrm, ws, 0, st), 'seed norm')
      call ck(nkv_normalize_dev(L, Qb, nrm, c_null_ptr, 0, st), 'normalise')
      call ck(nkv_op_diag(L, d, Qb, Qa, 0.0d0, st), 'A seed')                  ! Q(1) = A s/||s||
      call ck(nkv_op_diag(L, d, Qb, Qb, 0.0d0, st), 'A seed (in place)')
      call ck(nkv_copy(L, Qc, Qb, NKV_TIME, st), 'seed copy')
      call ck(nkv_arnoldi_factorization(L, w, Qa, 1, int(mm, c_int), Ha, int(mm + 1, c_int64_t), f, sc, ws, &
                                        c_funloc(diag_mv), c_null_ptr, c_null_funptr, c_null_ptr, NKV_MGS2, st), 'mgs2')
      call ck(nkv_arnoldi_factorization(L, w, Qb, 1, int(mm, c_int), Hb, int(mm + 1, c_int64_t), f, sc, ws, &
                                        c_funloc(diag_mv), c_null_ptr, c_null_funptr, c_null_ptr, NKV_MGS_ICWY, st), 'icwy')
      call ck(nkv_arnoldi_factorization(L, w, Qc, 1, int(mm, c_int), Hc, int(mm + 1, c_int64_t), f, sc, ws, &
                                        c_funloc(diag_mv), c_null_ptr, c_null_funptr, c_null_ptr, NKV_MGS_LAGGED, st), &
              'lagged')
      call ck(nkv_check_status(ws, st), 'NaN check')
      allocate (Hah(mm + 1, mm), Hbh(mm + 1, mm), Hch(mm + 1, mm))
      call ck(hipMemcpy(c_loc(Hah), Ha, int(mm*(mm + 1), c_size_t)*8, hipMemcpyDeviceToHost), 'Ha down')
      call ck(hipMemcpy(c_loc(Hbh), Hb, int(mm*(mm + 1), c_size_t)*8, hipMemcpyDeviceToHost), 'Hb down')
      call ck(hipMemcpy(c_loc(Hch), Hc, int(mm*(mm + 1), c_size_t)*8, hipMemcpyDeviceToHost), 'Hc down')
      dmax = maxval(abs(Hah - Hbh))/maxval(abs(Hah))
      dmaxl = maxval(abs(Hah - Hch))/maxval(abs(Hah))
      print '(a,i0,a,es10.3,a,es10.3)', 'arnoldi_f: unnormalised Q(1), ', mm, &
         ' MGS2 steps: max|H - H(NKV_MGS2)|/max|H| = ', dmax, ' (NKV_MGS_ICWY), ', dmaxl
      print '(a)', 'arnoldi_f:   (NKV_MGS_LAGGED, two reads of Q per step)'
      ok = dmax < 1.0d-12 .and. dmaxl < 1.0d-12
   end subroutine mgs_leg

   subroutine gmres_leg(ok)
      ! ts_gmres: Q(:,1) = r/||r||; inner loop = nkv_gmres_dcgs2; y = argmin ||beta e1 - H y||;
      ! x += Q y; r = b - A x (initialize_gmres_vector); 3 restarts of m columns
      logical, intent(out) :: ok
      type(c_ptr) :: b, x, dq, rv, yd, Qg, Hg
      real(c_double), allocatable, target :: Hh(:, :), res(:), y(:), cs(:), sn(:), gv(:), Rm(:, :)
      real(c_double), target :: bb
      real(c_double) :: beta, bnorm, lsres, v, last_res
      integer(c_int), target :: k
      integer :: it, cc, rr
      call ck(hipMalloc(b, vbytes), 'b'); call ck(hipMalloc(x, vbytes), 'x')
      call ck(hipMalloc(dq, vbytes), 'dq'); call ck(hipMalloc(rv, vbytes), 'r')
      call ck(hipMalloc(yd, int(m, c_size_t)*8), 'yd')
      call ck(hipMalloc(Qg, (m + 1)*vbytes), 'Qg'); call ck(hipMalloc(Hg, int(m*(m + 1), c_size_t)*8), 'Hg')
      call ck(hipMemset(b, 0, vbytes), 'b0'); call ck(hipMemset(x, 0, vbytes), 'x0')
      call ck(hipMemset(Qg, 0, (m + 1)*vbytes), 'Q0')
      allocate (Hh(m + 1, m), res(m), y(m), cs(m + 2), sn(m + 2), gv(m + 2), Rm(m + 2, m))
      call ck(nkv_fill_hash(L, b, 3_c_int64_t, 0_c_int64_t, 0_c_int64_t, st), 'rhs')
      call ck(nkv_copy(L, rv, b, NKV_TIME, st), 'r = b')                        ! x = 0: r = b
      call ck(nkv_dot(L, w, b, b, nrm, ws, 0, st), 'rhs norm')
      call ck(hipMemcpy(c_loc(bb), nrm, 8_c_size_t, hipMemcpyDeviceToHost), 'bb')
      bnorm = sqrt(bb); beta = bnorm
      Lcb = L; dcb = d
      do it = 1, 3
         call ck(nkv_copy(L, Qg, rv, NKV_TIME, st), 'Q(1) = r')
         call ck(nkv_dot(L, w, Qg, Qg, nrm, ws, 0, st), 'r norm')
         call ck(nkv_normalize_dev(L, Qg, nrm, c_null_ptr, 0, st), 'Q(1) = r/|r|')
         call ck(hipMemset(Hg, 0, int(m*(m + 1), c_size_t)*8), 'H0')
         call ck(nkv_gmres_dcgs2(L, w, Qg, int(m, c_int), beta, 1.0d-30, Hg, int(m + 1, c_int64_t), f, scr, ws, &
                                 c_funloc(diag_mv), c_null_ptr, c_null_funptr, c_null_ptr, res, k, 0, st), 'gmres')
         call ck(hipMemcpy(c_loc(Hh), Hg, int(m*(m + 1), c_size_t)*8, hipMemcpyDeviceToHost), 'H down')
         cs = 0; sn = 0; gv = 0; gv(1) = beta; Rm = 0
         do cc = 1, k
            Rm(1:cc + 1, cc) = Hh(1:cc + 1, cc)
            lsres = nkv_givens_column(int(cc - 1, c_int), Rm(1, cc), cs, sn, gv)
         end do
         do rr = k, 1, -1
            v = gv(rr)
            do cc = rr + 1, k
               v = v - Rm(rr, cc)*y(cc)
            end do
            y(rr) = v/Rm(rr, rr)
         end do
         call ck(hipMemcpy(yd, c_loc(y), int(k, c_size_t)*8, hipMemcpyHostToDevice), 'y up')
         call ck(nkv_combine(L, Qg, k, yd, dq, NKV_TIME, st), 'dq = Q y')             ! k_matmul
         call ck(nkv_axpby(L, x, 1.0d0, dq, 1.0d0, NKV_TIME, st), 'x += dq')         ! k_add2
         call ck(nkv_op_diag(L, d, x, rv, 0.0d0, st), 'A x')                          ! initialize_gmres_vector
         call ck(nkv_axpby(L, rv, -1.0d0, b, 1.0d0, NKV_TIME, st), 'r = b - A x')
         call ck(nkv_dot(L, w, rv, rv, nrm, ws, 0, st), 'residual')
         call ck(hipMemcpy(c_loc(bb), nrm, 8_c_size_t, hipMemcpyDeviceToHost), 'res down')
         last_res = res(k); beta = sqrt(bb)
         print '(a,i0,a,i0,a,es10.3,a,es10.3,a,es10.3)', 'arnoldi_f: gmres restart ', it, ': ', k, &
            ' columns, reported ', last_res, ', least-squares ', lsres, ', ||b - A x||_W ', beta
      end do
      ok = abs(beta - lsres) <= 1.0d-10*bnorm .and. beta < 1.0d-6*bnorm
   end subroutine gmres_leg
end program arnoldi_f
