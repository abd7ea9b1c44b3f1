! nkv_bindings.f90 — the Fortran side of the drop-in boundary: the bind(C) interface a nekStab
! maintainer adds (INTEGRATION.md §2) to call include/nekkrylov.h from core/krylov_*.f90, plus the
! few HIP runtime calls a host needs for device memory.  Compiled with amdflang and exercised by
! arnoldi_f.f90 (tests/test_gpu_kernels.py::test_fortran_host_example_runs).
module nkv_bindings
   use iso_c_binding
   implicit none

   integer(c_int), parameter :: NKV_OK = 0, NKV_TILE = 4096
   integer(c_int), parameter :: NKV_TIME = 1, NKV_NORM2 = 8, NKV_OVERWRITE = 4, NKV_TIME_DOT = 16
   integer(c_int), parameter :: NKV_MGS_ICWY = 256
   integer(c_int), parameter :: NKV_MGS_LAGGED = 512
   integer(c_int), parameter :: NKV_X_IS_LAST = 32, NKV_MGS2 = 64, NKV_CHECK_BREAKDOWN = 128
   integer(c_int), parameter :: NKV_ECALLBACK = 5, NKV_EBREAKDOWN = 6

   type, bind(C) :: nkv_layout
      integer(c_int64_t) :: n_v, n_p, sv, sp, ld
      integer(c_int32_t) :: n_wf, rank0
   end type nkv_layout

   interface
      integer(c_int) function nkv_abi_version() bind(C, name="nkv_abi_version")
         import :: c_int
      end function
      integer(c_int) function nkv_layout_init(L, ldim, lx1, lx2, nelv, nelt, n_scalars, ifpo, rank0) &
         bind(C, name="nkv_layout_init")
         import :: c_int, c_int64_t, nkv_layout
         type(nkv_layout), intent(out) :: L
         integer(c_int), value :: ldim, lx1, lx2, n_scalars, ifpo, rank0
         integer(c_int64_t), value :: nelv, nelt
      end function
      type(c_ptr) function nkv_last_error() bind(C, name="nkv_last_error")
         import :: c_ptr
      end function
      integer(c_size_t) function nkv_workspace_bytes(L, max_cols) bind(C, name="nkv_workspace_bytes")
         import :: c_size_t, c_int, nkv_layout
         type(nkv_layout), intent(in) :: L
         integer(c_int), value :: max_cols
      end function
      integer(c_int) function nkv_check_status(ws, stream) bind(C, name="nkv_check_status")
         import :: c_int, c_ptr
         type(c_ptr), value :: ws, stream
      end function
      integer(c_int) function nkv_fill_hash(L, x, seed, voff, poff, stream) bind(C, name="nkv_fill_hash")
         import :: c_int, c_ptr, c_int64_t, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: x, stream
         integer(c_int64_t), value :: seed, voff, poff
      end function
      integer(c_int) function nkv_op_diag(L, d, x, y, ts, stream) bind(C, name="nkv_op_diag")
         import :: c_int, c_ptr, c_double, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: d, x, y, stream
         real(c_double), value :: ts
      end function
      integer(c_int) function nkv_dot(L, w, a, b, out, ws, flags, stream) bind(C, name="nkv_dot")
         import :: c_int, c_ptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: w, a, b, out, ws, stream
         integer(c_int), value :: flags
      end function
      integer(c_int) function nkv_normalize_dev(L, x, nrm2, beta, flags, stream) bind(C, name="nkv_normalize_dev")
         import :: c_int, c_ptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: x, nrm2, beta, stream
         integer(c_int), value :: flags
      end function
      integer(c_int) function nkv_copy(L, dst, src, flags, stream) bind(C, name="nkv_copy")
         import :: c_int, c_ptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: dst, src, stream
         integer(c_int), value :: flags
      end function
      integer(c_int) function nkv_axpby(L, x, a, y, b, flags, stream) bind(C, name="nkv_axpby")
         import :: c_int, c_ptr, c_double, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: x, y, stream
         real(c_double), value :: a, b
         integer(c_int), value :: flags
      end function
      integer(c_int) function nkv_combine(L, Q, k, y, out, flags, stream) bind(C, name="nkv_combine")
         import :: c_int, c_ptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: Q, y, out, stream
         integer(c_int), value :: k, flags
      end function
      real(c_double) function nkv_givens_column(k, h, cs, sn, g) bind(C, name="nkv_givens_column")
         import :: c_int, c_double
         integer(c_int), value :: k
         real(c_double), intent(inout) :: h(*), cs(*), sn(*), g(*)
      end function
      integer(c_int) function nkv_block_dot(L, w, Q, j, f, h, ws, flags, stream) bind(C, name="nkv_block_dot")
         import :: c_int, c_ptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: w, Q, f, h, ws, stream
         integer(c_int), value :: j, flags
      end function
      integer(c_int) function nkv_block_update(L, w, Q, j, h, f, nrm2, ws, flags, stream) &
            bind(C, name="nkv_block_update")
         import :: c_int, c_ptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: w, Q, h, f, nrm2, ws, stream
         integer(c_int), value :: j, flags
      end function
      integer(c_int) function nkv_block_dot2(L, w, Q, j, x, y, h, ws, flags, stream) bind(C, name="nkv_block_dot2")
         import :: c_int, c_ptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: w, Q, x, y, h, ws, stream
         integer(c_int), value :: j, flags
      end function
      integer(c_int) function nkv_dcgs2_coef(m, hq, hw, nrm_prev, H, ldh, coef, ws, stream) &
            bind(C, name="nkv_dcgs2_coef")
         import :: c_int, c_ptr, c_int64_t
         integer(c_int), value :: m
         type(c_ptr), value :: hq, hw, nrm_prev, H, coef, ws, stream
         integer(c_int64_t), value :: ldh
      end function
      integer(c_int) function nkv_dcgs2_update(L, w, Q, m, coef, qj, win, fout, nrm2, ws, flags, stream) &
            bind(C, name="nkv_dcgs2_update")
         import :: c_int, c_ptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: w, Q, coef, qj, win, fout, nrm2, ws, stream
         integer(c_int), value :: m, flags
      end function
      ! the whole DCGS2 factorisation in one call (replaces `call arnoldi_factorization(...)`);
      ! matvec / allreduce are c_funloc's of bind(C) procedures (allreduce: c_null_funptr on one rank)
      integer(c_size_t) function nkv_arnoldi_scratch_doubles(m) bind(C, name="nkv_arnoldi_scratch_doubles")
         import :: c_size_t, c_int
         integer(c_int), value :: m
      end function
      integer(c_int) function nkv_arnoldi_dcgs2(L, w, Q, mstart, mend, H, ldh, f, scratch, ws, matvec, mv_user, &
            allreduce, ar_user, flags, stream) bind(C, name="nkv_arnoldi_dcgs2")
         import :: c_int, c_int64_t, c_ptr, c_funptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: w, Q, H, f, scratch, ws, mv_user, ar_user, stream
         integer(c_int), value :: mstart, mend, flags
         integer(c_int64_t), value :: ldh
         type(c_funptr), value :: matvec, allreduce
      end function
      ! ts_gmres's inner loop (newton_krylov.f90:250-276) as one call: k_out columns, res_hist(1:k_out) the
      ! per-column least-squares residuals; the host then calls lstsq (dgels) on H and nkv_combine
      integer(c_int) function nkv_gmres_dcgs2(L, w, Q, kmax, beta, tol2, H, ldh, f, scratch, ws, matvec, mv_user, &
            allreduce, ar_user, res_hist, k_out, flags, stream) bind(C, name="nkv_gmres_dcgs2")
         import :: c_int, c_int64_t, c_double, c_ptr, c_funptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: w, Q, H, f, scratch, ws, mv_user, ar_user, stream
         integer(c_int), value :: kmax, flags
         real(c_double), value :: beta, tol2
         integer(c_int64_t), value :: ldh
         type(c_funptr), value :: matvec, allreduce
         real(c_double), intent(out) :: res_hist(*)
         integer(c_int), intent(out) :: k_out
      end function
      ! per-column factorisation (CGS2, or the reference's MGS2 order with NKV_MGS2): same arguments
      integer(c_int) function nkv_arnoldi_factorization(L, w, Q, mstart, mend, H, ldh, f, scratch, ws, matvec, &
            mv_user, allreduce, ar_user, flags, stream) bind(C, name="nkv_arnoldi_factorization")
         import :: c_int, c_int64_t, c_ptr, c_funptr, nkv_layout
         type(nkv_layout), intent(in) :: L
         type(c_ptr), value :: w, Q, H, f, scratch, ws, mv_user, ar_user, stream
         integer(c_int), value :: mstart, mend, flags
         integer(c_int64_t), value :: ldh
         type(c_funptr), value :: matvec, allreduce
      end function
      ! HIP runtime (device memory for the host's arrays)
      integer(c_int) function hipMalloc(p, bytes) bind(C, name="hipMalloc")
         import :: c_int, c_ptr, c_size_t
         type(c_ptr) :: p
         integer(c_size_t), value :: bytes
      end function
      integer(c_int) function hipMemset(p, v, bytes) bind(C, name="hipMemset")
         import :: c_int, c_ptr, c_size_t
         type(c_ptr), value :: p
         integer(c_int), value :: v
         integer(c_size_t), value :: bytes
      end function
      integer(c_int) function hipMemcpy(dst, src, bytes, kind) bind(C, name="hipMemcpy")
         import :: c_int, c_ptr, c_size_t
         type(c_ptr), value :: dst, src
         integer(c_size_t), value :: bytes
         integer(c_int), value :: kind
      end function
      integer(c_int) function hipDeviceSynchronize() bind(C, name="hipDeviceSynchronize")
         import :: c_int
      end function
   end interface

   integer(c_int), parameter :: hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2

contains

   ! address of column c (0-based) of a basis with leading dimension ld doubles
   type(c_ptr) function col(Q, c, ld)
      type(c_ptr), intent(in) :: Q
      integer, intent(in) :: c
      integer(c_int64_t), intent(in) :: ld
      integer(c_intptr_t) :: a
      a = transfer(Q, a) + int(c, c_intptr_t)*ld*8_c_intptr_t
      col = transfer(a, col)
   end function col

   type(c_ptr) function off(p, n)   ! p + n doubles
      type(c_ptr), intent(in) :: p
      integer, intent(in) :: n
      integer(c_intptr_t) :: a
      a = transfer(p, a) + int(n, c_intptr_t)*8_c_intptr_t
      off = transfer(a, off)
   end function off

   subroutine ck(rc, what)
      integer(c_int), intent(in) :: rc
      character(len=*), intent(in) :: what
      if (rc /= 0) then
         print *, 'FAILED: ', what, ' rc=', rc
         stop 1
      end if
   end subroutine ck
end module nkv_bindings
