!! poissbox_gpu.f90 -- Fortran (iso_c_binding) host interface to libpoissbox_gpu.so.
!
! Mirrors the reference's Fortran/PETSc API so a poissbox driver switches by changing its `use`
! lines. Reference -> here:
!   tDM / tMat / tVec / tKSP handles (PETSc)         -> type(tDM) / type(tMat) / type(tVec) / type(tKSP)
!   initialise_grid(nglobal, da)        (src/poissbox.f90:183-204)  -> same name and arguments
!   initialise_linear_system(da, ctx, P, A, x, b) (:206-240)        -> same (ctx = mat_ctx)
!   solve(P, A, x, b)                   (:269-298)                   -> same, options from argv
!   mfmult / MatMult(A, x, f, ierr)     (:300-322)                   -> MatMult(A, x, f, ierr)
!   compute_lapl_pointwise(da, grid_deltas, x, b) (:84-126)          -> same
!   DMDAGetCorners, VecDuplicate, VecCopy, VecAXPY, VecNorm, VecSum, VecSet, VecDestroy,
!   DMDAVecGetArrayF90 (copy-out form: VecGetValues / VecSetValues)
! Every routine returns ierr (0 = success) as the last argument, PETSc style; unlike the
! reference, ierr is always set.
module poissbox_gpu

  use iso_c_binding

  implicit none

  private

  integer, parameter, public :: pb_dp = c_double

  type, public :: tDM
     type(c_ptr) :: h = c_null_ptr
  end type tDM
  type, public :: tMat
     type(c_ptr) :: h = c_null_ptr
  end type tMat
  type, public :: tVec
     type(c_ptr) :: h = c_null_ptr
  end type tVec
  type, public :: tKSP
     type(c_ptr) :: h = c_null_ptr
  end type tKSP

  !! Shell-matrix context of the reference (src/poissbox.f90:17-20)
  type, public :: mat_ctx
     type(tDM) :: da
     real(pb_dp), dimension(3) :: grid_deltas
  end type mat_ctx

  type, bind(C), public :: pb_ksp_opts
     real(c_double) :: rtol, atol, dtol
     integer(c_int64_t) :: max_it
     integer(c_int) :: ksp_type, pc_type, nullspace, monitor, converged_reason, check_every
     integer(c_int) :: mg_levels, mg_coarse_its
     real(c_double) :: sor_omega
  end type pb_ksp_opts

  type, bind(C), public :: pb_ksp_result
     integer(c_int) :: reason
     integer(c_int64_t) :: its
     real(c_double) :: rnorm, rnorm0
     integer(c_int64_t) :: nhist  ! residual norms logged (its + 1; its after a breakdown exit)
  end type pb_ksp_result

  integer(c_int), parameter, public :: PB_OP_STAR7 = 0, PB_OP_COMPACT = 1, PB_OP_ASSEMBLED27 = 2

  type(c_ptr), save :: g_ctx = c_null_ptr  ! one context per process (one GPU), like PETSC_COMM_WORLD

  public :: PoissboxInitialize, PoissboxFinalize
  public :: initialise_grid, initialise_linear_system, solve, compute_lapl_pointwise
  public :: DMDAGetCorners, MatMult, MatDestroy, MatGetOwnershipRange, VecGetOwnershipRange
  public :: VecDuplicate, VecCopy, VecAXPY, VecNorm, VecSum, VecSet, VecDestroy
  public :: VecSetRandom, VecGetValues, VecSetValues, pb_error_string

  interface
     integer(c_int) function c_pb_ctx_create(device, rank, nranks, uid, ctx) bind(C, name="pb_ctx_create")
       import :: c_int, c_ptr
       integer(c_int), value :: device, rank, nranks
       type(c_ptr), value :: uid
       type(c_ptr) :: ctx
     end function
     integer(c_int) function c_pb_ctx_destroy(ctx) bind(C, name="pb_ctx_destroy")
       import :: c_int, c_ptr
       type(c_ptr), value :: ctx
     end function
     type(c_ptr) function c_pb_last_error() bind(C, name="pb_last_error")
       import :: c_ptr
     end function
     integer(c_int) function c_pb_grid_create(ctx, n, L, grid) bind(C, name="pb_grid_create")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int64_t), dimension(3) :: n
       real(c_double), dimension(3) :: L
       type(c_ptr) :: grid
     end function
     integer(c_int) function c_pb_grid_get_corners(grid, start, size) bind(C, name="pb_grid_get_corners")
       import :: c_int, c_ptr, c_int64_t
       type(c_ptr), value :: grid
       integer(c_int64_t), dimension(3) :: start, size
     end function
     integer(c_int) function c_pb_vec_create(grid, v) bind(C, name="pb_vec_create")
       import :: c_int, c_ptr
       type(c_ptr), value :: grid
       type(c_ptr) :: v
     end function
     integer(c_int) function c_pb_vec_duplicate(v, out) bind(C, name="pb_vec_duplicate")
       import :: c_int, c_ptr
       type(c_ptr), value :: v
       type(c_ptr) :: out
     end function
     integer(c_int) function c_pb_vec_destroy(v) bind(C, name="pb_vec_destroy")
       import :: c_int, c_ptr
       type(c_ptr), value :: v
     end function
     integer(c_int) function c_pb_vec_set(v, a) bind(C, name="pb_vec_set")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: v
       real(c_double), value :: a
     end function
     integer(c_int) function c_pb_vec_copy(src, dst) bind(C, name="pb_vec_copy")
       import :: c_int, c_ptr
       type(c_ptr), value :: src, dst
     end function
     integer(c_int) function c_pb_vec_axpy(y, a, x) bind(C, name="pb_vec_axpy")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: y, x
       real(c_double), value :: a
     end function
     integer(c_int) function c_pb_vec_norm2(v, out) bind(C, name="pb_vec_norm2")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: v
       real(c_double) :: out
     end function
     integer(c_int) function c_pb_vec_sum(v, out) bind(C, name="pb_vec_sum")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: v
       real(c_double) :: out
     end function
     integer(c_int) function c_pb_vec_set_random(v, seed) bind(C, name="pb_vec_set_random")
       import :: c_int, c_ptr, c_int64_t
       type(c_ptr), value :: v
       integer(c_int64_t), value :: seed
     end function
     integer(c_int) function c_pb_vec_get_values_host(v, owned) bind(C, name="pb_vec_get_values_host")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: v
       real(c_double), dimension(*) :: owned
     end function
     integer(c_int) function c_pb_vec_set_values_host(v, owned) bind(C, name="pb_vec_set_values_host")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: v
       real(c_double), dimension(*) :: owned
     end function
     integer(c_int) function c_pb_op_create(grid, kind, deltas, op) bind(C, name="pb_op_create")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: grid
       integer(c_int), value :: kind
       real(c_double), dimension(3) :: deltas
       type(c_ptr) :: op
     end function
     integer(c_int) function c_pb_op_apply(op, x, y) bind(C, name="pb_op_apply")
       import :: c_int, c_ptr
       type(c_ptr), value :: op, x, y
     end function
     integer(c_int) function c_pb_op_destroy(op) bind(C, name="pb_op_destroy")
       import :: c_int, c_ptr
       type(c_ptr), value :: op
     end function
     integer(c_int) function c_pb_op_get_ownership_range(op, first, next) &
          bind(C, name="pb_op_get_ownership_range")
       import :: c_int, c_ptr, c_int64_t
       type(c_ptr), value :: op
       integer(c_int64_t) :: first, next
     end function
     integer(c_int) function c_pb_vec_get_ownership_range(v, first, next) &
          bind(C, name="pb_vec_get_ownership_range")
       import :: c_int, c_ptr, c_int64_t
       type(c_ptr), value :: v
       integer(c_int64_t) :: first, next
     end function
     integer(c_int) function c_pb_ksp_opts_default(o) bind(C, name="pb_ksp_opts_default")
       import :: c_int, pb_ksp_opts
       type(pb_ksp_opts) :: o
     end function
     integer(c_int) function c_pb_ksp_opts_parse(o, argc, argv) bind(C, name="pb_ksp_opts_parse")
       import :: c_int, c_ptr, pb_ksp_opts
       type(pb_ksp_opts) :: o
       integer(c_int), value :: argc
       type(c_ptr), dimension(*) :: argv
     end function
     integer(c_int) function c_pb_solve(A, P, o, b, x, res, hist, cap) bind(C, name="pb_solve")
       import :: c_int, c_ptr, c_int64_t, pb_ksp_opts, pb_ksp_result
       type(c_ptr), value :: A, P, b, x, hist
       type(pb_ksp_opts) :: o
       type(pb_ksp_result) :: res
       integer(c_int64_t), value :: cap
     end function
  end interface

contains

  function pb_error_string() result(msg)
    character(len=:), allocatable :: msg
    character(kind=c_char), pointer :: s(:)
    integer :: n
    call c_f_pointer(c_pb_last_error(), s, [1024])
    n = 0
    do while (n < 1024)
       if (s(n + 1) == c_null_char) exit
       n = n + 1
    end do
    allocate(character(len=n) :: msg)
    msg = transfer(s(1:n), msg)
  end function pb_error_string

  subroutine check(ierr, where)
    integer, intent(in) :: ierr
    character(len=*), intent(in) :: where
    if (ierr /= 0) print *, "poissbox_gpu: ", where, " failed (", ierr, "): ", pb_error_string()
  end subroutine check

  !! ≙ MPI_Init + PetscInitialize (src/example.f90:43-47); one GPU per process
  subroutine PoissboxInitialize(device, ierr)
    integer, intent(in) :: device
    integer, intent(out) :: ierr
    ierr = c_pb_ctx_create(int(device, c_int), 0_c_int, 1_c_int, c_null_ptr, g_ctx)
    call check(ierr, "PoissboxInitialize")
  end subroutine PoissboxInitialize

  subroutine PoissboxFinalize(ierr)
    integer, intent(out) :: ierr
    ierr = c_pb_ctx_destroy(g_ctx)
    g_ctx = c_null_ptr
  end subroutine PoissboxFinalize

  !! src/poissbox.f90:183-204 (periodic x3, width 1; L = 1 as in src/example.f90:30-32)
  subroutine initialise_grid(nglobal, da, ierr)
    integer, dimension(3), intent(in) :: nglobal
    type(tDM), intent(out) :: da
    integer, intent(out) :: ierr
    integer(c_int64_t), dimension(3) :: n
    real(c_double), dimension(3) :: L
    n = int(nglobal, c_int64_t)
    L = 1.0_c_double
    ierr = c_pb_grid_create(g_ctx, n, L, da%h)
    call check(ierr, "initialise_grid")
  end subroutine initialise_grid

  !! ≙ DMDAGetCorners: 0-based start, owned extent
  subroutine DMDAGetCorners(da, istart, jstart, kstart, ni, nj, nk, ierr)
    type(tDM), intent(in) :: da
    integer, intent(out) :: istart, jstart, kstart, ni, nj, nk
    integer, intent(out) :: ierr
    integer(c_int64_t), dimension(3) :: s, z
    ierr = c_pb_grid_get_corners(da%h, s, z)
    istart = int(s(1)); jstart = int(s(2)); kstart = int(s(3))
    ni = int(z(1)); nj = int(z(2)); nk = int(z(3))
  end subroutine DMDAGetCorners

  !! src/poissbox.f90:206-240: P = assembled 27-entry BOX operator, A = matrix-free 7-point
  !! shell (mfmult) when matrix_free (src/example.f90:60-65), x and b global vectors.
  subroutine initialise_linear_system(da, ctx, P, A, x, b, ierr, matrix_free)
    type(tDM), intent(in) :: da
    type(mat_ctx), intent(in) :: ctx
    type(tMat), intent(out) :: P, A
    type(tVec), intent(out) :: x, b
    integer, intent(out) :: ierr
    logical, intent(in), optional :: matrix_free
    logical :: mf
    real(c_double), dimension(3) :: d
    mf = .true.
    if (present(matrix_free)) mf = matrix_free
    print *, "Initialising linear system"
    d = ctx%grid_deltas
    ierr = c_pb_op_create(da%h, PB_OP_ASSEMBLED27, d, P%h)
    if (ierr /= 0) return
    if (mf) then
       print *, "- Initialising matrix-free system"
       ierr = c_pb_op_create(da%h, PB_OP_STAR7, d, A%h)
       if (ierr /= 0) return
       print *, "- Done"
    else
       A = P
    end if
    ierr = c_pb_vec_create(da%h, x%h)
    if (ierr /= 0) return
    ierr = c_pb_vec_create(da%h, b%h)
    call check(ierr, "initialise_linear_system")
    print *, "Done"
  end subroutine initialise_linear_system

  !! src/poissbox.f90:269-298 with KSPSetFromOptions: PETSc-style options from the command line
  subroutine solve(P, A, x, b, ierr, its, reason, rnorm)
    type(tMat), intent(in) :: P, A
    type(tVec), intent(inout) :: x
    type(tVec), intent(in) :: b
    integer, intent(out) :: ierr
    integer, intent(out), optional :: its, reason
    real(pb_dp), intent(out), optional :: rnorm
    type(pb_ksp_opts) :: o
    type(pb_ksp_result) :: res
    integer :: nargs, i, l, lmax
    character(len=:), allocatable, target :: args(:)
    type(c_ptr), allocatable :: argv(:)

    ierr = c_pb_ksp_opts_default(o)
    nargs = command_argument_count()
    lmax = 1  ! buffers sized from the longest argument (+1 for the C terminator)
    do i = 1, nargs
       call get_command_argument(i, length=l)
       lmax = max(lmax, l + 1)
    end do
    allocate(character(len=lmax) :: args(max(nargs, 1)))
    allocate(argv(max(nargs, 1)))
    do i = 1, nargs
       call get_command_argument(i, args(i), l)
       args(i)(l + 1:l + 1) = c_null_char
       argv(i) = c_loc(args(i))
    end do
    ierr = c_pb_ksp_opts_parse(o, int(nargs, c_int), argv)
    if (ierr /= 0) then
       call check(ierr, "KSPSetFromOptions")
       return
    end if
    if (c_associated(A%h, P%h) .eqv. .false.) print *, "Setting nullspace on A"
    ierr = c_pb_solve(A%h, P%h, o, b%h, x%h, res, c_null_ptr, 0_c_int64_t)
    call check(ierr, "KSPSolve")
    if (present(its)) its = int(res%its)
    if (present(reason)) reason = int(res%reason)
    if (present(rnorm)) rnorm = res%rnorm
  end subroutine solve

  !! ≙ MatMult(A, x, f, ierr) -> mfmult (src/poissbox.f90:300-322)
  subroutine MatMult(A, x, f, ierr)
    type(tMat), intent(in) :: A
    type(tVec), intent(in) :: x
    type(tVec), intent(inout) :: f
    integer, intent(out) :: ierr
    ierr = c_pb_op_apply(A%h, x%h, f%h)
    call check(ierr, "MatMult")
  end subroutine MatMult

  !! src/poissbox.f90:84-126
  subroutine compute_lapl_pointwise(da, grid_deltas, x, b, ierr)
    type(tDM), intent(in) :: da
    real(pb_dp), dimension(3), intent(in) :: grid_deltas
    type(tVec), intent(in) :: x
    type(tVec), intent(inout) :: b
    integer, intent(out) :: ierr
    type(tMat) :: op
    real(c_double), dimension(3) :: d
    integer :: l
    d = grid_deltas
    ierr = c_pb_op_create(da%h, PB_OP_STAR7, d, op%h)
    if (ierr /= 0) return
    ierr = c_pb_op_apply(op%h, x%h, b%h)
    call check(ierr, "compute_lapl_pointwise")
    if (ierr /= 0) then  ! keep the apply's error; still release the operator
       l = c_pb_op_destroy(op%h)
       return
    end if
    ierr = c_pb_op_destroy(op%h)
  end subroutine compute_lapl_pointwise

  !! ≙ MatGetOwnershipRange (src/example.f90:137): rows [myrow, nextrow) on this rank
  subroutine MatGetOwnershipRange(A, myrow, nextrow, ierr)
    type(tMat), intent(in) :: A
    integer, intent(out) :: myrow, nextrow, ierr
    integer(c_int64_t) :: f, n
    ierr = c_pb_op_get_ownership_range(A%h, f, n)
    myrow = int(f)
    nextrow = int(n)
  end subroutine MatGetOwnershipRange

  !! ≙ VecGetOwnershipRange (src/example.f90:142,147)
  subroutine VecGetOwnershipRange(x, myrow, nextrow, ierr)
    type(tVec), intent(in) :: x
    integer, intent(out) :: myrow, nextrow, ierr
    integer(c_int64_t) :: f, n
    ierr = c_pb_vec_get_ownership_range(x%h, f, n)
    myrow = int(f)
    nextrow = int(n)
  end subroutine VecGetOwnershipRange

  subroutine MatDestroy(A, ierr)
    type(tMat), intent(inout) :: A
    integer, intent(out) :: ierr
    ierr = c_pb_op_destroy(A%h)
    A%h = c_null_ptr
  end subroutine MatDestroy

  subroutine VecDuplicate(x, y, ierr)
    type(tVec), intent(in) :: x
    type(tVec), intent(out) :: y
    integer, intent(out) :: ierr
    ierr = c_pb_vec_duplicate(x%h, y%h)
  end subroutine VecDuplicate

  subroutine VecCopy(x, y, ierr)
    type(tVec), intent(in) :: x
    type(tVec), intent(inout) :: y
    integer, intent(out) :: ierr
    ierr = c_pb_vec_copy(x%h, y%h)
  end subroutine VecCopy

  subroutine VecAXPY(y, alpha, x, ierr)  ! y = y + alpha*x
    type(tVec), intent(inout) :: y
    real(pb_dp), intent(in) :: alpha
    type(tVec), intent(in) :: x
    integer, intent(out) :: ierr
    ierr = c_pb_vec_axpy(y%h, real(alpha, c_double), x%h)
  end subroutine VecAXPY

  subroutine VecNorm(x, nrm, ierr)  ! NORM_2
    type(tVec), intent(in) :: x
    real(pb_dp), intent(out) :: nrm
    integer, intent(out) :: ierr
    ierr = c_pb_vec_norm2(x%h, nrm)
  end subroutine VecNorm

  subroutine VecSum(x, s, ierr)
    type(tVec), intent(in) :: x
    real(pb_dp), intent(out) :: s
    integer, intent(out) :: ierr
    ierr = c_pb_vec_sum(x%h, s)
  end subroutine VecSum

  subroutine VecSet(x, alpha, ierr)
    type(tVec), intent(inout) :: x
    real(pb_dp), intent(in) :: alpha
    integer, intent(out) :: ierr
    ierr = c_pb_vec_set(x%h, real(alpha, c_double))
  end subroutine VecSet

  !! set_solution's x = 2(0.5 - U) (src/example.f90:180-181) with a decomposition-independent
  !! generator (SplitMix64 by global index) instead of the compiler's random_number
  subroutine VecSetRandom(x, seed, ierr)
    type(tVec), intent(inout) :: x
    integer(c_int64_t), intent(in) :: seed
    integer, intent(out) :: ierr
    ierr = c_pb_vec_set_random(x%h, seed)
  end subroutine VecSetRandom

  !! copy-out / copy-in forms of DMDAVecGetArrayF90 / Restore on the owned block
  subroutine VecGetValues(x, owned, ierr)
    type(tVec), intent(in) :: x
    real(pb_dp), dimension(:, :, :), intent(out) :: owned
    integer, intent(out) :: ierr
    ierr = c_pb_vec_get_values_host(x%h, owned)
  end subroutine VecGetValues

  subroutine VecSetValues(x, owned, ierr)
    type(tVec), intent(inout) :: x
    real(pb_dp), dimension(:, :, :), intent(in) :: owned
    integer, intent(out) :: ierr
    ierr = c_pb_vec_set_values_host(x%h, owned)
  end subroutine VecSetValues

  subroutine VecDestroy(x, ierr)
    type(tVec), intent(inout) :: x
    integer, intent(out) :: ierr
    ierr = c_pb_vec_destroy(x%h)
    x%h = c_null_ptr
  end subroutine VecDestroy

end module poissbox_gpu
