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
!   MPI_Init / MPI_Comm_rank / MPI_Comm_size / MPI_Allreduce(SUM) / MPI_Barrier
!     (src/example.f90:43-52,108,137-147,194) -> PoissboxInitialize (launcher environment:
!     torchrun --no-python, mpirun, PMI), PoissboxCommRank, PoissboxAllreduceSum, PoissboxBarrier
!   assemble_laplacian(da, dx, dy, dz, M) (src/coefficients.f90:50-113) -> same
! The module procedures of src/tridsol.f90 and src/compact_schemes.f90 keep their own module
! names (poissbox_modules.f90: modules tridsol, compact_schemes, coefficients; constants in
! poissbox_constants.f90); the device-pointer C entry points are bound here as c_pb_*.
! Every routine returns ierr (0 = success) as the last argument, PETSc style; unlike the
! reference, ierr is always set.
module poissbox_gpu

  use iso_c_binding
  use constants, only: pb_dp

  implicit none

  private

  public :: pb_dp

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
     integer(c_int) :: cg_single_reduction
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
  public :: PoissboxContext, PoissboxCommRank, PoissboxAllreduceSum, PoissboxBarrier
  public :: assemble_laplacian
  public :: CompactGrad, CompactDiv, CompactInterp, CompactLapl, CompactLaplFast
  ! C entry points on device pointers / host arrays (batched line solvers, compact operators)
  public :: c_pb_comm_unique_id, c_pb_tdma_batched, c_pb_tdma_sweeps_batched
  public :: c_pb_pcr_alpha_batched, c_pb_compact_1d_batched
  public :: c_pb_tdma_batched_host, c_pb_tdma_sweeps_batched_host, c_pb_compact_1d_batched_host
  public :: c_pb_compact_grad_host, c_pb_compact_div_host, c_pb_compact_interp_host
  public :: c_pb_compact_lapl_host, c_pb_lapl_1d_coeffs, c_pb_lapl_star_coeffs

  interface PoissboxAllreduceSum  ! ≙ MPI_Allreduce(..., MPI_SUM, MPI_COMM_WORLD)
     module procedure allreduce_sum_int, allreduce_sum_real
  end interface PoissboxAllreduceSum

  interface
     integer(c_int) function c_pb_ctx_create(device, rank, nranks, uid, ctx) bind(C, name="pb_ctx_create")
       import :: c_int, c_ptr
       integer(c_int), value :: device, rank, nranks
       type(c_ptr), value :: uid
       type(c_ptr) :: ctx
     end function
     integer(c_int) function c_pb_ctx_create_from_env(device, ctx) &
          bind(C, name="pb_ctx_create_from_env")
       import :: c_int, c_ptr
       integer(c_int), value :: device
       type(c_ptr) :: ctx
     end function
     integer(c_int) function c_pb_ctx_get_rank(ctx, rank, nranks) bind(C, name="pb_ctx_get_rank")
       import :: c_int, c_ptr
       type(c_ptr), value :: ctx
       integer(c_int) :: rank, nranks
     end function
     integer(c_int) function c_pb_ctx_comm_info(ctx, transport, comm_nranks, comm_rank) &
          bind(C, name="pb_ctx_comm_info")
       import :: c_int, c_ptr
       type(c_ptr), value :: ctx
       integer(c_int) :: transport, comm_nranks, comm_rank
     end function
     integer(c_int) function c_pb_ctx_allreduce_host(ctx, vals, count) &
          bind(C, name="pb_ctx_allreduce_host")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: ctx
       real(c_double), dimension(*) :: vals
       integer(c_int), value :: count
     end function
     integer(c_int) function c_pb_ctx_barrier(ctx) bind(C, name="pb_ctx_barrier")
       import :: c_int, c_ptr
       type(c_ptr), value :: ctx
     end function
     integer(c_int) function c_pb_comm_unique_id(uid) bind(C, name="pb_comm_unique_id")
       import :: c_int, c_char
       character(kind=c_char), dimension(128) :: uid
     end function
     integer(c_int) function c_pb_op_set_deltas(op, deltas) bind(C, name="pb_op_set_deltas")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: op
       real(c_double), dimension(3) :: deltas
     end function
     ! src/tridsol.f90 on device pointers (element e of line l at ptr[l*line_stride + e*elem_stride])
     integer(c_int) function c_pb_tdma_batched(ctx, n, nbatch, ls, es, a, b, c, d, periodic) &
          bind(C, name="pb_tdma_batched")
       import :: c_int, c_ptr, c_int64_t
       type(c_ptr), value :: ctx, a, b, c, d
       integer(c_int64_t), value :: n, nbatch, ls, es
       integer(c_int), value :: periodic
     end function
     integer(c_int) function c_pb_tdma_sweeps_batched(ctx, n, nbatch, ls, es, a, b, c, d, which) &
          bind(C, name="pb_tdma_sweeps_batched")
       import :: c_int, c_ptr, c_int64_t
       type(c_ptr), value :: ctx, a, b, c, d
       integer(c_int64_t), value :: n, nbatch, ls, es
       integer(c_int), value :: which
     end function
     integer(c_int) function c_pb_pcr_alpha_batched(ctx, n, nbatch, ls, es, alpha, d) &
          bind(C, name="pb_pcr_alpha_batched")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx, d
       integer(c_int64_t), value :: n, nbatch, ls, es
       real(c_double), value :: alpha
     end function
     integer(c_int) function c_pb_compact_1d_batched(ctx, kind, stagger, dx, n, nbatch, ls, es, &
          f, out) bind(C, name="pb_compact_1d_batched")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx, f, out
       integer(c_int), value :: kind, stagger
       real(c_double), value :: dx
       integer(c_int64_t), value :: n, nbatch, ls, es
     end function
     ! the same on host arrays (copied through device memory)
     integer(c_int) function c_pb_tdma_batched_host(ctx, n, nbatch, ls, es, a, b, c, d, periodic) &
          bind(C, name="pb_tdma_batched_host")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int64_t), value :: n, nbatch, ls, es
       real(c_double), dimension(*) :: a, b, c, d
       integer(c_int), value :: periodic
     end function
     integer(c_int) function c_pb_tdma_sweeps_batched_host(ctx, n, nbatch, ls, es, a, b, c, d, &
          which) bind(C, name="pb_tdma_sweeps_batched_host")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int64_t), value :: n, nbatch, ls, es
       real(c_double), dimension(*) :: a, b, c, d
       integer(c_int), value :: which
     end function
     integer(c_int) function c_pb_compact_1d_batched_host(ctx, kind, stagger, dx, n, nbatch, ls, &
          es, f, out) bind(C, name="pb_compact_1d_batched_host")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int), value :: kind, stagger
       real(c_double), value :: dx
       integer(c_int64_t), value :: n, nbatch, ls, es
       real(c_double), dimension(*) :: f, out
     end function
     integer(c_int) function c_pb_compact_grad_host(ctx, n, dx, f, df) &
          bind(C, name="pb_compact_grad_host")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int64_t), dimension(3) :: n
       real(c_double), dimension(3) :: dx
       real(c_double), dimension(*) :: f, df
     end function
     integer(c_int) function c_pb_compact_div_host(ctx, n, dx, f, df) &
          bind(C, name="pb_compact_div_host")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int64_t), dimension(3) :: n
       real(c_double), dimension(3) :: dx
       real(c_double), dimension(*) :: f, df
     end function
     integer(c_int) function c_pb_compact_interp_host(ctx, n, stagger, f, fi) &
          bind(C, name="pb_compact_interp_host")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int64_t), dimension(3) :: n
       integer(c_int), value :: stagger
       real(c_double), dimension(*) :: f, fi
     end function
     integer(c_int) function c_pb_compact_lapl_host(ctx, n, dx, f, out) &
          bind(C, name="pb_compact_lapl_host")
       import :: c_int, c_ptr, c_int64_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int64_t), dimension(3) :: n
       real(c_double), dimension(3) :: dx
       real(c_double), dimension(*) :: f, out
     end function
     pure integer(c_int) function c_pb_lapl_1d_coeffs(dx, c) bind(C, name="pb_lapl_1d_coeffs")
       import :: c_int, c_double
       real(c_double), value, intent(in) :: dx
       real(c_double), dimension(3), intent(out) :: c
     end function
     pure integer(c_int) function c_pb_lapl_star_coeffs(dx, dy, dz, c) &
          bind(C, name="pb_lapl_star_coeffs")
       import :: c_int, c_double
       real(c_double), value, intent(in) :: dx, dy, dz
       real(c_double), dimension(27), intent(out) :: c
     end function
     ! compact operators on grid vectors (z-slab split grids included)
     integer(c_int) function c_pb_compact_grad(grid, dx, f, df) bind(C, name="pb_compact_grad")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: grid, f
       real(c_double), dimension(3) :: dx
       type(c_ptr), dimension(3) :: df
     end function
     integer(c_int) function c_pb_compact_div(grid, dx, f, df) bind(C, name="pb_compact_div")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: grid, df
       real(c_double), dimension(3) :: dx
       type(c_ptr), dimension(3) :: f
     end function
     integer(c_int) function c_pb_compact_interp(grid, stagger, f, fi) &
          bind(C, name="pb_compact_interp")
       import :: c_int, c_ptr
       type(c_ptr), value :: grid, f, fi
       integer(c_int), value :: stagger
     end function
     integer(c_int) function c_pb_compact_lapl(grid, dx, f, out) bind(C, name="pb_compact_lapl")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: grid, f, out
       real(c_double), dimension(3) :: dx
     end function
     integer(c_int) function c_pb_compact_lapl_fast(grid, dx, f, out) &
          bind(C, name="pb_compact_lapl_fast")
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: grid, f, out
       real(c_double), dimension(3) :: dx
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

  !! ≙ MPI_Init + PetscInitialize (src/example.f90:43-47). One process: rank 0 of 1 on GPU
  !! `device`. Under a launcher (torchrun --no-python, mpirun, PMI) every process is one rank on
  !! GPU LOCAL_RANK, connected over RCCL, or over the built-in shared-memory transport when ranks
  !! outnumber GPUs (PB_TRANSPORT, include/poissbox_gpu.h pb_ctx_create_from_env).
  subroutine PoissboxInitialize(device, ierr)
    integer, intent(in) :: device
    integer, intent(out) :: ierr
    ierr = c_pb_ctx_create_from_env(int(device, c_int), g_ctx)
    call check(ierr, "PoissboxInitialize")
  end subroutine PoissboxInitialize

  !! the process's context; created on first use (GPU LOCAL_RANK) when a program calls a module
  !! procedure without PoissboxInitialize (the reference's compact / tridiagonal routines need no
  !! set-up either)
  function PoissboxContext() result(ctx)
    type(c_ptr) :: ctx
    integer :: ierr
    if (.not. c_associated(g_ctx)) then
       ierr = c_pb_ctx_create_from_env(-1_c_int, g_ctx)
       if (ierr /= 0) then
          call check(ierr, "PoissboxContext")
          error stop 1
       end if
    end if
    ctx = g_ctx
  end function PoissboxContext

  !! ≙ MPI_Comm_rank + MPI_Comm_size on MPI_COMM_WORLD
  subroutine PoissboxCommRank(rank, nranks, ierr)
    integer, intent(out) :: rank, nranks, ierr
    integer(c_int) :: r, n
    ierr = c_pb_ctx_get_rank(PoissboxContext(), r, n)
    rank = int(r)
    nranks = int(n)
  end subroutine PoissboxCommRank

  !! ≙ MPI_Barrier(MPI_COMM_WORLD)
  subroutine PoissboxBarrier(ierr)
    integer, intent(out) :: ierr
    ierr = c_pb_ctx_barrier(PoissboxContext())
    call check(ierr, "PoissboxBarrier")
  end subroutine PoissboxBarrier

  subroutine allreduce_sum_real(v, ierr)
    real(pb_dp), intent(inout) :: v
    integer, intent(out) :: ierr
    real(c_double), dimension(1) :: t
    t(1) = v
    ierr = c_pb_ctx_allreduce_host(PoissboxContext(), t, 1_c_int)
    call check(ierr, "PoissboxAllreduceSum")
    v = t(1)
  end subroutine allreduce_sum_real

  subroutine allreduce_sum_int(v, ierr)  ! exact for |sum| < 2**53
    integer, intent(inout) :: v
    integer, intent(out) :: ierr
    real(c_double), dimension(1) :: t
    t(1) = real(v, c_double)
    ierr = c_pb_ctx_allreduce_host(PoissboxContext(), t, 1_c_int)
    call check(ierr, "PoissboxAllreduceSum")
    v = nint(t(1))
  end subroutine allreduce_sum_int

  !! src/coefficients.f90:50-113: the operator's coefficients from the spacings (the 27-entry
  !! BOX rows are implicit: PB_OP_ASSEMBLED27 sums them in PETSc AIJ order)
  subroutine assemble_laplacian(da, dx, dy, dz, M)
    type(tDM), intent(in) :: da
    real(pb_dp), intent(in) :: dx, dy, dz
    type(tMat), intent(inout) :: M
    real(c_double), dimension(3) :: d
    integer :: ierr
    d = [dx, dy, dz]
    if (.not. c_associated(M%h)) then
       ierr = c_pb_op_create(da%h, PB_OP_ASSEMBLED27, d, M%h)
    else
       ierr = c_pb_op_set_deltas(M%h, d)
    end if
    call check(ierr, "assemble_laplacian")
  end subroutine assemble_laplacian

  !! compact operators on grid vectors (src/compact_schemes.f90:17-257), split grids included
  subroutine CompactGrad(da, dx, f, df, ierr)
    type(tDM), intent(in) :: da
    real(pb_dp), dimension(3), intent(in) :: dx
    type(tVec), intent(in) :: f
    type(tVec), dimension(3), intent(inout) :: df
    integer, intent(out) :: ierr
    real(c_double), dimension(3) :: d
    type(c_ptr), dimension(3) :: h
    d = dx
    h = [df(1)%h, df(2)%h, df(3)%h]
    ierr = c_pb_compact_grad(da%h, d, f%h, h)
    call check(ierr, "CompactGrad")
  end subroutine CompactGrad

  subroutine CompactDiv(da, dx, f, df, ierr)
    type(tDM), intent(in) :: da
    real(pb_dp), dimension(3), intent(in) :: dx
    type(tVec), dimension(3), intent(in) :: f
    type(tVec), intent(inout) :: df
    integer, intent(out) :: ierr
    real(c_double), dimension(3) :: d
    type(c_ptr), dimension(3) :: h
    d = dx
    h = [f(1)%h, f(2)%h, f(3)%h]
    ierr = c_pb_compact_div(da%h, d, h, df%h)
    call check(ierr, "CompactDiv")
  end subroutine CompactDiv

  subroutine CompactInterp(da, stagger, f, fi, ierr)
    type(tDM), intent(in) :: da
    integer, intent(in) :: stagger
    type(tVec), intent(in) :: f
    type(tVec), intent(inout) :: fi
    integer, intent(out) :: ierr
    ierr = c_pb_compact_interp(da%h, int(stagger, c_int), f%h, fi%h)
    call check(ierr, "CompactInterp")
  end subroutine CompactInterp

  subroutine CompactLapl(da, dx, f, out, ierr)
    type(tDM), intent(in) :: da
    real(pb_dp), dimension(3), intent(in) :: dx
    type(tVec), intent(in) :: f
    type(tVec), intent(inout) :: out
    integer, intent(out) :: ierr
    real(c_double), dimension(3) :: d
    d = dx
    ierr = c_pb_compact_lapl(da%h, d, f%h, out%h)
    call check(ierr, "CompactLapl")
  end subroutine CompactLapl

  !! the 3-pass factorised compact Laplacian (what PB_OP_COMPACT applies)
  subroutine CompactLaplFast(da, dx, f, out, ierr)
    type(tDM), intent(in) :: da
    real(pb_dp), dimension(3), intent(in) :: dx
    type(tVec), intent(in) :: f
    type(tVec), intent(inout) :: out
    integer, intent(out) :: ierr
    real(c_double), dimension(3) :: d
    d = dx
    ierr = c_pb_compact_lapl_fast(da%h, d, f%h, out%h)
    call check(ierr, "CompactLaplFast")
  end subroutine CompactLaplFast

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
    ierr = c_pb_grid_create(PoissboxContext(), n, L, da%h)
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
