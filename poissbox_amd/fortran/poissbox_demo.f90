!! poissbox_demo.f90 -- the reference demo flow (src/example.f90) on 1..N MI355X ranks.
!
! Same sequence of steps as poissbox_example (src/example.f90:55-84): grid + check_grid, linear
! system + check_linear_system, assemble_laplacian, x = random in [-1,1], b = A x, check_lapl
! (A x vs pointwise stencil), check_matrices (A x vs P x), KSP solve from PETSc-style options,
! final residual ||A x - b||_2. One process per rank, started by any launcher
! (`torchrun --no-python --nproc-per-node N poissbox_demo ...`, mpirun, or RANK/WORLD_SIZE set by
! hand): the per-rank lines reproduce README.md:25-33 (64^3 on 3 ranks: 90112/86016/86016).
! Usage: poissbox_demo [-n N] [-ksp_rtol 1e-10] [-ksp_monitor] [-ksp_converged_reason] ...
program poissbox_demo

  use iso_c_binding, only: c_int64_t
  use poissbox_gpu

  implicit none

  integer :: ierr, n1, its, reason, irank, nproc
  integer, dimension(3) :: n
  real(pb_dp), dimension(3) :: h
  real(pb_dp) :: error, rnorm
  type(tDM) :: da
  type(tMat) :: P, A
  type(tVec) :: x, b, x2
  type(mat_ctx) :: ctx

  n1 = arg_int("-n", 64)
  n = [n1, n1, n1]
  h = 1.0_pb_dp / real(n, pb_dp)  ! src/example.f90:33-35, L = 1

  call PoissboxInitialize(0, ierr)
  if (ierr /= 0) stop 1
  call PoissboxCommRank(irank, nproc, ierr)
  if (irank == 0) print *, "Running poissbox on ", nproc, " ranks"
  call PoissboxBarrier(ierr)
  print *, "Hello from ", irank

  call initialise_grid(n, da, ierr)
  call check_grid(n, da)

  ctx%da = da
  ctx%grid_deltas = h
  call initialise_linear_system(da, ctx, P, A, x, b, ierr)
  if (ierr /= 0) stop 1
  call check_linear_system(n, P, x, b)
  call assemble_laplacian(da, h(1), h(2), h(3), P)

  call set_solution(da, x)
  print *, "Calling MatMult"
  call MatMult(A, x, b, ierr)
  call check_lapl(da, x, b)
  call check_matrices(A, P, x)

  call solve(P, A, x, b, ierr, its, reason, rnorm)
  if (ierr /= 0) stop 1
  call VecDuplicate(x, x2, ierr)
  print *, "Calling MatMult"
  call MatMult(A, x, x2, ierr)
  call VecAXPY(x2, -1.0_pb_dp, b, ierr)
  call VecNorm(x2, error, ierr)
  print *, "KSP iterations: ", its, " reason: ", reason, " ||z||: ", rnorm
  print *, "Solution residual (L2 norm): ", error

  call VecDestroy(x2, ierr)
  call VecDestroy(x, ierr)
  call VecDestroy(b, ierr)
  call PoissboxFinalize(ierr)

contains

  integer function arg_int(name, dflt)
    character(len=*), intent(in) :: name
    integer, intent(in) :: dflt
    character(len=64) :: a
    integer :: i
    arg_int = dflt
    do i = 1, command_argument_count() - 1
       call get_command_argument(i, a)
       if (trim(a) == name) then
          call get_command_argument(i + 1, a)
          read(a, *) arg_int
       end if
    end do
  end function arg_int

  !! src/example.f90:92-116: owned DoF vs global DoF (sum over ranks)
  subroutine check_grid(nglobal, da)
    integer, dimension(3), intent(in) :: nglobal
    type(tDM), intent(in) :: da
    integer :: istart, jstart, kstart, ni, nj, nk, ierr, nloc, nglob
    call DMDAGetCorners(da, istart, jstart, kstart, ni, nj, nk, ierr)
    nloc = ni * nj * nk
    nglob = nloc
    call PoissboxAllreduceSum(nglob, ierr)
    print *, "(DMDA): Rank ", irank, " has ", nloc, " of ", nglob, " expected: ", product(nglobal)
  end subroutine check_grid

  !! src/example.f90:118-152: row ownership of P, x and b against the global DoF count
  subroutine check_linear_system(nglobal, M, x, b)
    integer, dimension(3), intent(in) :: nglobal
    type(tMat), intent(in) :: M
    type(tVec), intent(in) :: x, b
    integer :: myrow, nextrow, ierr, nloc, nglob
    call MatGetOwnershipRange(M, myrow, nextrow, ierr)
    nloc = nextrow - myrow
    nglob = nloc
    call PoissboxAllreduceSum(nglob, ierr)
    print *, "(M): Rank ", irank, " has ", nloc, " rows of ", nglob, " expected: ", product(nglobal)
    call VecGetOwnershipRange(x, myrow, nextrow, ierr)
    nloc = nextrow - myrow
    nglob = nloc
    call PoissboxAllreduceSum(nglob, ierr)
    print *, "(x): Rank ", irank, " has ", nloc, " rows of ", nglob, " expected: ", product(nglobal)
    call VecGetOwnershipRange(b, myrow, nextrow, ierr)
    nloc = nextrow - myrow
    nglob = nloc
    call PoissboxAllreduceSum(nglob, ierr)
    print *, "(b): Rank ", irank, " has ", nloc, " rows of ", nglob, " expected: ", product(nglobal)
  end subroutine check_linear_system

  !! src/example.f90:154-199: x = 2(0.5 - U) on the owned block; the sum computed directly over
  !! the owned values (host loop, as the reference's xsum, summed over ranks) against VecSum
  subroutine set_solution(da, x)
    type(tDM), intent(in) :: da
    type(tVec), intent(inout) :: x
    integer :: istart, jstart, kstart, ni, nj, nk, ierr, i, j, k
    real(pb_dp), allocatable :: xdof(:, :, :)
    real(pb_dp) :: xs, xsum_v
    call DMDAGetCorners(da, istart, jstart, kstart, ni, nj, nk, ierr)
    call VecSetRandom(x, 20231015_c_int64_t, ierr)
    allocate(xdof(ni, nj, nk))
    call VecGetValues(x, xdof, ierr)
    xs = 0.0_pb_dp
    do k = 1, nk
       do j = 1, nj
          do i = 1, ni
             xs = xs + xdof(i, j, k)
          end do
       end do
    end do
    deallocate(xdof)
    call VecSum(x, xsum_v, ierr)
    call PoissboxAllreduceSum(xs, ierr)
    print *, "Rank ", irank, "Delta of XSUM norms computed directly and from X: ", xsum_v - xs, &
         xsum_v, xs
  end subroutine set_solution

  !! src/example.f90:201-233: ||A x - pointwise(x)||_2 (identical kernels -> 0)
  subroutine check_lapl(da, x, b)
    type(tDM), intent(in) :: da
    type(tVec), intent(in) :: x, b
    type(tVec) :: b2, c
    real(pb_dp) :: residual
    integer :: ierr
    call VecDuplicate(b, b2, ierr)
    call VecCopy(b, b2, ierr)
    call VecDuplicate(b, c, ierr)
    call compute_lapl_pointwise(da, h, x, c, ierr)
    call VecAXPY(b2, -1.0_pb_dp, c, ierr)
    call VecNorm(b2, residual, ierr)
    print *, "Rank ", irank, "Delta between b=Mx and pointwise calculation: ", residual
    call VecDestroy(b2, ierr)
    call VecDestroy(c, ierr)
  end subroutine check_lapl

  !! src/example.f90:235-261: ||A x - P x||_2
  subroutine check_matrices(A, P, x)
    type(tMat), intent(in) :: A, P
    type(tVec), intent(in) :: x
    type(tVec) :: bP, bA
    real(pb_dp) :: delta
    integer :: ierr
    call VecDuplicate(x, bP, ierr)
    call VecDuplicate(x, bA, ierr)
    call MatMult(P, x, bP, ierr)
    call MatMult(A, x, bA, ierr)
    call VecAXPY(bA, -1.0_pb_dp, bP, ierr)
    call VecNorm(bA, delta, ierr)
    print *, "Ax - Px = ", delta
    call VecDestroy(bP, ierr)
    call VecDestroy(bA, ierr)
  end subroutine check_matrices

end program poissbox_demo
