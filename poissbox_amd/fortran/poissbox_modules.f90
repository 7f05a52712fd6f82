!! poissbox_modules.f90 -- the reference's Fortran module procedures on the MI355X library, under
!! the reference's module names, so code written against them (including the reference's own test
!! programs, tests/test_reference_suite.py) builds unchanged against this library:
!!   module coefficients   (src/coefficients.f90:16-18)   lapl_1d_coeffs, lapl_star_coeffs,
!!                                                          assemble_laplacian (poissbox_gpu)
!!   module tridsol        (src/tridsol.f90:16-18)        tdma, tdma_periodic, fwd_sweep, bwd_sweep
!!   module compact_schemes (src/compact_schemes.f90:9-13) grad, grad_1d, interp, interp_1d, div,
!!                                                          div_1d, interp_div, interp_1d_div, lapl
!! Same assumed-shape signatures. Arrays are process-local host arrays, as in the reference; each
!! call stages them through device memory and runs the HIP kernels (pb_*_host in
!! include/poissbox_gpu.h), whose results are bit-identical to the reference's. There is no
!! error argument in the reference API: a library failure prints the reason and stops.

module coefficients

  use iso_c_binding, only: c_int, c_double
  use constants
  use poissbox_gpu, only: c_pb_lapl_1d_coeffs, c_pb_lapl_star_coeffs, assemble_laplacian

  implicit none

  private
  public :: lapl_1d_coeffs, lapl_star_coeffs, assemble_laplacian

contains

  !! src/coefficients.f90:22-35
  pure function lapl_1d_coeffs(dx) result(coeffs)
    real(pb_dp), intent(in) :: dx
    real(pb_dp), dimension(3) :: coeffs
    integer(c_int) :: rc
    rc = c_pb_lapl_1d_coeffs(real(dx, c_double), coeffs)
  end function lapl_1d_coeffs

  !! src/coefficients.f90:38-48: the 3x3x3 coefficient box of the 7-point star
  pure function lapl_star_coeffs(dx, dy, dz) result(coeffs)
    real(pb_dp), intent(in) :: dx, dy, dz
    real(pb_dp), dimension(3, 3, 3) :: coeffs
    real(c_double), dimension(27) :: c
    integer(c_int) :: rc
    rc = c_pb_lapl_star_coeffs(real(dx, c_double), real(dy, c_double), real(dz, c_double), c)
    coeffs = reshape(c, [3, 3, 3])
  end function lapl_star_coeffs

end module coefficients

module tridsol

  use iso_c_binding, only: c_int, c_int64_t
  use constants
  use poissbox_gpu, only: PoissboxContext, pb_error_string, c_pb_tdma_batched_host, &
       c_pb_tdma_sweeps_batched_host

  implicit none

  private
  public :: tdma, tdma_periodic
  public :: fwd_sweep, bwd_sweep

contains

  subroutine must(rc, what)
    integer(c_int), intent(in) :: rc
    character(len=*), intent(in) :: what
    if (rc /= 0) then
       print *, "tridsol: ", what, " failed: ", pb_error_string()
       error stop 1
    end if
  end subroutine must

  !! src/tridsol.f90:22-32 (b and d are overwritten, as in the reference)
  subroutine tdma(a, b, c, d)
    real(pb_dp), dimension(:), intent(in) :: a
    real(pb_dp), dimension(:), intent(inout) :: b
    real(pb_dp), dimension(:), intent(in) :: c
    real(pb_dp), dimension(:), intent(inout) :: d
    integer(c_int64_t) :: n
    n = size(d, kind=c_int64_t)
    call must(c_pb_tdma_batched_host(PoissboxContext(), n, 1_c_int64_t, n, 1_c_int64_t, a, b, c, &
         d, 0_c_int), "tdma")
  end subroutine tdma

  !! src/tridsol.f90:34-74 (Sherman-Morrison; b unchanged)
  subroutine tdma_periodic(a, b, c, d)
    real(pb_dp), dimension(:), intent(in) :: a
    real(pb_dp), dimension(:), intent(inout) :: b
    real(pb_dp), dimension(:), intent(in) :: c
    real(pb_dp), dimension(:), intent(inout) :: d
    integer(c_int64_t) :: n
    n = size(d, kind=c_int64_t)
    call must(c_pb_tdma_batched_host(PoissboxContext(), n, 1_c_int64_t, n, 1_c_int64_t, a, b, c, &
         d, 1_c_int), "tdma_periodic")
  end subroutine tdma_periodic

  !! src/tridsol.f90:76-96
  subroutine fwd_sweep(a, b, c, d)
    real(pb_dp), dimension(:), intent(in) :: a
    real(pb_dp), dimension(:), intent(inout) :: b
    real(pb_dp), dimension(:), intent(in) :: c
    real(pb_dp), dimension(:), intent(inout) :: d
    integer(c_int64_t) :: n
    n = size(d, kind=c_int64_t)
    call must(c_pb_tdma_sweeps_batched_host(PoissboxContext(), n, 1_c_int64_t, n, 1_c_int64_t, &
         a, b, c, d, 1_c_int), "fwd_sweep")
  end subroutine fwd_sweep

  !! src/tridsol.f90:98-115
  subroutine bwd_sweep(b, c, d)
    real(pb_dp), dimension(:), intent(in) :: b
    real(pb_dp), dimension(:), intent(in) :: c
    real(pb_dp), dimension(:), intent(inout) :: d
    integer(c_int64_t) :: n
    real(pb_dp), dimension(size(b)) :: bc
    n = size(d, kind=c_int64_t)
    bc = b  ! the C entry point takes b writable (fwd_sweep's signature); bwd leaves it unchanged
    call must(c_pb_tdma_sweeps_batched_host(PoissboxContext(), n, 1_c_int64_t, n, 1_c_int64_t, &
         bc, bc, c, d, 2_c_int), "bwd_sweep")
  end subroutine bwd_sweep

end module tridsol

module compact_schemes

  use iso_c_binding, only: c_int, c_int64_t, c_double
  use constants
  use poissbox_gpu, only: PoissboxContext, pb_error_string, c_pb_compact_1d_batched_host, &
       c_pb_compact_grad_host, c_pb_compact_div_host, c_pb_compact_interp_host, &
       c_pb_compact_lapl_host

  implicit none

  private
  public :: grad, grad_1d
  public :: interp, interp_1d
  public :: div, div_1d
  public :: interp_div, interp_1d_div
  public :: lapl

contains

  subroutine must(rc, what)
    integer(c_int), intent(in) :: rc
    character(len=*), intent(in) :: what
    if (rc /= 0) then
       print *, "compact_schemes: ", what, " failed: ", pb_error_string()
       error stop 1
    end if
  end subroutine must

  function shape3(f) result(n)
    real(pb_dp), dimension(:, :, :), intent(in) :: f
    integer(c_int64_t), dimension(3) :: n
    n = int(shape(f), c_int64_t)
  end function shape3

  integer(c_int) function stagger_of(opt_stagger)
    integer, intent(in), optional :: opt_stagger
    stagger_of = -1_c_int  ! cell -> vertex by default (src/compact_schemes.f90:108-112)
    if (present(opt_stagger)) stagger_of = int(opt_stagger, c_int)
  end function stagger_of

  !! src/compact_schemes.f90:17-37
  subroutine lapl(f, dx, d2fdx2)
    real(pb_dp), dimension(:, :, :), intent(in) :: f
    real(pb_dp), dimension(3), intent(in) :: dx
    real(pb_dp), dimension(:, :, :), intent(out) :: d2fdx2
    real(c_double), dimension(3) :: h
    h = dx
    call must(c_pb_compact_lapl_host(PoissboxContext(), shape3(f), h, f, d2fdx2), "lapl")
  end subroutine lapl

  !! src/compact_schemes.f90:42-88 (df(:, :, :, 1:3))
  subroutine grad(f, dx, df)
    real(pb_dp), dimension(:, :, :), intent(in) :: f
    real(pb_dp), dimension(3), intent(in) :: dx
    real(pb_dp), dimension(:, :, :, :), intent(out) :: df
    real(c_double), dimension(3) :: h
    h = dx
    call must(c_pb_compact_grad_host(PoissboxContext(), shape3(f), h, f, df), "grad")
  end subroutine grad

  !! src/compact_schemes.f90:93-142
  subroutine interp(f, fi, opt_stagger)
    real(pb_dp), dimension(:, :, :), intent(in) :: f
    real(pb_dp), dimension(:, :, :), intent(out) :: fi
    integer, intent(in), optional :: opt_stagger
    call must(c_pb_compact_interp_host(PoissboxContext(), shape3(f), stagger_of(opt_stagger), f, &
         fi), "interp")
  end subroutine interp

  !! src/compact_schemes.f90:144-152
  subroutine interp_div(f, fi)
    real(pb_dp), dimension(:, :, :), intent(in) :: f
    real(pb_dp), dimension(:, :, :), intent(out) :: fi
    call interp(f, fi, +1)
  end subroutine interp_div

  !! src/compact_schemes.f90:207-257 (f(:, :, :, 1:3))
  subroutine div(f, dx, df)
    real(pb_dp), dimension(:, :, :, :), intent(in) :: f
    real(pb_dp), dimension(3), intent(in) :: dx
    real(pb_dp), dimension(:, :, :), intent(out) :: df
    real(c_double), dimension(3) :: h
    h = dx
    call must(c_pb_compact_div_host(PoissboxContext(), shape3(df), h, f, df), "div")
  end subroutine div

  subroutine line_op(kind, stagger, dx, f, df, what)
    integer(c_int), intent(in) :: kind, stagger
    real(pb_dp), intent(in) :: dx
    real(pb_dp), dimension(:), intent(in) :: f
    real(pb_dp), dimension(:), intent(out) :: df
    character(len=*), intent(in) :: what
    integer(c_int64_t) :: n
    n = size(f, kind=c_int64_t)
    if (size(df) /= n) then  ! src/compact_schemes.f90:177-180, :292-295
       print *, "ERROR: periodic gradient is same length as field!"
       stop 7
    end if
    call must(c_pb_compact_1d_batched_host(PoissboxContext(), kind, stagger, real(dx, c_double), &
         n, 1_c_int64_t, n, 1_c_int64_t, f, df), what)
  end subroutine line_op

  !! src/compact_schemes.f90:155-204
  subroutine grad_1d(f, dx, df, opt_stagger)
    real(pb_dp), dimension(:), intent(in) :: f
    real(pb_dp), intent(in) :: dx
    real(pb_dp), dimension(:), intent(out) :: df
    integer, intent(in), optional :: opt_stagger
    call line_op(0_c_int, stagger_of(opt_stagger), dx, f, df, "grad_1d")
  end subroutine grad_1d

  !! src/compact_schemes.f90:260-268
  subroutine div_1d(f, dx, df)
    real(pb_dp), dimension(:), intent(in) :: f
    real(pb_dp), intent(in) :: dx
    real(pb_dp), dimension(:), intent(out) :: df
    call grad_1d(f, dx, df, +1)
  end subroutine div_1d

  !! src/compact_schemes.f90:271-319
  subroutine interp_1d(f, fi, opt_stagger)
    real(pb_dp), dimension(:), intent(in) :: f
    real(pb_dp), dimension(:), intent(out) :: fi
    integer, intent(in), optional :: opt_stagger
    call line_op(1_c_int, stagger_of(opt_stagger), 0.0_pb_dp, f, fi, "interp_1d")
  end subroutine interp_1d

  !! src/compact_schemes.f90:322-329
  subroutine interp_1d_div(f, fi)
    real(pb_dp), dimension(:), intent(in) :: f
    real(pb_dp), dimension(:), intent(out) :: fi
    call interp_1d(f, fi, +1)
  end subroutine interp_1d_div

end module compact_schemes
