!! oracle/gen_fixtures.f90 -- golden-vector generator (TEST INFRASTRUCTURE ONLY).
!
! Our own driver program (not reference source). It is linked against the reference's own
! modules compiled where they lie (/root/reference/src/{constants,tridsol,compact_schemes}.f90,
! see oracle/Makefile target `ref`) and evaluates them on inputs written by
! tests/golden/make_golden.py, so the committed fixtures are outputs of the real reference. The
! 7-point operator (`star`) calls the reference's evaluate_laplacian_pointwise
! (src/poissbox.f90:128-148) with lapl_star_coeffs (src/coefficients.f90:22-48), cut out of those
! PETSc-dependent files by the Makefile, on each point's periodic 3x3x3 neighbourhood -- the loop
! of compute_lapl_pointwise (src/poissbox.f90:112-119) on a one-rank periodic DMDA.
!
! Manifest (text, one case per line):  op nx ny nz dx dy dz infile outfile
!   tdma | tdma_periodic | fwd_sweep : in = [a, b, c, d] (4*nx), out = [b', d'] (2*nx)
!   bwd_sweep                        : in = [b, c, d] (3*nx),    out = d' (nx)
!   grad_1d | div_1d                 : in = f (nx), out = df (nx), uses dx
!   interp_1d | interp_1d_div        : in = f (nx), out = fi (nx)
!   grad                             : in = f (N),  out = df (3N)
!   div                              : in = f (3N), out = df (N)
!   interp | interp_div              : in = f (N),  out = fi (N)
!   lapl                             : in = f (N),  out = d2f (N)
!   star                             : in = f (N),  out = A f (N), uses dx, dy, dz
program gen_fixtures

  use constants
  use tridsol
  use compact_schemes
  use ref_pointwise, only: evaluate_laplacian_pointwise

  implicit none

  character(len=512) :: manifest, op, infile, outfile
  integer :: nx, ny, nz, ios, u
  real(pb_dp) :: dx, dy, dz

  call get_command_argument(1, manifest)
  open(newunit=u, file=trim(manifest), status='old', action='read')
  do
     read(u, *, iostat=ios) op, nx, ny, nz, dx, dy, dz, infile, outfile
     if (ios /= 0) exit
     call run_case(trim(op), nx, ny, nz, [dx, dy, dz], trim(infile), trim(outfile))
  end do
  close(u)

contains

  subroutine read_vec(fname, v)
    character(len=*), intent(in) :: fname
    real(pb_dp), dimension(:), intent(out) :: v
    integer :: iu
    open(newunit=iu, file=fname, access='stream', form='unformatted', status='old', action='read')
    read(iu) v
    close(iu)
  end subroutine read_vec

  subroutine write_vec(fname, v)
    character(len=*), intent(in) :: fname
    real(pb_dp), dimension(:), intent(in) :: v
    integer :: iu
    open(newunit=iu, file=fname, access='stream', form='unformatted', status='replace', &
         action='write')
    write(iu) v
    close(iu)
  end subroutine write_vec

  subroutine run_case(op, nx, ny, nz, h, infile, outfile)
    character(len=*), intent(in) :: op, infile, outfile
    integer, intent(in) :: nx, ny, nz
    real(pb_dp), dimension(3), intent(in) :: h

    real(pb_dp), allocatable :: buf(:), a(:), b(:), c(:), d(:)
    real(pb_dp), allocatable :: f3(:, :, :), g3(:, :, :), v4(:, :, :, :)
    integer :: n

    n = nx
    select case (op)
    case ('tdma', 'tdma_periodic', 'fwd_sweep')
       allocate(buf(4 * n))
       call read_vec(infile, buf)
       a = buf(1:n); b = buf(n+1:2*n); c = buf(2*n+1:3*n); d = buf(3*n+1:4*n)
       if (op == 'tdma') then
          call tdma(a, b, c, d)
       else if (op == 'tdma_periodic') then
          call tdma_periodic(a, b, c, d)
       else
          call fwd_sweep(a, b, c, d)
       end if
       call write_vec(outfile, [b, d])
    case ('bwd_sweep')
       allocate(buf(3 * n))
       call read_vec(infile, buf)
       b = buf(1:n); c = buf(n+1:2*n); d = buf(2*n+1:3*n)
       call bwd_sweep(b, c, d)
       call write_vec(outfile, d)
    case ('grad_1d', 'div_1d', 'interp_1d', 'interp_1d_div')
       allocate(a(n), d(n))
       call read_vec(infile, a)
       if (op == 'grad_1d') call grad_1d(a, h(1), d)
       if (op == 'div_1d') call div_1d(a, h(1), d)
       if (op == 'interp_1d') call interp_1d(a, d)
       if (op == 'interp_1d_div') call interp_1d_div(a, d)
       call write_vec(outfile, d)
    case ('grad')
       allocate(f3(nx, ny, nz), v4(nx, ny, nz, 3), buf(nx * ny * nz))
       call read_vec(infile, buf)
       f3 = reshape(buf, [nx, ny, nz])
       call grad(f3, h, v4)
       call write_vec(outfile, reshape(v4, [3 * nx * ny * nz]))
    case ('div')
       allocate(v4(nx, ny, nz, 3), g3(nx, ny, nz), buf(3 * nx * ny * nz))
       call read_vec(infile, buf)
       v4 = reshape(buf, [nx, ny, nz, 3])
       call div(v4, h, g3)
       call write_vec(outfile, reshape(g3, [nx * ny * nz]))
    case ('interp', 'interp_div', 'lapl')
       allocate(f3(nx, ny, nz), g3(nx, ny, nz), buf(nx * ny * nz))
       call read_vec(infile, buf)
       f3 = reshape(buf, [nx, ny, nz])
       if (op == 'interp') call interp(f3, g3)
       if (op == 'interp_div') call interp_div(f3, g3)
       if (op == 'lapl') call lapl(f3, h, g3)
       call write_vec(outfile, reshape(g3, [nx * ny * nz]))
    case ('star')
       allocate(f3(nx, ny, nz), g3(nx, ny, nz), buf(nx * ny * nz))
       call read_vec(infile, buf)
       f3 = reshape(buf, [nx, ny, nz])
       call star_apply(f3, h, g3)
       call write_vec(outfile, reshape(g3, [nx * ny * nz]))
    case default
       print *, "unknown op ", op
       stop 2
    end select
  end subroutine run_case

  ! b(i,j,k) = evaluate_laplacian_pointwise(x(i-1:i+1, j-1:j+1, k-1:k+1)) with periodic wrap (the
  ! ghosted local vector DMGlobalToLocal fills on one rank)
  subroutine star_apply(x, h, b)
    real(pb_dp), dimension(:, :, :), intent(in) :: x
    real(pb_dp), dimension(3), intent(in) :: h
    real(pb_dp), dimension(:, :, :), intent(out) :: b
    real(pb_dp) :: nb(3, 3, 3)
    integer :: i, j, k, di, dj, dk, nx, ny, nz
    nx = size(x, 1); ny = size(x, 2); nz = size(x, 3)
    do k = 1, nz
       do j = 1, ny
          do i = 1, nx
             do dk = -1, 1
                do dj = -1, 1
                   do di = -1, 1
                      nb(di + 2, dj + 2, dk + 2) = x(modulo(i + di - 1, nx) + 1, &
                           modulo(j + dj - 1, ny) + 1, modulo(k + dk - 1, nz) + 1)
                   end do
                end do
             end do
             b(i, j, k) = evaluate_laplacian_pointwise(nb, h)
          end do
       end do
    end do
  end subroutine star_apply

end program gen_fixtures
