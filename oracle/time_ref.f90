!! oracle/time_ref.f90 -- CPU timing of the REAL reference routines (TEST/MEASUREMENT INFRASTRUCTURE).
!
! Our own driver program (not reference source), linked like gen_fixtures.f90 against the
! reference's constants/tridsol/compact_schemes modules compiled where they lie under
! /root/reference (oracle/Makefile target `ref`, outputs only in oracle/_ref/). It gives
! scripts/bench_rows.py the reference's own single-core CPU rate beside each GPU row
! (kind "reference"):
!
!   time_ref <op> <n> <min_seconds>
!     tdma | tdma_periodic | grad_1d : one line of n points (diagonally dominant system / random
!                                      field), repeated until min_seconds have passed
!     lapl                           : the 3-D compact Laplacian on an n^3 grid, repeated likewise
!
! Prints one line: {"op": ..., "n": ..., "reps": ..., "seconds": ..., "dofs_per_s": ...}
program time_ref

  use constants
  use tridsol
  use compact_schemes

  implicit none

  character(len=64) :: op, arg
  integer :: n, reps
  integer(8) :: t0, t1, rate
  real(pb_dp) :: tmin, secs, dofs
  real(pb_dp), allocatable :: a(:), b(:), c(:), d(:), a0(:), b0(:), c0(:), d0(:)
  real(pb_dp), allocatable :: f3(:, :, :), g3(:, :, :)
  real(pb_dp) :: h(3), sink

  call get_command_argument(1, op)
  call get_command_argument(2, arg)
  read(arg, *) n
  call get_command_argument(3, arg)
  read(arg, *) tmin

  sink = 0.0_pb_dp
  reps = 0
  call system_clock(t0, rate)
  select case (trim(op))
  case ('tdma', 'tdma_periodic')
     allocate(a0(n), b0(n), c0(n), d0(n))
     call random_number(a0)
     call random_number(c0)
     call random_number(d0)
     call random_number(b0)
     b0 = 10.0_pb_dp * b0 + 3.0_pb_dp  ! diagonally dominant
     dofs = real(n, pb_dp)
     do
        a = a0; b = b0; c = c0; d = d0
        if (trim(op) == 'tdma') then
           call tdma(a, b, c, d)
        else
           call tdma_periodic(a, b, c, d)
        end if
        sink = sink + d(1)
        reps = reps + 1
        call system_clock(t1)
        if (real(t1 - t0, pb_dp) / real(rate, pb_dp) >= tmin) exit
     end do
  case ('grad_1d')
     allocate(a0(n), d(n))
     call random_number(a0)
     dofs = real(n, pb_dp)
     do
        call grad_1d(a0, 0.01_pb_dp, d)
        sink = sink + d(1)
        reps = reps + 1
        call system_clock(t1)
        if (real(t1 - t0, pb_dp) / real(rate, pb_dp) >= tmin) exit
     end do
  case ('lapl')
     allocate(f3(n, n, n), g3(n, n, n))
     call random_number(f3)
     h = 2.0_pb_dp * acos(-1.0_pb_dp) / real(n, pb_dp)
     dofs = real(n, pb_dp)**3
     do
        call lapl(f3, h, g3)
        sink = sink + g3(1, 1, 1)
        reps = reps + 1
        call system_clock(t1)
        if (real(t1 - t0, pb_dp) / real(rate, pb_dp) >= tmin) exit
     end do
  case default
     print *, "unknown op ", trim(op)
     stop 2
  end select
  call system_clock(t1)
  secs = real(t1 - t0, pb_dp) / real(rate, pb_dp)
  ! the copies of the inputs (tdma*) are inside the timed loop, as a caller's would be
  write(*, '(A,A,A,I0,A,I0,A,ES12.5,A,ES12.5,A,ES10.3,A)') '{"op": "', trim(op), '", "n": ', n, &
       ', "reps": ', reps, ', "seconds": ', secs, ', "dofs_per_s": ', dofs * reps / secs, &
       ', "checksum": ', sink, '}'

end program time_ref
