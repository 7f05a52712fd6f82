!! poissbox_constants.f90 -- the working precision shared by every module here, under the module
!! name the reference's code expects (`use constants`, src/constants.f90): fp64, matching the
!! C ABI's double.
module constants
  use iso_c_binding, only: c_double
  implicit none
  private
  integer, parameter, public :: pb_dp = c_double
end module constants
