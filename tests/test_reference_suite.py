"""The reference's OWN test programs, run against this library.

poissbox_amd/fortran provides the reference's module names and procedures (constants,
coefficients, tridsol, compact_schemes) on the MI355X library. `make -C poissbox_amd/fortran
reftests` (run by __graft_entry__.build() where /root/reference exists) compiles the reference's
PETSc-free CTest programs from where they lie -- tests/tridiag/test_tdma{,_periodic,_sweeps}.f90,
tests/grad/test_grad_{1d,3d}.f90, tests/div/test_div_{1d,3d}.f90, tests/lapl/test_lapl.f90,
tests/coefficients/test_{compact,d2dx2,star}.f90 -- and links them against these modules; the
binaries (tests/_reftests, git-ignored) travel to the GPU box. Each program exits non-zero (`stop
1`) when one of its own checks fails, with the reference's own tolerances. The coefficient tests
need no GPU; the rest run the HIP kernels. (tests/coefficients/test_lapl.f90 is the reference's
always-failing stub, `stop 1` before any check, and is not built.)"""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(REPO, "tests", "_reftests")
CPU_PROGS = ["test_compact", "test_d2dx2", "test_star"]
GPU_PROGS = ["test_tdma", "test_tdma_periodic", "test_tdma_sweeps", "test_grad_1d",
             "test_grad_3d", "test_div_1d", "test_div_3d", "test_lapl"]


def _run(prog, env=None):
    path = os.path.join(RT, prog)
    if not os.path.exists(path):
        pytest.skip(f"{prog} not built (needs /root/reference at build time)")
    out = subprocess.run([path], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, f"{prog} failed (rc {out.returncode}):\n{out.stdout[-3000:]}{out.stderr[-2000:]}"
    return out.stdout


@pytest.mark.parametrize("prog", CPU_PROGS)
def test_reference_program_cpu(prog):
    _run(prog, env=dict(os.environ, HIP_VISIBLE_DEVICES=""))


@pytest.mark.gpu
@pytest.mark.parametrize("prog", GPU_PROGS)
def test_reference_program_gpu(prog):
    _run(prog)


def test_star_coeffs_match_oracle():
    """pb_lapl_star_coeffs / pb_lapl_1d_coeffs (src/coefficients.f90:22-48) bit-identical to the
    oracle's restatement, for non-uniform spacings."""
    import ctypes as C

    from oracle import oracle as O
    from poissbox_amd import _lib as L
    lib = L.load()
    for h in [(0.1, 0.2, 0.3), (1 / 64, 1 / 64, 1 / 64), (2.718, 0.155, 1e-3)]:
        c = np.zeros(27)
        assert lib.pb_lapl_star_coeffs(h[0], h[1], h[2], c.ctypes.data_as(L.P_d)) == 0
        assert np.array_equal(c, O.star_coeffs(h))
        c3 = np.zeros(3)
        assert lib.pb_lapl_1d_coeffs(C.c_double(h[0]), c3.ctypes.data_as(L.P_d)) == 0
        assert c3[0] == c[12] and c3[2] == c[14] and c3[1] == -2.0 * c3[0]  # x line; the centre
        assert c[13] == (c3[1] + (-2.0 * c[10])) + (-2.0 * c[4])              # sums x, y, z
