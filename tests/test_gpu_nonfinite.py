"""GPU tier: non-finite inputs end every CG path with PETSc's reason, not a convergence.

PETSc's KSPSolve_CG checks every norm (KSPCheckNorm) and dot (KSPCheckDot) it forms and stops
with KSP_DIVERGED_NANORINF (-9) on a NaN or Inf; the oracle restates exactly that
(oracle/pb_oracle.c pbo_cg_solve / cg_solve_single_reduction). The GPU iteration forms ||z|| from
shifted sums (sum z^2 - N mu^2), whose NaN once clamped to 0 and reported CONVERGED_ATOL with
x = 0. Cases: a right-hand side with one NaN, +Inf or -Inf (stage 0: the
shifted sum is NaN), and one scaled to 1e150 (the norms stay finite, a later dot or norm may
overflow) -- for -pc_type jacobi / none / mg / fft, with and without -ksp_cg_single_reduction, on
1 and 2 ranks (host transport). Bars: the oracle's reason and iteration count, NaN where its
logged history has NaN, finite entries within HIST_RTOL.
Reference: src/poissbox.f90:296 (KSPSolve), SURVEY.md §5 (NaN/Inf guard).
"""
import numpy as np
import pytest

import poissbox_amd as pb
from oracle import oracle as O
from parity_bars import HIST_RTOL, HIST_RTOL_PC

pytestmark = pytest.mark.gpu

SEED = 20231015
KINDS = ["nan", "inf", "-inf", "big"]


def _rhs(pc, kind):
    n3 = (64, 64, 64) if pc == "fft" else (16, 16, 16)  # the spectral PC takes extents >= 64
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    if kind == "big":
        b = b * 1e150
    else:
        b[37] = {"nan": np.nan, "inf": np.inf, "-inf": -np.inf}[kind]
    return n3, h, b


def _check(reason, its, hist, ro, itso, ho, pc, tag):
    assert (reason, its) == (ro, itso), (tag, reason, its, ro, itso)
    hist, ho = np.asarray(hist), np.asarray(ho)
    assert hist.shape == ho.shape, (tag, hist, ho)
    bad = ~np.isfinite(ho)
    assert np.array_equal(bad, ~np.isfinite(hist)), (tag, hist, ho)
    if (~bad).any():
        bar = HIST_RTOL_PC if pc == "mg" else HIST_RTOL
        rel = np.max(np.abs(hist[~bad] - ho[~bad]) / ho[~bad])
        assert rel < bar, (tag, rel)


def _oracle_sr(pc, sr):
    # the single-reduction iteration runs with the Jacobi / no PC; with a stored-z PC (mg, fft)
    # the library runs KSPSolve_CG (include/poissbox_gpu.h), so that is the oracle's form there
    return sr if pc in ("jacobi", "none") else 0


def _opts(pc, sr):
    return ["-pc_type", pc, "-ksp_rtol", "1e-8"] + (["-ksp_cg_single_reduction"] if sr else [])


def _mats(da, h, pc):
    if pc == "fft":  # the spectral PC inverts P's symbol: P = A = the 7-point operator
        A = pb.Mat(da, pb.STAR7, h)
        return A, A
    P, A, _, _ = pb.initialise_linear_system(da, h)
    return P, A


@pytest.mark.parametrize("sr", [0, 1])
@pytest.mark.parametrize("pc", ["jacobi", "none", "mg", "fft"])
@pytest.mark.parametrize("kind", KINDS)
def test_nonfinite_rhs_one_rank(ctx, pc, sr, kind):
    n3, h, b = _rhs(pc, kind)
    _, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-8, pc=pc, single_reduction=_oracle_sr(pc, sr))
    if kind != "big":
        assert (ro, itso) == (-9, 0)
    da = pb.DA(ctx, n3)
    P, A = _mats(da, h, pc)
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, _opts(pc, sr))
    _check(reason, its, hist, ro, itso, ho, pc, f"{pc} sr={sr} {kind}")


@pytest.mark.parametrize("sr", [0, 1])
@pytest.mark.parametrize("pc", ["jacobi", "none", "mg", "fft"])
@pytest.mark.parametrize("kind", ["nan", "inf", "big"])
def test_nonfinite_rhs_two_ranks(pc, sr, kind):
    from test_gpu_parity import run_ranks
    n3, h, b = _rhs(pc, kind)
    _, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-8, pc=pc, single_reduction=_oracle_sr(pc, sr),
                                 nranks=2)

    def body(ctx, rank):
        da = pb.DA(ctx, n3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        P, A = _mats(da, h, pc)
        x, bv = pb.Vec(da), pb.Vec(da)
        bv.set_values(b.reshape(n3[2], -1)[k0:k0 + nk])
        return pb.solve(P, A, x, bv, _opts(pc, sr))

    for reason, its, hist in run_ranks(2, body):
        _check(reason, its, hist, ro, itso, ho, pc, f"2 ranks {pc} sr={sr} {kind}")


@pytest.mark.parametrize("sr", [0, 1])
def test_nan_operator_is_nanorinf(ctx, sr):
    """A finite right-hand side but a NaN grid spacing in A only (P's diagonal stays finite): the
    first p.w is NaN -> KSPCheckDot (KSPSolve_CG: its 1); the single-reduction iteration, which
    checks only beta, stops at the next norm -- as the oracle's restatements of both."""
    n3 = (16, 16, 16)
    h = (1.0 / 16,) * 3
    b = O.stencil(O.fill_random(4096, SEED), n3, h)
    da = pb.DA(ctx, n3)
    P = pb.Mat(da, pb.ASSEMBLED27, h)
    A = pb.Mat(da, pb.STAR7, (np.nan, h[1], h[2]))
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, _opts("jacobi", sr))
    assert reason == -9 and its == 1, (reason, its, hist)
    assert np.isfinite(hist[0])
