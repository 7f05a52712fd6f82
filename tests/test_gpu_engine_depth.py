"""GPU tier: the stencil engine's two-plane look-ahead (tuning engine_depth = 2, star7_kernel
DEPTH 2: CG pass A) against the one-plane form -- the same loads and the same
per-point arithmetic in the same order, so reason, iteration count, history and x are bit for bit
equal. Shapes cover odd z-chunk lengths (the 2-unrolled march's tail step), one-plane chunks, odd
x (one point per lane), TY 1 / 2 / 4, 8-row tiles, and a 2-rank split grid (interior and boundary
launches, folded and unfolded).
Reference: src/poissbox.f90:112-119 (the stencil), :296 (KSPSolve)."""
import numpy as np
import pytest

import poissbox_amd as pb
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 20231015
SHAPES = [(64, 32, 16), (32, 24, 17), (16, 16, 3), (34, 10, 5), (33, 9, 7), (128, 64, 9),
          (256, 64, 13)]


def _solve(ctx, n3, h, b, opts):
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, opts)
    return reason, its, np.asarray(hist), x.get_values()


@pytest.mark.parametrize("fold", ["1", "0"])
@pytest.mark.parametrize("n3", SHAPES)
def test_engine_depth_bit_identical(ctx, n3, fold, tune):
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    opts = ["-ksp_rtol", "0", "-ksp_max_it", "13"]
    out = {}
    for depth in ("1", "2"):
        tune.set("cg_fold", fold)
        tune.set("engine_depth", depth)
        out[depth] = _solve(ctx, n3, h, b, opts)
    (r1, i1, h1, x1), (r2, i2, h2, x2) = out["1"], out["2"]
    assert (r1, i1) == (r2, i2) == (-3, 13)
    assert np.array_equal(h1, h2) and np.array_equal(x1, x2)
    _, ro, itso, ho = O.cg_solve(b, n3, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=13)
    assert (ro, itso) == (r2, i2)
    assert np.max(np.abs(h2 - np.asarray(ho)) / np.asarray(ho)) < 1e-11


@pytest.mark.parametrize("fold", ["1", "0"])
def test_engine_depth_two_ranks_bit_identical(fold, tune):
    from test_gpu_parity import run_ranks
    n3 = (64, 48, 18)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    opts = ["-ksp_rtol", "0", "-ksp_max_it", "11"]

    def body(ctx, rank):
        da = pb.DA(ctx, n3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        P, A, x, bv = pb.initialise_linear_system(da, h)
        bv.set_values(b.reshape(n3[2], -1)[k0:k0 + nk])
        reason, its, hist = pb.solve(P, A, x, bv, opts)
        return reason, its, np.asarray(hist), x.get_values()

    res = {}
    for depth in ("1", "2"):
        tune.set("cg_fold", fold)
        tune.set("engine_depth", depth)
        res[depth] = run_ranks(2, body)
    for a, c in zip(res["1"], res["2"]):
        assert a[:2] == c[:2] == (-3, 11)
        assert np.array_equal(a[2], c[2]) and np.array_equal(a[3], c[3])
