"""GPU tier: single-reduction CG (-ksp_cg_single_reduction, PETSc KSPSolve_CG_SingleReduction).

The GPU iteration is two stencil-engine passes and ONE reduction: pass P forms p from (r, p_old) on
load, w = A p, r' = r - alpha w (p, r' stored; the deferred x update every 4th iteration), pass S
takes t = dinv r' - mu on load, s = A t and the five sums (z'z, z'r, the mean, z'As); p'w comes from
PETSc's recurrence delta - beta^2 dpiold / betaold^2. It differs from PETSc's own single-reduction
form only in recomputing w = A p instead of the recurrence w = s + (beta/betaold) w (equal in exact
arithmetic; oracle form 2 restates exactly that). Bars: the oracle's faithful PETSc restatement
(form 1) -- same reason and iteration count, history within HIST_RTOL, x within X_RTOL -- and the
KSPSolve_CG oracle's iteration count (oracle/pb_oracle.c cg_solve_single_reduction).
"""
import numpy as np
import pytest

import poissbox_amd as pb
from oracle import oracle as O
from parity_bars import HIST_RTOL, check_history, check_x

pytestmark = pytest.mark.gpu

SEED = 20231015
SR = ["-ksp_cg_single_reduction"]


def _case(n3, seed=SEED, nthreads=1):
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, seed), n3, h, nthreads=nthreads)
    return h, b


def _solve(ctx, n3, h, b, opts, **kw):
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    k = pb.KSP(A, P, pb.ksp_options(opts, **kw))
    reason, its, hist = k.solve(bv, x)
    xs = x.get_values()
    k.destroy()
    return reason, its, np.asarray(hist), xs


@pytest.mark.parametrize("n3,rtol", [((16, 16, 16), 1e-5), ((32, 32, 32), 1e-10),
                                     ((64, 64, 64), 1e-10), ((24, 20, 12), 1e-8),
                                     # odd x (one point per lane), 2 / 1 rows per wave, odd z
                                     ((17, 18, 9), 1e-8), ((130, 6, 33), 1e-8),
                                     # 512^2 planes (8-row tiles of the read-only pass S,
                                     # the x-update pass), short z
                                     ((512, 512, 4), 1e-6), ((256, 256, 6), 1e-6)])
def test_single_reduction_matches_oracle(ctx, n3, rtol):
    h, b = _case(n3)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=rtol, single_reduction=1)
    _, ro0, itso0, _ = O.cg_solve(b, n3, h, rtol=rtol)
    assert (ro, itso) == (ro0, itso0) == (2, itso)  # same its as KSPSolve_CG
    reason, its, hist, xs = _solve(ctx, n3, h, b, SR + ["-ksp_rtol", str(rtol)])
    assert (reason, its) == (ro, itso)
    check_history(hist, ho, tag="sr")
    check_x(xs, xo)


def test_single_reduction_after_nan_in_lds(ctx):
    """The one-pass kernel's warm-up steps read its LDS row exchange before any wave wrote it:
    stale LDS of an earlier kernel (here the spectral PC's tiles, fed NaN) must not reach the
    sums (a 16^3 solve once stopped at its 1, reason ATOL, after 380 other GPU tests)."""
    n3 = (16, 16, 16)
    h, b = _case(n3)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-5, single_reduction=1)
    for _ in range(2):
        m = (64, 64, 64)
        da = pb.DA(ctx, m, (2 * np.pi,) * 3)
        P = pb.Mat(da, pb.COMPACT, tuple(2 * np.pi / v for v in m))
        k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
        rv, zv = pb.Vec(da), pb.Vec(da)
        rv.set_values(np.full(int(np.prod(m)), np.nan))
        k.pc_apply(rv, zv)
        k.destroy()
        reason, its, hist, xs = _solve(ctx, n3, h, b, SR + ["-ksp_rtol", "1e-5"])
        assert (reason, its) == (ro, itso)
        check_history(hist, ho)


@pytest.mark.parametrize("defer", ["0", "2", "4"])
@pytest.mark.parametrize("max_it", [1, 2, 3, 4, 5, 8, 9, 11])
def test_single_reduction_deferred_x_max_it(ctx, defer, max_it, tune):
    """Stopping at every position of the deferred-x cycle (DIVERGED_ITS at max_it): x and the
    history as the oracle's."""
    tune.setenv("PB_CG_DEFER_X", defer)
    n3 = (32, 24, 16)
    h, b = _case(n3)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=max_it,
                                  single_reduction=1)
    reason, its, hist, xs = _solve(ctx, n3, h, b, SR + ["-ksp_rtol", "0", "-ksp_atol", "0",
                                                        "-ksp_divtol", "1e300",
                                                        "-ksp_max_it", str(max_it)])
    assert (reason, its) == (ro, itso) == (-3, max_it)
    check_history(hist, ho)
    check_x(xs, xo, bar=1e-12)


@pytest.mark.parametrize("case", ["rtol", "max_it1", "max_it2", "max_it9", "split_iterate"])
def test_single_reduction_folded_bit_identical(ctx, case):
    """One rank: the residual-sum stage folded into the next pass P's prologue (check_every >= 2)
    against the separate finalize launch (check_every 1) -- bit for bit (same partial-sum
    order); split begin / iterate(3) / iterate(5) / iterate(rest) / end swaps the state slots'
    parity across calls."""
    n3 = (64, 32, 16)
    h, b = _case(n3)
    opts = {"rtol": ["-ksp_rtol", "1e-9"], "max_it1": ["-ksp_rtol", "0", "-ksp_max_it", "1"],
            "max_it2": ["-ksp_rtol", "0", "-ksp_max_it", "2"],
            "max_it9": ["-ksp_rtol", "0", "-ksp_max_it", "9"],
            "split_iterate": ["-ksp_rtol", "1e-9"]}[case]
    out = {}
    for check in (8, 1):
        da = pb.DA(ctx, n3)
        P, A, x, bv = pb.initialise_linear_system(da, h)
        bv.set_values(b)
        k = pb.KSP(A, P, pb.ksp_options(SR + opts, check_every=check))
        if case == "split_iterate":
            k.begin(bv, x)
            k.iterate(3)
            k.iterate(5)
            k.iterate(10000)
            reason, its, hist = k.end()
        else:
            reason, its, hist = k.solve(bv, x)
        k.destroy()
        out[check] = (reason, its, np.asarray(hist), x.get_values())
    (r1, i1, h1, x1), (r0, i0, h0, x0) = out[8], out[1]
    assert (r1, i1) == (r0, i0)
    assert np.array_equal(h1, h0) and np.array_equal(x1, x0)
    kw = {"rtol": float(opts[1])} if opts[1] != "0" else {"rtol": 0.0, "max_it": int(opts[3])}
    xo, ro, itso, ho = O.cg_solve(b, n3, h, single_reduction=1, **kw)
    assert (r1, i1) == (ro, itso)
    check_history(h1, ho)
    check_x(x1, xo)


def test_single_reduction_pc_none(ctx):
    n3 = (16, 16, 16)
    h, b = _case(n3, seed=5)
    _, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-8, pc="none", single_reduction=1)
    reason, its, hist, _ = _solve(ctx, n3, h, b, SR + ["-pc_type", "none", "-ksp_rtol", "1e-8"])
    assert (reason, its) == (ro, itso)
    check_history(hist, ho)


def test_single_reduction_zero_rhs(ctx):
    n3 = (8, 8, 8)
    reason, its, hist, xs = _solve(ctx, n3, (1 / 8,) * 3, np.zeros(512), SR)
    assert reason == 3 and its == 0 and len(hist) == 1 and hist[0] == 0.0
    assert not np.any(xs)


def test_single_reduction_nonzero_mean_rhs(ctx):
    """b with a constant component (not in the range of A): the null-space projection of z keeps
    the iteration well defined. r keeps the constant (sum r = sum b), so every rounding of r is
    relative to a vector far larger than z: the oracle's own three forms (KSPSolve_CG, PETSc's
    single reduction, w recomputed) agree to 1e-12 while ||z_k|| > 1e-4 ||z_0|| and drift apart to
    2.4e-2 at ||z_k|| ~ 1e-9 ||z_0|| (same reason and its). Bars: same reason / its; history
    within HIST_RTOL down to 1e-4 ||z_0||, and at every entry within HIST_RTOL plus three times
    the spread, at that entry, of 14 equivalent runs of the oracle (its three forms, each with its
    sums in 1, 2, 3, 4 and 8 thread orders): the rounding the reference algorithm itself leaves
    undetermined there. Leave-one-out over those runs, a single-reduction run in another sum
    order stays within 0.9 of twice the others' spread. x (mean removed) within 1e-8."""
    n3 = (32, 16, 16)
    h, b = _case(n3)
    b = b + 3.0
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-9, single_reduction=1)
    reason, its, hist, xs = _solve(ctx, n3, h, b, SR + ["-ksp_rtol", "1e-9"])
    assert (reason, its) == (ro, itso)
    head = ho > 1e-4 * ho[0]
    check_history(hist[head], ho[head])
    ho = np.asarray(ho)
    spread = np.zeros_like(ho)
    for form in (0, 1, 2):  # KSPSolve_CG, PETSc's single reduction, w recomputed
        for nt in (1, 2, 3, 4, 8):
            if (form, nt) == (1, 1):
                continue
            _, rf, itf, hf = O.cg_solve(b, n3, h, rtol=1e-9, single_reduction=form, nthreads=nt)
            assert (rf, itf) == (ro, itso), (form, nt)
            spread = np.maximum(spread, np.abs(np.asarray(hf) - ho))
    bar = HIST_RTOL * ho + 3.0 * spread
    dev = np.abs(np.asarray(hist) - ho)
    assert np.all(dev <= bar), np.max(dev / bar)
    xm, xom = xs - xs.mean(), xo - xo.mean()
    assert np.max(np.abs(xm - xom)) < 1e-8 * np.max(np.abs(xom))


def test_single_reduction_option_off_and_other_pcs(ctx):
    """-ksp_cg_single_reduction false is the KSPSolve_CG iteration; with a stored-z PC (mg) the
    KSPSolve_CG iteration runs (include/poissbox_gpu.h) -- bit-identical to no option."""
    n3 = (32, 32, 32)
    h, b = _case(n3)
    base = _solve(ctx, n3, h, b, ["-ksp_rtol", "1e-8"])
    off = _solve(ctx, n3, h, b, SR + ["false", "-ksp_rtol", "1e-8"])
    assert base[:2] == off[:2] and np.array_equal(base[2], off[2])
    mg0 = _solve(ctx, n3, h, b, ["-pc_type", "mg", "-ksp_rtol", "1e-8"])
    mg1 = _solve(ctx, n3, h, b, SR + ["-pc_type", "mg", "-ksp_rtol", "1e-8"])
    assert mg0[:2] == mg1[:2] and np.array_equal(mg0[2], mg1[2])


def test_single_reduction_full_256(ctx):
    """The whole 256^3 solve (config 2's grid) to rtol 1e-10: the faithful restatement's reason
    and iteration count, every history entry within the bar (oracle on 8 threads)."""
    n3 = (256, 256, 256)
    h, b = _case(n3, nthreads=8)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, single_reduction=1, nthreads=8)
    reason, its, hist, xs = _solve(ctx, n3, h, b, SR + ["-ksp_rtol", "1e-10"])
    assert (reason, its) == (ro, itso)
    check_history(hist, ho, tag="sr256")
    check_x(xs, xo)


@pytest.mark.parametrize("nranks,n", [(2, (16, 16, 12)), (3, (16, 16, 12)), (3, (20, 16, 7)),
                                       # 1- and 2-plane slabs (no interior launch)
                                       (4, (16, 12, 6)),
                                       # config 4's rank count (two-plane slabs)
                                       (8, (16, 16, 16)),
                                       (2, (512, 512, 12))])
def test_multirank_single_reduction(nranks, n):
    """N ranks (host transport, one GPU): p's boundary planes and r''s raw boundary planes are
    exchanged, the five sums allreduced once per iteration; history / x as the oracle's."""
    from test_gpu_parity import run_ranks
    N = int(np.prod(n))
    h = tuple(1.0 / m for m in n)
    b = O.stencil(O.fill_random(N, SEED), n, h)
    xo, ro, itso, ho = O.cg_solve(b, n, h, rtol=1e-8, single_reduction=1)

    def body(ctx, rank):
        da = pb.DA(ctx, n)
        (_, _, k0), (_, _, nk) = da.get_corners()
        P, A, x, bv = pb.initialise_linear_system(da, h)
        bv.set_values(b.reshape(n[2], -1)[k0:k0 + nk])
        reason, its, hist = pb.solve(P, A, x, bv, SR + ["-ksp_rtol", "1e-8"])
        return reason, its, hist, k0, nk, x.get_values()

    for reason, its, hist, k0, nk, xs in run_ranks(nranks, body):
        assert (reason, its) == (ro, itso)
        check_history(hist, ho)
        check_x(xs, xo.reshape(n[2], -1)[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


@pytest.mark.parametrize("ddiff", [0, 1])
@pytest.mark.parametrize("n3", [(32, 32, 32), (24, 20, 12), (17, 18, 9), (130, 6, 33),
                                (512, 512, 4), (64, 13, 16)])
def test_single_reduction_delta_forms(ctx, tune, n3, ddiff):
    """The one-pass kernel's delta = z'A z as t.(A t) (two halo rows per block side) or in the
    difference form (-sum c (forward difference)^2, one row fewer to fetch twice; r06): both on
    the oracle's reason, iterations and history (PETSc's single-reduction form)."""
    tune.set("sr_ddiff", ddiff)
    h, b = _case(n3)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-9, single_reduction=1)
    reason, its, hist, xs = _solve(ctx, n3, h, b, SR + ["-ksp_rtol", "1e-9"])
    assert (reason, its) == (ro, itso)
    check_history(hist, ho, tag=f"sr_ddiff{ddiff}")
    check_x(xs, xo)
