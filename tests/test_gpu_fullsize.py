"""GPU tier at the BASELINE.json sizes: 512^3 on one GPU (config 3) and the 1024x1024x128 slab
one GPU holds of the 1024^3 grid on 8 GPUs (config 4).

The operator and the synthetic input are checked bit-exact against the oracle over the whole grid
(the oracle's C stencil finishes 512^3 in about a second on 16 host threads). CG is checked
through size-independent properties: the stopping reason, the true residual ||b - A x|| / ||b||
recomputed with the product's own MatMult, the error against x_true (mean-free, the null space),
the grid-independent MG iteration count (13, as from 32^3 up; test_gpu_parity checks it against
the oracle at small sizes), and a fixed-iteration CG history against the oracle's at 512^3.
"""
import os

import numpy as np
import pytest

import poissbox_amd as pb
from oracle import oracle as O
from parity_bars import check_history, check_x

pytestmark = pytest.mark.gpu

SEED = 20231015
THREADS = min(16, os.cpu_count() or 1)


def _system(ctx, n):
    h = tuple(1.0 / m for m in n)
    da = pb.DA(ctx, n)
    P, A, x, b = pb.initialise_linear_system(da, h)
    xt = pb.Vec(da)
    xt.set_random(SEED)
    A.mult(xt, b)  # b = A x_true (src/example.f90:70-72)
    return da, h, P, A, x, b, xt


def _true_residual(A, x, b):
    r = b.duplicate()
    A.mult(x, r)
    r.aypx(-1.0, b)  # r = b - A x
    out = r.norm() / b.norm()
    r.destroy()
    return out


def _mean_free_err(x, xt):
    e = x.duplicate()
    x.copy_to(e)
    e.axpy(-1.0, xt)
    s = e.sum()
    ev = e.get_values()
    ev -= s / ev.size
    ref = xt.get_values()
    e.destroy()
    return np.max(np.abs(ev)) / np.max(np.abs(ref - ref.mean()))


@pytest.mark.parametrize("n", [(512, 512, 512), (1024, 1024, 128)])
def test_matvec_full_grid_bit_exact(ctx, n):
    """Synthetic x_true and A x_true over the whole grid, both z-march directions."""
    N = int(np.prod(n))
    h = tuple(1.0 / m for m in n)
    xs = O.fill_random(N, SEED)
    ref = O.stencil(xs, n, h, nthreads=THREADS)
    da = pb.DA(ctx, n)
    A = pb.Mat(da, pb.STAR7)
    x, y = pb.Vec(da), pb.Vec(da)
    x.set_random(SEED)
    assert np.array_equal(x.get_values(), xs)
    del xs
    for _ in range(2):  # consecutive applies march in opposite z directions
        A.mult(x, y)
        assert np.array_equal(y.get_values(), ref)
    for o in (A, x, y):
        o.destroy()
    da.destroy()


def test_cg_jacobi_512_fixed_iterations_vs_oracle(ctx):
    """30 CG + Jacobi iterations at 512^3: the ||z_k|| history against the oracle's."""
    n = (512, 512, 512)
    its = 30
    da, h, P, A, x, b, xt = _system(ctx, n)
    bo = b.get_values()
    _, ro, itso, ho = O.cg_solve(bo, n, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=its,
                                 nthreads=THREADS)
    del bo
    opts = ["-ksp_type", "cg", "-pc_type", "jacobi", "-ksp_rtol", "0", "-ksp_atol", "0",
            "-ksp_max_it", str(its), "-ksp_divtol", "1e300"]
    reason, it, hist = pb.solve(P, A, x, b, opts)
    assert (reason, it) == (ro, itso) == (reason, its)
    check_history(hist, ho)
    for o in (P, A, x, b, xt):
        o.destroy()
    da.destroy()


def test_cg_jacobi_256_full_history_vs_oracle(ctx):
    """BASELINE config 2: 256^3 fp64 CG + Jacobi to rtol 1e-10 on one GPU. Same stopping reason
    and iteration count as the oracle (its restatement of PETSc KSPSolve_CG, src/poissbox.f90:
    269-298), every ||z_k|| of the ~674-iteration history within the CG bar, x within its bar."""
    n = (256, 256, 256)
    da, h, P, A, x, b, xt = _system(ctx, n)
    bo = b.get_values()
    xo, ro, itso, ho = O.cg_solve(bo, n, h, rtol=1e-10, nthreads=THREADS)
    del bo
    reason, its, hist = pb.solve(P, A, x, b, ["-ksp_type", "cg", "-pc_type", "jacobi",
                                              "-ksp_rtol", "1e-10"])
    assert reason == ro == 2
    assert its == itso and 600 < its < 750  # 674 measured (profiles/r01/solve_star7.jsonl)
    check_history(hist, ho)
    check_x(x.get_values(), xo)
    assert _true_residual(A, x, b) < 1e-8
    for o in (P, A, x, b, xt):
        o.destroy()
    da.destroy()


@pytest.mark.parametrize("pc,rtol", [("mg", 1e-10), ("jacobi", 1e-10)])
def test_cg_full_solve_512(ctx, pc, rtol):
    """Solve to rtol 1e-10 (the north-star tolerance): converged on the preconditioned norm, true
    residual below 1e-8 relative, x_true recovered up to the null space."""
    n = (512, 512, 512)
    da, h, P, A, x, b, xt = _system(ctx, n)
    reason, its, hist = pb.solve(P, A, x, b, ["-ksp_type", "cg", "-pc_type", pc,
                                              "-ksp_rtol", str(rtol)])
    assert reason == 2  # KSP_CONVERGED_RTOL
    assert hist[-1] <= rtol * hist[0]
    if pc == "mg":
        assert its == 13
    else:
        assert 1000 < its < 1400  # 1182 measured (profiles/r01/solve_star7.jsonl)
    assert _true_residual(A, x, b) < 1e-8
    assert _mean_free_err(x, xt) < 1e-5  # cond(A) ~ (n/pi)^2 ~ 2.7e4 times the residual
    for o in (P, A, x, b, xt):
        o.destroy()
    da.destroy()


def test_config5_compact_fft_solve_512(ctx):
    """BASELINE config 5 at full size on one GPU: the compact-scheme Laplacian (A = P = compact,
    src/compact_schemes.f90:17-37) in CG with the spectral preconditioner built from it, to the
    north-star rtol 1e-10 (r01: 7-point MG stalled, 10,000 iterations, DIVERGED_ITS). The compact
    operator's null space holds every mode with two or more Nyquist components, so x_true is
    recovered only up to it: the bar is the true residual."""
    n = (512, 512, 512)
    h = tuple(2 * np.pi / m for m in n)
    da = pb.DA(ctx, n, (2 * np.pi,) * 3)
    A = pb.Mat(da, pb.COMPACT, h)
    x, b, xt = pb.Vec(da), pb.Vec(da), pb.Vec(da)
    xt.set_random(SEED)
    A.mult(xt, b)
    reason, its, hist = pb.solve(A, A, x, b, ["-ksp_type", "cg", "-pc_type", "fft",
                                              "-ksp_rtol", "1e-10"])
    assert reason == 2 and its <= 3
    assert hist[-1] <= 1e-10 * hist[0]
    assert _true_residual(A, x, b) < 1e-12
    for o in (A, x, b, xt):
        o.destroy()
    da.destroy()


def test_config5_eight_ranks_512():
    """BASELINE config 5's decomposition: 512^3 over 8 ranks (512x512x64 z-slabs, the Z passes on
    64-row y-slabs through all-to-all transposes), 8 contexts on the one GPU joined by the
    in-process host transport. Against the 1-rank run of the same problem: A x_true (compact
    operator) and the spectral PC apply bit-identical on every slab; the CG solve to rtol 1e-10
    with the same reason and iteration count, x within the CG bar (the dot products sum per-rank
    partials in another order, so x differs at rounding level) and ||b - A x|| / ||b|| < 1e-12."""
    from test_gpu_parity import run_ranks
    n = (512, 512, 512)
    plane = n[0] * n[1]
    h = tuple(2 * np.pi / m for m in n)
    argv = ["-ksp_type", "cg", "-pc_type", "fft", "-ksp_rtol", "1e-10"]

    def system(ctx):
        da = pb.DA(ctx, n, (2 * np.pi,) * 3)
        A = pb.Mat(da, pb.COMPACT, h)
        x, b, xt, z = pb.Vec(da), pb.Vec(da), pb.Vec(da), pb.Vec(da)
        xt.set_random(SEED)
        A.mult(xt, b)
        k = pb.KSP(A, A, pb.ksp_options(argv))
        k.pc_apply(b, z)
        return da, A, x, b, xt, z, k

    ctx1 = pb.Context(0)
    da, A, x, b, xt, z, k = system(ctx1)
    reason1, its1, _ = k.solve(b, x)
    ref_b, ref_z, ref_x = b.get_values(), z.get_values(), x.get_values()
    for o in (k, A, x, b, xt, z):
        o.destroy()
    da.destroy()
    ctx1.destroy()
    assert reason1 == 2 and its1 <= 3
    xscale = float(np.max(np.abs(ref_x)))

    def body(ctx, rank):
        da, A, x, b, xt, z, k = system(ctx)
        (_, _, k0), (_, _, nk) = da.get_corners()
        sl = slice(k0 * plane, (k0 + nk) * plane)
        same_b = bool(np.array_equal(b.get_values(), ref_b[sl]))
        same_z = bool(np.array_equal(z.get_values(), ref_z[sl]))
        reason, its, _ = k.solve(b, x)
        xerr = float(np.max(np.abs(x.get_values() - ref_x[sl]))) / xscale
        res = _true_residual(A, x, b)  # collective: every rank takes part
        for o in (k, A, x, b, xt, z):
            o.destroy()
        da.destroy()
        return k0, nk, same_b, same_z, reason, its, xerr, res

    out = run_ranks(8, body)
    assert [(r[0], r[1]) for r in out] == [(64 * q, 64) for q in range(8)]
    for k0, nk, same_b, same_z, reason, its, xerr, res in out:
        assert same_b and same_z, (k0, same_b, same_z)
        assert (reason, its) == (reason1, its1)
        assert xerr <= 1e-10, xerr  # parity_bars.X_RTOL
        assert res < 1e-12, res


def test_mg_pc_apply_512_bit_exact(ctx):
    """One V-cycle (8 levels, fused sweeps on the 512^3 and 256^3 levels) bit-identical to the
    oracle's over the whole grid."""
    n = (512, 512, 512)
    N = int(np.prod(n))
    h = tuple(1.0 / m for m in n)
    r = O.fill_random(N, 3)
    ref = O.mg_apply(r, n, h, pc="mg")
    da = pb.DA(ctx, n)
    P, A, _, _ = pb.initialise_linear_system(da, h)
    k = pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg"]))
    rv, zv = pb.Vec(da), pb.Vec(da)
    rv.set_values(r)
    del r
    k.pc_apply(rv, zv)
    assert np.array_equal(zv.get_values(), ref)
    for o in (k, P, A, rv, zv):
        o.destroy()
    da.destroy()


def test_compact_lapl_fast_512_analytic(ctx):
    """Config 5's operator at 512^3 (tests/lapl/test_lapl.f90:87-130 bars): const -> 0,
    sum sin -> -sum sin to 1e-9 (6th order: h^6 ~ 4e-12 at n = 512)."""
    m = 512
    h = 2 * np.pi / m
    da = pb.DA(ctx, (m, m, m), (2 * np.pi,) * 3)
    f, out = pb.Vec(da), pb.Vec(da)
    f.set(2.8170923)
    pb.compact_lapl_fast(da, (h, h, h), f, out)
    assert np.sqrt(np.mean(out.get_values() ** 2)) <= 100 * np.finfo(float).eps
    x = (np.arange(m) + 0.5) * h
    s = np.sin(x)
    fs = (s[None, None, :] + s[None, :, None] + s[:, None, None]).reshape(-1)
    f.set_values(fs)
    pb.compact_lapl_fast(da, (h, h, h), f, out)
    assert np.sqrt(np.mean((out.get_values() + fs) ** 2)) <= 1e-9
    for o in (f, out):
        o.destroy()
    da.destroy()


@pytest.mark.parametrize("periodic", [False, True])
def test_tdma_full_batch(ctx, periodic):
    """512^2 lines of 512 points, interleaved (the rows bench layout): 512 sampled lines
    bit-identical to the reference-order restatement, every line satisfying its system."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    n, nb = 512, 512 * 512
    rng = np.random.default_rng(11)
    host = {k: rng.random((n, nb)) for k in "abcd"}
    host["b"] = host["b"] * 10 + 3  # diagonally dominant (tests/tridiag/test_tdma_utils.f90)
    ptr = {}
    for k, v in host.items():
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(8 * v.size)) == 0
        assert hip.hipMemcpy(p, v.ctypes.data_as(C.c_void_p), C.c_size_t(8 * v.size), 1) == 0
        ptr[k] = p
    assert hip.hipDeviceSynchronize() == 0
    pb.tdma_batched(ctx, n, nb, 1, nb, ptr["a"], ptr["b"], ptr["c"], ptr["d"], periodic=periodic)
    x = np.empty((n, nb))
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipMemcpy(x.ctypes.data_as(C.c_void_p), ptr["d"], C.c_size_t(8 * x.size), 2) == 0
    for p in ptr.values():
        hip.hipFree(p)
    a, b, c, d = host["a"], host["b"], host["c"], host["d"]
    for l in np.random.default_rng(5).choice(nb, 512, replace=False):
        _, ref = O.tdma(a[:, l], b[:, l], c[:, l], d[:, l], periodic=periodic)
        assert np.array_equal(x[:, l], ref), l
    # a_i x_{i-1} + b_i x_i + c_i x_{i+1} = d_i (a_1 / c_n couple x_n / x_1 when periodic)
    lhs = b * x
    lhs[1:] += a[1:] * x[:-1]
    lhs[:-1] += c[:-1] * x[1:]
    if periodic:
        lhs[0] += a[0] * x[-1]
        lhs[-1] += c[-1] * x[0]
    assert np.max(np.abs(lhs - d)) <= 1e-12 * np.max(np.abs(d))
