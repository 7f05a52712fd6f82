"""GPU tier: the HIP path (through the C ABI) against the oracle and the reference fixtures.

Bars (stated per test): bit-exact for the 7-point operator, the vector updates, the synthetic
input, the tridiagonal solvers and the compact operators (same operation order, no FMA
contraction); CG residual history within a stated relative tolerance of the PETSc-semantics
restatement (reduction order differs), same iteration count and stopping reason.
"""
import ctypes as C
import queue
import os
import threading

import numpy as np
import pytest

import poissbox_amd as pb
from oracle import oracle as O
from parity_bars import HIST_RTOL, HIST_RTOL_PC, X_RTOL, check_history, check_x

pytestmark = pytest.mark.gpu

SEED = 20231015


# ---------------------------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------------------------
class Dev:
    """Raw device buffer through the HIP runtime (ctypes, no torch needed)."""

    _hip = None

    def __init__(self, arr):
        if Dev._hip is None:
            Dev._hip = C.CDLL("libamdhip64.so")
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        self.n = arr.size
        self.p = C.c_void_p()
        assert Dev._hip.hipMalloc(C.byref(self.p), C.c_size_t(max(8, 8 * self.n))) == 0
        assert Dev._hip.hipMemcpy(self.p, arr.ctypes.data_as(C.c_void_p), C.c_size_t(8 * self.n), 1) == 0
        assert Dev._hip.hipDeviceSynchronize() == 0  # pageable H2D may return before the DMA lands

    def get(self):
        out = np.empty(self.n)
        assert Dev._hip.hipDeviceSynchronize() == 0
        assert Dev._hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), self.p, C.c_size_t(8 * self.n), 2) == 0
        return out

    def free(self):
        Dev._hip.hipFree(self.p)


def grid_vec(ctx, n, values=None, L=(1.0, 1.0, 1.0)):
    da = pb.DA(ctx, n, L)
    v = pb.Vec(da)
    if values is not None:
        v.set_values(values)
    return da, v


# ---------------------------------------------------------------------------------------------
# 7-point operator (mfmult / compute_lapl_pointwise)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [(3, 3, 3), (16, 16, 16), (17, 12, 9), (130, 18, 7), (64, 64, 64),
                               (256, 8, 5), (20, 36, 11), (128, 128, 4), (512, 64, 128),
                               # planes of >= 512^2 points: 8 rows per wave (StoreY::TALL)
                               (512, 512, 6), (1024, 256, 5), (512, 520, 3)])
def test_stencil_bit_exact(ctx, n):
    N = int(np.prod(n))
    x = O.fill_random(N, SEED + N)
    h = tuple(1.0 / m for m in n)
    da, xv = grid_vec(ctx, n, x)
    yv = pb.Vec(da)
    A = pb.Mat(da, pb.STAR7)
    A.mult(xv, yv)
    y = yv.get_values()
    ref = O.stencil(x, n, h, faithful=N <= 40000)
    assert np.array_equal(y, ref), np.max(np.abs(y - ref))
    # assembled P: the same 7 non-zeros, summed in AIJ order on the seams (this second apply
    # marches the other z direction: consecutive applies alternate, so both are checked)
    P = pb.Mat(da, pb.ASSEMBLED27)
    P.mult(xv, yv)
    assert np.array_equal(yv.get_values(), O.assembled(x, n, h))
    for o in (A, P, xv, yv):
        o.destroy()
    da.destroy()


def test_stencil_matches_reference_fixtures(ctx, golden):
    """SURVEY.md §8(c) golden vector 4, pinned to the reference's own arithmetic: A x (the
    matvec kernel, MatMult through the shell operator) and compute_lapl_pointwise equal the
    outputs of the reference's evaluate_laplacian_pointwise + lapl_star_coeffs (flang-built,
    tests/golden/make_golden.py) bit for bit, uniform and non-uniform spacings; the assembled
    P's rows away from the seams as well (its seam rows sum in AIJ order: test_stencil_bit_exact)."""
    names = [n for n in sorted({k.rsplit("__", 1)[0] for k in golden.files})
             if n.startswith("star__")]
    assert len(names) >= 6
    for name in names:
        m = golden[name + "__meta"]
        n3, h = tuple(int(v) for v in m[:3]), tuple(float(v) for v in m[3:])
        x, ref = golden[name + "__in"], golden[name + "__out"]
        da, xv = grid_vec(ctx, n3, x)
        yv = pb.Vec(da)
        A = pb.Mat(da, pb.STAR7, h)
        A.mult(xv, yv)
        assert np.array_equal(yv.get_values(), ref), name
        yv.set(0.0)
        pb.compute_lapl_pointwise(da, h, xv, yv)
        assert np.array_equal(yv.get_values(), ref), name
        P = pb.Mat(da, pb.ASSEMBLED27, h)
        P.mult(xv, yv)
        yp, r3 = yv.get_values().reshape(n3[::-1]), ref.reshape(n3[::-1])
        assert np.array_equal(yp[1:-1, 1:-1, 1:-1], r3[1:-1, 1:-1, 1:-1]), name
        for o in (A, P, xv, yv):
            o.destroy()
        da.destroy()


def test_stencil_nonuniform_spacing(ctx):
    n = (24, 20, 10)
    L = (1.0, 2.5, 0.3)
    da = pb.DA(ctx, n, L)
    h = da.spacing
    assert np.allclose(h, [L[i] / n[i] for i in range(3)])
    x = O.fill_random(int(np.prod(n)), 11)
    xv, yv = pb.Vec(da), pb.Vec(da)
    xv.set_values(x)
    pb.compute_lapl_pointwise(da, h, xv, yv)
    assert np.array_equal(yv.get_values(), O.stencil(x, n, h, faithful=True))


def test_stencil_polynomial_known_answer(ctx):
    """Quadratic field a*(x^2+y^2+z^2) -> 3*2a away from the periodic seam
    (tests/coefficients/test_star.f90:108-116)."""
    n = (16, 16, 16)
    a = 2.718
    h = 0.155
    i = np.arange(16) * h
    f = a * (i[None, None, :] ** 2 + i[None, :, None] ** 2 + i[:, None, None] ** 2)
    da = pb.DA(ctx, n, (16 * h,) * 3)
    xv, yv = pb.Vec(da), pb.Vec(da)
    xv.set_values(f.reshape(-1))
    pb.Mat(da, pb.STAR7, (h, h, h)).mult(xv, yv)
    y = yv.get_values().reshape(16, 16, 16)[1:-1, 1:-1, 1:-1]
    assert np.allclose(y, 6 * a, rtol=0, atol=1e-9 * 6 * a / h ** 2 * h ** 2 + 1e-9)


# ---------------------------------------------------------------------------------------------
# vectors
# ---------------------------------------------------------------------------------------------
def test_vector_ops(ctx):
    n = (40, 30, 20)
    N = 40 * 30 * 20
    a, b = O.fill_random(N, 1), O.fill_random(N, 2)
    da = pb.DA(ctx, n)
    va, vb = pb.Vec(da), pb.Vec(da)
    va.set_values(a)
    vb.set_values(b)
    assert np.isclose(va.dot(vb), np.dot(a, b), rtol=1e-13)
    assert np.isclose(va.norm(), np.linalg.norm(a), rtol=1e-13)
    assert np.isclose(va.sum(), a.sum(), rtol=1e-12, atol=1e-12)
    vc = va.duplicate()
    va.copy_to(vc)
    vc.axpy(-0.37, vb)
    assert np.array_equal(vc.get_values(), a + (-0.37) * b)
    vc.aypx(1.5, vb)
    assert np.array_equal(vc.get_values(), b + 1.5 * (a + (-0.37) * b))
    vc.scale(-2.0)
    vc.set(3.25)
    assert np.all(vc.get_values() == 3.25)


def test_random_fill_matches_oracle(ctx):
    n = (33, 17, 9)
    da = pb.DA(ctx, n)
    v = pb.Vec(da)
    v.set_random(SEED)
    assert np.array_equal(v.get_values(), O.fill_random(33 * 17 * 9, SEED))


# ---------------------------------------------------------------------------------------------
# CG (KSPSolve -ksp_type cg -pc_type jacobi, constant null space)
# ---------------------------------------------------------------------------------------------
# CG bars: tests/parity_bars.py (history 1e-11, x 1e-10 relative; reduction order differs)


@pytest.mark.parametrize("n,rtol", [(16, 1e-5), (32, 1e-5), (32, 1e-10), (64, 1e-10),
                                    ((24, 20, 12), 1e-8),
                                    # odd x (one point per lane), rows per wave 2 / 1, odd z,
                                    # several x-segments, partial segment, long z-chunks
                                    ((17, 18, 9), 1e-8), ((130, 6, 33), 1e-8),
                                    ((256, 64, 96), 1e-6),
                                    # planes of 512^2: pass A with 8 rows per wave (TALL);
                                    # 256^2: 4 rows, short z
                                    ((512, 512, 4), 1e-6), ((256, 256, 6), 1e-6)])
def test_cg_matches_petsc_semantics(ctx, n, rtol):
    n3 = (n, n, n) if isinstance(n, int) else n
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    xt = O.fill_random(N, SEED)
    b = O.stencil(xt, n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=rtol)
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, ["-ksp_type", "cg", "-pc_type", "jacobi",
                                               "-ksp_rtol", str(rtol)])
    assert reason == ro == 2
    assert its == itso
    check_history(hist, ho)
    xs = x.get_values()
    check_x(xs, xo)
    # residual ||A x - b|| like src/example.f90:79-84
    r = pb.Vec(da)
    A.mult(x, r)
    r.axpy(-1.0, bv)
    assert r.norm() <= 1e3 * rtol * np.linalg.norm(b) + 1e-9


def test_cg_wide_planes_vs_oracle(ctx):
    """Planes of 1024 x 1024 (config 4's per-GPU slab width) on one rank: the CG passes run
    8-row tiles (WIDE8) with the residency cap -- against the oracle: 20 fixed iterations'
    history, x. (r04 also measured 4 points per lane on 4-row tiles there: no faster,
    profiles/r04/shapes/slab_v4_ab.jsonl.)"""
    n3 = (1024, 1024, 16)
    its = 20
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h, nthreads=8)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=its,
                                  nthreads=8)
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    reason, it, hist = pb.solve(P, A, x, bv, ["-ksp_rtol", "0", "-ksp_atol", "0", "-ksp_max_it",
                                              str(its), "-ksp_divtol", "1e300"])
    assert (reason, it) == (ro, itso) == (reason, its)
    check_history(hist, ho)
    check_x(x.get_values(), xo)


def test_cg_pc_none_and_max_it(ctx):
    n3 = (16, 16, 16)
    h = (1 / 16,) * 3
    xt = O.fill_random(4096, 5)
    b = O.stencil(xt, n3, h)
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    _, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-8, pc="none")
    reason, its, hist = pb.solve(P, A, x, bv, ["-pc_type", "none", "-ksp_rtol", "1e-8"])
    assert (reason, its) == (ro, itso)
    check_history(hist, ho)
    # DIVERGED_ITS at max_it
    _, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-12, max_it=7)
    reason, its, hist = pb.solve(P, A, x, bv, ["-ksp_rtol", "1e-12", "-ksp_max_it", "7"])
    assert (reason, its) == (ro, itso) == (-3, 7)
    check_history(hist, ho)


@pytest.mark.parametrize("defer", ["0", "2", "4"])
@pytest.mark.parametrize("max_it", [1, 2, 3, 8, 9, 10, 11])
def test_cg_deferred_x_update(ctx, defer, max_it, tune):
    """The solution update deferred over D iterations (tuning cg_defer_x = D; 4 is the default):
    stopping at every position of the cycle (0-3 updates still pending, flushed at the end)
    gives the oracle's x (summation order differs: rounding level) and the same history."""
    tune.setenv("PB_CG_DEFER_X", defer)
    n3 = (32, 24, 16)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=max_it)
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, ["-ksp_rtol", "0", "-ksp_atol", "0",
                                               "-ksp_divtol", "1e300",
                                               "-ksp_max_it", str(max_it)])
    assert (reason, its) == (ro, itso) == (-3, max_it)
    check_history(hist, ho)
    check_x(x.get_values(), xo, bar=1e-12)


@pytest.mark.parametrize("case", ["rtol", "rtol_tight", "max_it1", "max_it2", "max_it9",
                                  "split_iterate", "check1"])
def test_cg_folded_finalize_bit_identical(ctx, case, tune):
    """One-rank Jacobi CG with the finalize steps folded into the passes' prologues (default)
    against the separate finalize launches (PB_CG_FOLD=0): same reason, iteration count,
    history and x, bit for bit -- stopping at every kind of place (rtol inside a poll interval,
    max_it 1 / 2 / 9, a begin / iterate(3) / iterate(n) / end sequence, check_every 1 which
    cannot fold)."""
    n3 = (64, 32, 16)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    opts = {"rtol": ["-ksp_rtol", "1e-5"], "rtol_tight": ["-ksp_rtol", "1e-11"],
            "max_it1": ["-ksp_rtol", "0", "-ksp_max_it", "1"],
            "max_it2": ["-ksp_rtol", "0", "-ksp_max_it", "2"],
            "max_it9": ["-ksp_rtol", "0", "-ksp_max_it", "9"],
            "split_iterate": ["-ksp_rtol", "1e-7"], "check1": ["-ksp_rtol", "1e-6"]}[case]
    out = {}
    for fold in ("1", "0"):
        tune.setenv("PB_CG_FOLD", fold)
        da = pb.DA(ctx, n3)
        P, A, x, bv = pb.initialise_linear_system(da, h)
        bv.set_values(b)
        if case == "split_iterate":
            k = pb.KSP(A, P, pb.ksp_options(opts))
            k.begin(bv, x)
            k.iterate(3)
            k.iterate(5)
            k.iterate(1000)
            reason, its, hist = k.end()
            k.destroy()
        elif case == "check1":
            k = pb.KSP(A, P, pb.ksp_options(opts, check_every=1))
            reason, its, hist = k.solve(bv, x)
            k.destroy()
        else:
            reason, its, hist = pb.solve(P, A, x, bv, opts)
        out[fold] = (reason, its, np.asarray(hist), x.get_values())
    (r1, i1, h1, x1), (r0, i0, h0, x0) = out["1"], out["0"]
    assert (r1, i1) == (r0, i0)
    assert np.array_equal(h1, h0) and np.array_equal(x1, x0)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, **({"rtol": float(opts[1])} if opts[1] != "0" else
                                                {"rtol": 0.0, "max_it": int(opts[3])}))
    assert (r1, i1) == (ro, itso)
    check_history(h1, ho)


def test_cg_zero_rhs_converges_immediately(ctx):
    n3 = (8, 8, 8)
    da = pb.DA(ctx, n3)
    P, A, x, b = pb.initialise_linear_system(da, (1 / 8,) * 3)
    reason, its, hist = pb.solve(P, A, x, b)
    # ||z0|| = 0 <= max(rtol*0, atol) -> CONVERGED_ATOL at iteration 0, one norm logged
    assert reason == 3 and its == 0 and len(hist) == 1 and hist[0] == 0.0


def test_cg_split_iterate_equals_solve(ctx):
    """pb_ksp_begin / iterate / end (the benchmark form) gives the same iterates as KSPSolve."""
    n3 = (32, 16, 8)
    N = 32 * 16 * 8
    h = (1 / 32, 1 / 16, 1 / 8)
    b = O.stencil(O.fill_random(N, 9), n3, h)
    da = pb.DA(ctx, n3)
    P, A, x1, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    x2 = pb.Vec(da)
    opts = pb.ksp_options(["-ksp_rtol", "0", "-ksp_max_it", "40"], atol=0.0)
    k = pb.KSP(A, P, opts)
    k.begin(bv, x1)
    k.iterate(15)
    k.iterate(25)
    r1, its1, h1 = k.end()
    r2, its2, h2 = pb.KSP(A, P, opts).solve(bv, x2)
    assert its1 == its2 == 40 and np.array_equal(h1, h2)
    assert np.array_equal(x1.get_values(), x2.get_values())


# ---------------------------------------------------------------------------------------------
# multi-rank (host transport: N contexts on one GPU, one thread per rank)
# ---------------------------------------------------------------------------------------------
def run_ranks(nranks, body):
    """Run body(ctx, rank) on nranks contexts (same GPU, one thread each) connected by an
    in-process host transport: keyed mailboxes for the halo planes, a barrier allreduce."""
    box = [{"from_up": queue.Queue(), "from_down": queue.Queue(),
            "a2a": [queue.Queue() for _ in range(nranks)]} for _ in range(nranks)]
    barrier = threading.Barrier(nranks)
    red = [None] * nranks
    results, errors = [None] * nranks, []

    def worker(rank):
        try:
            ctx = pb.Context(0, rank, nranks)
            down, up = (rank - 1) % nranks, (rank + 1) % nranks

            def sendrecv(lo, hi):
                box[down]["from_up"].put(lo)    # my first plane sits above rank-1's last
                box[up]["from_down"].put(hi)    # my last plane sits below rank+1's first
                return box[rank]["from_down"].get(timeout=120), box[rank]["from_up"].get(timeout=120)

            def allreduce(vals):
                red[rank] = vals.copy()
                barrier.wait(timeout=120)
                total = red[0].copy()
                for r in range(1, nranks):
                    total = total + red[r]
                barrier.wait(timeout=120)
                return total

            def alltoallv(blocks, rsizes):
                for p in range(nranks):
                    box[p]["a2a"][rank].put(np.array(blocks[p], copy=True))
                return [box[rank]["a2a"][p].get(timeout=120) for p in range(nranks)]

            ctx.set_host_transport(sendrecv, allreduce, alltoallv)
            results[rank] = body(ctx, rank)
        except Exception as e:  # pragma: no cover
            errors.append(e)
            barrier.abort()

    ts = [threading.Thread(target=worker, args=(r,)) for r in range(nranks)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    if errors:
        raise errors[0]
    return results


def test_assembled_check_matrices(ctx):
    """src/example.f90:235-261 check_matrices: ||A x - P x|| is a rounding-level number (the seam
    rows sum in AIJ column order), and the GPU reproduces P x bit for bit, so the printed value
    is the reference's own."""
    n = (64, 48, 40)
    h = tuple(1.0 / m for m in n)
    x = O.fill_random(int(np.prod(n)), SEED)
    da, xv = grid_vec(ctx, n, x)
    ya, yp = pb.Vec(da), pb.Vec(da)
    A, P = pb.Mat(da, pb.STAR7), pb.Mat(da, pb.ASSEMBLED27)
    A.mult(xv, ya)
    P.mult(xv, yp)
    ref_a, ref_p = O.stencil(x, n, h), O.assembled(x, n, h)
    assert np.array_equal(ya.get_values(), ref_a) and np.array_equal(yp.get_values(), ref_p)
    ya.axpy(-1.0, yp)
    d_gpu, d_ref = ya.norm(), float(np.sqrt(np.sum((ref_a - ref_p) ** 2)))
    assert d_ref > 0 and abs(d_gpu - d_ref) <= 1e-12 * d_ref
    for o in (A, P, xv, ya, yp):
        o.destroy()
    da.destroy()


@pytest.mark.parametrize("n", [(16, 12, 10), (31, 12, 10)])
def test_cg_assembled_operator(ctx, n):
    """A = P (the demo's assembled branch, src/example.f90:62-64): CG runs on the AIJ-order
    MatMult and matches the oracle's restatement of the same sums."""
    h = tuple(1.0 / m for m in n)
    N = int(np.prod(n))
    b = O.assembled(O.fill_random(N, SEED), n, h)
    xo, ro, itso, ho = O.cg_solve(b, n, h, rtol=1e-10, op="assembled")
    da = pb.DA(ctx, n)
    P = pb.Mat(da, pb.ASSEMBLED27, h)
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, P, x, bv, ["-ksp_rtol", "1e-10"])
    assert (reason, its) == (ro, itso)
    check_history(hist, ho)
    check_x(x.get_values(), xo)
    for o in (P, x, bv):
        o.destroy()
    da.destroy()


@pytest.mark.parametrize("nranks,n", [(2, (16, 12, 10)), (3, (20, 16, 7)), (4, (12, 10, 5)),
                                      (3, (64, 32, 40))])
def test_multirank_assembled_aij_order(nranks, n):
    """MatMult_MPIAIJ order on z-slabs: owned columns first, then the off-rank (halo) columns --
    bit-exact against the oracle on every rank, including 1-plane slabs."""
    N = int(np.prod(n))
    x = O.fill_random(N, SEED + 1)
    h = tuple(1.0 / m for m in n)
    ref = O.assembled(x, n, h, nranks=nranks).reshape(n[2], -1)

    def body(ctx, rank):
        da = pb.DA(ctx, n)
        (_, _, k0), (_, _, nk) = da.get_corners()
        xv, yv = pb.Vec(da), pb.Vec(da)
        xv.set_values(x.reshape(n[2], -1)[k0:k0 + nk])
        pb.Mat(da, pb.ASSEMBLED27).mult(xv, yv)
        return k0, nk, yv.get_values()

    for k0, nk, y in run_ranks(nranks, body):
        assert np.array_equal(y, ref[k0:k0 + nk].reshape(-1))


@pytest.mark.parametrize("nranks,n", [(2, (16, 12, 10)), (3, (20, 16, 7)), (4, (32, 32, 8))])
def test_multirank_stencil_bit_exact(nranks, n):
    N = int(np.prod(n))
    x = O.fill_random(N, SEED)
    h = tuple(1.0 / m for m in n)
    ref = O.stencil(x, n, h).reshape(n[2], n[1] * n[0])

    def body(ctx, rank):
        da = pb.DA(ctx, n)
        (_, _, k0), (_, _, nk) = da.get_corners()
        xv, yv = pb.Vec(da), pb.Vec(da)
        xv.set_values(x.reshape(n[2], -1)[k0:k0 + nk])
        pb.Mat(da, pb.STAR7).mult(xv, yv)
        return k0, nk, yv.get_values()

    for k0, nk, y in run_ranks(nranks, body):
        assert np.array_equal(y, ref[k0:k0 + nk].reshape(-1))


@pytest.mark.parametrize("nranks,n", [(2, (16, 16, 12)), (3, (16, 16, 12)),
                                       # 512^2 planes: tall pass A / matvec on the interior and
                                       # boundary launches of a decomposed step (nzl = 6, 4)
                                       (2, (512, 512, 12)), (3, (512, 512, 12))])
def test_multirank_cg(nranks, n):
    N = int(np.prod(n))
    h = tuple(1.0 / m for m in n)
    b = O.stencil(O.fill_random(N, SEED), n, h)
    xo, ro, itso, ho = O.cg_solve(b, n, h, rtol=1e-8)

    def body(ctx, rank):
        da = pb.DA(ctx, n)
        (_, _, k0), (_, _, nk) = da.get_corners()
        P, A, x, bv = pb.initialise_linear_system(da, h)
        xt = pb.Vec(da)  # decomposition-independent synthetic input ...
        xt.set_random(SEED)
        A.mult(xt, bv)        # ... b = A x_true, as src/example.f90:70-72
        reason, its, hist = pb.solve(P, A, x, bv, ["-ksp_rtol", "1e-8"])
        return reason, its, hist, k0, nk, x.get_values()

    out = run_ranks(nranks, body)
    for reason, its, hist, k0, nk, xs in out:
        assert (reason, its) == (ro, itso)
        check_history(hist, ho)
        check_x(xs, xo.reshape(n[2], -1)[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


# ---------------------------------------------------------------------------------------------
# tridiagonal + compact schemes against the reference fixtures (bit-exact)
# ---------------------------------------------------------------------------------------------
def _cases(golden, prefix):
    names = sorted({k.rsplit("__", 1)[0] for k in golden.files})
    return [n for n in names if n.split("__")[0] == prefix]


@pytest.mark.parametrize("op", ["tdma", "tdma_periodic"])
def test_tdma_batched_bit_exact(ctx, golden, op):
    for name in _cases(golden, op):
        n = int(golden[name + "__meta"][0])
        inp, out = golden[name + "__in"], golden[name + "__out"]
        # batch of 3 copies, interleaved layout (line stride 1, element stride 3)
        rep = lambda v: np.repeat(v[:, None], 3, axis=1).reshape(-1)
        bufs = [Dev(rep(inp[i * n:(i + 1) * n])) for i in range(4)]
        pb.tdma_batched(ctx, n, 3, 1, 3, *[d.p for d in bufs], periodic=(op == "tdma_periodic"))
        d = bufs[3].get().reshape(n, 3)
        for j in range(3):
            assert np.array_equal(d[:, j], out[n:]), name
        for bb in bufs:
            bb.free()


@pytest.mark.parametrize("op,kind,stagger", [("grad_1d", 0, -1), ("div_1d", 0, 1),
                                              ("interp_1d", 1, -1), ("interp_1d_div", 1, 1)])
def test_compact_1d_bit_exact(ctx, golden, op, kind, stagger):
    for name in _cases(golden, op):
        m = golden[name + "__meta"]
        n, dx = int(m[0]), float(m[3])
        f = Dev(golden[name + "__in"])
        o = Dev(np.zeros(n))
        pb.compact_1d_batched(ctx, kind, stagger, dx, n, 1, n, 1, f.p, o.p)
        assert np.array_equal(o.get(), golden[name + "__out"]), name
        f.free()
        o.free()


@pytest.mark.parametrize("op", ["grad", "div", "interp", "interp_div", "lapl"])
def test_compact_3d_bit_exact(ctx, golden, op):
    for name in _cases(golden, op):
        m = golden[name + "__meta"]
        n3, h3 = tuple(int(v) for v in m[:3]), tuple(float(v) for v in m[3:])
        N = int(np.prod(n3))
        da = pb.DA(ctx, n3)
        inp = golden[name + "__in"]
        if op == "div":
            fs = [pb.Vec(da) for _ in range(3)]
            for c in range(3):
                fs[c].set_values(inp[c * N:(c + 1) * N])
            out = pb.Vec(da)
            pb.compact_div(da, h3, fs, out)
            got = out.get_values()
        elif op == "grad":
            f = pb.Vec(da)
            f.set_values(inp)
            dfs = [pb.Vec(da) for _ in range(3)]
            pb.compact_grad(da, h3, f, dfs)
            got = np.concatenate([v.get_values() for v in dfs])
        else:
            f, out = pb.Vec(da), pb.Vec(da)
            f.set_values(inp)
            if op == "lapl":
                pb.compact_lapl(da, h3, f, out)
            else:
                pb.compact_interp(da, -1 if op == "interp" else 1, f, out)
            got = out.get_values()
        assert np.array_equal(got, golden[name + "__out"]), name


def test_pcr_alpha_matches_thomas(ctx):
    for n, alpha in ((64, 3 / 10), (512, 9 / 62), (8, 3 / 10)):
        rng = np.random.default_rng(n)
        nb = 5
        d = rng.random((nb, n)) * 2 - 1
        ref = np.stack([O.tdma(np.full(n, alpha), np.ones(n), np.full(n, alpha), row,
                               periodic=True)[1] for row in d])
        buf = Dev(d.reshape(-1))
        pb.pcr_alpha_batched(ctx, n, nb, n, 1, alpha, buf.p)
        got = buf.get().reshape(nb, n)
        assert np.max(np.abs(got - ref)) <= 1e-14 * np.max(np.abs(ref)) * 10
        buf.free()


@pytest.mark.parametrize("n,nb,layout,alpha", [(512, 37, "contig", 3 / 10), (512, 64, "inter", 9 / 62),
                                               (192, 20, "contig", 3 / 10), (128, 33, "inter", 3 / 10),
                                               (64, 6, "contig", 9 / 62), (1024, 8, "inter", 3 / 10),
                                               (96, 4, "contig", 3 / 10), (64, 20005, "inter", 9 / 62),
                                               (128, 9001, "inter", 3 / 10)])
def test_pcr_batched_layouts(ctx, n, nb, layout, alpha):
    """Batched periodic (alpha,1,alpha) solve in both layouts of the batched API: contiguous lines
    (register path, one wave per line), interleaved lines (LDS tile transpose), and an n the
    register path does not take (96: LDS PCR fallback is power-of-two only -> error). The large
    interleaved batches give every persistent block several tiles (two-deep input prefetch) and a
    ragged last tile."""
    rng = np.random.default_rng(n + nb)
    d = rng.random((nb, n)) * 2 - 1
    ref = np.stack([O.tdma(np.full(n, alpha), np.ones(n), np.full(n, alpha), row,
                           periodic=True)[1] for row in d])
    host = d if layout == "contig" else np.ascontiguousarray(d.T)
    buf = Dev(host.reshape(-1))
    ls, es = (n, 1) if layout == "contig" else (1, nb)
    if n == 96:
        with pytest.raises(pb.PbError):
            pb.pcr_alpha_batched(ctx, n, nb, ls, es, alpha, buf.p)
        buf.free()
        return
    pb.pcr_alpha_batched(ctx, n, nb, ls, es, alpha, buf.p)
    got = buf.get().reshape(host.shape)
    got = got if layout == "contig" else got.T
    assert np.max(np.abs(got - ref)) <= 1e-13 * np.max(np.abs(ref))
    buf.free()


# ---------------------------------------------------------------------------------------------
# compact Laplacian fast path (3-pass factorisation + PCR) and CG with the compact operator
# ---------------------------------------------------------------------------------------------
FAST_RTOL = 1e-12  # relative to max|reference|; operation order differs from the reference


def test_compact_lapl_fast_matches_reference(ctx, golden):
    names = _cases(golden, "lapl")
    assert names
    for name in names:
        m = golden[name + "__meta"]
        n3, h3 = tuple(int(v) for v in m[:3]), tuple(float(v) for v in m[3:])
        da = pb.DA(ctx, n3)
        f, out = pb.Vec(da), pb.Vec(da)
        f.set_values(golden[name + "__in"])
        pb.compact_lapl_fast(da, h3, f, out)
        ref = golden[name + "__out"]
        err = np.max(np.abs(out.get_values() - ref))
        assert err <= FAST_RTOL * np.max(np.abs(ref)), (name, err)


@pytest.mark.parametrize("n3", [(64, 48, 40), (33, 17, 9), (128, 128, 64), (256, 192, 64),
                                (1024, 64, 64), (64, 768, 64), (128, 64, 384)])
def test_compact_lapl_fast_vs_oracle_sizes(ctx, n3):
    from oracle import oracle as O
    N = int(np.prod(n3))
    h3 = tuple(2 * np.pi / m for m in n3)
    f = O.fill_random(N, 77)
    ref = O.lapl(f, n3, h3)
    da = pb.DA(ctx, n3)
    fv, out = pb.Vec(da), pb.Vec(da)
    fv.set_values(f)
    pb.compact_lapl_fast(da, h3, fv, out)
    assert np.max(np.abs(out.get_values() - ref)) <= FAST_RTOL * np.max(np.abs(ref))
    # analytic pin (tests/lapl/test_lapl.f90): sum of sines -> minus itself at RMS <= 1e-9 (64^3)
    if n3 == (64, 48, 40):
        return


def test_compact_lapl_fast_analytic_64(ctx):
    """tests/lapl/test_lapl.f90:87-130 on the GPU fast path: const -> 0, sum sin -> -sum sin."""
    n3 = (64, 64, 64)
    h = 2 * np.pi / 64
    da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
    f, out = pb.Vec(da), pb.Vec(da)
    f.set(2.8170923)
    pb.compact_lapl_fast(da, (h, h, h), f, out)
    assert np.sqrt(np.mean(out.get_values() ** 2)) <= 100 * np.finfo(float).eps
    x = (np.arange(64) + 0.5) * h
    s = np.sin(x)
    fs = (s[None, None, :] + s[None, :, None] + s[:, None, None]).reshape(-1)
    f.set_values(fs)
    pb.compact_lapl_fast(da, (h, h, h), f, out)
    assert np.sqrt(np.mean((out.get_values() + fs) ** 2)) <= 1e-9


def test_cg_with_compact_operator(ctx):
    """compact A inside KSPSolve, Jacobi from the 7-point P (A != P as
    src/poissbox.f90:226-228,294)."""
    from oracle import oracle as O
    n3 = (16, 16, 16)
    h3 = (1 / 16,) * 3
    N = 4096
    b = O.lapl(O.fill_random(N, SEED), n3, h3)
    xo, ro, itso, ho = O.cg_solve(b, n3, h3, rtol=1e-8, op="compact")
    da = pb.DA(ctx, n3)
    P = pb.Mat(da, pb.ASSEMBLED27, h3)
    A = pb.Mat(da, pb.COMPACT, h3)
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, ["-ksp_rtol", "1e-8"])
    assert (reason, its) == (ro, itso)
    check_history(hist, ho)
    check_x(x.get_values(), xo)


# ---------------------------------------------------------------------------------------------
# SOR / geometric multigrid preconditioners -- parity against the oracle's
# restatement of the same V-cycle (bit-exact PC apply), CG histories within HIST_RTOL
# ---------------------------------------------------------------------------------------------
# kernel selections of the V-cycle (all bit-identical): default thresholds (small test grids run
# the per-pair kernels), every level forced onto the stencil-engine SOR / residual kernels and the
# z-marching restriction / prolongation, and every level on the per-pair / per-cell kernels
MG_KERNELS = {"default": {},
              "engine": {"PB_MG_ENGINE_MIN_PLANE": "0", "PB_MG_RESTRICT_Z_MIN_COLS": "0"},
              "legacy": {"PB_MG_ENGINE_MIN_PLANE": "1000000000",
                         "PB_MG_RESTRICT_Z_MIN_COLS": "1000000000"},
              # half-sweeps and residual as separate engine passes (no fused sweeps)
              "unfused": {"PB_MG_ENGINE_MIN_PLANE": "0", "PB_MG_SWEEP2": "0"},
              # a longer one-launch tail (every level up to 32^3)
              "bigtail": {"PB_MG_TAIL_MAX": "40000"},
              # decomposed grids: coarse levels with halo exchanges instead of gathered onto
              # every rank (the pre-r04 N > 1 path)
              "noagg": {"PB_MG_AGGLOMERATE": "0"},
              # decomposed grids: every level on the fused unrolled passes (deep ghost planes)
              "splitfused": {"PB_MG_ENGINE_MIN_PLANE": "0", "PB_MG_RESTRICT_Z_MIN_COLS": "0"},
              # ... and the pre-r04 decomposed V-cycle (per-pass kernels, halos on every level)
              "nosplitfused": {"PB_MG_ENGINE_MIN_PLANE": "0", "PB_MG_RESTRICT_Z_MIN_COLS": "0",
                               "PB_MG_SPLIT_FUSED": "0", "PB_MG_AGGLOMERATE": "0"}}


@pytest.mark.parametrize("kern", sorted(MG_KERNELS))
@pytest.mark.parametrize("pc,n3,levels", [("sor", (16, 12, 8), 0), ("mg", (32, 32, 32), 0),
                                          ("mg", (64, 48, 32), 0), ("mg", (32, 16, 24), 2),
                                          ("mg", (8, 8, 8), 0), ("mg", (256, 256, 32), 0)])
def test_pc_apply_bit_exact(ctx, kern, pc, n3, levels, tune):
    for k_, v_ in MG_KERNELS[kern].items():
        tune.setenv(k_, v_)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    r = O.fill_random(N, 11)
    ref = O.mg_apply(r, n3, h, pc=pc, levels=levels)
    da = pb.DA(ctx, n3)
    P, A, _, _ = pb.initialise_linear_system(da, h)
    k = pb.KSP(A, P, pb.ksp_options(["-pc_type", pc, "-pc_mg_levels", str(levels)]))
    assert k.pc_levels == (O.mg_plan_levels(n3, 1, levels) if pc == "mg" else 1)
    rv, zv = pb.Vec(da), pb.Vec(da)
    rv.set_values(r)
    k.pc_apply(rv, zv)
    assert np.array_equal(zv.get_values(), ref)
    k.destroy()


@pytest.mark.parametrize("m", [64, 128])
def test_cg_compact_fft_padded_bit_identical(ctx, m, tune):
    """Config 5's CG (compact A, spectral PC, fused passes) with the PC's padded Z buffer:
    reason, iterations, history and x bit-identical to the unpadded run."""
    n3 = (m, m, m)
    h = (2 * np.pi / m,) * 3
    b = O.lapl(O.fill_random(m ** 3, SEED), n3, h)
    tune.setenv("PB_FFT_ZPAD_MIN_PLANE", "0")
    res = []
    for pad in ("0", "32"):
        tune.setenv("PB_FFT_ZPAD", pad)
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        A = pb.Mat(da, pb.COMPACT, h)
        x, bv = pb.Vec(da), pb.Vec(da)
        bv.set_values(b)
        reason, its, hist = pb.solve(A, A, x, bv, ["-pc_type", "fft", "-ksp_rtol", "1e-10"])
        res.append((reason, its, np.asarray(hist), x.get_values()))
    assert res[0][:2] == res[1][:2] and res[0][0] == 2
    assert np.array_equal(res[0][2], res[1][2]) and np.array_equal(res[0][3], res[1][3])


@pytest.mark.parametrize("kern", ["default", "engine"])
@pytest.mark.parametrize("pc,n", [("sor", 32), ("mg", 32), ("mg", 64)])
def test_cg_sor_mg_matches_oracle(ctx, kern, pc, n, tune):
    """CG + SOR / MG. 'engine': every level on the stencil-engine kernels, so the last half-sweep
    of each PC apply also takes the CG residual sums (no separate pass)."""
    for k_, v_ in MG_KERNELS[kern].items():
        tune.setenv(k_, v_)
    n3 = (n, n, n)
    N = n ** 3
    h = (1.0 / n,) * 3
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, pc=pc)
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, ["-pc_type", pc, "-ksp_rtol", "1e-10"])
    assert reason == ro == 2 and its == itso
    check_history(hist, ho, bar=HIST_RTOL_PC)
    check_x(x.get_values(), xo)
    if pc == "mg":
        assert its <= 16  # h-independent V-cycle preconditioning


@pytest.mark.parametrize("kern", ["default", "engine", "legacy", "unfused"])
def test_cg_mg_fused_post_smoothing(ctx, kern, tune):
    """x extent >= 128: the V-cycle's post-smoothing runs as ONE fused two-colour pass (out of
    place, with CG's residual sums on level 0); history / solution within the CG bar, PC apply
    bit-identical to the oracle."""
    for k_, v_ in MG_KERNELS[kern].items():
        tune.setenv(k_, v_)
    n3 = (128, 128, 32)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, pc="mg")
    r = O.fill_random(N, 7)
    zref = O.mg_apply(r, n3, h, pc="mg")
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    k = pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg", "-ksp_rtol", "1e-10"]))
    rv, zv = pb.Vec(da), pb.Vec(da)
    rv.set_values(r)
    k.pc_apply(rv, zv)
    assert np.array_equal(zv.get_values(), zref)
    bv.set_values(b)
    reason, its, hist = k.solve(bv, x)
    assert reason == ro == 2 and its == itso
    check_history(hist, ho, bar=HIST_RTOL_PC)
    check_x(x.get_values(), xo)
    k.destroy()


# the fused pre-smoothing + residual + restriction and prolongation + post-smoothing passes (rows
# shared between the waves of a block through LDS, plane loop unrolled by four) on every level: y
# extents that are no multiple of a block's stored rows (24 / 28), one smaller than a block (8
# rows: the block's rows wrap several times), four planes (the unrolled kernels' spare planes
# wrap around the grid more than once), plane counts that are no multiple of the unrolled loop's
# four (6, 12), and the full-size test's 256^2 planes
POSTX_SHAPES = [(256, 256, 32), (128, 40, 16), (256, 8, 8), (128, 96, 24), (256, 16, 4),
                (128, 24, 6), (256, 16, 12)]


@pytest.mark.parametrize("n3", POSTX_SHAPES)
def test_mg_fused_passes_bit_exact(ctx, n3, tune):
    tune.setenv("PB_MG_ENGINE_MIN_PLANE", "0")
    tune.setenv("PB_MG_RESTRICT_Z_MIN_COLS", "0")
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    r = O.fill_random(N, 5)
    ref = O.mg_apply(r, n3, h, pc="mg")
    da = pb.DA(ctx, n3)
    P, A, _, _ = pb.initialise_linear_system(da, h)
    k = pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg"]))
    rv, zv = pb.Vec(da), pb.Vec(da)
    rv.set_values(r)
    k.pc_apply(rv, zv)
    assert np.array_equal(zv.get_values(), ref)
    k.destroy()


@pytest.mark.parametrize("split", [1, 2, 7, 64])
@pytest.mark.parametrize("n3", POSTX_SHAPES)
def test_mg_u4_balanced_split_bit_exact(ctx, split, n3, tune):
    """The unrolled fused passes with the balanced work split (mg_u4_split = workgroups per CU): the columns' planes cut into equal pieces, so one workgroup may run the
    end of one column and the start of the next, or several columns (64 per CU: pieces of 2 or 4
    planes, shorter than the passes' warm-up) -- PC apply bit-identical to the oracle."""
    tune.set("mg_u4_split", split)
    tune.set("mg_engine_min_plane", 0)
    tune.set("mg_restrict_z_min_cols", 0)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    r = O.fill_random(N, 8)
    ref = O.mg_apply(r, n3, h, pc="mg")
    da = pb.DA(ctx, n3)
    P, A, _, _ = pb.initialise_linear_system(da, h)
    k = pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg"]))
    rv, zv = pb.Vec(da), pb.Vec(da)
    rv.set_values(r)
    k.pc_apply(rv, zv)
    assert np.array_equal(zv.get_values(), ref)
    k.destroy()


@pytest.mark.parametrize("split", [0, 1, 7])
def test_cg_mg_post_sweep_xch_sums(ctx, split, tune):
    """The LDS-shared post-smoothing also takes CG's residual sums on level 0 (a partial per
    block; split > 0: a partial per balanced-split workgroup, whatever ranges it ran): CG + MG
    history / solution within the CG bar."""
    tune.set("mg_u4_split", split)
    tune.setenv("PB_MG_ENGINE_MIN_PLANE", "0")
    tune.setenv("PB_MG_RESTRICT_Z_MIN_COLS", "0")
    n3 = (128, 96, 24)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, pc="mg")
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, ["-pc_type", "mg", "-ksp_rtol", "1e-10"])
    assert reason == ro == 2 and its == itso
    check_history(hist, ho, bar=HIST_RTOL_PC)
    check_x(x.get_values(), xo)


def test_cg_compact_operator_mg_pc(ctx):
    """Config 5 shape: compact A inside CG, MG-SOR preconditioner on the 7-point P."""
    n3 = (32, 32, 32)
    h = (2 * np.pi / 32,) * 3
    N = 32 ** 3
    b = O.lapl(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-8, op="compact", pc="mg")
    da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
    P = pb.Mat(da, pb.ASSEMBLED27, h)
    A = pb.Mat(da, pb.COMPACT, h)
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, ["-pc_type", "mg", "-ksp_rtol", "1e-8"])
    assert reason == ro == 2 and its == itso
    check_history(hist, ho, bar=HIST_RTOL_PC)
    check_x(x.get_values(), xo)


@pytest.mark.parametrize("pc", ["fft", "mg"])
def test_cg_compact_lazy_initial_state(ctx, pc, tune):
    """Stored-z CG on the compact operator leaves r0 = b, x0 = 0 and p0 = 0 implicit
    (PB_KSP_LAZY0, default on): the setup reads b in place of r and the first iteration writes
    p = z, x = alpha p, r = b - alpha w without reading them. Same reason, iterations, history and
    x as the explicit setup passes, whatever x held before (KSPSolve_CG's zero initial guess); a
    right-hand side that converges at the setup returns x = 0."""
    m = 64 if pc == "fft" else 32  # the spectral PC takes extents 64..1024
    n3 = (m, m, m)
    h = (2 * np.pi / m,) * 3
    N = m ** 3
    b = O.lapl(O.fill_random(N, SEED), n3, h)
    da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
    P = pb.Mat(da, pb.ASSEMBLED27, h)
    A = pb.Mat(da, pb.COMPACT, h)
    Pm = A if pc == "fft" else P  # the spectral PC inverts the compact symbol (config 5)
    opts = ["-pc_type", pc, "-ksp_rtol", "1e-8"]
    x, bv = pb.Vec(da), pb.Vec(da)
    res = {}
    for lazy in ("1", "0"):
        tune.setenv("PB_KSP_LAZY0", lazy)
        x.set_random(99)  # stale content
        bv.set_values(b)
        reason, its, hist = pb.solve(Pm, A, x, bv, opts)
        res[lazy] = (reason, its, np.asarray(hist), x.get_values())
    (r1, i1, h1, x1), (r0, i0, h0, x0) = res["1"], res["0"]
    assert (r1, i1) == (r0, i0) and r1 == 2 and i1 >= 1
    assert np.array_equal(h1, h0) and np.array_equal(x1, x0)
    tune.setenv("PB_KSP_LAZY0", "1")
    x.set_random(99)
    bv.set_values(np.zeros(N))
    reason, its, hist = pb.solve(Pm, A, x, bv, opts)
    assert reason > 0 and its == 0
    assert np.all(x.get_values() == 0.0)


@pytest.mark.parametrize("pc,m", [("fft", 64), ("fft", 128), ("mg", 64), ("sor", 64)])
def test_cg_compact_fused_passes(ctx, pc, m, tune):
    """Stored-z CG on the compact operator with the CgFuse passes (default): the compact Z pass
    forms p = (z - mu) + beta/beta_old p_old (cg_gen_p_kernel's arithmetic) and the X pass takes
    the p . w partial sums. Against PB_CG_FUSE=0 (separate p and dot passes): same reason and
    iterations, p . w summed in another order so the history and x agree to rounding; and the
    oracle's reason / its / history at the CG bars (fixed 6 iterations for the slow MG / SOR)."""
    n3 = (m, m, m)
    h = (2 * np.pi / m,) * 3
    N = m ** 3
    b = O.lapl(O.fill_random(N, SEED), n3, h)
    da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
    P = pb.Mat(da, pb.ASSEMBLED27, h)
    A = pb.Mat(da, pb.COMPACT, h)
    Pm = A if pc == "fft" else P
    if pc == "fft":
        opts = ["-pc_type", pc, "-ksp_rtol", "1e-10"]
        kw = dict(rtol=1e-10)
    else:
        opts = ["-pc_type", pc, "-ksp_rtol", "0", "-ksp_atol", "0", "-ksp_max_it", "6",
                "-ksp_divtol", "1e300"]
        kw = dict(rtol=0.0, atol=0.0, dtol=1e300, max_it=6)
    x, bv = pb.Vec(da), pb.Vec(da)
    res = {}
    for fuse in ("1", "0"):
        tune.setenv("PB_CG_FUSE", fuse)
        bv.set_values(b)
        reason, its, hist = pb.solve(Pm, A, x, bv, opts)
        res[fuse] = (reason, its, np.asarray(hist), x.get_values())
    tune.setenv("PB_CG_FUSE", "1")
    (r1, i1, h1, x1), (r0, i0, h0, x0) = res["1"], res["0"]
    assert (r1, i1) == (r0, i0)
    # with the spectral PC the converged norm is rounding noise (~1e-14 of the first): measured
    # against ||z_0|| there; every norm against itself for the slowly converging MG / SOR runs
    scale = h0[0] if pc == "fft" else h0
    assert np.max(np.abs(h1 - h0) / scale) < 1e-12
    assert np.max(np.abs(x1 - x0)) <= 1e-12 * np.max(np.abs(x0))
    xo, ro, itso, ho = O.cg_solve(b, n3, h, pc=pc, op="compact",
                                  pc_compact=(pc == "fft"), nthreads=8, **kw)
    assert (r1, i1) == (ro, itso)
    if pc == "fft":
        assert abs(h1[0] - ho[0]) / ho[0] < 1e-12
    else:
        check_history(h1, ho, bar=HIST_RTOL_PC)
    check_x(x1, xo, scale=np.max(np.abs(xo)))


@pytest.mark.parametrize("pc", ["fft", "mg"])
def test_cg_compact_lines_off(ctx, pc, tune):
    """with the register line solves off (compact_lines = 0: the LDS-PCR passes, which
    take no CgFuse) stored-z CG on the compact operator must take the unfused iteration, not fail
    -- reason / its / x against the oracle (fixed 6 iterations for MG)."""
    m = 64
    n3 = (m, m, m)
    h = (2 * np.pi / m,) * 3
    b = O.lapl(O.fill_random(m ** 3, SEED), n3, h)
    tune.set("compact_lines", 0)
    da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
    P = pb.Mat(da, pb.ASSEMBLED27, h)
    A = pb.Mat(da, pb.COMPACT, h)
    if pc == "fft":
        opts, kw = ["-pc_type", pc, "-ksp_rtol", "1e-10"], dict(rtol=1e-10)
    else:
        opts = ["-pc_type", pc, "-ksp_rtol", "0", "-ksp_atol", "0", "-ksp_max_it", "6",
                "-ksp_divtol", "1e300"]
        kw = dict(rtol=0.0, atol=0.0, dtol=1e300, max_it=6)
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its, hist = pb.solve(A if pc == "fft" else P, A, x, bv, opts)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, pc=pc, op="compact", pc_compact=(pc == "fft"),
                                  nthreads=8, **kw)
    assert (reason, its) == (ro, itso)
    check_x(x.get_values(), xo, scale=np.max(np.abs(xo)))


@pytest.mark.parametrize("kern", ["default", "engine"])
@pytest.mark.parametrize("pc,omega,n3", [("sor", 2.5, (16, 12, 8)), ("mg", 2.2, (16, 16, 16)),
                                         ("mg", 2.2, (32, 32, 32))])
def test_cg_indefinite_pc(ctx, kern, pc, omega, n3, tune):
    """KSP_DIVERGED_INDEFINITE_PC (PETSc KSPSolve_CG: beta*betaold < 0 at the top of an
    iteration), reached from src/poissbox.f90:296 with -pc_type sor|mg and an SOR factor outside
    (0, 2): same reason, iteration and logged history as the oracle; no norm is logged for the
    iteration that stopped (history length = its)."""
    for k_, v_ in MG_KERNELS[kern].items():
        tune.setenv(k_, v_)
    tune.setenv("PB_SOR_OMEGA_ANY", "1")  # PETSc's PCSOR would reject omega >= 2
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, pc=pc, omega=omega)
    assert ro == -8
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, ["-pc_type", pc, "-pc_sor_omega", str(omega),
                                               "-ksp_rtol", "1e-10"])
    assert pb.REASONS[reason] == "DIVERGED_INDEFINITE_PC"
    assert (reason, its) == (ro, itso) and len(hist) == its
    check_history(hist, ho, bar=HIST_RTOL_PC)
    check_x(x.get_values(), xo)


def test_mg_rejects_odd_extents(ctx):
    da = pb.DA(ctx, (17, 16, 16))
    P, A, _, _ = pb.initialise_linear_system(da, (1 / 17, 1 / 16, 1 / 16))
    with pytest.raises(pb.PbError):
        pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg"]))


@pytest.mark.parametrize("kern", ["default", "engine", "noagg", "splitfused", "nosplitfused"])
@pytest.mark.parametrize("nranks,n", [(2, (16, 16, 32)), (4, (16, 16, 32)), (3, (16, 16, 12)),
                                        (2, (128, 16, 32)), (3, (128, 8, 12)),
                                        (8, (32, 32, 64)), (8, (128, 16, 64))])
def test_multirank_mg_bit_exact_and_cg(kern, nranks, n, tune):
    """Slab-decomposed V-cycle equals the single-grid restatement: halo exchanges on the
    decomposed levels, the coarse levels gathered onto every rank and run as the one-launch tail
    (default since r04; "noagg": halo exchanges on every level).

    nx = 128 cases take the fused two-colour sweeps on the fine level (two-deep z ghosts,
    nzl = 16, 8 and 4 planes per rank); 8 ranks: the GPU count of the driver's scaling runs."""
    for k_, v_ in MG_KERNELS[kern].items():
        tune.setenv(k_, v_)
    N = int(np.prod(n))
    h = tuple(1.0 / m for m in n)
    r = O.fill_random(N, 3)
    ref = O.mg_apply(r, n, h, pc="mg", nranks=nranks).reshape(n[2], -1)
    b = O.stencil(O.fill_random(N, SEED), n, h)
    xo, ro, itso, ho = O.cg_solve(b, n, h, rtol=1e-8, pc="mg", nranks=nranks)

    def body(ctx, rank):
        da = pb.DA(ctx, n)
        (_, _, k0), (_, _, nk) = da.get_corners()
        P, A, x, bv = pb.initialise_linear_system(da, h)
        k = pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg", "-ksp_rtol", "1e-8"]))
        rv, zv = pb.Vec(da), pb.Vec(da)
        rv.set_values(r.reshape(n[2], -1)[k0:k0 + nk])
        k.pc_apply(rv, zv)
        bv.set_values(b.reshape(n[2], -1)[k0:k0 + nk])
        reason, its, hist = k.solve(bv, x)
        return k0, nk, zv.get_values(), reason, its, hist, x.get_values(), k.pc_levels

    for k0, nk, z, reason, its, hist, xs, lv in run_ranks(nranks, body):
        assert lv == O.mg_plan_levels(n, nranks)
        assert np.array_equal(z, ref[k0:k0 + nk].reshape(-1))
        assert (reason, its) == (ro, itso)
        check_history(hist, ho, bar=HIST_RTOL_PC)
        check_x(xs, xo.reshape(n[2], -1)[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


# ---------------------------------------------------------------------------------------------
# spectral preconditioner (-pc_type fft, pb_fft.hip): z = P^+ r by separable Hartley transforms;
# against the oracle's naive-sum restatement (tests/test_oracle.py pins that to the reference
# operators). FFT and naive sums round differently: measured differences ~1e-14 of max|z|.
# ---------------------------------------------------------------------------------------------
FFT_PC_RTOL = 1e-11


def _fft_case(n3, compact):
    h = tuple(2 * np.pi / m for m in n3) if compact else tuple(1.0 / m for m in n3)
    return h, (pb.COMPACT if compact else pb.STAR7)


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("n3", [(64, 64, 64), (128, 64, 256), (256, 128, 64), (1024, 64, 64),
                                (64, 1024, 64), (64, 64, 512), (32, 32, 32), (32, 64, 1024),
                                # mixed radix (r03): 3 * 2^a and 5 * 2^a line lengths
                                (96, 96, 96), (48, 80, 40), (192, 160, 128), (64, 768, 48),
                                (640, 40, 32), (384, 32, 320)])
def test_fft_pc_apply_vs_oracle(ctx, n3, compact):
    N = int(np.prod(n3))
    h, kind = _fft_case(n3, compact)
    r = O.fill_random(N, 17)
    ref = O.fft_pc_apply(r, n3, h, compact)
    da = pb.DA(ctx, n3)
    P = pb.Mat(da, kind, h)
    k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
    rv, zv = pb.Vec(da), pb.Vec(da)
    rv.set_values(r)
    k.pc_apply(rv, zv)
    z = zv.get_values()
    assert np.isfinite(z).all()
    err = float(np.max(np.abs(z - ref)) / np.max(np.abs(ref)))
    assert err < FFT_PC_RTOL, err
    k.destroy()


@pytest.mark.parametrize("pad", [1, 512, 65536])
@pytest.mark.parametrize("n3", [(64, 64, 64), (128, 64, 256), (96, 96, 96), (64, 64, 512),
                                (512, 32, 64)])
def test_fft_pc_padded_z_buffer_bit_identical(ctx, n3, pad, tune):
    """PB_FFT_ZPAD: the Y forward pass writes a buffer with padded planes, the Z pass runs there
    and the Y inverse pass reads it back; the same operations on the same values, so the PC
    apply is bit-identical to the in-place passes (and so within the oracle bar)."""
    N = int(np.prod(n3))
    h, kind = _fft_case(n3, True)
    r = O.fill_random(N, 23)
    outs = []
    for zp in ("0", str(pad)):
        tune.setenv("PB_FFT_ZPAD", zp)
        tune.setenv("PB_FFT_ZPAD_MIN_PLANE", "0")
        da = pb.DA(ctx, n3)
        P = pb.Mat(da, kind, h)
        k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
        rv, zv = pb.Vec(da), pb.Vec(da)
        rv.set_values(r)
        k.pc_apply(rv, zv)
        outs.append(zv.get_values())
        k.destroy()
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("n3", [(64, 64, 64), (128, 64, 128), (512, 64, 64)])
def test_cg_fft_pc_matches_oracle(ctx, n3, compact):
    """CG + the spectral PC: A = P (7-point star, or config 5's compact operator). One iteration
    reaches rounding level, so after ||z_0|| the logged norms are rounding noise: they are checked
    against ||z_0|| (absolute), reason / its / x against the oracle."""
    N = int(np.prod(n3))
    h, kind = _fft_case(n3, compact)
    x0 = O.fill_random(N, SEED)
    b = O.lapl(x0, n3, h) if compact else O.stencil(x0, n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, pc="fft",
                                  op="compact" if compact else "star7", nthreads=8)
    assert ro == 2 and itso <= 3
    da = pb.DA(ctx, n3)
    A = pb.Mat(da, kind, h)
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its, hist = pb.solve(A, A, x, bv, ["-pc_type", "fft", "-ksp_rtol", "1e-10"])
    assert (reason, its) == (ro, itso)
    assert abs(hist[0] - ho[0]) / ho[0] < 1e-12
    assert np.max(np.abs(np.asarray(hist[1:]) - ho[1:])) / ho[0] < 1e-10
    check_x(x.get_values(), xo)


@pytest.mark.parametrize("n3", [(512, 64, 64), (1024, 32, 64)])
def test_cg_fft_r_update_fused(ctx, n3, tune):
    """512- and 1024-point x lines: the spectral PC's first (register-edge) X pass forms CG's
    residual r = r_in - alpha w as it loads it (PB_FFT_RUPD, default on) with cg_pc_xr_kernel's
    rounding, and x is updated on its own: reason, iterations, history and x bit-identical to the
    separate x / r pass (PB_FFT_RUPD=0)."""
    N = int(np.prod(n3))
    h, kind = _fft_case(n3, True)
    b = O.lapl(O.fill_random(N, SEED), n3, h)
    da = pb.DA(ctx, n3)
    A = pb.Mat(da, kind, h)
    x, bv = pb.Vec(da), pb.Vec(da)
    res = {}
    for rupd in ("1", "0"):
        tune.setenv("PB_FFT_RUPD", rupd)
        x.set_random(5)
        bv.set_values(b)
        reason, its, hist = pb.solve(A, A, x, bv, ["-pc_type", "fft", "-ksp_rtol", "1e-12"])
        res[rupd] = (reason, its, np.asarray(hist), x.get_values())
    (r1, i1, h1, x1), (r0, i0, h0, x0) = res["1"], res["0"]
    assert (r1, i1) == (r0, i0) and r1 > 0 and i1 >= 1
    assert np.array_equal(h1, h0) and np.array_equal(x1, x0)


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("nranks,n3", [(2, (64, 64, 64)), (4, (128, 64, 64)), (3, (64, 64, 64)),
                                       (2, (96, 80, 48)), (3, (40, 96, 96))])
def test_multirank_fft_pc(nranks, n3, compact):
    """Split grid: the Z pass runs on y-slabs (z-slab <-> y-slab transposes); per-rank result
    equals the single-grid oracle."""
    N = int(np.prod(n3))
    h, kind = _fft_case(n3, compact)
    r = O.fill_random(N, 23)
    ref = O.fft_pc_apply(r, n3, h, compact).reshape(n3[2], -1)
    scale = float(np.max(np.abs(ref)))

    def body(ctx, rank):
        da = pb.DA(ctx, n3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        P = pb.Mat(da, kind, h)
        k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
        rv, zv = pb.Vec(da), pb.Vec(da)
        rv.set_values(r.reshape(n3[2], -1)[k0:k0 + nk])
        k.pc_apply(rv, zv)
        return k0, nk, zv.get_values()

    for k0, nk, z in run_ranks(nranks, body):
        err = float(np.max(np.abs(z - ref[k0:k0 + nk].reshape(-1)))) / scale
        assert err < FFT_PC_RTOL, err


@pytest.mark.parametrize("nranks,n3", [(2, (64, 64, 64)), (3, (64, 64, 64)), (4, (64, 64, 64)),
                                       (8, (64, 64, 64)), (8, (128, 64, 128))])
def test_multirank_cg_compact_fft(nranks, n3):
    """Config 5 decomposed: compact A = P on z-slabs (Z passes on y-slabs via all-to-all
    transposes), spectral PC, CG to rtol 1e-10 -- reason / its equal to the single-grid oracle,
    x within the CG bar on every rank. 8 ranks: config 5's GPU count (8-plane / 16-plane slabs,
    8-row y-slabs)."""
    N = int(np.prod(n3))
    h = tuple(2 * np.pi / m for m in n3)
    b = O.lapl(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, pc="fft", op="compact", nthreads=8)
    assert ro == 2

    def body(ctx, rank):
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        A = pb.Mat(da, pb.COMPACT, h)
        x, bv = pb.Vec(da), pb.Vec(da)
        bv.set_values(b.reshape(n3[2], -1)[k0:k0 + nk])
        reason, its, hist = pb.solve(A, A, x, bv, ["-pc_type", "fft", "-ksp_rtol", "1e-10"])
        return k0, nk, reason, its, hist, x.get_values()

    for k0, nk, reason, its, hist, xs in run_ranks(nranks, body):
        assert (reason, its) == (ro, itso)
        assert abs(hist[0] - ho[0]) / ho[0] < 1e-12
        check_x(xs, xo.reshape(n3[2], -1)[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


def test_multirank_cg_compact_fft_register_edges():
    """Config 5 decomposed with 512-point x lines: the spectral PC's X passes on the register-edge
    kernel, its first X pass carrying CG's x / r update and its last the residual sums, on two
    z-slab ranks (Z pass on y-slabs) -- reason / its / x against the single-grid oracle."""
    n3 = (512, 32, 64)
    N = int(np.prod(n3))
    h = tuple(2 * np.pi / m for m in n3)
    b = O.lapl(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, pc="fft", op="compact", nthreads=8)
    assert ro == 2

    def body(ctx, rank):
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        A = pb.Mat(da, pb.COMPACT, h)
        x, bv = pb.Vec(da), pb.Vec(da)
        bv.set_values(b.reshape(n3[2], -1)[k0:k0 + nk])
        reason, its, hist = pb.solve(A, A, x, bv, ["-pc_type", "fft", "-ksp_rtol", "1e-10"])
        return k0, nk, reason, its, hist, x.get_values()

    for k0, nk, reason, its, hist, xs in run_ranks(2, body):
        assert (reason, its) == (ro, itso)
        assert abs(hist[0] - ho[0]) / ho[0] < 1e-12
        check_x(xs, xo.reshape(n3[2], -1)[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


def _compact_star_symbol_case(n3):
    """Config 5's operator with the spectral PC of the 7-point symbol (P = STAR7): the symbols
    part at the multi-Nyquist modes (compact A near zero there, the star not), so CG runs many
    iterations -- a long history of the fused compact passes and the spectral PC, which the
    config-5 solve (A = P, one iteration) cannot give. Fixed iteration count, no convergence
    test; measured oracle-vs-oracle (1 vs 8 threads) history spread 2.6e-13 at 64^3."""
    N = int(np.prod(n3))
    h = tuple(2 * np.pi / m for m in n3)
    b = O.lapl(O.fill_random(N, SEED), n3, h)
    return h, b


@pytest.mark.parametrize("n3,its", [((32, 32, 32), 40), ((64, 64, 64), 24)])
def test_cg_compact_star_symbol_fft_history(ctx, n3, its):
    """Compact A, spectral PC of the 7-point P, fixed iterations: reason, iterations, the whole
    ||z_k|| history and x against the oracle's same KSPSolve."""
    h, b = _compact_star_symbol_case(n3)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=its, pc="fft",
                                  op="compact", pc_compact=False, nthreads=8)
    assert ro == -3 and itso == its and ho[-1] < 1e-3 * ho[0]
    da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
    A = pb.Mat(da, pb.COMPACT, h)
    P = pb.Mat(da, pb.STAR7, h)
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its_g, hist = pb.solve(P, A, x, bv, ["-pc_type", "fft", "-ksp_rtol", "0", "-ksp_atol",
                                                 "0", "-ksp_max_it", str(its), "-ksp_divtol",
                                                 "1e300"])
    assert (reason, its_g) == (ro, itso)
    check_history(hist, ho, bar=HIST_RTOL_PC)
    check_x(x.get_values(), xo)


@pytest.mark.parametrize("nranks,n3", [(2, (32, 32, 32)), (8, (64, 64, 64))])
def test_multirank_cg_compact_star_symbol_fft_history(nranks, n3):
    """The same decomposed: z-slab ranks, compact Z passes and the PC's Z pass on y-slabs through
    the all-to-all transposes (8 ranks: config 5's count), 20 fixed iterations -- every rank's
    history and x slab against the single-grid oracle."""
    its = 20
    h, b = _compact_star_symbol_case(n3)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=its, pc="fft",
                                  op="compact", pc_compact=False, nthreads=8)

    def body(ctx, rank):
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        A = pb.Mat(da, pb.COMPACT, h)
        P = pb.Mat(da, pb.STAR7, h)
        x, bv = pb.Vec(da), pb.Vec(da)
        bv.set_values(b.reshape(n3[2], -1)[k0:k0 + nk])
        reason, its_g, hist = pb.solve(P, A, x, bv, ["-pc_type", "fft", "-ksp_rtol", "0",
                                                     "-ksp_atol", "0", "-ksp_max_it", str(its),
                                                     "-ksp_divtol", "1e300"])
        return k0, nk, reason, its_g, hist, x.get_values()

    for k0, nk, reason, its_g, hist, xs in run_ranks(nranks, body):
        assert (reason, its_g) == (ro, itso)
        check_history(hist, ho, bar=HIST_RTOL_PC)
        check_x(xs, xo.reshape(n3[2], -1)[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


@pytest.mark.parametrize("n3", [(96, 96, 96), (192, 160, 128)])
def test_cg_compact_fft_mixed_radix(ctx, n3):
    """Config 5 beyond powers of two: compact A = P on 3 * 2^a and 5 * 2^a extents, spectral PC
    (mixed-radix Stockham transforms), CG to rtol 1e-10 -- the oracle's reason / its / x."""
    N = int(np.prod(n3))
    h = tuple(2 * np.pi / m for m in n3)
    b = O.lapl(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-10, pc="fft", op="compact", nthreads=8)
    assert ro == 2 and itso <= 3
    da = pb.DA(ctx, n3, tuple(2 * np.pi for _ in n3))
    A = pb.Mat(da, pb.COMPACT, h)
    x, bv = pb.Vec(da), pb.Vec(da)
    bv.set_values(b)
    reason, its, hist = pb.solve(A, A, x, bv, ["-pc_type", "fft", "-ksp_rtol", "1e-10"])
    assert (reason, its) == (ro, itso)
    assert abs(hist[0] - ho[0]) / ho[0] < 1e-12
    check_x(x.get_values(), xo)
    r = pb.Vec(da)
    A.mult(x, r)
    r.axpy(-1.0, bv)
    assert r.norm() <= 1e-9 * bv.norm()


def test_fft_pc_rejects_bad_extents(ctx):
    for n3 in [(70, 64, 64), (64, 24, 64), (64, 64, 2048), (64, 64, 75), (64, 1280, 64)]:
        da = pb.DA(ctx, n3)
        P = pb.Mat(da, pb.STAR7, tuple(1.0 / m for m in n3))
        with pytest.raises(pb.PbError):
            pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))


# ---------------------------------------------------------------------------------------------
# compact Laplacian / compact CG on a split grid (z-slab <-> y-slab all-to-all transposes)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("op", ["grad", "div", "interp", "interp_div", "lapl"])
@pytest.mark.parametrize("nranks,n", [(2, (16, 12, 10)), (3, (12, 9, 7)), (4, (8, 8, 13)),
                                       # odd x extent: the per-element transpose kernel, whose
                                       # rank-own block is written in place (r06 host transport)
                                       (3, (9, 8, 6))])
def test_multirank_compact_reference_order(nranks, n, op):
    """src/compact_schemes.f90:17-257 in the reference's operation order on a split grid: the Z
    steps run on y-slabs (complete z-lines), so every rank's slab is bit-identical to the
    oracle's single-domain result (itself bit-exact against the flang-built reference)."""
    N = int(np.prod(n))
    h = tuple(2 * np.pi / m for m in n)
    f = O.fill_random(3 * N if op == "div" else N, 91)
    if op == "grad":
        ref = O.grad(f, n, h).reshape(3, n[2], -1)
    elif op == "div":
        ref = O.div(f, n, h).reshape(1, n[2], -1)
    elif op == "lapl":
        ref = O.lapl(f, n, h).reshape(1, n[2], -1)
    else:
        ref = O.interp(f, n, -1 if op == "interp" else 1).reshape(1, n[2], -1)

    def body(ctx, rank):
        da = pb.DA(ctx, n, (2 * np.pi,) * 3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        comps = f.reshape(-1, n[2], n[1] * n[0])
        ins = [pb.Vec(da) for _ in range(comps.shape[0])]
        for c, v in enumerate(ins):
            v.set_values(comps[c, k0:k0 + nk])
        outs = [pb.Vec(da) for _ in range(3 if op == "grad" else 1)]
        if op == "grad":
            pb.compact_grad(da, h, ins[0], outs)
        elif op == "div":
            pb.compact_div(da, h, ins, outs[0])
        elif op == "lapl":
            pb.compact_lapl(da, h, ins[0], outs[0])
        else:
            pb.compact_interp(da, -1 if op == "interp" else 1, ins[0], outs[0])
        return k0, nk, [o.get_values() for o in outs]

    for k0, nk, got in run_ranks(nranks, body):
        for c, y in enumerate(got):
            assert np.array_equal(y, ref[c, k0:k0 + nk].reshape(-1)), (op, c, k0)


@pytest.mark.parametrize("nranks,n", [(2, (64, 32, 128)), (3, (64, 48, 64)), (4, (32, 16, 20))])
def test_multirank_compact_lapl(nranks, n):
    N = int(np.prod(n))
    h = tuple(2 * np.pi / m for m in n)
    f = O.fill_random(N, 77)
    ref = O.lapl(f, n, h).reshape(n[2], -1)
    one = {}

    def body(ctx, rank):
        da = pb.DA(ctx, n, (2 * np.pi,) * 3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        fv, out = pb.Vec(da), pb.Vec(da)
        fv.set_values(f.reshape(n[2], -1)[k0:k0 + nk])
        pb.compact_lapl_fast(da, h, fv, out)
        A = pb.Mat(da, pb.COMPACT, h)   # the operator form (MatMult) takes the same path
        out2 = pb.Vec(da)
        A.mult(fv, out2)
        return k0, nk, out.get_values(), out2.get_values()

    ctx1 = pb.Context(0)
    da1 = pb.DA(ctx1, n, (2 * np.pi,) * 3)
    f1, o1 = pb.Vec(da1), pb.Vec(da1)
    f1.set_values(f)
    pb.compact_lapl_fast(da1, h, f1, o1)
    one = o1.get_values().reshape(n[2], -1)
    for k0, nk, y, y2 in run_ranks(nranks, body):
        # the Z pass sees the same complete lines: bit-identical to the single-rank result
        assert np.array_equal(y, one[k0:k0 + nk].reshape(-1))
        assert np.array_equal(y2, y)
        assert np.max(np.abs(y - ref[k0:k0 + nk].reshape(-1))) <= FAST_RTOL * np.max(np.abs(ref))


def test_multirank_cg_compact_operator_mg():
    """Config 5 shape on 2 ranks: compact A, MG-SOR preconditioner, z-slabs."""
    n = (32, 32, 32)
    N = 32 ** 3
    h = (2 * np.pi / 32,) * 3
    b = O.lapl(O.fill_random(N, SEED), n, h)
    xo, ro, itso, ho = O.cg_solve(b, n, h, rtol=1e-8, op="compact", pc="mg", nranks=2)

    def body(ctx, rank):
        da = pb.DA(ctx, n, (2 * np.pi,) * 3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        P = pb.Mat(da, pb.ASSEMBLED27, h)
        A = pb.Mat(da, pb.COMPACT, h)
        x, bv = pb.Vec(da), pb.Vec(da)
        bv.set_values(b.reshape(32, -1)[k0:k0 + nk])
        reason, its, hist = pb.solve(P, A, x, bv, ["-pc_type", "mg", "-ksp_rtol", "1e-8"])
        return k0, nk, reason, its, hist, x.get_values()

    for k0, nk, reason, its, hist, xs in run_ranks(2, body):
        assert reason == ro == 2 and its == itso
        check_history(hist, ho, bar=HIST_RTOL_PC)
        check_x(xs, xo.reshape(32, -1)[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


def test_rccl_code_paths_one_rank_communicator(tune):
    """force_comm = 1 gives a 1-rank context an RCCL communicator and the decomposed code paths:
    the halo exchange (ncclSend/ncclRecv to self, interior/boundary overlap split), the RCCL
    allreduce of the CG sums, the compact transposes and the MG level halos -- the paths the
    multi-GPU driver runs, exercised on one GPU (two ranks cannot share a device under RCCL)."""
    tune.set("force_comm", 1)
    ctx = pb.Context(0)
    tune.set("force_comm", 0)
    n3 = (32, 24, 16)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    xt = O.fill_random(N, SEED)
    b = O.stencil(xt, n3, h)
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    y = pb.Vec(da)
    xv = pb.Vec(da)
    xv.set_values(xt)
    A.mult(xv, y)
    assert np.array_equal(y.get_values(), b)
    bv.set_values(b)
    for pc in ("jacobi", "mg"):
        xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-9, pc=pc)
        reason, its, hist = pb.solve(P, A, x, bv, ["-pc_type", pc, "-ksp_rtol", "1e-9"])
        assert (reason, its) == (ro, itso)
        check_history(hist, ho, bar=HIST_RTOL if pc == "jacobi" else HIST_RTOL_PC)
    # single-reduction CG on the decomposed path (boundary-plane fold, one RCCL allreduce)
    for check in (8, 1):
        xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-9, single_reduction=1)
        k = pb.KSP(A, P, pb.ksp_options(["-ksp_cg_single_reduction", "-ksp_rtol", "1e-9"],
                                        check_every=check))
        reason, its, hist = k.solve(bv, x)
        k.destroy()
        assert (reason, its) == (ro, itso)
        check_history(np.asarray(hist), ho)
    hc = tuple(2 * np.pi / m for m in n3)
    ref = O.lapl(xt, n3, hc)
    pb.compact_lapl_fast(da, hc, xv, y)
    assert np.max(np.abs(y.get_values() - ref)) <= FAST_RTOL * np.max(np.abs(ref))
    # 512^2 planes (tall pass A / matvec) on the interior + boundary launches with RCCL halos
    n3 = (512, 512, 6)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    b = O.stencil(O.fill_random(N, SEED), n3, h)
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=1e-6)
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    bv.set_values(b)
    reason, its, hist = pb.solve(P, A, x, bv, ["-ksp_rtol", "1e-6"])
    assert (reason, its) == (ro, itso)
    check_history(hist, ho)
    # fused MG sweeps on a decomposed grid: two-deep z ghosts through ncclSend/ncclRecv
    n3 = (128, 16, 16)
    N = int(np.prod(n3))
    h = tuple(1.0 / m for m in n3)
    r = O.fill_random(N, 3)
    ref = O.mg_apply(r, n3, h, pc="mg")
    for k_, v_ in MG_KERNELS["engine"].items():
        tune.setenv(k_, v_)
    da = pb.DA(ctx, n3)
    P, A, _, _ = pb.initialise_linear_system(da, h)
    k = pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg"]))
    rv, zv = pb.Vec(da), pb.Vec(da)
    rv.set_values(r)
    k.pc_apply(rv, zv)
    assert np.array_equal(zv.get_values(), ref)
    ctx.destroy()


@pytest.mark.parametrize("n3", [(64, 64, 64), (64, 40, 32)])
def test_rccl_self_block_elision_bit_identical(tune, n3):
    """force_comm (a one-rank RCCL communicator): the all-to-all transposes of the compact
    operator and the spectral PC do not copy the rank's own block -- its producer writes it where
    its consumer reads it (YSlabPlan::self_direct; 2^k rows: the blocked Y passes, 40 rows: the
    pack / unpack kernels). Bit-identical to the copying form (tuning a2a_copy_self = 1) and to
    the one-rank path."""
    N = int(np.prod(n3))
    hc = tuple(2 * np.pi / m for m in n3)
    f = O.fill_random(N, 11)

    def run(ctx):
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        xv, y = pb.Vec(da), pb.Vec(da)
        xv.set_values(f)
        pb.compact_lapl_fast(da, hc, xv, y)
        P = pb.Mat(da, pb.COMPACT, hc)
        k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
        z = pb.Vec(da)
        k.pc_apply(xv, z)
        out = (y.get_values(), z.get_values())
        k.destroy()
        return out

    res = {}
    for name, fc, copy in (("one", 0, 0), ("elide", 1, 0), ("copy", 1, 1)):
        tune.set("force_comm", fc)
        ctx = pb.Context(0)
        tune.set("force_comm", 0)
        tune.set("a2a_copy_self", copy)
        res[name] = run(ctx)
        tune.set("a2a_copy_self", 0)
        ctx.destroy()
    for name in ("elide", "copy"):
        for a, b in zip(res[name], res["one"]):
            assert np.array_equal(a, b), name
    assert np.isfinite(res["elide"][1]).all()


def test_split_apply_timers_cover_whole_applies(tune):
    """On a decomposed grid a matvec / CG pass A is two launches (interior planes, then the
    boundary planes after the halo exchange). The "stencil" and "cg_pass_a" timers that bench.py
    prices against all owned DoF count one entry per complete apply; the launches keep their own
    "_interior" / "_boundary" names."""
    tune.set("force_comm", 1)
    ctx = pb.Context(0)
    tune.set("force_comm", 0)
    n3 = (64, 64, 16)
    h = tuple(1.0 / m for m in n3)
    da = pb.DA(ctx, n3)
    P, A, x, bv = pb.initialise_linear_system(da, h)
    xv, y = pb.Vec(da), pb.Vec(da)
    xv.set_values(O.fill_random(int(np.prod(n3)), SEED))
    A.mult(xv, bv)
    ctx.sync()
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(5):
        A.mult(xv, y)
    pb.solve(P, A, x, bv, ["-ksp_rtol", "0", "-ksp_atol", "0", "-ksp_max_it", "6"])
    ctx.sync()
    ms, cnt = ctx.timing("stencil")
    assert cnt == 5 and ms > 0
    for part in ("stencil_interior", "stencil_boundary"):
        assert ctx.timing(part)[1] == 5
    a_ms, a_cnt = ctx.timing("cg_pass_a")
    ai, bi = ctx.timing("cg_pass_a_interior"), ctx.timing("cg_pass_a_boundary")
    assert a_cnt == ai[1] == bi[1] >= 6
    assert a_ms >= ai[0] + bi[0] - 1e-6  # the apply spans both launches
    ctx.set_timing(False)


@pytest.mark.parametrize("sr", [False, True])
@pytest.mark.parametrize("nranks,n", [(2, (16, 16, 12)), (3, (32, 16, 12)), (2, (32, 16, 4))])
def test_multirank_cg_folded_bit_identical(nranks, n, sr):
    """Split grids, Jacobi CG (and -ksp_cg_single_reduction): the state stages folded into the
    next kernel's prologue, the allreduced sums read as a one-block partial (check_every >= 2,
    r05) against the separate finalize launches (check_every 1) -- reason, its, history and x
    bit-identical on every rank, begin / iterate(3) / iterate(rest) included (state slots across
    calls); and the oracle's history."""
    N = int(np.prod(n))
    h = tuple(1.0 / m for m in n)
    b = O.stencil(O.fill_random(N, SEED), n, h)
    xo, ro, itso, ho = O.cg_solve(b, n, h, rtol=1e-9, single_reduction=int(sr))
    argv = ["-ksp_rtol", "1e-9"] + (["-ksp_cg_single_reduction"] if sr else [])

    def body(ctx, rank):
        da = pb.DA(ctx, n)
        (_, _, k0), (_, _, nk) = da.get_corners()
        out = {}
        for check in (8, 1):
            P, A, x, bv = pb.initialise_linear_system(da, h)
            bv.set_values(b.reshape(n[2], -1)[k0:k0 + nk])
            k = pb.KSP(A, P, pb.ksp_options(argv, check_every=check))
            k.begin(bv, x)
            k.iterate(3)
            k.iterate(100000)
            reason, its, hist = k.end()
            k.destroy()
            out[check] = (reason, its, np.asarray(hist), x.get_values())
        return out, k0, nk

    for out, k0, nk in run_ranks(nranks, body):
        (r8, i8, h8, x8), (r1, i1, h1, x1) = out[8], out[1]
        assert (r8, i8) == (r1, i1) == (ro, itso)
        assert np.array_equal(h8, h1) and np.array_equal(x8, x1)
        check_history(h8, ho)
        check_x(x8, xo.reshape(n[2], -1)[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


@pytest.mark.parametrize("nranks,n3", [(2, (64, 64, 64)), (4, (64, 64, 64)), (3, (64, 40, 32)),
                                       (2, (64, 40, 32))])
def test_multirank_self_block_elision_bit_identical(tune, nranks, n3):
    """the all-to-all's self-block elision (YSlabPlan::self_direct, the producer
    writes the rank's own block at ybuf + self_shift) had run only on a one-rank communicator,
    where self_shift is 0. The host transport now elides it the same way, so ranks > 0 use their
    real offsets here: the compact operator and the spectral PC on 2 - 4 ranks (2^k rows per rank:
    the blocked Y passes; 40 rows: the pack / unpack kernels), bit-identical to the copying form
    (a2a_copy_self = 1) and to one rank."""
    N = int(np.prod(n3))
    hc = tuple(2 * np.pi / m for m in n3)
    f = O.fill_random(N, 11)

    def run(ctx, rank=0):
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        xv, y = pb.Vec(da), pb.Vec(da)
        xv.set_values(f.reshape(n3[2], -1)[k0:k0 + nk])
        pb.compact_lapl_fast(da, hc, xv, y)
        P = pb.Mat(da, pb.COMPACT, hc)
        k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
        z = pb.Vec(da)
        k.pc_apply(xv, z)
        out = (k0, nk, y.get_values(), z.get_values())
        k.destroy()
        return out

    _, _, y1, z1 = run(ctx_one := pb.Context(0))
    ctx_one.destroy()
    plane = n3[0] * n3[1]
    for copy in (0, 1):
        tune.set("a2a_copy_self", copy)
        for k0, nk, y, z in run_ranks(nranks, run):
            assert np.array_equal(y, y1[k0 * plane:(k0 + nk) * plane]), (copy, k0)
            assert np.array_equal(z, z1[k0 * plane:(k0 + nk) * plane]), (copy, k0)
    tune.set("a2a_copy_self", 0)


@pytest.mark.parametrize("nranks,n3,pc", [(2, (64, 32, 32), "fft"), (3, (64, 48, 32), "fft"),
                                          (2, (64, 32, 16), "mg")])
def test_multirank_compact_cg_fused(tune, nranks, n3, pc):
    """Split grids, compact A (r06): the transpose's pack forms CG's p = (z - mu) + b/b0 p_old
    (cg_gen_p_kernel's arithmetic) and the X pass takes p . w (CgFuse), against the separate
    kernels (cg_fuse = 0): same reason and iterations, histories within 1e-12 of each other (p . w
    summed in another order), both on the oracle's history; x alike. Fixed iterations with the
    7-point symbol's spectral PC / the 7-point MG (long histories)."""
    its = 12
    h = tuple(2 * np.pi / m for m in n3)
    b = O.lapl(O.fill_random(int(np.prod(n3)), SEED), n3, h)
    opts = ["-pc_type", pc, "-ksp_rtol", "0", "-ksp_atol", "0", "-ksp_max_it", str(its),
            "-ksp_divtol", "1e300"]
    xo, ro, itso, ho = O.cg_solve(b, n3, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=its, pc=pc,
                                  op="compact", pc_compact=False, nthreads=8, nranks=nranks)

    def body(ctx, rank):
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        (_, _, k0), (_, _, nk) = da.get_corners()
        A = pb.Mat(da, pb.COMPACT, h)
        P = pb.Mat(da, pb.STAR7 if pc == "fft" else pb.ASSEMBLED27, h)
        x, bv = pb.Vec(da), pb.Vec(da)
        bv.set_values(b.reshape(n3[2], -1)[k0:k0 + nk])
        reason, its_g, hist = pb.solve(P, A, x, bv, opts)
        return k0, nk, reason, its_g, np.asarray(hist), x.get_values()

    res = {}
    for fuse in (1, 0):
        tune.set("cg_fuse", fuse)
        res[fuse] = run_ranks(nranks, body)
    tune.set("cg_fuse", 1)
    for (k0, nk, r1, i1, h1, x1), (_, _, r0, i0, h0, x0) in zip(res[1], res[0]):
        assert (r1, i1) == (r0, i0) == (ro, itso)
        assert np.max(np.abs(h1 - h0) / h0) < 1e-12
        check_history(h1, ho, bar=HIST_RTOL_PC)
        xs = np.max(np.abs(xo))
        assert np.max(np.abs(x1 - x0)) <= 1e-12 * xs
        check_x(x1, xo.reshape(n3[2], -1)[k0:k0 + nk].reshape(-1), scale=xs)


@pytest.mark.parametrize("pc", ["fft", "mg"])
def test_rccl_compact_cg_fused_split(tune, pc):
    """The split-grid compact CG fusions (the transpose's pack forms p, the X pass takes p . w;
    r06) on a one-rank RCCL communicator (force_comm: the RCCL all-to-all path, self block
    elided) against the one-rank context: same reason and iterations, histories within 1e-12,
    x alike; 12 fixed iterations with the 7-point symbol's spectral PC / the 7-point MG."""
    n3 = (64, 32, 32)
    its = 12
    h = tuple(2 * np.pi / m for m in n3)
    b = O.lapl(O.fill_random(int(np.prod(n3)), SEED), n3, h)
    opts = ["-pc_type", pc, "-ksp_rtol", "0", "-ksp_atol", "0", "-ksp_max_it", str(its),
            "-ksp_divtol", "1e300"]
    res = {}
    for fc in (0, 1):
        tune.set("force_comm", fc)
        c = pb.Context(0)
        tune.set("force_comm", 0)
        da = pb.DA(c, n3, (2 * np.pi,) * 3)
        A = pb.Mat(da, pb.COMPACT, h)
        P = pb.Mat(da, pb.STAR7 if pc == "fft" else pb.ASSEMBLED27, h)
        x, bv = pb.Vec(da), pb.Vec(da)
        bv.set_values(b)
        reason, its_g, hist = pb.solve(P, A, x, bv, opts)
        res[fc] = (reason, its_g, np.asarray(hist), x.get_values())
        for o in (A, P, x, bv):
            o.destroy()
        da.destroy()
        c.destroy()
    (r0, i0, h0, x0), (r1, i1, h1, x1) = res[0], res[1]
    assert (r0, i0) == (r1, i1) == (-3, its)
    assert np.max(np.abs(h1 - h0) / h0) < 1e-12
    assert np.max(np.abs(x1 - x0)) <= 1e-12 * np.max(np.abs(x0))
