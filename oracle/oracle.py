"""ctypes front-end of the CPU restatement (oracle/pb_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker. The product package (poissbox_amd) never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_d = C.POINTER(C.c_double)
_i64 = C.c_int64


def build():
    subprocess.run(["make", "-s", "-C", _HERE, "libpb_oracle.so"], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libpb_oracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.pbo_diag.restype = C.c_double
        L.pbo_cg_solve.restype = C.c_int
        L.pbo_cg_fixed.restype = C.c_double
        L.pbo_splitmix64.restype = C.c_uint64
        L.pbo_splitmix64.argtypes = [C.c_uint64]
        _LIB = L
    return _LIB


class KspOpts(C.Structure):
    _fields_ = [("rtol", C.c_double), ("atol", C.c_double), ("dtol", C.c_double),
                ("max_it", C.c_int64), ("pc_type", C.c_int), ("nullspace", C.c_int),
                ("op_kind", C.c_int), ("nthreads", C.c_int), ("mg_levels", C.c_int),
                ("mg_coarse_its", C.c_int), ("omega", C.c_double), ("nranks", C.c_int),
                ("pc_compact", C.c_int), ("single_reduction", C.c_int)]

PC_CODES = {"none": 0, "jacobi": 1, "sor": 2, "mg": 3, "fft": 4}


def _p(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_d)


def _n3(n):
    return (C.c_int64 * 3)(*[int(v) for v in n])


def _h3(h):
    return (C.c_double * 3)(*[float(v) for v in h])


def star_coeffs(h):
    c = np.zeros(27)
    lib().pbo_lapl_star_coeffs(C.c_double(h[0]), C.c_double(h[1]), C.c_double(h[2]), _p(c))
    return c


def diag(h):
    return lib().pbo_diag(_h3(h))


def stencil(x, n, h, faithful=False, nthreads=1):
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    y = np.empty_like(x)
    if faithful:
        lib().pbo_stencil_apply27(_n3(n), _h3(h), _p(x), _p(y))
    else:
        lib().pbo_stencil_apply7(_n3(n), _h3(h), _p(x), _p(y), C.c_int(nthreads))
    return y


def stencil_slab(x, n_local, h, ghost_lo, ghost_hi):
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    glo = np.ascontiguousarray(ghost_lo, dtype=np.float64).reshape(-1)
    ghi = np.ascontiguousarray(ghost_hi, dtype=np.float64).reshape(-1)
    y = np.empty_like(x)
    lib().pbo_stencil_slab(_n3(n_local), _h3(h), _p(x), _p(glo), _p(ghi), _p(y))
    return y


def assembled(x, n, h, nranks=1):
    """MatMult of the assembled 27-entry P (AIJ row order; MPIAIJ block order on nranks z-slabs)."""
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    y = np.empty_like(x)
    lib().pbo_assembled_apply(_n3(n), _h3(h), C.c_int(nranks), _p(x), _p(y))
    return y


def fill_random(count, seed, g0=0):
    x = np.empty(int(count))
    lib().pbo_fill_random(_i64(int(count)), C.c_uint64(seed), _i64(int(g0)), _p(x))
    return x


def cg_solve(b, n, h, rtol=1e-5, atol=1e-50, dtol=1e5, max_it=10000, pc="jacobi",
             nullspace=True, faithful=False, nthreads=1, op="star7", mg_levels=0,
             mg_coarse_its=8, omega=1.0, nranks=1, pc_compact=None, single_reduction=0):
    """KSPSolve(-ksp_type cg -pc_type jacobi|none|sor|mg|fft) with the constant null space.
    pc_compact: the fft PC inverts the compact operator's symbol (default: when op is compact).
    single_reduction: 1 = PETSc KSPSolve_CG_SingleReduction (-ksp_cg_single_reduction), 2 = the
    same iteration with w = A p recomputed (the GPU pass's arithmetic).
    Returns (x, reason, its, history): the norms KSPLogResidualHistory logged (its + 1 of them,
    its after a breakdown exit)."""
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1)
    x = np.empty_like(b)
    hist = np.zeros(int(max_it) + 2)
    its, nlog = C.c_int64(0), C.c_int64(0)
    if op == "assembled":  # A = P (src/example.f90:62-64), MatMult in AIJ order on nranks slabs
        kind = 2 + max(1, nranks)
    else:
        kind = 2 if op == "compact" else (1 if faithful else 0)
    if pc_compact is None:
        pc_compact = op == "compact"
    o = KspOpts(rtol, atol, dtol, max_it, PC_CODES[pc], int(nullspace), kind, nthreads,
                mg_levels, mg_coarse_its, omega, nranks, int(pc_compact), int(single_reduction))
    reason = lib().pbo_cg_solve(_n3(n), _h3(h), C.byref(o), _p(b), _p(x), _p(hist), C.byref(its),
                                C.byref(nlog))
    return x, reason, its.value, hist[:nlog.value].copy()


def mg_plan_levels(n, nranks=1, levels=0):
    return lib().pbo_mg_plan_levels(_n3(n), C.c_int(nranks), C.c_int(levels))


def mg_apply(r, n, h, pc="mg", levels=0, coarse_its=8, omega=1.0, nranks=1):
    """z = M^-1 r for the red-black SOR / geometric MG preconditioner (pb_mg.hip restatement)."""
    r = np.ascontiguousarray(r, dtype=np.float64).reshape(-1)
    z = np.empty_like(r)
    lib().pbo_mg_apply(_n3(n), _h3(h), C.c_int(PC_CODES[pc]), C.c_int(levels),
                       C.c_int(coarse_its), C.c_double(omega), C.c_int(nranks), _p(r), _p(z))
    return z


def fft_pc_apply(r, n, h, compact=False):
    """z = P^+ r, the spectral preconditioner (pb_fft.hip restatement by naive Hartley sums)."""
    r = np.ascontiguousarray(r, dtype=np.float64).reshape(-1)
    z = np.empty_like(r)
    lib().pbo_fft_pc_apply(_n3(n), _h3(h), C.c_int(int(compact)), _p(r), _p(z))
    return z


def cg_fixed(b, n, h, iters, nthreads=1):
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1)
    x = np.empty_like(b)
    work = np.empty(4 * b.size)
    dp = lib().pbo_cg_fixed(_n3(n), _h3(h), _i64(int(iters)), C.c_int(nthreads), _p(b), _p(x),
                            _p(work))
    return x, dp


# ---- tridiagonal (src/tridsol.f90) ----
def tdma(a, b, c, d, periodic=False):
    a, c = (np.ascontiguousarray(v, dtype=np.float64) for v in (a, c))
    b, d = (np.array(v, dtype=np.float64) for v in (b, d))
    fn = lib().pbo_tdma_periodic if periodic else lib().pbo_tdma
    fn(_i64(len(d)), _p(a), _p(b), _p(c), _p(d))
    return b, d


def fwd_sweep(a, b, c, d):
    a, c = (np.ascontiguousarray(v, dtype=np.float64) for v in (a, c))
    b, d = (np.array(v, dtype=np.float64) for v in (b, d))
    lib().pbo_fwd_sweep(_i64(len(d)), _p(a), _p(b), _p(c), _p(d))
    return b, d


def bwd_sweep(b, c, d):
    b, c = (np.ascontiguousarray(v, dtype=np.float64) for v in (b, c))
    d = np.array(d, dtype=np.float64)
    lib().pbo_bwd_sweep(_i64(len(d)), _p(b), _p(c), _p(d))
    return d


# ---- compact schemes (src/compact_schemes.f90) ----
def grad_1d(f, dx, stagger=-1):
    f = np.ascontiguousarray(f, dtype=np.float64)
    g = np.empty_like(f)
    lib().pbo_grad_1d(_i64(f.size), _p(f), C.c_double(dx), _p(g), C.c_int(stagger))
    return g


def interp_1d(f, stagger=-1):
    f = np.ascontiguousarray(f, dtype=np.float64)
    g = np.empty_like(f)
    lib().pbo_interp_1d(_i64(f.size), _p(f), _p(g), C.c_int(stagger))
    return g


def grad(f, n, h):
    f = np.ascontiguousarray(f, dtype=np.float64).reshape(-1)
    g = np.empty(3 * f.size)
    lib().pbo_grad(_n3(n), _p(f), _h3(h), _p(g))
    return g


def div(f, n, h):
    f = np.ascontiguousarray(f, dtype=np.float64).reshape(-1)
    g = np.empty(f.size // 3)
    lib().pbo_div(_n3(n), _p(f), _h3(h), _p(g))
    return g


def interp(f, n, stagger=-1):
    f = np.ascontiguousarray(f, dtype=np.float64).reshape(-1)
    g = np.empty_like(f)
    lib().pbo_interp(_n3(n), _p(f), _p(g), C.c_int(stagger))
    return g


def lapl(f, n, h):
    f = np.ascontiguousarray(f, dtype=np.float64).reshape(-1)
    g = np.empty_like(f)
    lib().pbo_lapl(_n3(n), _p(f), _h3(h), _p(g))
    return g
