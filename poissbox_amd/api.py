"""Python host side of the poissbox KSPSolve path, mirroring the reference's Fortran/PETSc interface.

Reference (3decomp/poissbox) -> here:
  MPI_Init + PetscInitialize (src/example.f90:43-47)        -> Context(device, rank, nranks, uid)
  initialise_grid(nglobal, da) (src/poissbox.f90:183-204)   -> initialise_grid(ctx, nglobal) -> DA
  DMDAGetCorners (src/poissbox.f90:107)                     -> DA.get_corners()
  initialise_linear_system(da, ctx, P, A, x, b) (:206-240)  -> initialise_linear_system(da, deltas)
  MatCreateShell + MATOP_MULT = mfmult (:242-267, :300-322) -> Mat(kind=STAR7) .mult(x, y)
  compute_lapl_pointwise(da, grid_deltas, x, b) (:84-126)   -> compute_lapl_pointwise(da, deltas, x, b)
  solve(P, A, x, b) (:269-298) + KSPSetFromOptions          -> solve(P, A, x, b, options=argv)
  Vec* (VecAXPY/VecNorm/VecSum/VecDuplicate/...)            -> Vec methods
  tdma / tdma_periodic (src/tridsol.f90)                    -> tdma_batched(...)
  grad/div/interp/interp_div/lapl (src/compact_schemes.f90) -> compact_* functions

All compute runs in libpoissbox_gpu.so (HIP kernels for gfx950); there is no CPU fallback.
"""
import ctypes as C

import numpy as np

from . import _lib as L

STAR7, COMPACT, ASSEMBLED27 = 0, 1, 2
PC_NONE, PC_JACOBI, PC_SOR, PC_MG, PC_FFT = 0, 1, 2, 3, 4

REASONS = {0: "CONVERGED_ITERATING", 2: "CONVERGED_RTOL", 3: "CONVERGED_ATOL",
           4: "CONVERGED_ITS", -3: "DIVERGED_ITS", -4: "DIVERGED_DTOL",
           -8: "DIVERGED_INDEFINITE_PC", -9: "DIVERGED_NANORINF",
           -10: "DIVERGED_INDEFINITE_MAT"}


def _i64_3(v):
    return (C.c_int64 * 3)(*[int(t) for t in v])


def _d_3(v):
    return (C.c_double * 3)(*[float(t) for t in v])


def _dptr(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(L.P_d)


def comm_unique_id():
    buf = C.create_string_buffer(128)
    L.call("pb_comm_unique_id", buf)
    return bytes(buf.raw)


def slab_partition(nz, nranks, rank):
    k0, nk = C.c_int64(), C.c_int64()
    L.call("pb_slab_partition", int(nz), int(nranks), int(rank), C.byref(k0), C.byref(nk))
    return k0.value, nk.value


def tune_set(name, value):
    """pb_tune_set: a kernel-selection / launch-shape parameter (INTEGRATION.md lists them)."""
    L.call("pb_tune_set", name.encode(), int(value))


def tune_get(name):
    """The value set for a tuning parameter, or None when it runs at its measured default."""
    v, s = C.c_int(), C.c_int()
    L.call("pb_tune_get", name.encode(), C.byref(v), C.byref(s))
    return v.value if s.value else None


def tune_reset():
    L.call("pb_tune_reset")


class Context:
    """One GPU, one rank. nranks > 1 needs either an RCCL unique id (uid, from rank 0's
    comm_unique_id()) or a host transport (set_host_transport) before the grid is created."""

    def __init__(self, device=0, rank=0, nranks=1, uid=None):
        h = C.c_void_p()
        L.call("pb_ctx_create", int(device), int(rank), int(nranks), uid, C.byref(h))
        self.h = h
        self.device = device
        self.rank, self.nranks = rank, nranks
        self._keep = []

    @classmethod
    def from_env(cls, device=-1):
        """pb_ctx_create_from_env: rank layout from the launcher's environment (torchrun / mpirun /
        PMI), RCCL or the built-in shared-memory transport (PB_TRANSPORT)."""
        self = cls.__new__(cls)
        h = C.c_void_p()
        L.call("pb_ctx_create_from_env", int(device), C.byref(h))
        self.h = h
        self.device = device
        r, n = C.c_int(), C.c_int()
        L.call("pb_ctx_get_rank", h, C.byref(r), C.byref(n))
        self.rank, self.nranks = r.value, n.value
        self._keep = []
        return self

    def allreduce_sum(self, vals):
        """SUM over ranks of a few host doubles (MPI_Allreduce of the reference's checks)."""
        a = np.ascontiguousarray(vals, dtype=np.float64).reshape(-1).copy()
        L.call("pb_ctx_allreduce_host", self.h, _dptr(a), a.size)
        return a

    def set_host_transport(self, sendrecv, allreduce, alltoallv=None):
        """sendrecv(send_lo, send_hi) -> (recv_lo, recv_hi) numpy arrays; allreduce(vals) -> vals;
        alltoallv(list of per-rank send blocks, list of per-rank receive sizes) -> list of
        per-rank received blocks (optional; the compact operator on a split grid needs it)."""

        def _sr(user, s_lo, s_hi, r_lo, r_hi, count):
            try:
                a = np.ctypeslib.as_array(s_lo, shape=(count,)).copy()
                b = np.ctypeslib.as_array(s_hi, shape=(count,)).copy()
                lo, hi = sendrecv(a, b)
                np.ctypeslib.as_array(r_lo, shape=(count,))[:] = lo
                np.ctypeslib.as_array(r_hi, shape=(count,))[:] = hi
                return 0
            except Exception as e:  # pragma: no cover - reported through the C error path
                print("host sendrecv failed:", e)
                return 1

        def _ar(user, vals, count):
            try:
                v = np.ctypeslib.as_array(vals, shape=(count,))
                v[:] = allreduce(v.copy())
                return 0
            except Exception as e:  # pragma: no cover
                print("host allreduce failed:", e)
                return 1

        f1, f2 = L.SENDRECV_FN(_sr), L.ALLREDUCE_FN(_ar)
        self._keep += [f1, f2]
        L.call("pb_ctx_set_host_transport", self.h, f1, f2, None)
        if alltoallv is None:
            return

        def _a2a(user, send, scount, recv, rcount):
            try:
                P = self.nranks
                sc = [int(scount[p]) for p in range(P)]
                rc = [int(rcount[p]) for p in range(P)]
                sa = np.ctypeslib.as_array(send, shape=(max(sum(sc), 1),))
                so = np.concatenate([[0], np.cumsum(sc)])
                blocks = [sa[so[p]:so[p + 1]].copy() for p in range(P)]
                got = alltoallv(blocks, rc)
                ra = np.ctypeslib.as_array(recv, shape=(max(sum(rc), 1),))
                ro = np.concatenate([[0], np.cumsum(rc)])
                for p in range(P):
                    assert got[p].size == rc[p], (p, got[p].size, rc[p])
                    ra[ro[p]:ro[p + 1]] = got[p]
                return 0
            except Exception as e:  # pragma: no cover
                print("host alltoallv failed:", e)
                return 1

        f3 = L.ALLTOALLV_FN(_a2a)
        self._keep.append(f3)
        L.call("pb_ctx_set_host_alltoallv", self.h, f3, None)

    def sync(self):
        L.call("pb_ctx_sync", self.h)

    def barrier(self):
        L.call("pb_ctx_barrier", self.h)

    @property
    def comm_failed(self):
        """True after a communication failure (timeout, RCCL error, failing host callback)."""
        v = C.c_int(0)
        L.call("pb_ctx_comm_status", self.h, C.byref(v))
        return bool(v.value)

    TRANSPORTS = {0: "none", 1: "rccl", 2: "host"}

    def comm_info(self):
        """(transport, communicator size, rank in it) as the transport itself reports them:
        RCCL's ncclCommCount / ncclCommUserRank, the host transport's rank layout, or
        ("none", 1, 0) on one rank (pb_ctx_comm_info)."""
        t, n, r = C.c_int(), C.c_int(), C.c_int()
        L.call("pb_ctx_comm_info", self.h, C.byref(t), C.byref(n), C.byref(r))
        return self.TRANSPORTS.get(t.value, t.value), n.value, r.value

    def set_timing(self, on=True, only=None, every=1):
        """HIP-event timing of the library's phases; only: phase names (str or list) to time,
        every: time one launch in `every` of each (pb_ctx_set_timing_filter)."""
        if isinstance(only, (list, tuple)):
            only = ",".join(only)
        L.call("pb_ctx_set_timing_filter", self.h, int(bool(on)),
               only.encode() if only else None, int(every))

    def timing(self, name):
        ms, cnt = C.c_double(), C.c_int64()
        L.call("pb_ctx_get_timing", self.h, name.encode(), C.byref(ms), C.byref(cnt))
        return ms.value, cnt.value

    def timing_samples(self, name):
        """Per-launch durations (ms) of a timed phase since the last reset (numpy float32)."""
        cnt = C.c_int64()
        L.call("pb_ctx_get_timing_samples", self.h, name.encode(), None, 0, C.byref(cnt))
        out = np.zeros(cnt.value, dtype=np.float32)
        if cnt.value:
            L.call("pb_ctx_get_timing_samples", self.h, name.encode(),
                   out.ctypes.data_as(C.POINTER(C.c_float)), cnt.value, C.byref(cnt))
        return out

    def copy_probe(self, n=1 << 27, reps=10):
        """HBM calibration: (best, median) GB/s of a flat fp64 copy of n doubles."""
        best, med = C.c_double(), C.c_double()
        L.call("pb_ctx_copy_probe", self.h, int(n), int(reps), C.byref(best), C.byref(med))
        return best.value, med.value

    def reset_timing(self):
        L.call("pb_ctx_reset_timing", self.h)

    def destroy(self):
        if self.h:
            L.call("pb_ctx_destroy", self.h)
            self.h = None


class DA:
    """DMDA analogue: periodic grid, z-slab per rank (src/poissbox.f90:191-202)."""

    def __init__(self, ctx, nglobal, L_=(1.0, 1.0, 1.0)):
        h = C.c_void_p()
        L.call("pb_grid_create", ctx.h, _i64_3(nglobal), _d_3(L_), C.byref(h))
        self.h, self.ctx = h, ctx
        n, hh, nl = (C.c_int64 * 3)(), (C.c_double * 3)(), C.c_int64()
        L.call("pb_grid_get_info", h, n, hh, C.byref(nl))
        self.n = tuple(n)
        self.spacing = tuple(hh)
        self.nlocal = nl.value

    def get_corners(self):
        """0-based (start, size) of the owned block, like DMDAGetCorners."""
        s, z = (C.c_int64 * 3)(), (C.c_int64 * 3)()
        L.call("pb_grid_get_corners", self.h, s, z)
        return tuple(s), tuple(z)

    def create_global_vector(self):
        return Vec(self)

    def destroy(self):
        if self.h:
            L.call("pb_grid_destroy", self.h)
            self.h = None


class Vec:
    def __init__(self, da, _handle=None):
        self.da = da
        if _handle is None:
            h = C.c_void_p()
            L.call("pb_vec_create", da.h, C.byref(h))
            _handle = h
        self.h = _handle

    def duplicate(self):
        return Vec(self.da)

    def set(self, a):
        L.call("pb_vec_set", self.h, float(a))
        return self

    def copy_to(self, dst):
        L.call("pb_vec_copy", self.h, dst.h)

    def axpy(self, a, x):  # VecAXPY(self, a, x): self = self + a*x
        L.call("pb_vec_axpy", self.h, float(a), x.h)

    def aypx(self, b, x):  # VecAYPX(self, b, x): self = x + b*self
        L.call("pb_vec_aypx", self.h, float(b), x.h)

    def scale(self, a):
        L.call("pb_vec_scale", self.h, float(a))

    def dot(self, y):
        out = C.c_double()
        L.call("pb_vec_dot", self.h, y.h, C.byref(out))
        return out.value

    def norm(self):
        out = C.c_double()
        L.call("pb_vec_norm2", self.h, C.byref(out))
        return out.value

    def sum(self):
        out = C.c_double()
        L.call("pb_vec_sum", self.h, C.byref(out))
        return out.value

    def set_values(self, owned):
        a = np.ascontiguousarray(owned, dtype=np.float64).reshape(-1)
        if a.size != self.da.nlocal:
            raise ValueError(f"expected {self.da.nlocal} owned values, got {a.size}")
        L.call("pb_vec_set_values_host", self.h, _dptr(a))

    def get_values(self):
        a = np.empty(self.da.nlocal)
        L.call("pb_vec_get_values_host", self.h, _dptr(a))
        return a

    def set_random(self, seed):
        L.call("pb_vec_set_random", self.h, C.c_uint64(int(seed)))

    def copy_probe(self, y, reps=10):
        """HBM calibration over this vector's and y's own buffers (y is overwritten): flat copy
        self -> y, the matvec's access mix. Returns (best, median) GB/s."""
        best, med = C.c_double(), C.c_double()
        L.call("pb_vec_copy_probe", self.h, y.h, int(reps), C.byref(best), C.byref(med))
        return best.value, med.value

    def device_ptr(self):
        p, n = C.c_void_p(), C.c_int64()
        L.call("pb_vec_device_ptr", self.h, C.byref(p), C.byref(n))
        return p.value, n.value

    def destroy(self):
        if self.h:
            L.call("pb_vec_destroy", self.h)
            self.h = None


class Mat:
    """MatShell analogue (kind STAR7 = mfmult's compute_lapl_pointwise) or the assembled P."""

    def __init__(self, da, kind=STAR7, deltas=None):
        h = C.c_void_p()
        d = _d_3(deltas) if deltas is not None else None
        L.call("pb_op_create", da.h, int(kind), d, C.byref(h))
        self.h, self.da, self.kind = h, da, kind

    def mult(self, x, y):  # MatMult(self, x, y)
        L.call("pb_op_apply", self.h, x.h, y.h)

    def diagonal(self):
        d = C.c_double()
        L.call("pb_op_get_diagonal", self.h, C.byref(d))
        return d.value

    def destroy(self):
        if self.h:
            L.call("pb_op_destroy", self.h)
            self.h = None


def MatMult(A, x, y):
    A.mult(x, y)


def ksp_options(argv=(), **kw):
    o = L.KspOpts()
    L.call("pb_ksp_opts_default", C.byref(o))
    if argv:
        arr = (C.c_char_p * len(argv))(*[str(a).encode() for a in argv])
        L.call("pb_ksp_opts_parse", C.byref(o), len(argv), arr)
    for k, v in kw.items():
        setattr(o, k, v)
    return o


class KSP:
    """KSPCreate + KSPSetOperators(ksp, A, P) + KSPSetFromOptions (src/poissbox.f90:293-295)."""

    def __init__(self, A, P=None, options=None):
        self.opts = options if isinstance(options, L.KspOpts) else ksp_options(options or ())
        h = C.c_void_p()
        L.call("pb_ksp_create", A.h, (P or A).h, C.byref(self.opts), C.byref(h))
        self.h = h

    def solve(self, b, x):
        """Returns (reason, its, history): the res.nhist logged norms (its + 1 of them, its
        after a breakdown exit)."""
        res = L.KspResult()
        hist = np.zeros(int(self.opts.max_it) + 1)
        L.call("pb_ksp_solve", self.h, b.h, x.h, C.byref(res), _dptr(hist), hist.size)
        self.result = res
        return res.reason, res.its, hist[: res.nhist].copy()

    def begin(self, b, x):
        L.call("pb_ksp_begin", self.h, b.h, x.h)

    def iterate(self, n):
        L.call("pb_ksp_iterate", self.h, int(n))

    def end(self):
        res = L.KspResult()
        hist = np.zeros(int(self.opts.max_it) + 1)
        L.call("pb_ksp_end", self.h, C.byref(res), _dptr(hist), hist.size)
        self.result = res
        return res.reason, res.its, hist[: res.nhist].copy()

    def pc_apply(self, r, z):
        """PCApply: z = M^-1 r (no null-space removal)."""
        L.call("pb_ksp_pc_apply", self.h, r.h, z.h)

    @property
    def pc_levels(self):
        v = C.c_int(0)
        L.call("pb_ksp_pc_levels", self.h, C.byref(v))
        return v.value

    def destroy(self):
        if self.h:
            L.call("pb_ksp_destroy", self.h)
            self.h = None


# ---- reference-named entry points ----------------------------------------------------------
def initialise_grid(ctx, nglobal, L_=(1.0, 1.0, 1.0)):
    """src/poissbox.f90:183-204"""
    return DA(ctx, nglobal, L_)


def initialise_linear_system(da, grid_deltas, matrix_free=True):
    """src/poissbox.f90:206-240: returns (P, A, x, b); A is the matrix-free operator when
    matrix_free (src/example.f90:60-65), else A = P."""
    P = Mat(da, ASSEMBLED27, grid_deltas)
    A = Mat(da, STAR7, grid_deltas) if matrix_free else P
    return P, A, Vec(da), Vec(da)


def compute_lapl_pointwise(da, grid_deltas, x, b):
    """src/poissbox.f90:84-126 (one pass of the stencil, same kernel as mfmult)."""
    op = Mat(da, STAR7, grid_deltas)
    try:
        op.mult(x, b)
    finally:
        op.destroy()


def solve(P, A, x, b, options=("-ksp_type", "cg", "-pc_type", "jacobi")):
    """src/poissbox.f90:269-298: constant null space on A and P, KSPSolve(b -> x)."""
    ksp = KSP(A, P, options)
    try:
        return ksp.solve(b, x)
    finally:
        ksp.destroy()


# ---- tridiagonal / compact ------------------------------------------------------------------
def tdma_batched(ctx, n, nbatch, line_stride, elem_stride, a_ptr, b_ptr, c_ptr, d_ptr,
                 periodic=False):
    L.call("pb_tdma_batched", ctx.h, int(n), int(nbatch), int(line_stride), int(elem_stride),
           a_ptr, b_ptr, c_ptr, d_ptr, int(bool(periodic)))


def pcr_alpha_batched(ctx, n, nbatch, line_stride, elem_stride, alpha, d_ptr):
    L.call("pb_pcr_alpha_batched", ctx.h, int(n), int(nbatch), int(line_stride),
           int(elem_stride), float(alpha), d_ptr)


def compact_1d_batched(ctx, kind, stagger, dx, n, nbatch, line_stride, elem_stride, f_ptr,
                       out_ptr):
    L.call("pb_compact_1d_batched", ctx.h, int(kind), int(stagger), float(dx), int(n),
           int(nbatch), int(line_stride), int(elem_stride), f_ptr, out_ptr)


def compact_grad(da, dx, f, df3):
    arr = (C.c_void_p * 3)(*[v.h.value for v in df3])
    L.call("pb_compact_grad", da.h, _d_3(dx), f.h, arr)


def compact_div(da, dx, f3, df):
    arr = (C.c_void_p * 3)(*[v.h.value for v in f3])
    L.call("pb_compact_div", da.h, _d_3(dx), arr, df.h)


def compact_interp(da, stagger, f, fi):
    L.call("pb_compact_interp", da.h, int(stagger), f.h, fi.h)


def compact_lapl(da, dx, f, out):
    L.call("pb_compact_lapl", da.h, _d_3(dx), f.h, out.h)


# host-array forms (the reference's module procedures on process-local arrays)
def tdma_host(ctx, a, b, c, d, periodic=False):
    """tdma / tdma_periodic (src/tridsol.f90:22-74) on host arrays, batched over leading axes:
    the last axis is the line. b and d are updated in place like the reference."""
    for v in (a, b, c, d):
        assert v.dtype == np.float64 and v.flags.c_contiguous and v.shape == d.shape
    n = d.shape[-1]
    L.call("pb_tdma_batched_host", ctx.h, n, d.size // n, n, 1, _dptr(a), _dptr(b), _dptr(c),
           _dptr(d), int(bool(periodic)))


def compact_host(ctx, op, f, n, dx=(1.0, 1.0, 1.0), stagger=-1):
    """grad / div / interp / lapl (src/compact_schemes.f90) on whole host arrays (C order
    [c][k][j][i] == Fortran (i, j, k, c)); returns the result array."""
    f = np.ascontiguousarray(f, dtype=np.float64).reshape(-1)
    N = int(np.prod(n))
    out = np.empty(3 * N if op == "grad" else N)
    if op == "interp":
        L.call("pb_compact_interp_host", ctx.h, _i64_3(n), int(stagger), _dptr(f), _dptr(out))
    else:
        L.call(f"pb_compact_{op}_host", ctx.h, _i64_3(n), _d_3(dx), _dptr(f), _dptr(out))
    return out


def compact_lapl_fast(da, dx, f, out):
    """3-pass factorised compact Laplacian with PCR line solves (agrees with compact_lapl to
    rounding); the operator PB_OP_COMPACT applies."""
    L.call("pb_compact_lapl_fast", da.h, _d_3(dx), f.h, out.h)
