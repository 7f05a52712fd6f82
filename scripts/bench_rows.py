"""Per-row measurement of SURVEY.md §8 kernels on one MI355X against their HBM roofline, with the
oracle's CPU restatement of the same reference function timed beside it (1 core unless noted).

Prints one JSON line per row: {"row", "kernel", "size", "avg_ms", "bytes_per_dof",
"GBps", "frac_of_8TBps", "cpu": {...}}. Rows:
  a6/a7 matvec (7-point)            16 B/DoF    512^3
  a2 CG iteration (fused, deferred) 60 B/DoF    512^3 (passes reported by bench.py)
  a12 tdma (general, batched)       48 B/DoF    512 x 512^2 lines (read a,b,c,d; write b,d)
  a13 tdma_periodic (batched)       40 B/DoF    512 x 512^2 lines (read a,b,c,d; write d)
  PCR (alpha,1,alpha) batched       16 B/DoF    512 x 512^2 lines, interleaved and contiguous
  a15 compact 1-D (grad_1d)         16 B/DoF    512 x 512^2 lines (reference order, bit-exact)
  a16 compact lapl, reference order 80 B/DoF*   256^3   (*the 3-pass algorithmic minimum)
  a16 compact lapl, 3-pass + PCR    80 B/DoF    512^3 and 256^3
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import poissbox_amd as pb  # noqa: E402
from oracle import oracle as O  # noqa: E402

PEAK = 8000.0
hip = C.CDLL("libamdhip64.so")


def timed(ctx, fn, reps, name, warm_s=0.5):
    """Average launch time of fn under HIP events, after warming up for warm_s seconds of the same
    launches: r03's single warm-up launch left the first rows (the matvec ran first in the process)
    timing the GPU before its clocks had settled -- 0.423 ms against 0.369 ms from the §8(d)
    protocol's 10 warm-ups on the same box."""
    fn()
    ctx.sync()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(8):
            fn()
        ctx.sync()
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(reps):
        fn()
    ctx.sync()
    ms, cnt = ctx.timing(name)
    ctx.set_timing(False)
    return ms / max(cnt, 1)


def wall(fn, reps):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps


TIME_REF = os.path.join(REPO, "oracle", "_ref", "time_ref")


def ref_cpu(op, n, seconds, port_fn, port_sample):
    """CPU rate of the REAL reference routine (flang-built from /root/reference sources by
    `make -C oracle ref`, oracle/time_ref.f90), one core; the oracle's restatement when that
    binary is absent."""
    import subprocess
    if os.path.exists(TIME_REF):
        try:
            out = subprocess.run([TIME_REF, op, str(n), str(seconds)], capture_output=True, text=True,
                                 timeout=60 + 4 * seconds, check=True).stdout
            d = json.loads(out.strip().splitlines()[-1])
            return {"dofs_per_s_1core": d["dofs_per_s"], "kind": "reference",
                    "sample": f"reference {op} (src/tridsol.f90 / src/compact_schemes.f90 via "
                              f"oracle/time_ref.f90), n={n}, {d['reps']} reps in {d['seconds']:.2f} s"}
        except Exception as e:  # fall back to the restatement
            print(f"time_ref {op}: {e}", file=sys.stderr)
    return {"dofs_per_s_1core": port_fn(), "kind": "port", "sample": port_sample}


def row(name, kernel, size, dofs, bytes_per_dof, ms, cpu=None):
    gbps = bytes_per_dof * dofs / (ms / 1e3) / 1e9
    out = {"row": name, "kernel": kernel, "size": size, "avg_ms": ms, "bytes_per_dof": bytes_per_dof,
           "GBps": gbps, "frac_of_8TBps": gbps / PEAK, "dofs_per_s": dofs / (ms / 1e3)}
    if cpu:
        out["cpu"] = cpu
    print(json.dumps(out), flush=True)


def dev_buf(n, fill=None):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(8 * n)) == 0
    if fill is not None:
        a = np.ascontiguousarray(fill, dtype=np.float64)
        assert hip.hipMemcpy(p, a.ctypes.data_as(C.c_void_p), C.c_size_t(8 * n), 1) == 0
        assert hip.hipDeviceSynchronize() == 0
    return p


def main():
    ctx = pb.Context(0)
    # ---- matvec 512^3 ----
    n3 = (512, 512, 512)
    N = 512 ** 3
    da = pb.DA(ctx, n3)
    A = pb.Mat(da, pb.STAR7)
    x, y = pb.Vec(da), pb.Vec(da)
    x.set_random(1)
    ms = timed(ctx, lambda: A.mult(x, y), 100, "stencil")
    n64 = (128, 128, 128)
    xs = O.fill_random(128 ** 3, 1)
    t1 = wall(lambda: O.stencil(xs, n64, (1 / 128,) * 3, faithful=True), 1)
    t7 = wall(lambda: O.stencil(xs, n64, (1 / 128,) * 3), 3)
    row("a6/a7", "star7 matvec", "512^3", N, 16, ms,
        {"faithful_27term_dofs_per_s_1core": 128 ** 3 / t1, "7term_dofs_per_s_1core": 128 ** 3 / t7,
         "sample": "128^3, oracle pbo_stencil_apply27 / apply7"})
    for o in (A, x, y):
        o.destroy()
    da.destroy()

    # ---- line solvers: 512-long lines, 512^2 of them, interleaved (line stride 1) ----
    n, nb = 512, 512 * 512
    rng = np.random.default_rng(3)
    host = {k: rng.random(n * nb) for k in "abcd"}
    host["b"] = host["b"] * 10 + 3  # diagonally dominant
    bufs = {k: dev_buf(n * nb, v) for k, v in host.items()}
    ms = timed(ctx, lambda: pb.tdma_batched(ctx, n, nb, 1, nb, bufs["a"], bufs["b"], bufs["c"],
                                            bufs["d"], periodic=False), 5, "tdma")
    a1, b1, c1, d1 = (host[k][:n * 64].reshape(n, 64)[:, 0].copy() for k in "abcd")
    row("a12", "tdma (Thomas, one lane per line)", "512 x 512^2", n * nb, 48, ms,
        ref_cpu("tdma", n, 2, lambda: n / wall(lambda: O.tdma(a1, b1, c1, d1), 200),
                "oracle pbo_tdma, one 512 line"))
    ms = timed(ctx, lambda: pb.tdma_batched(ctx, n, nb, 1, nb, bufs["a"], bufs["b"], bufs["c"],
                                            bufs["d"], periodic=True), 5, "tdma")
    row("a13", "tdma_periodic (Sherman-Morrison, one lane per line)", "512 x 512^2", n * nb, 40, ms,
        ref_cpu("tdma_periodic", n, 2,
                lambda: n / wall(lambda: O.tdma(a1, b1, c1, d1, periodic=True), 200),
                "oracle pbo_tdma_periodic, one 512 line"))
    ms = timed(ctx, lambda: pb.pcr_alpha_batched(ctx, n, nb, 1, nb, 0.3, bufs["d"]), 5, "pcr")
    row("PCR", "batched (a,1,a) solve, interleaved lines", "512 x 512^2", n * nb, 16, ms)
    ms = timed(ctx, lambda: pb.pcr_alpha_batched(ctx, n, nb, n, 1, 0.3, bufs["d"]), 5, "pcr")
    row("PCR", "batched (a,1,a) solve, contiguous lines", "512 x 512^2", n * nb, 16, ms)
    ms = timed(ctx, lambda: pb.compact_1d_batched(ctx, 0, -1, 0.01, n, nb, 1, nb, bufs["a"],
                                                  bufs["d"]), 5, "compact_1d")
    f1 = host["a"][:n].copy()
    row("a15", "grad_1d (reference order, one lane per line)", "512 x 512^2", n * nb, 16, ms,
        ref_cpu("grad_1d", n, 2, lambda: n / wall(lambda: O.grad_1d(f1, 0.01), 200),
                "oracle pbo_grad_1d, one 512 line"))
    for v in bufs.values():
        hip.hipFree(v)

    # ---- compact Laplacian ----
    for m in (256, 512):
        n3 = (m, m, m)
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        f, out = pb.Vec(da), pb.Vec(da)
        f.set_random(5)
        h = da.spacing
        ms = timed(ctx, lambda: pb.compact_lapl_fast(da, h, f, out), 5, "compact_lapl_fast")
        cpu = None
        if m == 256:
            fc = O.fill_random(64 ** 3, 5)
            cpu = ref_cpu("lapl", 64, 3,
                          lambda: 64 ** 3 / wall(lambda: O.lapl(fc, (64, 64, 64),
                                                                (2 * np.pi / 64,) * 3), 1),
                          "oracle pbo_lapl (reference order), 64^3")
        row("a16", "compact lapl 3-pass + PCR", f"{m}^3", m ** 3, 80, ms, cpu)
        if m == 256:
            ms = timed(ctx, lambda: pb.compact_lapl(da, h, f, out), 2, "compact_lapl")
            row("a16", "compact lapl, reference order (bit-exact)", f"{m}^3", m ** 3, 80, ms)
        for o in (f, out):
            o.destroy()
        da.destroy()
    ctx.destroy()


if __name__ == "__main__":
    main()
