"""SURVEY.md §8(d) timing protocol at 512^3 on one GPU, one JSON line per measurement:
  (i)   100 matvecs after 10 warm-ups (HIP events per launch),
  (ii)  a fixed 200 CG + Jacobi iterations with the reductions enabled (wall clock around
        pb_ksp_iterate, synchronised; rtol = 0 so every iteration runs the full scalar logic),
  (iii) a full solve to rtol 1e-10 (CG + Jacobi; CG + MG beside it),
each repeated 5 times; the median and the spread are reported.
usage: python scripts/bench_protocol.py [n]   (default 512)
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

SEED = 20231015
REPS = 5


def med(v):
    return {"median": statistics.median(v), "min": min(v), "max": max(v), "n": len(v)}


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = (m, m, m)
    N = m ** 3
    ctx = pb.Context(0)
    da = pb.DA(ctx, n)
    h = da.spacing
    P, A, x, b = pb.initialise_linear_system(da, h)
    xt = pb.Vec(da)
    xt.set_random(SEED)
    A.mult(xt, b)
    y = pb.Vec(da)

    # (i) matvec
    per = []
    for _ in range(REPS):
        for _ in range(10):
            A.mult(xt, y)
        ctx.sync()
        ctx.set_timing(True)
        ctx.reset_timing()
        for _ in range(100):
            A.mult(xt, y)
        ctx.sync()
        ms, cnt = ctx.timing("stencil")
        ctx.set_timing(False)
        per.append(ms / cnt)
    r = med(per)
    print(json.dumps({"n": m, "what": "(i) matvec, 100 after 10 warm-ups", "ms": r,
                      "dofs_per_s": N / (r["median"] / 1e3),
                      "GBps": 16 * N / (r["median"] / 1e3) / 1e9}), flush=True)

    # (ii) fixed 200 CG iterations
    per = []
    for _ in range(REPS):
        k = pb.KSP(A, P, pb.ksp_options(["-ksp_type", "cg", "-pc_type", "jacobi"], rtol=0.0,
                                        atol=0.0, dtol=1e300, max_it=260))
        k.begin(b, x)
        k.iterate(10)
        ctx.sync()
        t0 = time.perf_counter()
        k.iterate(200)
        ctx.sync()
        per.append((time.perf_counter() - t0) / 200 * 1e3)
        k.end()
        k.destroy()
    r = med(per)
    print(json.dumps({"n": m, "what": "(ii) 200 CG + Jacobi iterations, reductions enabled",
                      "ms_per_it": r, "dof_updates_per_s": N / (r["median"] / 1e3),
                      "it_per_s": 1e3 / r["median"]}), flush=True)

    # (iii) full solves to rtol 1e-10
    for pc in ("jacobi", "mg"):
        per, its_ = [], None
        for _ in range(REPS):
            k = pb.KSP(A, P, pb.ksp_options(["-ksp_type", "cg", "-pc_type", pc,
                                             "-ksp_rtol", "1e-10"]))
            ctx.sync()
            t0 = time.perf_counter()
            reason, its, hist = k.solve(b, x)
            ctx.sync()
            per.append((time.perf_counter() - t0) * 1e3)
            its_ = (reason, its)
            k.destroy()
        r = med(per)
        print(json.dumps({"n": m, "what": f"(iii) full solve, CG + {pc}, rtol 1e-10",
                          "reason": its_[0], "its": its_[1], "solve_ms": r}), flush=True)
    for o in (P, A, x, b, xt, y):
        o.destroy()
    da.destroy()
    ctx.destroy()


if __name__ == "__main__":
    main()
