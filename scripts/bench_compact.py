"""Fast compact Laplacian (pb_compact_lapl_fast, 3-pass factorisation) apply time per grid, with
per-pass averages (HIP events around each line pass); one JSON line per grid with the
knobs in the environment. usage: python scripts/bench_compact.py [n ...]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [512]
    ctx = pb.Context(0)
    for n in sizes:
        n3 = (n, n, n)
        h = (2 * np.pi / n,) * 3
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        f, out = pb.Vec(da), pb.Vec(da)
        f.set_random(7)
        for _ in range(3):
            pb.compact_lapl_fast(da, h, f, out)
        ctx.sync()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            pb.compact_lapl_fast(da, h, f, out)
        ctx.sync()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        ctx.set_timing(True)
        ctx.reset_timing()
        for _ in range(reps):
            pb.compact_lapl_fast(da, h, f, out)
        ctx.sync()
        passes = {}
        for nm, bpd in (("compact_lines_z", 24), ("compact_lines_y", 32), ("compact_lines_x", 24)):
            t, c = ctx.timing(nm)
            if c:
                passes[nm] = {"ms": round(t / c, 4), "GBps": round(bpd * n ** 3 / (t / c) / 1e6, 1)}
        ctx.set_timing(False)
        cfg = {}
        print(json.dumps({"n": n, "lapl_ms": ms, "GBps_80B": 80 * n ** 3 / ms / 1e6,
                          "frac": 80 * n ** 3 / ms / 1e6 / 8000.0, "passes": passes, "cfg": cfg}),
              flush=True)
        for o in (f, out):
            o.destroy()
        da.destroy()


if __name__ == "__main__":
    main()
