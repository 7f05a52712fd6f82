"""Spectral PC apply time (pb_ksp_pc_apply, -pc_type fft) per grid; one JSON line per grid with
the tuning settings. usage: python scripts/bench_fft.py [n | nx x ny x nz ...]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402


def main():
    sizes = sys.argv[1:] or ["512"]
    ctx = pb.Context(0)
    for arg in sizes:
        n3 = tuple(int(v) for v in arg.split("x")) if "x" in arg else (int(arg),) * 3
        n = n3[0] if len(set(n3)) == 1 else "x".join(map(str, n3))
        h = tuple(2 * np.pi / m for m in n3)
        da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
        P = pb.Mat(da, pb.COMPACT, h)
        k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
        r, z = pb.Vec(da), pb.Vec(da)
        r.set_random(7)
        for _ in range(3):
            k.pc_apply(r, z)
        ctx.sync()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            k.pc_apply(r, z)
        ctx.sync()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        # per-pass averages (HIP events around each line pass, a separate set of applies)
        ctx.set_timing(True)
        ctx.reset_timing()
        for _ in range(reps):
            k.pc_apply(r, z)
        ctx.sync()
        passes = {}
        for nm in ("pc_fft_x", "pc_fft_y", "pc_fft_z"):
            t, c = ctx.timing(nm)
            if c:
                passes[nm] = round(t / c, 4)
        ctx.set_timing(False)
        cfg = {}
        ndof = n3[0] * n3[1] * n3[2]
        print(json.dumps({"n": n, "pc_apply_ms": ms, "GBps_80B": 80 * ndof / ms / 1e6,
                          "passes_ms": passes, "cfg": cfg}), flush=True)
        for o in (k, r, z, P):
            o.destroy()
        da.destroy()


if __name__ == "__main__":
    main()
