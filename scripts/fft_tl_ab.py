"""Spectral PC apply at 512^3 under tuning variants, interleaved in one process (r06: 8-line
tiles for the strided passes, fft_tl8). Prints per variant the apply time and the Z / Y pass
averages, and whether z is bit-identical to the default's. usage: python scripts/fft_tl_ab.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

VARIANTS = [{}, {"fft_persist": 1}]


def main():
    n3 = (512, 512, 512)
    ctx = pb.Context(0)
    h = tuple(2 * np.pi / m for m in n3)
    da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
    P = pb.Mat(da, pb.COMPACT, h)
    k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
    r, z = pb.Vec(da), pb.Vec(da)
    r.set_random(7)
    ref = None
    for rnd in range(3):
        for v in VARIANTS:
            pb.tune_reset()
            for k_, v_ in v.items():
                pb.tune_set(k_, v_)
            for _ in range(3):
                k.pc_apply(r, z)
            ctx.sync()
            ctx.set_timing(True)
            ctx.reset_timing()
            t0 = time.perf_counter()
            for _ in range(20):
                k.pc_apply(r, z)
            ctx.sync()
            ms = (time.perf_counter() - t0) * 1e3 / 20
            row = {"rnd": rnd, "tune": v, "apply_ms": round(ms, 4)}
            for nm in ("pc_fft_x", "pc_fft_y", "pc_fft_z"):
                t_, c_ = ctx.timing(nm)
                row[nm] = round(t_ / c_, 4) if c_ else None
            ctx.set_timing(False)
            zv = z.get_values()
            if ref is None:
                ref = zv
            row["bit_identical"] = bool(np.array_equal(zv, ref))
            print(json.dumps(row), flush=True)
    pb.tune_reset()
    ctx.destroy()


if __name__ == "__main__":
    main()
