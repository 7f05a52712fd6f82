"""The spectral PC's Z pass on a y-slab-shaped grid (config 5 over 8 ranks: 512 x 64 x 512, 256 KiB
planes) with and without the padded Z buffer; interleaved rounds, per-pass HIP-event times.
usage: python scripts/ab_fft_zpad_shape.py [NXxNYxNZ ...]"""
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

configs = [{}, {"fft_zpad_min_plane": 0}, {"fft_zpad_min_plane": 0, "fft_zpad": 64}]
ctx = pb.Context(0)
for arg in sys.argv[1:] or ["512x64x512"]:
    n3 = tuple(int(v) for v in arg.split("x"))
    h = tuple(2 * np.pi / m for m in n3)
    da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
    P = pb.Mat(da, pb.COMPACT, h)
    r, z = pb.Vec(da), pb.Vec(da)
    r.set_random(7)
    acc = [{nm: [] for nm in ("pc_fft", "pc_fft_y", "pc_fft_z")} for _ in configs]
    for rnd in range(4):
        for i, cfg in enumerate(configs):
            pb.tune_reset()
            for key, v in cfg.items():
                pb.tune_set(key, int(v))
            k = pb.KSP(P, P, pb.ksp_options(["-pc_type", "fft"]))
            for _ in range(3):
                k.pc_apply(r, z)
            ctx.sync()
            ctx.set_timing(True)
            ctx.reset_timing()
            for _ in range(20):
                k.pc_apply(r, z)
            ctx.sync()
            for nm in acc[i]:
                ms, cnt = ctx.timing(nm)
                acc[i][nm].append(ms / cnt if cnt else 0.0)
            ctx.set_timing(False)
            k.destroy()
    pb.tune_reset()
    for i, cfg in enumerate(configs):
        print(json.dumps({"grid": arg, "cfg": cfg, **{nm: round(statistics.median(v), 4)
                                                     for nm, v in acc[i].items()}}), flush=True)
