"""Time the 3-pass compact Laplacian per pass at n^3 (default 512) on one GPU; one JSON line.
Tuning knobs come from the environment (PB_LINES_TL, PB_LINES_ABLATE, PB_COMPACT_LINES)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

BYTES = {"compact_lines_z": 24, "compact_lines_y": 32, "compact_lines_x": 24, "compact_lapl_fast": 80}


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    ctx = pb.Context(0)
    da = pb.DA(ctx, (m, m, m), (2 * np.pi,) * 3)
    f, out = pb.Vec(da), pb.Vec(da)
    f.set_random(5)
    h = da.spacing
    for _ in range(10):
        pb.compact_lapl_fast(da, h, f, out)
    ctx.sync()
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(30):
        pb.compact_lapl_fast(da, h, f, out)
    ctx.sync()
    res = {"n": m, "env": {k: v for k, v in os.environ.items() if k.startswith("PB_")}}
    for name, b in BYTES.items():
        ms, cnt = ctx.timing(name)
        if cnt:
            avg = ms / cnt
            res[name] = {"ms": round(avg, 4), "GBps": round(b * m ** 3 / avg / 1e6, 1)}
    # batched (alpha, 1, alpha) solve over m^2 interleaved lines of m points (the PCR row)
    dp, _ = out.device_ptr()
    for _ in range(5):
        pb.pcr_alpha_batched(ctx, m, m * m, 1, m * m, 0.3, dp)
    ctx.sync()
    ctx.reset_timing()
    for _ in range(20):
        pb.pcr_alpha_batched(ctx, m, m * m, 1, m * m, 0.3, dp)
    ctx.sync()
    ms, cnt = ctx.timing("pcr")
    if cnt:
        res["pcr_interleaved"] = {"ms": round(ms / cnt, 4), "GBps": round(16 * m ** 3 / (ms / cnt) / 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
