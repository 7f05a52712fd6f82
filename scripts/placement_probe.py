"""Placement probe: does the 7-point matvec's rate depend on where its x and y
buffers sit? One process, 512^3: NX input vectors x_s and NY output vectors y_t are allocated
(fresh device allocations), every (x_s, y_t) pair runs `reps` timed matvecs (HIP events per
launch) and a flat copy x_s -> y_t over the same buffers; the device addresses are printed mod
2 MiB and 1 GiB. One JSON line per pair, then a summary line.
Usage: python scripts/placement_probe.py [n] [NX] [NY] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

HBM = 8000.0


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    nx_ = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ny_ = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    ctx = pb.Context(0)
    da = pb.initialise_grid(ctx, (n, n, n))
    A = pb.Mat(da, pb.STAR7, da.spacing)
    xs = []
    for s in range(nx_):
        v = pb.Vec(da)
        v.set_random(1000 + s)
        xs.append(v)
    ys = [pb.Vec(da) for _ in range(ny_)]
    nloc = da.nlocal
    rows = []
    for si, x in enumerate(xs):
        for ti, y in enumerate(ys):
            for _ in range(3):
                A.mult(x, y)
            ctx.sync()
            ctx.set_timing(True)
            ctx.reset_timing()
            for _ in range(reps):
                A.mult(x, y)
            ctx.sync()
            smp = sorted(float(v) for v in ctx.timing_samples("stencil"))
            ctx.set_timing(False)
            cb, cm = x.copy_probe(y, reps=6)
            px, py = x.device_ptr()[0], y.device_ptr()[0]
            med = smp[len(smp) // 2]
            row = {"x": si, "y": ti, "mv_med_ms": med, "mv_best_ms": smp[0],
                   "mv_frac": 16 * nloc / (med * 1e-3) / 1e9 / HBM,
                   "copy_best_frac": cb / HBM, "copy_med_frac": cm / HBM,
                   "x_mod2M": px % (1 << 21), "y_mod2M": py % (1 << 21),
                   "x_mod1G": px % (1 << 30), "y_mod1G": py % (1 << 30),
                   "y_minus_x_mod1G": (py - px) % (1 << 30), "x_hex": hex(px), "y_hex": hex(py)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    fr = sorted(r["mv_frac"] for r in rows)
    cp = sorted(r["copy_med_frac"] for r in rows)
    print(json.dumps({"summary": True, "n": n, "pairs": len(rows), "mv_frac_min": fr[0],
                      "mv_frac_med": fr[len(fr) // 2], "mv_frac_max": fr[-1],
                      "copy_frac_min": cp[0], "copy_frac_max": cp[-1]}), flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
