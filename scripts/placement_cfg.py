"""Matvec launch configurations across buffer pairings: K fresh 512^3
vectors, every ordered pair (i, j) runs the matvec v_i -> v_j under each tuning configuration
(median of `reps` HIP-event-timed launches); prints per config the min / median / max over pairs
and the matrix. Usage: python scripts/placement_cfg.py [n] [K] [reps] [configs-json]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

CONFIGS = [{}, {"stencil_nt": 0}, {"stencil_tall": 0}, {"stencil_tall": 0, "stencil_wgcu": 1},
           {"stencil_wgcu": 2}, {"stencil_tall": 0, "stencil_nt": 0}]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    configs = json.loads(sys.argv[4]) if len(sys.argv) > 4 else CONFIGS
    ctx = pb.Context(0)
    da = pb.initialise_grid(ctx, (n, n, n))
    A = pb.Mat(da, pb.STAR7, da.spacing)
    vs = []
    for s in range(K):
        v = pb.Vec(da)
        v.set_random(1000 + s)
        vs.append(v)
    nloc = da.nlocal
    res = {}
    for rnd in range(2):  # two rounds, configs interleaved per pair
        for i in range(K):
            for j in range(K):
                if i == j:
                    continue
                for ci, cfg in enumerate(configs):
                    pb.tune_reset()
                    for k_, v_ in cfg.items():
                        pb.tune_set(k_, v_)
                    for _ in range(2):
                        A.mult(vs[i], vs[j])
                    ctx.sync()
                    ctx.set_timing(True)
                    ctx.reset_timing()
                    for _ in range(reps):
                        A.mult(vs[i], vs[j])
                    ctx.sync()
                    smp = sorted(float(v) for v in ctx.timing_samples("stencil"))
                    ctx.set_timing(False)
                    res.setdefault((ci, i, j), []).append(smp[len(smp) // 2])
                vs[j].set_random(1000 + j)
        print(json.dumps({"round_done": rnd}), flush=True)
    pb.tune_reset()
    for ci, cfg in enumerate(configs):
        M = [[None] * K for _ in range(K)]
        vals = []
        for (c, i, j), v in res.items():
            if c == ci:
                M[i][j] = round(min(v), 4)
                vals.append(min(v))
        vals.sort()
        fr = lambda t: 16 * nloc / (t * 1e-3) / 1e9 / 8000.0
        print(json.dumps({"config": cfg, "min_ms": vals[0], "med_ms": vals[len(vals) // 2],
                          "max_ms": vals[-1], "frac_worst": fr(vals[-1]),
                          "frac_med": fr(vals[len(vals) // 2]), "matrix": M}), flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
