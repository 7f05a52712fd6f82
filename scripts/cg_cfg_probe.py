"""CG iteration and matvec across buffer placements x tuning configurations:
R solver instances at n^3, each with fresh vectors (the earlier instances stay allocated, so each
gets other memory); every instance runs every configuration interleaved: `its` fixed CG + Jacobi
iterations (ms/iteration, per-pass HIP-event averages) and `mv` matvecs x -> y of its own vectors.
Prints per configuration min / median / max over instances.
Usage: python scripts/cg_cfg_probe.py [n | nxXnyXnz] [R] [configs-json] [alloc]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

PASSES = ("cg_pass_a", "cg_pass_b_even", "cg_pass_b_x4", "stencil")


def main():
    a1 = sys.argv[1] if len(sys.argv) > 1 else "512"
    n3 = tuple(int(v) for v in a1.split("x")) if "x" in a1 else (int(a1),) * 3
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    configs = json.loads(sys.argv[3]) if len(sys.argv) > 3 else [{}, {"engine_kc_skew": 4}]
    # alloc mode: every configuration gets its own instances (settings that act at allocation,
    # field_stagger_kib); otherwise every instance runs every configuration
    alloc_mode = len(sys.argv) > 4 and sys.argv[4] == "alloc"
    its, warm, mv = 32, 8, 10
    ctx = pb.Context(0)
    da = pb.initialise_grid(ctx, n3)
    P, A = pb.Mat(da, pb.ASSEMBLED27, da.spacing), pb.Mat(da, pb.STAR7, da.spacing)
    keep = []
    res = {}
    plan = [(inst, [ci]) for inst in range(R) for ci in range(len(configs))] if alloc_mode \
        else [(inst, list(range(len(configs)))) for inst in range(R)]
    for inst, cis in plan:
        if alloc_mode:
            pb.tune_reset()
            for k_, v_ in configs[cis[0]].items():
                pb.tune_set(k_, v_)
        x, b, xt, y = pb.Vec(da), pb.Vec(da), pb.Vec(da), pb.Vec(da)
        xt.set_random(20231015)
        A.mult(xt, b)
        opts = pb.ksp_options(["-ksp_type", "cg", "-pc_type", "jacobi"], rtol=0.0, atol=0.0,
                              dtol=1e300, max_it=len(configs) * 2 * (its + warm) + 64,
                              check_every=8)
        k = pb.KSP(A, P, opts)
        k.begin(b, x)
        keep.append((x, b, xt, y, k))
        for rnd in range(2):
            for ci in cis:
                cfg = configs[ci]
                pb.tune_reset()
                for k_, v_ in cfg.items():
                    pb.tune_set(k_, v_)
                k.iterate(warm)
                ctx.sync()
                ctx.set_timing(True)
                ctx.reset_timing()
                t0 = time.perf_counter()
                k.iterate(its)
                ctx.sync()
                dt = (time.perf_counter() - t0) / its * 1e3
                passes = {p_: ctx.timing(p_) for p_ in PASSES}
                pbs = [round(float(v), 4) for v in ctx.timing_samples("cg_pass_b_even")]
                ctx.reset_timing()
                for _ in range(mv):
                    A.mult(xt, y)
                ctx.sync()
                smp = sorted(float(v) for v in ctx.timing_samples("stencil"))
                ctx.set_timing(False)
                row = {"inst": inst, "rnd": rnd, "cfg": ci, "ms_per_it": dt,
                       "mv_med_ms": smp[len(smp) // 2], "pass_b_samples": pbs}
                for p_, (ms_, c_) in passes.items():
                    if c_ and p_ != "stencil":
                        row[p_] = ms_ / c_
                res.setdefault((ci, inst), []).append(row)
                print(json.dumps(row), flush=True)
    pb.tune_reset()
    for ci, cfg in enumerate(configs):
        out = {"config": cfg}
        for key in ("ms_per_it", "mv_med_ms", "cg_pass_a", "cg_pass_b_even"):
            vals = sorted(min(r[key] for r in res[(ci, i)] if key in r) for i in range(R)
                          if (ci, i) in res and any(key in r for r in res[(ci, i)]))
            if vals:
                out[key] = [round(vals[0], 4), round(vals[len(vals) // 2], 4), round(vals[-1], 4)]
        print(json.dumps(out), flush=True)
    for t in keep:
        t[4].end()
    ctx.destroy()


if __name__ == "__main__":
    main()
