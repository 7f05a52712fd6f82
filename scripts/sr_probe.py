"""Per-iteration time of the KSPSolve_CG and single-reduction CG iterations (fixed iterations, one
GPU), interleaved in one process, plus per-pass HIP-event averages. Usage:
  python scripts/sr_probe.py [N ...]   (default 512 256)   -> one JSON line per (N, variant, rep)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

PASSES = ("cg_pass_a", "cg_pass_b_even", "cg_pass_b_x4", "cg_sr_p", "cg_sr_p_x4", "cg_sr_s", "cg_sr1")


def run(ctx, n, sr, steps=100, warmup=12, diag=16):
    da = pb.initialise_grid(ctx, (n, n, n))
    P, A, x, b = pb.initialise_linear_system(da, da.spacing)
    xt = pb.Vec(da)
    xt.set_random(20231015)
    A.mult(xt, b)
    argv = ["-ksp_type", "cg", "-pc_type", "jacobi"] + (["-ksp_cg_single_reduction"] if sr else [])
    opts = pb.ksp_options(argv, rtol=0.0, atol=0.0, dtol=1e300,
                          max_it=warmup + steps + diag + 16, check_every=8)
    k = pb.KSP(A, P, opts)
    k.begin(b, x)
    k.iterate(warmup)
    ctx.sync()
    t0 = time.perf_counter()
    k.iterate(steps)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    ctx.set_timing(True)
    ctx.reset_timing()
    k.iterate(diag)
    ctx.sync()
    passes = {}
    for nm in PASSES:
        ms, cnt = ctx.timing(nm)
        if cnt:
            passes[nm] = round(ms / cnt, 4)
    ctx.set_timing(False)
    reason, its, hist = k.end()
    for o in (k, xt, x, b, A, P):
        o.destroy()
    da.destroy()
    return {"n": n, "sr": sr, "ms_per_it": round(dt * 1e3, 4), "passes_ms": passes,
            "its": its, "rnorm_last": float(hist[-1]), "gdofs": n ** 3 / dt / 1e9}


def main():
    """args: sizes (ints) and A/B settings "name=v[,name=v...]" (each one a variant, interleaved;
    "-" = defaults); with settings only the single-reduction iteration runs"""
    args = sys.argv[1:]
    combos = [a for a in args if "=" in a or a == "-"]
    sizes = [int(a) for a in args if a.isdigit()] or [512, 256]
    ctx = pb.Context(0)
    for n in sizes:
        for rep in range(int(os.environ.get("SR_REPS", "3"))):
            for c in (combos or [None]):
                for sr in ((1,) if combos else (0, 1)):
                    pb.tune_reset()
                    kv = {}
                    if c and c != "-":
                        for item in c.split(","):
                            k_, v_ = item.split("=")
                            kv[k_] = int(v_)
                            pb.tune_set(k_, int(v_))
                    r = run(ctx, n, sr)
                    r.update(rep=rep, tune=kv)
                    print(json.dumps(r), flush=True)
    pb.tune_reset()
    ctx.destroy()


if __name__ == "__main__":
    main()
