"""Per-iteration time of the CG iterations on the decomposed code path (force_comm: a one-rank
RCCL communicator -- boundary-plane kernel, halo exchange overlapped with the interior planes,
allreduced sums folded into the next launch's prologue) against one rank, interleaved in one
process, fixed iterations. usage: [FC=0,1] [SR=0,1] [REPS=3] python scripts/probe_decomposed_cg.py
[N ...] (default 512)
One JSON line per (N, force_comm, variant, rep)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

STEPS, WARMUP = 100, 12


def run(ctx, n, sr):
    da = pb.DA(ctx, (n, n, n))
    P, A, x, b = pb.initialise_linear_system(da, da.spacing)
    xt = pb.Vec(da)
    xt.set_random(20231015)
    A.mult(xt, b)
    argv = ["-ksp_type", "cg", "-pc_type", "jacobi"] + (["-ksp_cg_single_reduction"] if sr else [])
    k = pb.KSP(A, P, pb.ksp_options(argv, rtol=0.0, atol=0.0, dtol=1e300,
                                    max_it=WARMUP + STEPS + 16, check_every=8))
    k.begin(b, x)
    k.iterate(WARMUP)
    ctx.sync()
    t0 = time.perf_counter()
    k.iterate(STEPS)
    ctx.sync()
    dt = (time.perf_counter() - t0) / STEPS
    reason, its, hist = k.end()
    for o in (k, xt, x, b, A, P):
        o.destroy()
    da.destroy()
    return dt * 1e3, float(hist[-1])


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [512]
    for n in sizes:
        for rep in range(int(os.environ.get("REPS", "3"))):
            for fc in [int(v) for v in os.environ.get("FC", "0,1").split(",")]:
                pb.tune_reset()
                pb.tune_set("force_comm", fc)
                ctx = pb.Context(0)
                pb.tune_reset()
                for sr in [int(v) for v in os.environ.get("SR", "0,1").split(",")]:
                    ms, rl = run(ctx, n, sr)
                    print(json.dumps({"n": n, "force_comm": fc, "sr": sr, "rep": rep,
                                      "ms_per_it": round(ms, 4), "rnorm_last": rl}), flush=True)
                ctx.destroy()


if __name__ == "__main__":
    main()
