"""Full KSPSolve to rtol 1e-10 (SURVEY.md §8d timing (iii)) with -pc_type jacobi | sor | mg | fft on one
GPU: iterations, wall time of the solve (inputs resident, HIP-synchronised), per-iteration time,
and the multigrid V-cycle time. One JSON line per (n, pc). The oracle's CPU solve is timed at 64^3
beside it (1 core).

usage: python scripts/bench_solve.py [n ...]   (default 256 512)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

SEED = 20231015


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [256, 512]
    ctx = pb.Context(0)
    for n in sizes:
        n3 = (n, n, n)
        h = (1.0 / n,) * 3
        op = os.environ.get("OP", "star7")
        if op == "compact":  # config 5 shape: compact A, 7-point P, periodic 2*pi box
            h = (2 * np.pi / n,) * 3
            da = pb.DA(ctx, n3, (2 * np.pi,) * 3)
            P = pb.Mat(da, pb.ASSEMBLED27, h)
            A = pb.Mat(da, pb.COMPACT, h)
            x, b = pb.Vec(da), pb.Vec(da)
        else:
            da = pb.DA(ctx, n3)
            P, A, x, b = pb.initialise_linear_system(da, h)
        xt = pb.Vec(da)
        xt.set_random(SEED)
        A.mult(xt, b)
        for pc in os.environ.get("PCS", "mg,sor,jacobi").split(","):
            if pc == "sor" and n > 256:
                continue
            opts = pb.ksp_options(["-pc_type", pc, "-ksp_rtol", "1e-10"])
            # fft: the PC inverts P's symbol, so config 5 takes P = A = the compact operator
            k = pb.KSP(A, A if pc == "fft" else P, opts)
            k.solve(b, x)  # warm-up (allocations, first-touch)
            ctx.sync()
            ctx.set_timing(True)
            ctx.reset_timing()
            t0 = time.perf_counter()
            reason, its, hist = k.solve(b, x)
            ctx.sync()
            dt = time.perf_counter() - t0
            # per-launch averages over the launches that ran: the host enqueues iterations ahead
            # of its lagged convergence poll, and the launches after convergence exit at entry
            # (pb_ctx::op_skip, a few us) -- they are told apart by their duration and left out;
            # each part is divided by its own count of launches that ran
            def ran(nm):
                s = ctx.timing_samples(nm)
                if not len(s):
                    return None
                keep = s[s > 0.1 * float(s.max())]
                return {"avg_ms": float(keep.mean()), "launches": int(len(keep)),
                        "skipped": int(len(s) - len(keep))}
            pc_t = ran("pc_fft" if pc == "fft" else "mg_apply")
            parts = {}
            for nm in ("mg_fine_smooth_first", "mg_fine_resid_restrict", "mg_fine_prolong_post",
                       "mg_coarse_levels", "cg_pass_a", "cg_pass_b", "cg_pass_b_even",
                       "cg_pass_b_odd", "cg_pass_b_x4", "compact_lapl_fast", "cg_gen_p",
                       "cg_gen_dot", "cg_pc_xr", "pc_fft_x", "pc_fft_y", "pc_fft_z"):
                t_ = ran(nm)
                if t_:
                    parts[nm] = t_
            ctx.set_timing(False)
            r = pb.Vec(da)
            A.mult(x, r)
            r.axpy(-1.0, b)
            out = {"n": n, "op": op, "pc": pc, "reason": int(reason), "its": int(its), "solve_ms": dt * 1e3,
                   "ms_per_it": dt * 1e3 / max(its, 1), "levels": k.pc_levels,
                   "rel_residual": r.norm() / b.norm(),
                   "pc_apply_ms": pc_t["avg_ms"] if pc_t else None,
                   "pc_applies": pc_t, "per_launch": parts}
            out["cfg"] = {}
            print(json.dumps(out), flush=True)
            r.destroy()
            k.destroy()
        for o in (P, A, x, b, xt):
            o.destroy()
        da.destroy()
    if os.environ.get("NO_CPU"):
        return
    # CPU restatement at 64^3 (1 core)
    from oracle import oracle as O
    n3 = (64, 64, 64)
    h = (1 / 64,) * 3
    bb = O.stencil(O.fill_random(64 ** 3, SEED), n3, h)
    for pc in ("mg", "jacobi"):
        t0 = time.perf_counter()
        _, reason, its, _ = O.cg_solve(bb, n3, h, rtol=1e-10, pc=pc)
        print(json.dumps({"n": 64, "pc": pc, "cpu_oracle_1core": True, "its": its,
                          "solve_ms": (time.perf_counter() - t0) * 1e3}), flush=True)


if __name__ == "__main__":
    main()
