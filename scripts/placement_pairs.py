"""Placement probe, all ordered pairs: K fresh 512^3 vectors v_0 .. v_{K-1}
(each filled by set_random), then the 7-point matvec v_i -> v_j for every i != j (median of
`reps` HIP-event-timed launches) and the flat copy v_i -> v_j over the same buffers. A slow
output buffer shows as a slow column, a slow input as a slow row. One JSON line per pair, then a
matrix summary. Usage: python scripts/placement_pairs.py [n] [K] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    ctx = pb.Context(0)
    da = pb.initialise_grid(ctx, (n, n, n))
    A = pb.Mat(da, pb.STAR7, da.spacing)
    vs = []
    for s in range(K):
        v = pb.Vec(da)
        v.set_random(1000 + s)
        vs.append(v)
    ptr = [v.device_ptr()[0] for v in vs]
    M = [[None] * K for _ in range(K)]
    C = [[None] * K for _ in range(K)]
    for i in range(K):
        for j in range(K):
            if i == j:
                continue
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
            _, cm = vs[i].copy_probe(vs[j], reps=4)
            M[i][j] = round(smp[len(smp) // 2], 4)
            C[i][j] = round(cm / 8000.0, 3)
            print(json.dumps({"i": i, "j": j, "mv_med_ms": M[i][j], "mv_min_ms": round(smp[0], 4),
                              "copy_med_frac": C[i][j]}), flush=True)
            vs[j].set_random(1000 + j)  # restore the overwritten input
    print(json.dumps({"summary": True, "ptr": [hex(p) for p in ptr], "matvec_ms": M,
                      "copy_frac": C}), flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
