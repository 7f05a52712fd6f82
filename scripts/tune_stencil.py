"""Sweep the stencil launch knobs (PB_STENCIL_TY, PB_STENCIL_BLOCKS) at 512^3 on one GPU:
matvec and CG pass A/B average kernel times (HIP events), interleaved in one process."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

n = tuple(int(v) for v in os.environ.get("PB_TUNE_N", "512,512,512").split(","))
ctx = pb.Context(0)
da = pb.DA(ctx, n)
P, A, x, b = pb.initialise_linear_system(da, da.spacing)
xt = pb.Vec(da)
xt.set_random(1)
A.mult(xt, b)
y = pb.Vec(da)
N = da.nlocal
tys = [int(v) for v in os.environ.get("PB_TUNE_TY", "1,2,4").split(",")]
blocks = [int(v) for v in os.environ.get("PB_TUNE_BLOCKS", "512,1024,2048,4096,8192").split(",")]
res = []
for rnd in range(2):
    for ty in tys:
        for nb in blocks:
            os.environ["PB_STENCIL_TY"] = str(ty)
            os.environ["PB_STENCIL_BLOCKS"] = str(nb)
            for _ in range(2):
                A.mult(xt, y)
            ctx.sync()
            ctx.set_timing(True)
            ctx.reset_timing()
            for _ in range(10):
                A.mult(xt, y)
            opts = pb.ksp_options(rtol=0.0, atol=0.0, dtol=1e300, max_it=40)
            k = pb.KSP(A, P, opts)
            k.begin(b, x)
            k.iterate(12)
            ctx.sync()
            mv = ctx.timing("stencil")
            pa = ctx.timing("cg_pass_a")
            pbb = ctx.timing("cg_pass_b")
            ctx.set_timing(False)
            k.end()
            k.destroy()
            t_mv, t_a, t_b = mv[0] / mv[1], pa[0] / pa[1], pbb[0] / pbb[1]
            row = dict(round=rnd, ty=ty, blocks=nb, mv_ms=t_mv, mv_GBps=16 * N / t_mv / 1e6,
                       a_ms=t_a, a_GBps=24 * N / t_a / 1e6, b_ms=t_b, b_GBps=40 * N / t_b / 1e6)
            res.append(row)
            print(json.dumps(row), flush=True)
