import os, sys, time, json
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import poissbox_amd as pb
ctx = pb.Context(0)
da = pb.initialise_grid(ctx, (512, 512, 512))
P, A, x, b = pb.initialise_linear_system(da, da.spacing)
xt = pb.Vec(da); xt.set_random(1); A.mult(xt, b)
for timing in (False, True, False, True):
    k = pb.KSP(A, P, pb.ksp_options(["-ksp_type", "cg", "-pc_type", "jacobi"], rtol=0.0, atol=0.0, dtol=1e300, max_it=200, check_every=8))
    k.begin(b, x); k.iterate(10); ctx.sync()
    ctx.set_timing(timing); ctx.reset_timing()
    t0 = time.perf_counter(); k.iterate(100); ctx.sync(); t1 = time.perf_counter()
    ctx.set_timing(False)
    k.end(); k.destroy()
    print(json.dumps({"timing": timing, "ms_per_it": (t1 - t0) / 100 * 1e3}), flush=True)
