"""V-cycle phase times on the decomposed code path (force_comm: one-rank RCCL communicator) vs one
rank, 512^3: where the decomposed MG loses time. usage: python scripts/probe_mg_decomposed.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

names = ("mg_apply", "mg_fine_smooth_first", "mg_fine_resid_restrict", "mg_fine_prolong_post",
         "mg_coarse_levels", "halo", "mg_presmooth_residual", "mg_sor_sweep2", "mg_sor",
         "mg_residual")
for fc in (0, 1):
    pb.tune_reset()
    pb.tune_set("force_comm", fc)
    ctx = pb.Context(0)
    pb.tune_reset()
    da = pb.DA(ctx, (512, 512, 512))
    P, A, x, b = pb.initialise_linear_system(da, da.spacing)
    k = pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg"]))
    r, z = pb.Vec(da), pb.Vec(da)
    r.set_random(3)
    for _ in range(2):
        k.pc_apply(r, z)
    ctx.sync()
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(5):
        k.pc_apply(r, z)
    ctx.sync()
    out = {"force_comm": fc}
    for nm in names:
        ms, cnt = ctx.timing(nm)
        out[nm] = [round(ms / 5, 4), cnt / 5]
    print(json.dumps(out), flush=True)
    ctx.set_timing(False)
    k.destroy()
    for o in (P, A, x, b, r, z):
        o.destroy()
    da.destroy()
    ctx.destroy()
