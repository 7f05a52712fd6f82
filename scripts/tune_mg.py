"""A/B the V-cycle kernel knobs at 512^3 on one GPU: PC applies (-pc_type mg) with per-phase
HIP-event timing, interleaved rounds in ONE process.

PB_TUNE_CONFIGS: JSON list of tuning dicts (pb_tune_set names, e.g. {"mg_sweep2": 0}). Prints one JSON line per config (median over rounds).
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

n = tuple(int(v) for v in os.environ.get("PB_TUNE_N", "512,512,512").split(","))
rounds = int(os.environ.get("PB_TUNE_ROUNDS", "4"))
configs = json.loads(os.environ.get("PB_TUNE_CONFIGS", "[{}]"))
names = ("mg_apply", "mg_sor_sweep2", "mg_sor", "mg_residual", "mg_fine_smooth_first",
         "mg_fine_resid_restrict", "mg_fine_prolong_post", "mg_coarse_levels")
ctx = pb.Context(0)
da = pb.DA(ctx, n)
P, A, x, b = pb.initialise_linear_system(da, da.spacing)
k = pb.KSP(A, P, pb.ksp_options(["-pc_type", "mg"]))
r, z = pb.Vec(da), pb.Vec(da)
r.set_random(3)
acc = {i: {nm: [] for nm in names} for i in range(len(configs))}
for rnd in range(rounds):
    for i, cfg in enumerate(configs):
        pb.tune_reset()
        for key, v in cfg.items():  # tuning table (pb_tune_set), not the environment
            pb.tune_set(key[3:].lower() if key.startswith("PB_") else key, int(v))
        k.pc_apply(r, z)
        ctx.sync()
        ctx.set_timing(True)
        ctx.reset_timing()
        for _ in range(5):
            k.pc_apply(r, z)
        ctx.sync()
        for nm in names:
            ms, cnt = ctx.timing(nm)
            acc[i][nm].append(ms / 5 if cnt else 0.0)
        ctx.set_timing(False)
for i, cfg in enumerate(configs):
    print(json.dumps({"cfg": cfg, **{nm: round(statistics.median(v), 4) for nm, v in acc[i].items()}}),
          flush=True)
