"""A/B the stencil launch knobs at 512^3 on one GPU, interleaved rounds in ONE process.

PB_TUNE_CONFIGS: JSON list of tuning dicts (pb_tune_set names, e.g. [{"stencil_ty": 4, "xcd_remap": 0}, ...]).
Per config and round: 20 matvecs + 16 CG iterations with HIP-event kernel timing.
Prints one JSON line per config with min/median over rounds.
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

n = tuple(int(v) for v in os.environ.get("PB_TUNE_N", "512,512,512").split(","))
rounds = int(os.environ.get("PB_TUNE_ROUNDS", "4"))
configs = json.loads(os.environ.get("PB_TUNE_CONFIGS", "[{}]"))
ctx = pb.Context(0)
da = pb.DA(ctx, n)
P, A, x, b = pb.initialise_linear_system(da, da.spacing)
xt = pb.Vec(da)
xt.set_random(1)
A.mult(xt, b)
y = pb.Vec(da)
N = da.nlocal
acc = {i: {"mv": [], "a": [], "b": [], "be": [], "it": []} for i in range(len(configs))}
for rnd in range(rounds):
    for i, cfg in enumerate(configs):
        pb.tune_reset()
        for key, v in cfg.items():  # tuning table (pb_tune_set), not the environment
            pb.tune_set(key[3:].lower() if key.startswith("PB_") else key, int(v))
        for _ in range(3):
            A.mult(xt, y)
        ctx.sync()
        ctx.set_timing(True)
        ctx.reset_timing()
        for _ in range(20):
            A.mult(xt, y)
        k = pb.KSP(A, P, pb.ksp_options(rtol=0.0, atol=0.0, dtol=1e300, max_it=80))
        k.begin(b, x)
        k.iterate(4)
        ctx.sync()
        t0 = time.perf_counter()
        k.iterate(32)
        ctx.sync()
        it_ms = (time.perf_counter() - t0) / 32 * 1e3
        mv, pa = ctx.timing("stencil"), ctx.timing("cg_pass_a")
        # the pass B that applies the deferred x update (PB_CG_DEFER_X = 4 / 2 / 0)
        pbb = ctx.timing("cg_pass_b_x4")
        if pbb[1] == 0:
            pbb = ctx.timing("cg_pass_b_odd")
        if pbb[1] == 0:
            pbb = ctx.timing("cg_pass_b")
        pbe = ctx.timing("cg_pass_b_even")
        ctx.set_timing(False)
        k.end()
        k.destroy()
        acc[i]["mv"].append(mv[0] / mv[1])
        acc[i]["a"].append(pa[0] / pa[1])
        acc[i]["b"].append(pbb[0] / pbb[1])
        acc[i]["be"].append(pbe[0] / pbe[1] if pbe[1] else 0.0)
        acc[i]["it"].append(it_ms)
for i, cfg in enumerate(configs):
    out = {"cfg": cfg}
    dfx = int(cfg.get("cg_defer_x", cfg.get("PB_CG_DEFER_X", 4)))
    bx, it_b = {0: (40, 64), 2: (48, 60)}.get(dfx, (64, 58))
    for key, nbytes in (("mv", 16), ("a", 24), ("b", bx), ("be", 24), ("it", it_b)):
        v = acc[i][key]
        out[key + "_min_ms"] = min(v)
        out[key + "_med_ms"] = statistics.median(v)
        out[key + "_GBps_med"] = nbytes * N / max(statistics.median(v), 1e-9) / 1e6
    print(json.dumps(out), flush=True)
