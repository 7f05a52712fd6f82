"""A/B tuning settings on the bench: runs `bench.py --no-cpu-baseline --tune CFG` once per (config, rep),
interleaved (rep-major) so box drift hits every config alike, and prints one JSON line per run with
ms/step and the per-kernel averages.

usage: python scripts/ab_env.py REPS 'name=val[,name=val]' ['...' ...] [-- extra bench args]
('-' = defaults; names as pb_tune_set takes them)"""
import json
import os
import subprocess
import sys

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = sys.argv[1:]
extra = []
if "--" in args:
    i = args.index("--")
    args, extra = args[:i], args[i + 1:]
reps, cfgs = int(args[0]), args[1:]
for rep in range(reps):
    for cfg in cfgs:
        env = dict(os.environ)
        tune = [] if cfg == "-" else ["--tune", cfg]
        p = subprocess.run([sys.executable, os.path.join(here, "bench.py"), "--no-cpu-baseline",
                            "--secondary", "0", "--steps", "100", "--warmup", "10"] + tune + extra,
                           env=env, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(json.dumps({"cfg": cfg, "rep": rep, "rc": p.returncode,
                              "err": p.stderr[-800:]}), flush=True)
            sys.exit(p.returncode)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        ks = {k: round(v["avg_ms"], 4) for k, v in d.get("kernels", {}).items()}
        print(json.dumps({"cfg": cfg, "rep": rep, "ms_per_step": round(d["ms_per_step"], 4),
                          "frac": round(d["roofline"]["frac"], 4), "kernels": ks,
                          "ksp": d.get("ksp_state", {}).get("reason")}), flush=True)
