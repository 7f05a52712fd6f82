"""one line per bench JSON: grid, ms per iteration and the per-kernel averages"""
import json
import sys

r = json.load(open(sys.argv[2]))
k = r["kernels"]
print(sys.argv[1], round(r["ms_per_step"], 4), {n: round(v["avg_ms"], 4) for n, v in k.items()})
