#!/bin/bash
# CG + Jacobi iteration time per DoF on one GPU for several slab shapes of 2^27 DoF (the weak-
# scaling per-GPU geometries: N = 8 gives each GPU 1024 x 1024 x 128).
set -u
mkdir -p gpurun_out
# CFGS: ';'-separated settings per run ('-' = none): env assignments (PB_LIB=variants/x.so) or
# --tune name=val,..., crossed with GRIDS
IFS=';' read -ra CS <<< "${CFGS:--}"
for c in "${CS[@]}"; do
[ "$c" = "-" ] && c=""
for g in ${GRIDS:-512,512,512 1024,1024,128 1024,512,256 512,1024,256 1024,1024,128 512,512,512}; do
  tv=""; ev=""
  case "$c" in --tune*) tv="$c";; *) ev="$c";; esac
  env $ev timeout -k 10 200 python bench.py $tv --grid $g --secondary 0 --steps 40 --warmup 5 --no-cpu-baseline --matvecs 10 --sustained 10 > gpurun_out/grid_$g.json 2>>gpurun_out/grid.err || exit 1
  python3 - "$g" "$c" <<'PY'
import json, sys
g = sys.argv[1]
d = json.loads(open(f"gpurun_out/grid_{g}.json").read().strip().split("\n")[-1])
k = d["kernels"]
print(g, sys.argv[2], round(d["ms_per_step"], 4), round(d["value"] / 1e9, 2),
      {n: round(v["avg_ms"], 4) for n, v in k.items() if isinstance(v, dict) and "avg_ms" in v}, flush=True)
PY
done
done
