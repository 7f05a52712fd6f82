#!/bin/bash
# Config 5 (compact A, spectral PC, 512^3 solves): one rank against the decomposed code paths on a
# one-rank RCCL communicator (force_comm), per-kernel averages; then the compact X pass's fused
# p.w grid (x_dot_cu). Outputs in gpurun_out/.
set -u
mkdir -p gpurun_out
: > gpurun_out/config5_ab.txt
for xd in 16 0; do
for fc in 0 1; do
  timeout -k 10 300 python bench.py --workload compact-fft --tune force_comm=$fc,x_dot_cu=$xd --cpu-baseline none --steps 10 --warmup 2 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
  python - $fc $xd >> gpurun_out/config5_ab.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/c5.json").read().strip().splitlines()[-1])
print("force_comm", sys.argv[1], "x_dot_cu", sys.argv[2], round(d["ms_per_step"], 3), d["ksp_state"]["reason"],
      {k: (round(v["avg_ms"], 4), v["launches_per_solve"]) for k, v in d["kernels"].items()})
PY
done; done
cat gpurun_out/config5_ab.txt
