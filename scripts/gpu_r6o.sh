set -u
mkdir -p gpurun_out
: > gpurun_out/xdot_ab.txt
for rep in 1 2; do
for fc in 0 1; do
for xd in 16 64 0; do
  timeout -k 10 300 python bench.py --workload compact-fft --tune force_comm=$fc,x_dot_cu=$xd --cpu-baseline none --steps 10 --warmup 2 > gpurun_out/xd.json 2> gpurun_out/xd.err || exit 1
  python - $fc $xd >> gpurun_out/xdot_ab.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/xd.json").read().strip().splitlines()[-1])
print("fc", sys.argv[1], "x_dot_cu", sys.argv[2], round(d["ms_per_step"], 3), d["ksp_state"]["reason"], "x", round(d["kernels"]["compact_lines_x"]["avg_ms"], 4), "pcx", round(d["kernels"]["pc_fft_x"]["avg_ms"], 4))
PY
done; done; done
cat gpurun_out/xdot_ab.txt
