set -u
mkdir -p gpurun_out
for fc in 0 1; do
  timeout -k 10 300 python bench.py --workload compact-fft --tune force_comm=$fc --cpu-baseline none --steps 10 --warmup 2 > gpurun_out/cfft_fc$fc.json 2> gpurun_out/cfft_fc$fc.err || exit 1
done
python - <<'PY'
import json
for fc in (0, 1):
    d = json.loads(open(f"gpurun_out/cfft_fc{fc}.json").read().strip().splitlines()[-1])
    print(fc, round(d["ms_per_step"], 3), {k: (round(v["avg_ms"], 4), v["launches_per_solve"]) for k, v in d["kernels"].items()})
PY
