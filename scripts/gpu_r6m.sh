set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "compact_cg_fused or multirank_cg_compact or config5 or rccl or multirank_compact" -q -rf --timeout 400 --timeout-method thread > gpurun_out/t3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t3.log
[ $rc -le 1 ] || exit $rc
for fc in 0 1; do
  timeout -k 10 300 python bench.py --workload compact-fft --tune force_comm=$fc --cpu-baseline none --steps 10 --warmup 2 > gpurun_out/cfft2_fc$fc.json 2> gpurun_out/cfft2_fc$fc.err || exit 1
done
python - <<'PY'
import json
for fc in (0, 1):
    d = json.loads(open(f"gpurun_out/cfft2_fc{fc}.json").read().strip().splitlines()[-1])
    print(fc, round(d["ms_per_step"], 3), d["ksp_state"]["reason"], {k: (round(v["avg_ms"], 4), v["launches_per_solve"]) for k, v in d["kernels"].items()})
PY
