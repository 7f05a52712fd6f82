set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_single_reduction.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/t5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t5.log
[ $rc -le 1 ] || exit $rc
SR_REPS=3 timeout -k 10 600 python scripts/sr_probe.py 512 256 sr_ddiff=0 sr_ddiff=1 > gpurun_out/sr_ddiff_ab.jsonl 2>&1
rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/sr_ddiff_ab.jsonl"):
    r = json.loads(l)
    print(r["n"], r["tune"], r["ms_per_it"], r["passes_ms"])
PY
exit $rc
