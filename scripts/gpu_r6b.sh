set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nonfinite.py -q -rf --timeout 180 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t2.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/placement_probe.py 512 3 4 20 > gpurun_out/placement1.jsonl 2>&1
rc=$?; echo "placement rc=$rc"; cut -c1-250 gpurun_out/placement1.jsonl
exit $rc
