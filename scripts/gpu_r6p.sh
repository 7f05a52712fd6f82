set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_single_reduction.py tests/test_gpu_nonfinite.py tests/test_gpu_parity.py -k "single_reduction or nonfinite or nan or rccl" -q -rf --timeout 300 --timeout-method thread > gpurun_out/t4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t4.log
[ $rc -le 1 ] || exit $rc
VAR=srold bash scripts/gpu_sr_ab.sh > gpurun_out/sr_ab_ddiff.txt 2>&1
rc=$?; tail -14 gpurun_out/sr_ab_ddiff.txt
exit $rc
