set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_nonfinite.py tests/test_gpu_single_reduction.py tests/test_gpu_parity.py tests/test_abi.py -k "nonfinite or nan or reference_fixtures or self_block or single_reduction or folded or stencil_bit_exact or abi or rccl" -q -rf --timeout 180 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/t1.log
[ $rc -le 1 ] || exit $rc
SR_REPS=2 timeout -k 10 300 python scripts/sr_probe.py 512 256 > gpurun_out/sr_probe1.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/sr_probe1.jsonl | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/placement_probe.py 512 3 4 20 > gpurun_out/placement1.jsonl 2>&1
rc=$?; echo "placement rc=$rc"; tail -1 gpurun_out/placement1.jsonl
exit $rc
