#!/bin/bash
# compact-operator / spectral-PC / MG CG tests after the lazy initial-state setup, then the
# config-5 512^3 solve with PB_KSP_LAZY0 = 1 / 0
set -u
mkdir -p gpurun_out/lazy0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread -k "compact or fft or mg or config5" > gpurun_out/lazy0/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/lazy0/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 0 1; do
  for v in 1 0; do
    PB_KSP_LAZY0=$v OP=compact PCS=fft NO_CPU=1 timeout -k 10 200 python scripts/bench_solve.py 512 256 >> gpurun_out/lazy0/solve.jsonl 2>> gpurun_out/lazy0/err.log || exit $?
  done
done
cut -c1-200 gpurun_out/lazy0/solve.jsonl
