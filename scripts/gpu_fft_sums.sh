#!/bin/bash
# spectral-PC / compact / MG CG tests with CG's residual sums taken by the PC's last pass, then
# the config-5 solves with PB_FFT_SUMS = 1 / 0 (2 reps)
set -u
mkdir -p gpurun_out/fftsums
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread -k "compact or fft or mg or config5" > gpurun_out/fftsums/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fftsums/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 0 1; do
  for v in 1 0; do
    PB_FFT_SUMS=$v OP=compact PCS=fft NO_CPU=1 timeout -k 10 200 python scripts/bench_solve.py 512 256 | sed "s|^{|{\"PB_FFT_SUMS\": $v, |" >> gpurun_out/fftsums/solve.jsonl 2>> gpurun_out/fftsums/err.log || exit $?
  done
done
cut -c1-200 gpurun_out/fftsums/solve.jsonl
