#!/bin/bash
# spectral-PC / compact / MG / config-5 GPU tests, the PC apply per pass and the config-5 solves
set -u
mkdir -p gpurun_out/fftfinal
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread -k "compact or fft or mg or config5" > gpurun_out/fftfinal/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fftfinal/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/bench_fft.py 512 256 1024 > gpurun_out/fftfinal/fft.jsonl 2>> gpurun_out/fftfinal/err.log || exit $?
OP=compact PCS=fft NO_CPU=1 timeout -k 10 200 python scripts/bench_solve.py 512 256 > gpurun_out/fftfinal/solve.jsonl 2>> gpurun_out/fftfinal/err.log || exit $?
cut -c1-240 gpurun_out/fftfinal/fft.jsonl gpurun_out/fftfinal/solve.jsonl
