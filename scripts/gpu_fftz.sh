#!/bin/bash
# spectral-PC tests, then the Z pass A/B (register middle vs all-LDS build variants/zlds.so)
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "fft" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fft_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/fft_tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base zlds; do
    if [ $v = base ]; then unset PB_LIB; else export PB_LIB=variants/$v.so; fi
    timeout -k 10 120 python -u scripts/bench_fft.py 512 1024 | sed "s/^/$v /" >> gpurun_out/fftz_ab.txt || exit 1
  done
done
