#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/fft
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fft" > gpurun_out/fft/tests.log 2>&1
rc=$?; tail -2 gpurun_out/fft/tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/fft/tune.jsonl
for cfg in ${CFGS:-"X=16 Y=16 Z=8"}; do for bpc in ${BPCS:-0}; do
  set -- $cfg
  PB_FFT_BLOCKS_PER_CU=$bpc PB_FFT_TL_X=${1#X=} PB_FFT_TL_Y=${2#Y=} PB_FFT_TL_Z=${3#Z=} timeout -k 10 120 python scripts/bench_fft.py 512 256 >> gpurun_out/fft/tune.jsonl 2>> gpurun_out/fft/tune.err || exit $?
done; done
cat gpurun_out/fft/tune.jsonl
