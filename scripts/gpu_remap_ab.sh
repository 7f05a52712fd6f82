#!/bin/bash
# A/B of the XCD-aware tile order in the line-pass kernels (spectral PC passes, compact line
# passes): PB_FFT_REMAP / PB_LINES_REMAP = 1 (default) vs 0, interleaved, 3 reps
set -u
mkdir -p gpurun_out/remap
for rep in 0 1 2; do
  for v in 1 0; do
    PB_FFT_REMAP=$v PB_LINES_REMAP=$v timeout -k 10 120 python scripts/bench_fft.py 512 256 >> gpurun_out/remap/fft.jsonl 2>> gpurun_out/remap/err.log || exit $?
    PB_FFT_REMAP=$v PB_LINES_REMAP=$v timeout -k 10 120 python scripts/tune_compact.py 512 >> gpurun_out/remap/compact.jsonl 2>> gpurun_out/remap/err.log || exit $?
  done
done
