#!/bin/bash
# A/B: spectral PC with the twiddles held in registers (default build) vs read from the table
# where used (variants/twlazy.so, PB_FFT_TW_LAZY=1), Z-pass tiles of 8 and 16 lines; 3 reps.
# Variant: scripts/build_variant.sh twlazy -DPB_FFT_TW_LAZY=1 (with -DPB_FFT_SCALE_LDS=0 for the
# Z pass as it was then)
set -u
mkdir -p gpurun_out/fftlazy
for rep in 0 1 2; do
  for lib in "" variants/twlazy.so; do
    for tl in 8 16; do
      PB_LIB=$lib PB_FFT_TL_Z=$tl timeout -k 10 120 python scripts/bench_fft.py 512 256 | sed "s|^{|{\"lib\": \"${lib:-default}\", |" >> gpurun_out/fftlazy/fft.jsonl 2>> gpurun_out/fftlazy/err.log || exit $?
    done
  done
done
cut -c1-260 gpurun_out/fftlazy/fft.jsonl
