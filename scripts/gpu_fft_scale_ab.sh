#!/bin/bash
# A/B: Z-pass scaling as an LDS step (default) vs in the transform's registers (variants/scalereg.so),
# and with the twiddles held in registers (variants/nolazy.so); 3 reps, PC apply at 512^3 / 256^3.
# Variants (at the time the default read the Z pass's twiddles from the table; registers are now
# the default): scripts/build_variant.sh scalereg -DPB_FFT_SCALE_LDS=0 -DPB_FFT_TW_LAZY=1,
# scripts/build_variant.sh nolazy -DPB_FFT_TW_LAZY=0
set -u
mkdir -p gpurun_out/fftscale
for rep in 0 1 2; do
  for lib in "" variants/scalereg.so variants/nolazy.so; do
    PB_LIB=$lib timeout -k 10 120 python scripts/bench_fft.py 512 256 | sed "s|^{|{\"lib\": \"${lib:-default}\", |" >> gpurun_out/fftscale/fft.jsonl 2>> gpurun_out/fftscale/err.log || exit $?
  done
done
cut -c1-240 gpurun_out/fftscale/fft.jsonl
