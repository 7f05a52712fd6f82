#!/bin/bash
# 1024^3 spectral PC: tile widths of the strided passes with the padded Z buffer
set -u
mkdir -p gpurun_out
rm -f gpurun_out/fft_tl1024.jsonl
for c in "" "PB_FFT_TL_LONG=8" "" "PB_FFT_TL_LONG=8"; do
  env $c timeout -k 10 200 python scripts/bench_fft.py 1024 >> gpurun_out/fft_tl1024.jsonl 2>>gpurun_out/fft_tl1024.err || exit 1
done
cut -c1-250 gpurun_out/fft_tl1024.jsonl
