#!/bin/bash
# Spectral PC line-pass tile widths at 512^3 and 256^3 (PB_FFT_TL_X / _Y / _Z): the Z pass's row
# pieces are TL * 8 bytes (zpass_probe: 64-B pieces cap the pattern at ~2.6 TB/s, 128-B at ~4.9).
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fft_tl
for z in 8 16 32; do
  for xy in 16 32; do
    PB_FFT_TL_Z=$z PB_FFT_TL_X=$xy PB_FFT_TL_Y=$xy timeout -k 10 120 python scripts/bench_fft.py 512 256 >> gpurun_out/fft_tl/tl.jsonl 2>> gpurun_out/fft_tl/tl.err
    rc=$?; echo "z=$z xy=$xy rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
cat gpurun_out/fft_tl/tl.jsonl
