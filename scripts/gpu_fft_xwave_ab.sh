#!/bin/bash
# A/B: X pass with wave-private lines (default, tile loops unrolled 4), unrolled 2 / 8, and the
# block-wide tile (PB_FFT_X_WAVE=0, the previous form); 3 reps, PC apply at 512^3 / 256^3.
# Variants: scripts/build_variant.sh xwave_u2 -DPB_FFT_TILE_UNROLL=2 (u8: =8), xblock
# -DPB_FFT_X_WAVE=0 (built when the wave-private X pass applied to every line length)
set -u
mkdir -p gpurun_out/xwave
for rep in 0 1 2; do
  for lib in "" variants/xwave_u2.so variants/xwave_u8.so variants/xblock.so; do
    PB_LIB=$lib timeout -k 10 120 python scripts/bench_fft.py 512 256 | sed "s|^{|{\"lib\": \"${lib:-default}\", |" >> gpurun_out/xwave/fft.jsonl 2>> gpurun_out/xwave/err.log || exit $?
  done
done
