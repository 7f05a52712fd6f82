#!/bin/bash
# ring pass A variants (variants/*.so) against the engine's pass A (cg_pa_ring=0), interleaved
set -u
mkdir -p gpurun_out
: > gpurun_out/pa_ab.txt
for rep in 1 2; do
  for v in ${V:-base}; do
    if [ $v = base ]; then unset PB_LIB; else export PB_LIB=variants/$v.so; fi
    for ring in 1 0; do
      [ $ring = 0 ] && [ $v != base ] && continue
      timeout -k 10 200 python bench.py --steps 40 --warmup 5 --secondary 0 --cpu-baseline none --tune cg_pa_ring=$ring > gpurun_out/pa_ab.json 2> gpurun_out/pa_ab.err || exit 1
      python scripts/show_grid.py $v.ring$ring gpurun_out/pa_ab.json >> gpurun_out/pa_ab.txt
    done
  done
done
cat gpurun_out/pa_ab.txt
