#!/bin/bash
# A/B of library variants (variants/<name>.so, scripts/build_variant.sh) on the default bench line,
# interleaved: usage  V="base pa2 pa3" bash scripts/gpu_ab_lib.sh
set -u
mkdir -p gpurun_out
: > gpurun_out/ab_lib.txt
for rep in 1 2; do
  for v in ${V:-base}; do
    if [ $v = base ]; then unset PB_LIB; else export PB_LIB=variants/$v.so; fi
    timeout -k 10 200 python bench.py --steps 40 --warmup 5 --secondary 0 --cpu-baseline none > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
    python scripts/show_grid.py $v gpurun_out/ab.json >> gpurun_out/ab_lib.txt
  done
done
cat gpurun_out/ab_lib.txt
