#!/bin/bash
# per-GPU slab shapes of the weak-scaling runs (N = 1, 4, 8), interleaved, one process each
set -u
mkdir -p gpurun_out
for g in 512,512,512 1024,1024,128 512,1024,256 1024,1024,128 512,512,512 1024,1024,128; do
  timeout -k 10 200 python bench.py --grid $g --steps 40 --warmup 5 --secondary 0 --cpu-baseline none > gpurun_out/grid.json 2> gpurun_out/grid.err || exit 1
  python scripts/show_grid.py $g gpurun_out/grid.json >> gpurun_out/grids.txt
done
cat gpurun_out/grids.txt
