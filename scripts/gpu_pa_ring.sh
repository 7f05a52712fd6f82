#!/bin/bash
# ring-buffered pass A (pb_cg_pa.hip): parity tests, then the default bench line A/B against the
# engine's pass A (tuning cg_pa_ring=0), interleaved
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "ring_pass_a or folded_finalize or deferred_x_update or cg_matches or split_iterate or wide_planes or pc_none or indefinite" > gpurun_out/pa_tests.log 2>&1 || { tail -40 gpurun_out/pa_tests.log; exit 1; }
tail -3 gpurun_out/pa_tests.log
: > gpurun_out/pa_ab.txt
for rep in 1 2 3; do
  for ring in 1 0; do
    timeout -k 10 200 python bench.py --steps 40 --warmup 5 --secondary 0 --cpu-baseline none --tune cg_pa_ring=$ring > gpurun_out/pa_ab.json 2> gpurun_out/pa_ab.err || exit 1
    python scripts/show_grid.py ring$ring gpurun_out/pa_ab.json >> gpurun_out/pa_ab.txt
  done
done
cat gpurun_out/pa_ab.txt
