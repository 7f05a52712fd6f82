#!/bin/bash
# CG pass A with 8-row tiles from 256^2 planes (default) vs from 512^2 (the matvec's threshold,
# PB_STENCIL_TALL_MIN_PLANE=262144): CG parity cases first, then 256^3 and 512^3 bench.py runs
# in alternating processes.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "cg" > gpurun_out/pt_tall.log 2>&1
rc=$?; echo "cg tests rc=$rc"; tail -2 gpurun_out/pt_tall.log; [ $rc -eq 0 ] || exit $rc
for base in 256 512; do
  for i in 1 2 3; do
    for m in 65536 262144; do
      PB_STENCIL_TALL_MIN_PLANE=$m timeout -k 10 200 python bench.py --base $base --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/b_t$m.json 2> gpurun_out/b_t$m.err
      rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/b_t$m.err; exit $rc; }
      python3 -c "import json; d=json.load(open('gpurun_out/b_t$m.json')); print('base $base tall_min $m', round(d['ms_per_step'],4), {k: round(v['avg_ms'],4) for k, v in d['kernels'].items()})"
    done
  done
done
