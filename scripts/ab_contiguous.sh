#!/bin/bash
# A/B of PB_ALLOC_CONTIGUOUS (physically contiguous field allocations) in separate bench
# processes, alternating, to see whether the bimodal x-update pass follows the
# allocation. Prints ms/iteration and the per-kernel averages of every run.
set -u
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  for c in 0 1; do
    PB_ALLOC_CONTIGUOUS=$c timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/b_c$c.json 2> gpurun_out/b_c$c.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/b_c$c.err; exit $rc; }
    python3 -c "import json; d=json.load(open('gpurun_out/b_c$c.json')); print('contiguous=$c', round(d['ms_per_step'],4), {k: round(v['avg_ms'],4) for k, v in d['kernels'].items()})"
  done
done
