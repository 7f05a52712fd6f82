#!/bin/bash
# quick bench line (no secondary workloads, no CPU baseline) -> gpurun_out/bench_quick.json
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --secondary 0 --cpu-baseline none ${BENCH_EXTRA:-} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_quick.err
exit $rc
