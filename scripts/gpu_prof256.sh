#!/bin/bash
# 256^3 CG iteration: bench line + rocprofv3 kernel trace (per-kernel durations and the gaps
# between launches inside an iteration)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/p256
cd $R && timeout -k 10 300 python bench.py --base 256 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/p256/bench.json 2> gpurun_out/p256/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/p256/bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p256/prof -o p256 --output-format csv -- python3 $R/bench.py --base 256 --steps 200 --warmup 20 --no-cpu-baseline > $R/gpurun_out/p256/bench_prof.json 2> $R/gpurun_out/p256/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
