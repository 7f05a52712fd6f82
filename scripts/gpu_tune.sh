#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python scripts/tune_stencil.py > gpurun_out/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/tune.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2>$GRAFT_REPO_ROOT/gpurun_out/bench_prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
