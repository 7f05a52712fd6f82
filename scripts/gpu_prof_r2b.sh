#!/bin/bash
# rocprofv3 kernel-trace stats of the bench + the PMC passes (traffic) -> gpurun_out/r2b/
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2b
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "pstore" > gpurun_out/r2b/pstore_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r2b/pstore_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2b/prof -o bench --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r2b/bench_prof.json 2> $R/gpurun_out/r2b/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && bash scripts/gpu_pmc.sh
