#!/bin/bash
# r05 closing set on one box: every GPU test, smoke, the default bench (no flags), rocprofv3
# kernel stats of the bench, PMC traffic passes, MG / config-5 solves, the SR probe. Stops at the
# first crash-class failure.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/close5
mkdir -p $O
cd $R && PYTEST_ARGS="--timeout 300 --timeout-method thread" BENCH_ARGS=" " T_BENCH=900 bash scripts/gpu_check.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench.json gpurun_out/bench.err $O/
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --cpu-baseline none --secondary 0 > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 10 --warmup 2 --cpu-baseline none --secondary 0"
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 300 rocprofv3 --pmc $grp -d $O/pmc_$grp -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $O/pmc_$grp.json 2> $O/pmc_$grp.err
  rc=$?; echo "pmc $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $R
PCS=mg,jacobi NO_CPU=1 timeout -k 10 600 python scripts/bench_solve.py 256 512 > $O/solve_star7.jsonl 2> $O/solve.err
rc=$?; echo "solve rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/sr_probe.py 512 256 > $O/sr_probe.jsonl 2> $O/sr_probe.err
rc=$?; echo "sr probe rc=$rc"; exit $rc
