#!/bin/bash
# r04 closing set, part A (one box): every GPU test, smoke, bench (with its secondaries and the CPU
# baseline), rocprofv3 kernel stats of the headline bench and of the config-5 workload, PMC passes
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/close4
mkdir -p $O
cd $R && PYTEST_ARGS="--timeout 400 --timeout-method thread" BENCH_ARGS="--steps 50 --warmup 5" bash scripts/gpu_check.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench.json gpurun_out/bench.err $O/
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --secondary 0 > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_cfft -o cfft --output-format csv -- python3 $R/bench.py --workload compact-fft --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_cfft_prof.json 2> $O/bench_cfft_prof.err
rc=$?; echo "rocprof cfft rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && bash scripts/gpu_pmc.sh || exit $?
mv gpurun_out/pmc_* $O/ 2>/dev/null
exit 0
