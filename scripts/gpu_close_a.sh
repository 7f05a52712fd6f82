#!/bin/bash
# r03 closing profile set on one box: every GPU test, smoke, bench (gpu_check.sh); rocprofv3
# kernel-trace stats of the bench; PMC passes of the bench (gpu_pmc.sh) and of the spectral PC;
# (part a of gpu_close.sh: tests, smoke, bench, rocprof, PMC). Stops at the first failure.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/close
mkdir -p $O
cd $R && PYTEST_ARGS="--timeout 300 --timeout-method thread" bash scripts/gpu_check.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && bash scripts/gpu_pmc.sh || exit $?
cd /tmp
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/fftpmc_$grp -o pmc --output-format csv -- python3 $R/scripts/bench_fft.py 512 > $O/fftpmc_$grp.jsonl 2> $O/fftpmc_$grp.err
  rc=$?; echo "fft pmc $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
