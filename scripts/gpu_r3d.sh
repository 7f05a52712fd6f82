#!/bin/bash
# r03 mid-round check: every GPU test, smoke, bench (gpu_check.sh), then config-5 solves and the
# PC apply with the resident-grid sums
set -u
R=$GRAFT_REPO_ROOT
cd $R && PYTEST_ARGS="--timeout 300 --timeout-method thread" bash scripts/gpu_check.sh || exit $?
O=$R/gpurun_out/r3d
mkdir -p $O
for i in 1 2; do
  OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 >> $O/solve_fft_compact.jsonl 2>> $O/s1.err
  rc=$?; echo "cfg5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python scripts/bench_fft.py 512 256 >> $O/fft.jsonl 2>> $O/fft.err
cat $O/solve_fft_compact.jsonl $O/fft.jsonl
