#!/bin/bash
# r03: spectral-PC parity subset + PC timing, then the solve records (bench_solve.py, launches
# that ran only, each part by its own count) for config 5 (compact A + fft) and the 7-point
# MG / Jacobi solves, and a kernel trace of the config-5 solve at 512^3.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/solve
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "fft" --timeout 300 --timeout-method thread > gpurun_out/solve/pytest_fft.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/solve/pytest_fft.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_fft.py 512 256 1024 > gpurun_out/solve/fft_pc_apply.jsonl 2> gpurun_out/solve/fft.err
rc=$?; echo "fft rc=$rc"; cat gpurun_out/solve/fft_pc_apply.jsonl; [ $rc -eq 0 ] || exit $rc
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 > gpurun_out/solve/solve_fft_compact.jsonl 2> gpurun_out/solve/s1.err
rc=$?; echo "cfg5 rc=$rc"; cat gpurun_out/solve/solve_fft_compact.jsonl; [ $rc -eq 0 ] || exit $rc
PCS=mg,jacobi NO_CPU=1 timeout -k 10 600 python scripts/bench_solve.py 256 512 > gpurun_out/solve/solve_star7.jsonl 2> gpurun_out/solve/s2.err
rc=$?; echo "star7 rc=$rc"; cat gpurun_out/solve/solve_star7.jsonl; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/solve/kt_cfg5 -o cfg5 --output-format csv \
  -- python3 $R/scripts/bench_solve.py 512 > $R/gpurun_out/solve/kt_cfg5.jsonl 2> $R/gpurun_out/solve/kt_cfg5.err
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
for cfg in "TAG=default" "PB_LINES_ABLATE=1" "PB_LINES_ABLATE=2" "PB_LINES_CFG=6" "PB_LINES_CFG=7"; do
  env $cfg timeout -k 10 120 python scripts/bench_compact.py 512 256 >> gpurun_out/solve/compact_ab.jsonl 2>> gpurun_out/solve/compact_ab.err
  rc=$?; echo "compact $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/solve/compact_ab.jsonl
