#!/bin/bash
# spectral PC: parity tests, then config-5 solves (compact A = P + fft) and 7-point fft / mg solves
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/fft
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fft" > gpurun_out/fft/tests.log 2>&1
rc=$?; tail -5 gpurun_out/fft/tests.log; [ $rc -ne 0 ] && exit $rc
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 > gpurun_out/fft/solve_compact.jsonl 2> gpurun_out/fft/solve_compact.err
rc=$?; echo "compact rc=$rc"; cat gpurun_out/fft/solve_compact.jsonl; [ $rc -ne 0 ] && exit $rc
PCS=fft,mg NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 > gpurun_out/fft/solve_star.jsonl 2> gpurun_out/fft/solve_star.err
rc=$?; echo "star rc=$rc"; cat gpurun_out/fft/solve_star.jsonl; exit $rc
