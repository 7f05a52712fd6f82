#!/bin/bash
# MG change check: PC / MG parity tests, then MG solves at 512^3 (V-cycle part timers), product vs head
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/mg
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mg or sor or pc" > gpurun_out/mg/tests.log 2>&1
rc=$?; tail -3 gpurun_out/mg/tests.log; [ $rc -ne 0 ] && exit $rc
for lib in "" "$R/variants/head.so"; do
  PB_LIB=$lib PCS=mg NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 512 >> gpurun_out/mg/solve.jsonl 2>> gpurun_out/mg/solve.err || exit $?
done
cat gpurun_out/mg/solve.jsonl
