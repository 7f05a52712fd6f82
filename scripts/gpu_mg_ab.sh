#!/bin/bash
# MG V-cycle A/B of a variant build (variants/$VAR.so) against the default: the MG tests on the
# default build first, then scripts/tune_mg.py at 512^3 per build, alternating processes
set -u
mkdir -p gpurun_out
VAR=${VAR:-mgold}
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests \
  -m gpu -k "mg or sor or multigrid or fullsize" > gpurun_out/mg_ab_tests.log 2>&1 || { tail -30 gpurun_out/mg_ab_tests.log; exit 1; }
tail -2 gpurun_out/mg_ab_tests.log
: > gpurun_out/mg_ab.jsonl
for rep in 1 2 3; do
  for v in base $VAR; do
    if [ $v = base ]; then unset PB_LIB; else export PB_LIB=variants/$v.so; fi
    PB_TUNE_ROUNDS=3 timeout -k 10 200 python scripts/tune_mg.py | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/mg_ab.jsonl || exit 1
  done
done
cat gpurun_out/mg_ab.jsonl
