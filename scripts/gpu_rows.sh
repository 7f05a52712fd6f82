#!/bin/bash
# Parity tests of the line solvers / compact operators, then the per-row measurements.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "tdma or compact or pcr" > gpurun_out/pt_rows.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_rows.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/bench_rows.py > gpurun_out/rows.jsonl 2> gpurun_out/rows.err
rc=$?; echo "rows rc=$rc"; tail -3 gpurun_out/rows.err; cat gpurun_out/rows.jsonl; exit $rc
