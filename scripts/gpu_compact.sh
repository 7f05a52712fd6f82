#!/bin/bash
# compact-path GPU check: parity tests for the compact kernels, then the per-row bench
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "compact or tdma or pcr" > gpurun_out/compact_tests.log 2>&1
rc=$?; tail -5 gpurun_out/compact_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python scripts/bench_rows.py ${ROWS:-} > gpurun_out/rows.jsonl 2> gpurun_out/rows.err
rc=$?; echo "rows rc=$rc"; tail -3 gpurun_out/rows.err; exit $rc
