#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_single_reduction.py tests/test_gpu_faults.py tests/test_fortran.py -k "single_reduction or stalled or shm_options or three_ranks" > gpurun_out/sr2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/sr2_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u scripts/sr_probe.py 512 256 sr_s_shape=0/1/2/3/4/5 > gpurun_out/sr2_probe.jsonl 2> gpurun_out/sr2_probe.err
rc=$?; echo "probe rc=$rc"; tail -3 gpurun_out/sr2_probe.err
exit $rc
