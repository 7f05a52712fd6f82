#!/bin/bash
# single-reduction CG: GPU tests + existing CG tests + the per-iteration probe
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_single_reduction.py tests/test_gpu_parity.py tests/test_gpu_faults.py tests/test_fortran.py -k "single_reduction or test_cg_ or multirank_cg or stalled or shm_options or three_ranks" > gpurun_out/sr1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/sr1_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/sr_probe.py 512 256 > gpurun_out/sr1_probe.jsonl 2> gpurun_out/sr1_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/sr1_probe.jsonl; tail -3 gpurun_out/sr1_probe.err
exit $rc
