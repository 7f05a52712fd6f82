#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_single_reduction.py > gpurun_out/sr_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/sr_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u scripts/sr_probe.py 512 256 - cg_sr_fused=0 > gpurun_out/sr_probe.jsonl 2> gpurun_out/sr_probe.err
rc=$?; echo "probe rc=$rc"; tail -3 gpurun_out/sr_probe.err
exit $rc
