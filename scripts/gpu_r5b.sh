#!/bin/bash
# the NaN-in-LDS regression test against a build without the LDS zeroing (expected to fail), then
# the default build: the single-reduction file, then the whole GPU tier and the decomposed probe
set -u
mkdir -p gpurun_out
PB_LIB=variants/nozero.so timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -p no:cacheprovider tests/test_gpu_single_reduction.py -k nan_in_lds > gpurun_out/nozero.log 2>&1
echo "nozero variant rc=$? (1 expected)"; tail -2 gpurun_out/nozero.log
bash scripts/gpu_r5a.sh
