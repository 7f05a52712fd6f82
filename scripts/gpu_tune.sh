#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/tune_stencil.py > gpurun_out/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; [ $rc -eq 0 ] || tail -20 gpurun_out/tune.log; exit $rc
