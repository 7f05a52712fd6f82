#!/bin/bash
# engine change check: stencil / CG / MG parity tests, then A/B against variants/head.so at 512^3 and 256^3
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/eng
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/eng/tests.log 2>&1
rc=$?; tail -3 gpurun_out/eng/tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab.sh eng512 2 - PB_LIB=$R/variants/head.so ${EXTRA512:-} && bash scripts/gpu_ab.sh eng256 2 - PB_LIB=$R/variants/head.so ${EXTRA256:-} -- --base 256
