#!/bin/bash
# CG-path GPU tests (parity vs the oracle + fold/unfold identity), then the 512^3 and 256^3 bench
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/cg
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cg or fold or history or solve" > gpurun_out/cg/tests.log 2>&1
rc=$?; tail -5 gpurun_out/cg/tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab.sh fold 2 - PB_CG_FOLD=0 && bash scripts/gpu_ab.sh fold256 2 - PB_CG_FOLD=0 PB_STENCIL_KCMIN=16 -- --base 256
