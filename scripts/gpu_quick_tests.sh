#!/bin/bash
# quick GPU run of a -k selection of the parity tests (K overrides the selection)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -k "${K:-rccl_compact_cg_fused or compact_reference_order or compact_cg_fused}" -q -rf --timeout 300 --timeout-method thread > gpurun_out/t6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t6.log; exit $rc
