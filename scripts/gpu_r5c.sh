#!/bin/bash
# decomposed-path tests (multi-rank over the host transport, the one-rank RCCL communicator), then
# the interleaved decomposed-vs-one-rank CG probe and its kernel trace
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_single_reduction.py tests/test_fortran.py -m gpu -x -q -k "multirank or rccl or split or fortran or force_comm" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/decomp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/decomp_tests.log
[ $rc -eq 0 ] || exit $rc
REPS=5 SR=0 timeout -k 10 300 python -u scripts/probe_decomposed_cg.py 512 > gpurun_out/decomp_cg3.jsonl 2> gpurun_out/decomp_cg3.err
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_decomp_trace.sh
