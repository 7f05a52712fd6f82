#!/bin/bash
# whole GPU tier, then the decomposed-vs-one-rank CG probe
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -8 gpurun_out/full_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_decomposed_cg.py 512 > gpurun_out/decomp_cg.jsonl 2> gpurun_out/decomp_cg.err
rc=$?; echo "probe rc=$rc"; tail -3 gpurun_out/decomp_cg.err
exit $rc
