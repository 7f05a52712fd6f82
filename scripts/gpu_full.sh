#!/bin/bash
# whole GPU tier, then the single-reduction probe (A/B of the one-pass kernel's shapes)
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -8 gpurun_out/full_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u scripts/sr_probe.py 512 256 ${SR_AB:-- cg_sr_fused=0} > gpurun_out/sr_probe.jsonl 2> gpurun_out/sr_probe.err
rc=$?; echo "probe rc=$rc"; tail -3 gpurun_out/sr_probe.err
exit $rc
