#!/bin/bash
# compact Laplacian 3-pass: parity subset + per-pass timing and ablations
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/cab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "compact" --timeout 300 --timeout-method thread > gpurun_out/cab/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/cab/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "TAG=default" "PB_LINES_ABLATE=1" "PB_LINES_ABLATE=2" "PB_LINES_CFG=6" "PB_LINES_CFG=7" "TAG=default2"; do
  env $cfg timeout -k 10 120 python scripts/bench_compact.py 512 256 >> gpurun_out/cab/ab.jsonl 2>> gpurun_out/cab/ab.err
  rc=$?; echo "compact $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/cab/ab.jsonl
