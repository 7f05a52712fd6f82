#!/bin/bash
# r03 line passes after making every tile load unconditional: parity subsets (fft, compact),
# spectral-PC and compact-Laplacian timing with A/B knobs
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/lines
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "fft or compact" --timeout 300 --timeout-method thread > gpurun_out/lines/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/lines/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "TAG=default" "PB_FFT_PF_STRIDED=0" "PB_FFT_PF_STRIDED=1" "PB_FFT_ABLATE=1" "TAG=default2"; do
  env $cfg timeout -k 10 120 python scripts/bench_fft.py 512 256 >> gpurun_out/lines/fft.jsonl 2>> gpurun_out/lines/fft.err
  rc=$?; echo "fft $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for cfg in "TAG=default" "PB_LINES_ABLATE=1" "PB_LINES_CFG=6" "PB_LINES_CFG=7" "PB_LINES_CFG=2" "TAG=default2"; do
  env $cfg timeout -k 10 120 python scripts/bench_compact.py 512 256 >> gpurun_out/lines/compact.jsonl 2>> gpurun_out/lines/compact.err
  rc=$?; echo "compact $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/lines/fft.jsonl gpurun_out/lines/compact.jsonl
