#!/bin/bash
# r03 Stockham FFT engine: spectral-PC parity tests (incl. mixed radix), then PC-apply timing and a
# kernel trace at 256^3 / 512^3 / 1024^3.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/fftnew
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "fft" --timeout 300 --timeout-method thread > gpurun_out/fftnew/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/fftnew/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_fft.py 512 256 1024 > gpurun_out/fftnew/fft.jsonl 2> gpurun_out/fftnew/fft.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/fftnew/fft.jsonl; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fftnew/kt -o fft --output-format csv \
  -- python3 $R/scripts/bench_fft.py 512 256 > $R/gpurun_out/fftnew/kt.jsonl 2> $R/gpurun_out/fftnew/kt.err
rc=$?; echo "kt rc=$rc"; exit $rc
