#!/bin/bash
# spectral PC: parity subset, then A/B of persistent+prefetch on the strided passes and staggered
# co-resident blocks
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fftab4
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "fft" --timeout 300 --timeout-method thread > gpurun_out/fftab4/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fftab4/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { echo "== $*"; env "$@" timeout -k 10 120 python scripts/bench_fft.py 512 256 >> gpurun_out/fftab4/ab.jsonl 2>> gpurun_out/fftab4/ab.err; }
run TAG=default || exit $?
run PB_FFT_PF_STRIDED=0 || exit $?
run PB_FFT_TL_Z=32 || exit $?
run PB_FFT_TL_Z=32 PB_FFT_PF_STRIDED=0 || exit $?


run PB_FFT_TL_Z=32 PB_FFT_ABLATE=1 || exit $?
run TAG=default2 || exit $?
cat gpurun_out/fftab4/ab.jsonl
