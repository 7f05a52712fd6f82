#!/bin/bash
# spectral-PC kernels: parity subset, timing, and one SQ counter pass (LDS / VALU balance)
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/fftpmc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "fft" --timeout 300 --timeout-method thread > gpurun_out/fftpmc/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fftpmc/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_fft.py 512 256 > gpurun_out/fftpmc/fft.jsonl 2> gpurun_out/fftpmc/fft.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/fftpmc/fft.jsonl; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
  -d $R/gpurun_out/fftpmc/sq -o pmc --output-format csv -- python3 $R/scripts/bench_fft.py 512 > $R/gpurun_out/fftpmc/sq.jsonl 2> $R/gpurun_out/fftpmc/sq.err
rc=$?; echo "sq rc=$rc"; exit $rc
