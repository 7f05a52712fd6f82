#!/bin/bash
# r03: residual update on the spectral PC's first pass (parity + config-5 A/B), config-5 kernel
# trace, then the x-update bimodality runs (scripts/gpu_bimodal.sh)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3b
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "fft or compact" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "TAG=default" "PB_FFT_RUPD=0" "TAG=default2" "PB_FFT_RUPD=0"; do
  env $cfg OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 >> $O/solve_fft_compact.jsonl 2>> $O/s1.err
  rc=$?; echo "cfg5 $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o cfg5 --output-format csv \
  -- python3 $R/scripts/bench_solve.py 512 > $O/kt.jsonl 2> $O/kt.err
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && bash scripts/gpu_bimodal.sh
