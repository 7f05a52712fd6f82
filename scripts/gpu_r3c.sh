#!/bin/bash
# r03: resident-grid sums on the register-edge X pass; fft / compact parity, config-5 solves
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3c
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "fft or compact" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 >> $O/solve_fft_compact.jsonl 2>> $O/s1.err
  rc=$?; echo "cfg5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python scripts/bench_fft.py 512 256 >> $O/fft.jsonl 2>> $O/fft.err
cat $O/solve_fft_compact.jsonl $O/fft.jsonl
