#!/bin/bash
# r03 register edges in the spectral PC: X passes on dht_reg_x_kernel, the Z pass's symbol step
# on registers (MODE 2); fft / compact parity subsets, PC apply A/B, config-5 solves
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fftreg2
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "compact or fft" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "TAG=default" "PB_FFT_ZHYB=0" "PB_FFT_REG=0" "TAG=default2" "PB_FFT_ZHYB=0" ; do
  env $cfg timeout -k 10 200 python scripts/bench_fft.py 512 256 1024 >> $O/fft_ab.jsonl 2>> $O/fft_ab.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench_fft rc=$rc"; exit $rc; }
done
cat $O/fft_ab.jsonl
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 >> $O/solve_fft_compact.jsonl 2>> $O/s1.err
rc=$?; echo "cfg5 rc=$rc"; cat $O/solve_fft_compact.jsonl; exit $rc
