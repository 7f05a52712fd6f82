#!/bin/bash
# r03: V-cycle fused-sweep register budgets (build variants loaded with PB_LIB): default, 2 own
# rows per wave (PB_SWEEP2_TY=2), that plus 3 waves per SIMD for the post-smoothing, 3 waves per
# SIMD for both fused fine-level kernels (spills); V-cycle phase timers, then MG-PCG solves
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mgvar
cd $R && mkdir -p $O
for v in default ty2 ty2w3 w3 default; do
  if [ $v = default ]; then L=""; else L="PB_LIB=$R/variants/$v.so"; fi
  env $L PB_TUNE_ROUNDS=4 timeout -k 10 120 python scripts/tune_mg.py > $O/tune_$v.jsonl 2> $O/tune_$v.err
  rc=$?; echo "tune $v rc=$rc"; cat $O/tune_$v.jsonl; [ $rc -eq 0 ] || exit $rc
done
for v in default ty2 ty2w3; do
  if [ $v = default ]; then L=""; else L="PB_LIB=$R/variants/$v.so"; fi
  env $L PCS=mg NO_CPU=1 timeout -k 10 200 python scripts/bench_solve.py 512 > $O/solve_$v.jsonl 2> $O/solve_$v.err
  rc=$?; echo "solve $v rc=$rc"; cut -c1-200 $O/solve_$v.jsonl; [ $rc -eq 0 ] || exit $rc
done
# spectral PC on 1024-point lines: 8- vs 16-line tiles on the strided passes
for t in 8 16 8 16; do
  PB_FFT_TL_LONG=$t timeout -k 10 200 python scripts/bench_fft.py 1024 >> $O/fft1024.jsonl 2>> $O/fft1024.err
  rc=$?; echo "fft1024 $t rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat $O/fft1024.jsonl
