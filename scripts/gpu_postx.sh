#!/bin/bash
# MG post-smoothing with LDS-shared rows (PB_POSTX): bit-exact PC applies and CG histories, then
# the V-cycle phases at 512^3 per variant (interleaved in one process), then MG-PCG solves.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "post_sweep or pc_apply_bit_exact or fused_post" > gpurun_out/pt_postx.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_postx.log; [ $rc -eq 0 ] || exit $rc
PB_TUNE_ROUNDS=4 PB_TUNE_CONFIGS='[{"PB_POSTX":"0"},{"PB_POSTX":"1"},{"PB_POSTX":"3"},{"PB_POSTX":"3","PB_POSTX_WGCU":"8"},{"PB_POSTX":"3","PB_POSTX_WGCU":"16"},{"PB_POSTX":"6"},{"PB_POSTX":"6","PB_POSTX_WGCU":"8"},{"PB_POSTX":"4"},{"PB_POSTX":"2","PB_POSTX_WGCU":"8"}]' \
  timeout -k 10 300 python scripts/tune_mg.py > gpurun_out/postx_tune.jsonl 2> gpurun_out/postx_tune.err
rc=$?; echo "tune rc=$rc"; cat gpurun_out/postx_tune.jsonl; [ $rc -eq 0 ] || exit $rc
for v in ${POSTX_SOLVE:-0 3 6}; do
  PB_POSTX=$v NO_CPU=1 PCS=mg timeout -k 10 300 python scripts/bench_solve.py 512 > gpurun_out/postx_solve_$v.jsonl 2> gpurun_out/postx_solve_$v.err
  rc=$?; echo "solve postx=$v rc=$rc"; cut -c1-600 gpurun_out/postx_solve_$v.jsonl; [ $rc -eq 0 ] || exit $rc
done
