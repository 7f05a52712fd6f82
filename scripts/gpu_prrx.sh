#!/bin/bash
# MG fused sweeps with LDS-shared rows (PB_PRRX pre-smoothing + restriction, PB_POSTX
# post-smoothing): bit-exact PC applies and CG histories, then the V-cycle phases at 512^3 per
# variant (interleaved in one process), then MG-PCG solves.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "post_sweep or presmooth_restrict or pc_apply_bit_exact or fused_post or sor_mg" > gpurun_out/pt_prrx.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_prrx.log; [ $rc -eq 0 ] || exit $rc
: "${TUNE_CONFIGS:=[{\}]}"
PB_TUNE_ROUNDS=4 PB_TUNE_CONFIGS="$TUNE_CONFIGS" timeout -k 10 300 python scripts/tune_mg.py > gpurun_out/prrx_tune.jsonl 2> gpurun_out/prrx_tune.err
rc=$?; echo "tune rc=$rc"; cat gpurun_out/prrx_tune.jsonl; [ $rc -eq 0 ] || exit $rc
i=0
IFS=';' read -ra CFGS <<< "${SOLVE_CONFIGS:--}"
for c in "${CFGS[@]}"; do
  [ "$c" = "-" ] && c=""
  env $c NO_CPU=1 PCS=mg timeout -k 10 300 python scripts/bench_solve.py 512 > gpurun_out/prrx_solve_$i.jsonl 2> gpurun_out/prrx_solve_$i.err
  rc=$?; echo "solve [$c] rc=$rc"; cut -c1-420 gpurun_out/prrx_solve_$i.jsonl; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
if [ -n "${MG_TRACE:-}" ]; then  # kernel trace of the default V-cycle
  R=$(pwd)
  (cd /tmp && export TMPDIR=/tmp && PB_TUNE_ROUNDS=1 PB_TUNE_CONFIGS="[{}]" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mgtrace -o mg --output-format csv -- python3 $R/scripts/tune_mg.py > $R/gpurun_out/mgtrace.jsonl 2> $R/gpurun_out/mgtrace.err)
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
