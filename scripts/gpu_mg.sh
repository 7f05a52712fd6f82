#!/bin/bash
# MG preconditioner: bit-exact PC apply / CG parity tests, then full MG-PCG solves at 512^3 under
# several kernel configurations (MG_CONFIGS: ';'-separated env assignments, '-' = defaults).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "mg or sor or pc_apply or multirank or fused" > gpurun_out/pt_mg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_mg.log; [ $rc -eq 0 ] || exit $rc
IFS=';' read -ra CFGS <<< "${MG_CONFIGS:--}"
i=0
for c in "${CFGS[@]}"; do
  [ "$c" = "-" ] && c=""
  env $c NO_CPU=1 PCS=mg timeout -k 10 300 python scripts/bench_solve.py ${SIZES:-512} > gpurun_out/mg_cfg$i.jsonl 2> gpurun_out/mg_cfg$i.err
  rc=$?; echo "cfg[$c] rc=$rc"; cat gpurun_out/mg_cfg$i.jsonl; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
