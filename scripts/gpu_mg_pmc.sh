#!/bin/bash
# PMC passes over 512^3 V-cycles (scripts/tune_mg.py, one config): SQ issue / wait counters,
# fabric bytes and L2 hits of the fused fine-level sweeps. One counter group per run.
set -u
R=$(pwd)
mkdir -p gpurun_out/mgpmc
cd /tmp && export TMPDIR=/tmp
export PB_TUNE_ROUNDS=1 PB_TUNE_CONFIGS="${TUNE_CONFIGS:-[{\}]}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $R/gpurun_out/mgpmc/pmc_$i -o pmc --output-format csv -- python3 $R/scripts/tune_mg.py > $R/gpurun_out/mgpmc/run_$i.jsonl 2> $R/gpurun_out/mgpmc/run_$i.err
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
python3 $R/scripts/pmc_kernel_means.py $R/gpurun_out/mgpmc "presmooth|post_sweep|star7|sor_sweep2" > $R/gpurun_out/mgpmc/means.json
cat $R/gpurun_out/mgpmc/run_0.jsonl
