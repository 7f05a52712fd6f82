#!/bin/bash
# PMC passes (one counter group per run) over the single-reduction probe at 512^3
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/srpmc
cd /tmp && export TMPDIR=/tmp
export SR_REPS=1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp -d $R/gpurun_out/srpmc/p$i -o pmc --output-format csv -- python3 $R/scripts/sr_probe.py 512 ${SR_AB:--} > $R/gpurun_out/srpmc/p$i.jsonl 2> $R/gpurun_out/srpmc/p$i.err
  rc=$?; echo "$grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
