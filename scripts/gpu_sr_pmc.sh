#!/bin/bash
# PMC passes (one counter group per run) over the single-reduction probe (SIZE, default 512;
# SR_ARGS: the probe's settings, "-" = the single-reduction iteration only, "" = both iterations)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/srpmc${SIZE:+_$SIZE}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export SR_REPS=1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp -d $OUT/p$i -o pmc --output-format csv -- python3 $R/scripts/sr_probe.py ${SIZE:-512} ${SR_ARGS--} > $OUT/p$i.jsonl 2> $OUT/p$i.err
  rc=$?; echo "$grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
