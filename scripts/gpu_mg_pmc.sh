#!/bin/bash
# SQ issue / wait counters and fabric traffic of the MG-PCG solve's kernels (512^3)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mgpmc
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp -d $R/gpurun_out/mgpmc/p$i -o pmc --output-format csv -- python3 $R/bench.py --workload star7-mg --steps 1 --warmup 1 --cpu-baseline none > $R/gpurun_out/mgpmc/p$i.json 2> $R/gpurun_out/mgpmc/p$i.err
  rc=$?; echo "$grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
