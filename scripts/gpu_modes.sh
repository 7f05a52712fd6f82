#!/bin/bash
# several processes of scripts/probe_modes.py, each under one PMC pass with the kernel trace
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/modes
cd /tmp && export TMPDIR=/tmp
for p in 1 2 3 4 5 6; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum -d $R/gpurun_out/modes/p$p -o m --output-format csv -- python3 $R/scripts/probe_modes.py > $R/gpurun_out/modes/p$p.out 2> $R/gpurun_out/modes/p$p.err
  rc=$?; echo "p$p rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for p in 7 8 9; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/modes/p$p -o m --output-format csv -- python3 $R/scripts/probe_modes.py > $R/gpurun_out/modes/p$p.out 2> $R/gpurun_out/modes/p$p.err
  rc=$?; echo "p$p rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
