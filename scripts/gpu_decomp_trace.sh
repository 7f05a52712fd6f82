#!/bin/bash
# kernel trace of the decomposed (force_comm) and one-rank KSPSolve_CG iterations at 512^3
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/dtrace
cd /tmp && export TMPDIR=/tmp
export REPS=1 SR=0
for fc in 0 1; do
  FC=$fc timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dtrace/fc$fc -o kt --output-format csv -- python3 $R/scripts/probe_decomposed_cg.py 512 > $R/gpurun_out/dtrace/fc$fc.jsonl 2> $R/gpurun_out/dtrace/fc$fc.err
  rc=$?; echo "fc=$fc rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
