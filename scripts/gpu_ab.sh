#!/bin/bash
# usage: gpu_ab.sh OUTNAME REPS cfg... [-- bench args]  -> gpurun_out/ab/OUTNAME.jsonl
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/ab
out=$1; shift
cd $R && timeout -k 10 1000 python scripts/ab_env.py "$@" > gpurun_out/ab/$out.jsonl 2> gpurun_out/ab/$out.err
rc=$?; cat gpurun_out/ab/$out.jsonl; exit $rc
