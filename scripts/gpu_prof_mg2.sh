#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/pmg
cd /tmp && export TMPDIR=/tmp
PCS=mg NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmg/prof -o mg --output-format csv -- python3 $R/scripts/bench_solve.py 512 > $R/gpurun_out/pmg/solve.jsonl 2> $R/gpurun_out/pmg/solve.err
rc=$?; cat $R/gpurun_out/pmg/solve.jsonl; exit $rc
