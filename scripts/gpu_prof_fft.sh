#!/bin/bash
# config-5 solve (compact A = P, -pc_type fft) at 512^3 under rocprofv3 --kernel-trace --stats
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/pfft
cd /tmp && export TMPDIR=/tmp
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pfft/prof -o fft --output-format csv -- python3 $R/scripts/bench_solve.py 512 > $R/gpurun_out/pfft/solve.jsonl 2> $R/gpurun_out/pfft/solve.err
rc=$?; cat $R/gpurun_out/pfft/solve.jsonl; exit $rc
