#!/bin/bash
# Config 5 (compact A, spectral PC) 512^3 solve: kernel trace of two solves (warm-up + timed)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cfg5
cd /tmp && export TMPDIR=/tmp
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/cfg5/prof -o cfg5 -- python3 $R/scripts/bench_solve.py 512 > $R/gpurun_out/cfg5/solve.jsonl 2> $R/gpurun_out/cfg5/err.log
rc=$?; echo "rocprof rc=$rc"; cat $R/gpurun_out/cfg5/solve.jsonl; exit $rc
