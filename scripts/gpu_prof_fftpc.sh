#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/pfft2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pfft2/prof -o fft --output-format csv -- python3 $R/scripts/bench_fft.py 512 > $R/gpurun_out/pfft2/fft.jsonl 2> $R/gpurun_out/pfft2/fft.err
rc=$?; cat $R/gpurun_out/pfft2/fft.jsonl; exit $rc
