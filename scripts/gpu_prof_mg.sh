#!/bin/bash
# rocprofv3 kernel statistics of one MG-PCG solve at 512^3 (plus its warm-up solve)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
NO_CPU=1 PCS=mg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mg -o mg --output-format csv -- python3 $R/scripts/bench_solve.py 512 > $R/gpurun_out/prof_mg.jsonl 2> $R/gpurun_out/prof_mg.err
rc=$?; echo "rocprof rc=$rc"; cat $R/gpurun_out/prof_mg.jsonl
f=$(find $R/gpurun_out/prof_mg -name "*kernel_stats.csv" | head -1); cut -c1-200 "$f" | head -30
exit $rc
