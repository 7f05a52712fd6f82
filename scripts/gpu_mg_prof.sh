#!/bin/bash
# rocprofv3 kernel stats + trace of the MG-PCG solve workload (512^3)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mgprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mgprof -o mg --output-format csv -- python3 $R/bench.py --workload star7-mg --steps 2 --warmup 1 --cpu-baseline none > $R/gpurun_out/mgprof/bench.json 2> $R/gpurun_out/mgprof/bench.err
echo "rc=$?"
