set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_mg
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mg -o mg --output-format csv -- python3 bench.py --workload star7-mg --cpu-baseline none --steps 3 --warmup 1 > gpurun_out/prof_mg.json 2> gpurun_out/prof_mg.err
