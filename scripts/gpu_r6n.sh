set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof2_fc1
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof2_fc1 -o run -- python3 bench.py --workload compact-fft --tune force_comm=1 --cpu-baseline none --steps 5 --warmup 1 > gpurun_out/prof2_fc1.json 2> gpurun_out/prof2_fc1.err
