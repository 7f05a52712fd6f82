set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for fc in 0 1; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fc$fc -o run -- python3 bench.py --workload compact-fft --tune force_comm=$fc --cpu-baseline none --steps 5 --warmup 1 > gpurun_out/prof_fc$fc.json 2> gpurun_out/prof_fc$fc.err || exit 1
done
find gpurun_out/prof_fc0 gpurun_out/prof_fc1 -name "*kernel_stats.csv" | head
