# rocprofv3 kernel stats of the decomposed config-5 and MG solves (force_comm, one GPU)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cf -o cf -- python3 $R/bench.py --workload compact-fft --steps 6 --warmup 1 --no-cpu-baseline --tune force_comm=1 > $O/cf.json 2> $O/cf.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mg -o mg -- python3 $R/bench.py --workload star7-mg --steps 4 --warmup 1 --no-cpu-baseline --tune force_comm=1 > $O/mg.json 2> $O/mg.err || exit $?
