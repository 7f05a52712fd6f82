# decomposed CG iteration (force_comm) under a kernel trace: launches and gaps per iteration
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o cg -- python3 $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline --secondary 0 --tune force_comm=1 > $O/b.json 2> $O/b.err
