# MG solve kernel trace (gaps between launches), config-4 8-rank 30-iteration history test
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py -m gpu -x -v --timeout 500 --timeout-method thread -k config4 > $O/cfg4.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o mg -- python3 $R/bench.py --workload star7-mg --steps 4 --warmup 1 --no-cpu-baseline > $O/mg.json 2> $O/mg.err
