set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2
cd $R && timeout -k 10 600 python bench.py > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2/bench.json | cut -c1-600; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2/prof -o bench --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r2/bench_prof.json 2> $R/gpurun_out/r2/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
