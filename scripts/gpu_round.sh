#!/bin/bash
# Full GPU-box pass: parity tests + smoke + bench (gpu_check.sh), then a rocprofv3 kernel-trace
# stats run of the same bench, the PMC passes, the per-row measurements and full solves. Stops at the first
# failing step (exit status of that step).
set -u
R=$GRAFT_REPO_ROOT
cd $R && bash scripts/gpu_check.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && bash scripts/gpu_pmc.sh || exit $?
cd $R && timeout -k 10 900 python scripts/bench_rows.py > gpurun_out/rows.jsonl 2> gpurun_out/rows.err
rc=$?; echo "rows rc=$rc"; [ $rc -eq 0 ] || exit $rc
PCS=mg,jacobi timeout -k 10 600 python scripts/bench_solve.py 256 512 > gpurun_out/solve.jsonl 2> gpurun_out/solve.err
rc=$?; echo "solve rc=$rc"; exit $rc
