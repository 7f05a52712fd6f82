#!/bin/bash
# quick bench line, then rocprofv3 kernel stats and the PMC traffic passes of the same command
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
ARGS="--steps 30 --warmup 5 --secondary 0 --cpu-baseline none"
timeout -k 10 400 python $R/bench.py $ARGS > $R/gpurun_out/bq.json 2> $R/gpurun_out/bq.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bq_prof -o bq --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/bq_prof.json 2> $R/gpurun_out/bq_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -s KILL 300 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_$tag -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_$tag.json 2>$R/gpurun_out/pmc_$tag.err
  rc=$?; echo "$grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
