#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) over a short bench run.
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 2 --matvecs 10 --no-cpu-baseline --secondary 0"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_$tag -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_$tag.json 2>$R/gpurun_out/pmc_$tag.err
  rc=$?; echo "$grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
