#!/bin/bash
# r06 closing profiles: rocprofv3 kernel-trace stats of the default bench line (no CPU rows, no
# secondaries), the PMC traffic passes of the same command (FETCH_SIZE / WRITE_SIZE, one group
# per run) and the single-reduction probe. Outputs under gpurun_out/r6prof.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6prof
mkdir -p $O
ARGS="--steps 30 --warmup 5 --matvecs 20 --no-cpu-baseline --secondary 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py $ARGS > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 300 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_$grp -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_$grp.json 2>$R/gpurun_out/pmc_$grp.err
  rc=$?; echo "$grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $R && SR_REPS=2 timeout -k 10 300 python scripts/sr_probe.py 512 256 > $O/sr_probe.jsonl 2> $O/sr_probe.err
rc=$?; echo "sr rc=$rc"; exit $rc
