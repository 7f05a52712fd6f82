#!/bin/bash
# r03: the CG x-update pass's two modes. Six fresh bench processes without a
# profiler, then six under rocprofv3 with L2 / fabric request counters beside the kernel trace, so
# each process's x-update durations can be set against its counters (scripts/bimodal_summary.py)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bimodal
mkdir -p $O
cd $R
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python3 bench.py --steps 24 --warmup 4 --cpu-baseline none --matvecs 2 --sustained 2 > $O/plain$i.json 2> $O/plain$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "plain $i rc=$rc"; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/plain$i.json'));print('plain', $i, d['ms_per_step'], {k:v.get('avg_ms') for k,v in d['kernels'].items() if isinstance(v,dict)})"
done
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
    -d $O/p$i -o run --output-format csv -- python3 $R/bench.py --steps 24 --warmup 4 --cpu-baseline none --matvecs 2 --sustained 2 > $O/b$i.json 2> $O/b$i.err
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
