# decomposed MG: how many coarse levels to gather (force_comm, 512^3)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5l
mkdir -p $O
cd $R
for t in "force_comm=1" "force_comm=1,mg_agglomerate_max=32768" "force_comm=1,mg_agglomerate_max=262144" "force_comm=1" "force_comm=1,mg_agglomerate_max=32768" "force_comm=1,mg_agglomerate_max=262144"; do
  timeout -k 10 300 python bench.py --workload star7-mg --steps 6 --warmup 2 --no-cpu-baseline --tune $t > $O/w.json 2>> $O/err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/w.json').read()); print(sys.argv[1], round(d['ms_per_step'],3))" "$t" >> $O/ab.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "multirank_mg" > $O/tests.log 2>&1; tail -2 $O/tests.log
