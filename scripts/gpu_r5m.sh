# decomposed MG on the fused unrolled passes (deep ghosts): tests, phase probe, force_comm solves,
# and the one-rank V-cycle (must be unchanged)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5m
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread -k "mg or rccl_code_paths or multiproc or sor" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_mg_decomposed.py > $O/mg.jsonl 2> $O/err || exit $?
PB_TUNE_ROUNDS=4 timeout -k 10 200 python scripts/tune_mg.py > $O/vcycle_1rank.jsonl 2>> $O/err || exit $?
for t in "force_comm=1,mg_split_fused=0" "force_comm=1" "force_comm=1,mg_split_fused=0" "force_comm=1"; do
  timeout -k 10 300 python bench.py --workload star7-mg --steps 6 --warmup 2 --no-cpu-baseline --tune $t > $O/w.json 2>> $O/err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/w.json').read()); print(sys.argv[1], round(d['ms_per_step'],3))" "$t" >> $O/ab.txt
done
timeout -k 10 300 python bench.py --workload star7-mg --steps 6 --warmup 2 --no-cpu-baseline > $O/w1.json 2>> $O/err || exit $?
python3 -c "import json; d=json.loads(open('$O/w1.json').read()); print('1 rank', round(d['ms_per_step'],3))" >> $O/ab.txt
