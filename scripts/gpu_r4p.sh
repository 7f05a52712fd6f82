# pre-pass split default (auto) vs off: tests, V-cycle at 512^3 / 256^3, MG solves
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4p
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "balanced_split or post_sweep_xch_sums or presmooth_restrict_variants or mg" > $O/tests.log 2>&1 || exit $?
PB_TUNE_ROUNDS=6 PB_TUNE_CONFIGS='[{}, {"prrx_split": 0}]' timeout -k 10 300 python scripts/tune_mg.py > $O/vcycle_ab512.jsonl 2> $O/vcycle_ab.err || exit $?
PB_TUNE_N=256,256,256 PB_TUNE_ROUNDS=6 PB_TUNE_CONFIGS='[{}, {"prrx_split": 0}]' timeout -k 10 300 python scripts/tune_mg.py > $O/vcycle_ab256.jsonl 2>> $O/vcycle_ab.err || exit $?
for t in "" "--tune prrx_split=0" "" "--tune prrx_split=0"; do
  timeout -k 10 300 python bench.py --workload star7-mg --steps 8 --warmup 2 --no-cpu-baseline $t > $O/mg.json 2>> $O/mg.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/mg.json').read()); print(repr(sys.argv[1]), round(d['ms_per_step'],3))" "$t" >> $O/solve_ab.txt
done
