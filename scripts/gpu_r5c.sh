# decomposed code paths on one GPU (force_comm: 1-rank RCCL communicator, halos to self): the
# per-rank cost of the N > 1 paths for the headline, MG and config-5 workloads
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c
mkdir -p $O
cd $R
timeout -k 10 400 python scripts/ab_env.py 2 - force_comm=1 > $O/cg.jsonl 2> $O/err || exit $?
for t in "" "--tune force_comm=1"; do
  for w in star7-mg compact-fft; do
    timeout -k 10 300 python bench.py --workload $w --steps 6 --warmup 2 --no-cpu-baseline $t > $O/w.json 2>> $O/err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$O/w.json').read()); print(repr(sys.argv[1]), sys.argv[2], round(d['ms_per_step'],3), d.get('per_rank_comm'), d.get('diagnostics',{}).get('timers') if isinstance(d.get('diagnostics'),dict) else None)" "$t" $w >> $O/solves.txt
  done
done
