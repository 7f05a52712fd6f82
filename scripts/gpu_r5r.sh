# decomposed MG: the fused passes on the 128^3 level too (force_comm), 512^3
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5r
mkdir -p $O
cd $R
for t in "force_comm=1" "force_comm=1,mg_engine_min_plane=16384" "force_comm=1" "force_comm=1,mg_engine_min_plane=16384"; do
  timeout -k 10 300 python bench.py --workload star7-mg --steps 6 --warmup 2 --no-cpu-baseline --tune $t > $O/w.json 2>> $O/err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/w.json').read()); print(sys.argv[1], round(d['ms_per_step'],3))" "$t" >> $O/ab.txt
done
