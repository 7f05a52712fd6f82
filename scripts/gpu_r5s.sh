# decomposed MG with the 128^2-plane engine threshold: MG tests, force_comm solves, one rank unchanged
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread -k "mg or rccl_code_paths or multiproc or sor" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for t in "force_comm=1,mg_engine_min_plane=65536" "force_comm=1" "force_comm=1,mg_engine_min_plane=65536" "force_comm=1" "cg_fuse=1"; do
  timeout -k 10 300 python bench.py --workload star7-mg --steps 6 --warmup 2 --no-cpu-baseline --tune $t > $O/w.json 2>> $O/err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/w.json').read()); print(sys.argv[1], round(d['ms_per_step'],3))" "$t" >> $O/ab.txt
done
