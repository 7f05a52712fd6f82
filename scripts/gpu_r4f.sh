export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_faults.py "tests/test_gpu_parity.py::test_rccl_code_paths_one_rank_communicator" "tests/test_gpu_parity.py::test_split_apply_timers_cover_whole_applies" tests/test_gpu_multiproc.py::test_multiprocess_cg_on_one_gpu > gpurun_out/r4f/tests.log 2>&1 || exit 1
for rep in 1 2; do
for cfg in force_comm=1 force_comm=1,comm_mark_every=1000000000 force_comm=1,comm_mark_every=1; do
  timeout -k 10 200 python bench.py --tune $cfg --secondary 0 --no-cpu-baseline --steps 50 --warmup 5 --matvecs 5 --sustained 5 > gpurun_out/r4f/b.json 2>>gpurun_out/r4f/b.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4f/b.json').read()); print(sys.argv[1], round(d['ms_per_step'],4), {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" $cfg >> gpurun_out/r4f/marks_ab.txt
done
done
