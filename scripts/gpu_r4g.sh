# V-cycle coarse-level A/B: kernel thresholds through the tuning table
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
PB_TUNE_ROUNDS=4 PB_TUNE_CONFIGS='[{}, {"mg_engine_min_plane": 16384}, {"mg_engine_min_plane": 4096}, {"mg_tail_max": 32768}, {"mg_engine_min_plane": 16384, "mg_tail_max": 32768}, {"mg_engine_min_plane": 4096, "mg_tail_max": 32768}, {"mg_engine_min_plane": 16384, "mg_restrict_z_min_cols": 1024}, {"prrx_minz": 32}, {"prrx_minz": 64}, {"postx_minz": 64}, {"prrx_minz": 32, "postx_minz": 64}, {"prrx_wgcu": 2}]' timeout -k 10 300 python scripts/tune_mg.py > gpurun_out/r4g/vcycle_ab.jsonl 2> gpurun_out/r4g/vcycle_ab.err || exit 1
for rep in 1 2; do
for cfg in "" "--tune mg_engine_min_plane=16384" "--tune mg_engine_min_plane=16384,mg_tail_max=32768"; do
  timeout -k 10 200 python bench.py --workload star7-mg $cfg --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r4g/b.json 2>>gpurun_out/r4g/b.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4g/b.json').read()); print(repr(sys.argv[1]), round(d['ms_per_step'],3), d['its_per_solve'], {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" "$cfg" >> gpurun_out/r4g/solve_ab.txt
done
done
timeout -k 10 420 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_multiproc.py::test_bench_eight_ranks_default_run_host_transport > gpurun_out/r4g/eight.log 2>&1 || exit 1
