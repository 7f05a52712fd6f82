# compact CG fusion without the p_old fetch on a lazy first iteration: config-5 tests + bench
set -u
mkdir -p gpurun_out/r4k
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "compact or fft" tests/test_gpu_fullsize.py::test_config5_compact_fft_solve_512 > gpurun_out/r4k/tests.log 2>&1 || exit 1
rm -f gpurun_out/r4k/ab.txt
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --workload compact-fft --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/r4k/b.json 2>>gpurun_out/r4k/b.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4k/b.json').read()); print(round(d['ms_per_step'],4), d['ksp_state']['reason'], d['ksp_state']['true_residual_rel'], {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" >> gpurun_out/r4k/ab.txt
done
