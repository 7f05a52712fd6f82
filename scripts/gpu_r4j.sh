# LDS-resident V-cycle tail: MG parity tests, then V-cycle / solve A/B against the L2 tail
set -u
mkdir -p gpurun_out/r4j
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mg or sor" tests/test_gpu_fullsize.py::test_mg_pc_apply_512_bit_exact > gpurun_out/r4j/tests.log 2>&1 || exit 1
PB_TUNE_ROUNDS=6 PB_TUNE_CONFIGS='[{}, {"mg_tail_lds": 0}]' timeout -k 10 300 python scripts/tune_mg.py > gpurun_out/r4j/vcycle_ab.jsonl 2> gpurun_out/r4j/vcycle_ab.err || exit 1
rm -f gpurun_out/r4j/solve_ab.txt
for rep in 1 2; do
for cfg in "" "--tune mg_tail_lds=0"; do
  timeout -k 10 200 python bench.py --workload star7-mg $cfg --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r4j/b.json 2>>gpurun_out/r4j/b.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4j/b.json').read()); print(repr(sys.argv[1]), round(d['ms_per_step'],3), d['its_per_solve'], {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" "$cfg" >> gpurun_out/r4j/solve_ab.txt
done
done
