# spectral PC: the residual-sums X pass (prefetched r, resident-grid size) A/B in the config-5 solve
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
rm -f gpurun_out/r4h/ab.txt
for rep in 1 2; do
for cfg in "" "--tune fft_sums_pf=1" "--tune fft_sums_bpc=4" "--tune fft_sums_bpc=8" "--tune fft_sums_pf=1,fft_sums_bpc=8"; do
  timeout -k 10 200 python bench.py --workload compact-fft $cfg --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/r4h/b.json 2>>gpurun_out/r4h/b.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4h/b.json').read()); print(repr(sys.argv[1]), round(d['ms_per_step'],4), d['ksp_state']['reason'], {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" "$cfg" >> gpurun_out/r4h/ab.txt
done
done
