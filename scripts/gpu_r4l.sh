# data points: 256^3 (config 2) per-kernel breakdown; config 4's whole 1024^3 grid on one GPU
set -u
mkdir -p gpurun_out/r4l
export TMPDIR=/tmp
for g in 256,256,256 256,256,256; do
  timeout -k 10 200 python bench.py --grid $g --secondary 0 --no-cpu-baseline --steps 200 --warmup 20 --matvecs 20 --sustained 20 > gpurun_out/r4l/b.json 2>>gpurun_out/r4l/b.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4l/b.json').read()); print(sys.argv[1], round(d['ms_per_step'],4), {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" $g >> gpurun_out/r4l/summary.txt
done
timeout -k 10 400 python bench.py --base 1024 --secondary 0 --no-cpu-baseline --steps 20 --warmup 3 --matvecs 5 --sustained 5 > gpurun_out/r4l/b1024.json 2>>gpurun_out/r4l/b.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r4l/b1024.json').read()); print('1024^3', round(d['ms_per_step'],3), d['value']/1e9, {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" >> gpurun_out/r4l/summary.txt
