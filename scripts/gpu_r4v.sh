# per-GPU slab shapes of the weak-scaling bench (N = 1, 2, 4, 8: 512^3, 512^3, 512x1024x256, 1024x1024x128), interleaved
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4v
mkdir -p $O
cd $R
for rep in 1 2; do
for g in 512,512,512 512,1024,256 1024,1024,128; do
  timeout -k 10 200 python bench.py --grid $g --secondary 0 --no-cpu-baseline --steps 100 --warmup 10 --matvecs 20 --sustained 20 > $O/b.json 2>> $O/b.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/b.json').read()); print(sys.argv[1], round(d['ms_per_step'],4), {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})" $g >> $O/shapes.txt
done
done
