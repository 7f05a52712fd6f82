set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_d2.log 2>&1; rc=$?; echo "default tests rc=$rc"; tail -2 gpurun_out/pt_d2.log; [ $rc -eq 0 ] || exit $rc
PB_CG_DEFER_X=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread -k "cg or solve or multirank or rccl" > gpurun_out/pt_d4.log 2>&1; rc=$?; echo "defer4 tests rc=$rc"; tail -2 gpurun_out/pt_d4.log; [ $rc -eq 0 ] || exit $rc
for v in 2 4 2 4; do
  PB_CG_DEFER_X=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/b_d$v.json 2> gpurun_out/b_d$v.err; rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/b_d$v.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/b_d$v.json')); print('defer $v', round(d['ms_per_step'],4), round(d['value']/1e9,2))"
done
