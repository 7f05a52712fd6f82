#!/bin/bash
# spectral-PC / compact / decomposed tests, then config-5 solves (one rank vs force_comm)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "fft or compact or rccl or multirank or config5" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/c5_tests.log
[ $rc -eq 0 ] || exit $rc
for t in "" "--tune force_comm=1" "--tune force_comm=1,a2a_copy_self=1" "" "--tune force_comm=1"; do
  timeout -k 10 300 python -u bench.py --workload compact-fft --steps 5 --warmup 2 --secondary 0 --cpu-baseline none $t > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/c5_bench.json')); print(sys.argv[1] or 'default', round(r['ms_per_step'],3))" "$t"
done
