#!/bin/bash
# r03: x / r update on the spectral PC's first pass, poll every iteration; parity, config-5 A/B
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3e
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "fft or compact" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "TAG=default" "PB_FFT_POLL=2" "PB_FFT_RUPD=0" "TAG=default2" "PB_FFT_POLL=2" "PB_FFT_RUPD=0"; do
  env $cfg OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 >> $O/solve_fft_compact.jsonl 2>> $O/s1.err
  rc=$?; echo "cfg5 $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 -c "
import json
for l in open('$O/solve_fft_compact.jsonl'):
    d=json.loads(l); print(d['n'], round(d['solve_ms'],3), d['cfg'])
"
