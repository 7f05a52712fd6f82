set -u
mkdir -p gpurun_out
export PB_TUNE_ROUNDS=5
export PB_TUNE_CONFIGS='[{},{"PB_PASSA_WPE":"3"},{"PB_PASSA_WPE":"3","PB_STENCIL_BLOCKS":"1024"},{"PB_STENCIL_BLOCKS":"1024"},{"PB_STENCIL_TY":"2"}]'
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "stencil or cg" > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/tune_stencil.py > gpurun_out/tune.log 2>&1
rc=$?; cat gpurun_out/tune.log; exit $rc
