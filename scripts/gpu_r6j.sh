set -u
mkdir -p gpurun_out
PB_LIB=variants/kw8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "stencil_bit_exact or test_cg_matches_petsc_semantics" -x -q --timeout 120 --timeout-method thread > gpurun_out/kw8_tests.log 2>&1
rc=$?; echo "kw8 tests rc=$rc"; tail -3 gpurun_out/kw8_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/kw8_ab.jsonl
for rep in 1 2; do
  for v in base kw8; do
    if [ $v = base ]; then unset PB_LIB; else export PB_LIB=variants/$v.so; fi
    timeout -k 10 300 python scripts/cg_cfg_probe.py 512 3 '[{}]' | grep config | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/kw8_ab.jsonl || exit 1
  done
done
unset PB_LIB
cat gpurun_out/kw8_ab.jsonl
