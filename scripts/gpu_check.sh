#!/bin/bash
# GPU-box job: parity tests, smoke, short bench. Stops at the first crash-class exit status
# (fault/abort/segv/timeout); plain test failures (pytest exit 1) still let the bench run.
set -u
mkdir -p gpurun_out
ok_or_testfail() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok_or_testfail $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:---steps 50 --warmup 5} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
