#!/bin/bash
# pass-B-stores-p A/B (PB_CG_PSTORE_B): parity tests, then interleaved bench runs at 512^3 and 256^3,
# then the access-pattern probe. Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-.}
cd $R && mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "pstore or folded_finalize" > gpurun_out/pstore_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pstore_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh pstore_512 3 - PB_CG_PSTORE_B=1 || exit $?
bash scripts/gpu_ab.sh pstore_256 3 - PB_CG_PSTORE_B=1 -- --base 256 || exit $?
timeout -k 10 120 ./scripts/rw_mix_probe > gpurun_out/rw_mix.jsonl; echo "probe rc=$?"
