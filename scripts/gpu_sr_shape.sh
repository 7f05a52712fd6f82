#!/bin/bash
# single-reduction one-pass kernel shapes: the SR parity tests on a variant build (variants/$VAR.so),
# then the SR probe at 512^3 and 256^3, default build and variant interleaved per process
set -u
mkdir -p gpurun_out
VAR=${VAR:-sr4}
PB_LIB=variants/$VAR.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_single_reduction.py > gpurun_out/sr_shape_tests.log 2>&1 || { tail -30 gpurun_out/sr_shape_tests.log; exit 1; }
tail -2 gpurun_out/sr_shape_tests.log
: > gpurun_out/sr_shape.jsonl
for rep in 1 2 3; do
  for v in base $VAR; do
    if [ $v = base ]; then unset PB_LIB; else export PB_LIB=variants/$v.so; fi
    SR_REPS=1 timeout -k 10 200 python scripts/sr_probe.py 512 256 - | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/sr_shape.jsonl || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/sr_shape.jsonl"):
    r = json.loads(l)
    print(r["lib"], r["n"], r["ms_per_it"], r["passes_ms"])
PY
