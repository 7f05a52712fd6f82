#!/bin/bash
# compact / tridiagonal GPU tests, then the compact apply and line-solve benches
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multiproc.py -q -x --timeout 200 --timeout-method thread -k "compact or pcr or tdma or lines or fft" > gpurun_out/pt_compact.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt_compact.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/compact_dpp.jsonl
for i in 1 2; do
  timeout -k 10 120 python scripts/bench_compact.py 512 256 >> gpurun_out/compact_dpp.jsonl 2>>gpurun_out/compact_dpp.err || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/compact_dpp.jsonl"):
    d = json.loads(l)
    print(d["n"], round(d["lapl_ms"], 4), round(d["frac"], 3), {k: v["ms"] for k, v in d["passes"].items()})
PY
