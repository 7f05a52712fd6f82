#!/bin/bash
# single-reduction probe: default build vs variants/$VAR.so, alternating processes (512^3, 256^3)
set -u
mkdir -p gpurun_out
VAR=${VAR:-srnt}
: > gpurun_out/sr_ab.jsonl
for rep in 1 2 3; do
  for v in base $VAR; do
    if [ $v = base ]; then unset PB_LIB; else export PB_LIB=variants/$v.so; fi
    SR_REPS=1 timeout -k 10 200 python scripts/sr_probe.py 512 256 - | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/sr_ab.jsonl || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/sr_ab.jsonl"):
    r = json.loads(l)
    print(r["lib"], r["n"], r["ms_per_it"], r["passes_ms"])
PY
