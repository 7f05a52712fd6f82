#!/bin/bash
# single-reduction probe over library variants (V="base srt3 ..."), each with the z'Az forms
# (sr_ddiff=0 / 1) interleaved in one process; 512^3 and 256^3. Output gpurun_out/sr_variants.txt
set -u
mkdir -p gpurun_out
: > gpurun_out/sr_variants.jsonl
for rep in 1 2; do
  for v in ${V:-base}; do
    if [ $v = base ]; then unset PB_LIB; else export PB_LIB=variants/$v.so; fi
    SR_REPS=1 timeout -k 10 300 python scripts/sr_probe.py 512 256 sr_ddiff=0 sr_ddiff=1 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/sr_variants.jsonl || exit 1
  done
done
unset PB_LIB
python - <<'PY'
import json
for l in open("gpurun_out/sr_variants.jsonl"):
    r = json.loads(l)
    print(r["lib"], r["n"], r["tune"], r["ms_per_it"], r["passes_ms"].get("cg_sr1"))
PY
