#!/bin/bash
# run tune_compact.py under several knob settings (each its own process, knobs are read once)
set -u
mkdir -p gpurun_out
out=gpurun_out/tune_compact.jsonl; : > $out
for cfg in "${@:-PB_LINES_TL=16}"; do
  env $cfg timeout -k 10 120 python scripts/tune_compact.py ${N:-512} >> $out 2>> gpurun_out/tune_compact.err
  rc=$?; [ $rc -ne 0 ] && { echo "cfg $cfg rc=$rc"; exit $rc; }
done
cat $out
