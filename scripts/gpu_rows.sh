#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/bench_rows.py > gpurun_out/rows.jsonl 2> gpurun_out/rows.err
rc=$?; echo "rows rc=$rc"; tail -3 gpurun_out/rows.err; exit $rc
