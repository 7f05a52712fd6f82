#!/bin/bash
# per-row bench (scripts/bench_rows.py) alone, summary printed
set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/bench_rows.py > gpurun_out/rows_wall.jsonl 2> gpurun_out/rows_wall.err
rc=$?
python3 - <<'PY'
import json
for l in open("gpurun_out/rows_wall.jsonl"):
    d = json.loads(l)
    print(d["row"], d["kernel"][:45], d["size"], round(d["avg_ms"], 4), round(d["frac_of_8TBps"], 3))
PY
exit $rc
