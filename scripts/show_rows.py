"""Pretty-print the JSON lines of scripts/bench_rows.py."""
import json
import sys

for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rows.jsonl"):
    r = json.loads(line)
    c = r.get("cpu", {})
    cpu = c.get("dofs_per_s_1core", c.get("7term_dofs_per_s_1core", 0))
    print(f"{r['row']:6s} {r['kernel'][:46]:46s} {r['size']:12s} {r['avg_ms']:9.3f} ms "
          f"{r['GBps']:7.0f} GB/s {r['frac_of_8TBps'] * 100:5.1f}% | {r['dofs_per_s']:.3g} DoF/s"
          f" | cpu {cpu:.3g}")
