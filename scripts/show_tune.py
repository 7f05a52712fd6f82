import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
last = max(r["round"] for r in rows)
for r in rows:
    if r["round"] == last:
        print(f"TY={r['ty']} blocks={r['blocks']:5d}  mv {r['mv_ms']:.3f} ms {r['mv_GBps']:5.0f}  "
              f"A {r['a_ms']:.3f} {r['a_GBps']:5.0f}  B {r['b_ms']:.3f} {r['b_GBps']:5.0f}")
