import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"):
        continue
    r = json.loads(l)
    print(f"{json.dumps(r['cfg']):60s} mv {r['mv_min_ms']:.3f}/{r['mv_med_ms']:.3f} ({r['mv_GBps_med']:4.0f})  "
          f"A {r['a_min_ms']:.3f}/{r['a_med_ms']:.3f} ({r['a_GBps_med']:4.0f})  "
          f"B {r['b_min_ms']:.3f}/{r['b_med_ms']:.3f} ({r['b_GBps_med']:4.0f})")
