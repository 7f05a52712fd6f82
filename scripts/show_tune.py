import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"):
        continue
    r = json.loads(l)
    print(f"{json.dumps(r['cfg']):50s} mv {r['mv_med_ms']:.3f} ({r['mv_GBps_med']:4.0f}) "
          f"A {r['a_med_ms']:.3f} ({r['a_GBps_med']:4.0f}) B {r['b_med_ms']:.3f} "
          f"Be {r['be_med_ms']:.3f} | iter {r['it_min_ms']:.3f}/{r['it_med_ms']:.3f} ms")
