"""why the row bench (scripts/bench_rows.py) timed the 512^3 matvec at
0.423 ms while the §8(d) protocol (scripts/bench_protocol.py) timed 0.369 ms on the same box.
One process, the harnesses in sequence on the same operator and vectors, HIP events per launch:
  r03_rows   -- the r03 row bench: first GPU work of the process, 1 warm-up, 20 timed launches;
  rows_now   -- bench_rows.timed() as fixed: 0.5 s of warm-up launches, 100 timed;
  protocol   -- 10 warm-ups, 100 timed, 5 repetitions (median).
Per-launch samples (first / last 5) show whether the gap is a warm-up transient."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

ctx = pb.Context(0)
da = pb.DA(ctx, (512, 512, 512))
A = pb.Mat(da, pb.STAR7)
x, y = pb.Vec(da), pb.Vec(da)
x.set_random(1)


def run(tag, warm, reps, warm_s=0.0):
    for _ in range(warm):
        A.mult(x, y)
    ctx.sync()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(8):
            A.mult(x, y)
        ctx.sync()
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(reps):
        A.mult(x, y)
    ctx.sync()
    s = [float(v) for v in ctx.timing_samples("stencil")]
    ctx.set_timing(False)
    out = {"harness": tag, "avg_ms": sum(s) / len(s), "median_ms": statistics.median(s),
           "first5": [round(v, 4) for v in s[:5]], "last5": [round(v, 4) for v in s[-5:]]}
    print(json.dumps(out), flush=True)
    return out


run("r03_rows", 1, 20)
run("rows_now", 1, 100, warm_s=0.5)
for _ in range(5):
    run("protocol", 10, 100)
run("r03_rows_again", 1, 20)
