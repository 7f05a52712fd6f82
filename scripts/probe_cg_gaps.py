"""Kernel trace of plain CG iterations (no HIP-event timing at all) at n^3 (argv[1], default 512):
run under rocprofv3 --kernel-trace, then `python scripts/probe_cg_gaps.py --gaps <kernel_trace.csv>`
prints the per-iteration kernel time and the idle gaps between consecutive launches."""
import csv
import os
import sys

if len(sys.argv) > 2 and sys.argv[1] == "--gaps":
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"].split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
           for r in rows]
    ia = [i for i, s in enumerate(seq) if "PassAT" in s[0]]
    a, b = ia[len(ia) // 4], ia[len(ia) // 4 + 40]  # 40 iterations from the steady state
    busy = sum(e - s for _, s, e in seq[a:b]) / 1e3
    span = (seq[b][1] - seq[a][1]) / 1e3
    gaps = {}
    for j in range(a, b):
        nm = seq[j][0].split("pb::")[-1][:40]
        gaps.setdefault(nm, []).append((seq[j + 1][1] - seq[j][2]) / 1e3)
    print(f"40 iterations: span {span:.1f} us, kernels busy {busy:.1f} us, idle {span - busy:.1f} us "
          f"({(span - busy) / 40:.2f} us per iteration)")
    for nm, g in gaps.items():
        print(f"  after {nm:40s} mean gap {sum(g) / len(g):6.2f} us over {len(g)}")
    sys.exit(0)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

ctx = pb.Context(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
da = pb.initialise_grid(ctx, (n, n, n))
P, A, x, b = pb.initialise_linear_system(da, da.spacing)
xt = pb.Vec(da)
xt.set_random(1)
A.mult(xt, b)
k = pb.KSP(A, P, pb.ksp_options(["-ksp_type", "cg", "-pc_type", "jacobi"], rtol=0.0, atol=0.0,
                                dtol=1e300, max_it=200))
k.begin(b, x)
k.iterate(120)
ctx.sync()
k.end()
