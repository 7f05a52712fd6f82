"""Slow / fast process modes of the streaming kernels: one process runs 40
KSPSolve_CG iterations and 20 matvecs at 512^3; scripts/gpu_modes.sh runs it as several processes
under rocprofv3 --kernel-trace --pmc with the L2 -> fabric request, outstanding-level and DRAM
credit-stall counters, so per-dispatch durations and counters line up by process."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poissbox_amd as pb  # noqa: E402

ctx = pb.Context(0)
da = pb.DA(ctx, (512, 512, 512))
P, A, x, b = pb.initialise_linear_system(da, da.spacing)
xt = pb.Vec(da)
xt.set_random(20231015)
A.mult(xt, b)
k = pb.KSP(A, P, pb.ksp_options(["-ksp_type", "cg", "-pc_type", "jacobi"], rtol=0.0, atol=0.0,
                                dtol=1e300, max_it=64, check_every=8))
k.begin(b, x)
k.iterate(40)
ctx.sync()
y = pb.Vec(da)
for _ in range(20):
    A.mult(xt, y)
ctx.sync()
k.end()
print("ok", flush=True)
