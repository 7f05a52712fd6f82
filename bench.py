"""Benchmark: periodic 3-D Poisson CG (-ksp_type cg -pc_type jacobi, constant null space) at 512^3
fp64 per GPU -- BASELINE.json metric "CG iter/s and DoF-updates/s at 512^3; achieved HBM GB/s".

A step = one CG iteration over every DoF of the grid (one pass of the KSPSolve hot path).
Weak scaling: every GPU owns a 512^3 z-slab worth of DoF; the global grid doubles z, y, x in turn
(N=1: 512^3, N=2: 512x512x1024, N=4: 512x1024x1024, N=8: 1024^3 = SURVEY config 4).
Strong scaling (--scaling strong [--base 512|1024]): the base^3 grid split over all GPUs.
N > 1 lines carry per-rank halo / allreduce times (per_rank_comm).
Launch: python bench.py [--gpus N --steps K --warmup W]. For N > 1 either under
torch.distributed.run (one rank per GPU), or plain: with no WORLD_SIZE in the environment
bench.py starts the N rank processes itself (self_launch: child processes, no exec, before any
GPU call) and relays rank 0's line. RCCL unique id broadcast over the gloo process group; the line
records the transport and the size of the RCCL communicator as RCCL reports it (rccl_nranks).
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X spec (MI355X_MICROARCH.md "Chip-level parameters")
PASS_B_X_NAME = {0: "cg_pass_b", 2: "cg_pass_b_odd", 4: "cg_pass_b_x4"}
# Algorithmic bytes per DoF of each CG pass (Jacobi / none on the fused operator, pb_solver.cpp):
# pass A reads r, p_old (16, p.Ap only); pass B re-forms p from r, p_old, writes p and r into the
# other residual buffer (32); the x update every D-th iteration (cg_defer_x = D, default 4) adds x
# read / write and p_{i-2} .. p_{i-D+1} (p_{i-1} = p_old is already in the z-queue)
PASS_BYTES = {1: {"a": 16, "b_even": 32, "b_x": {0: 48, 2: 48, 4: 64}}}
MATVEC_BYTES = 16            # y = A x: read x, write y
# single-reduction CG (-ksp_cg_single_reduction, pb_solver.cpp enqueue_sr_iteration): pass P reads
# r, p_old and writes p, r' (32; + x read / write and p_{i-2}, p_{i-3} every 4th iteration: 64);
# pass S reads r' (8): 32 + 8 + 32/4 = 48 B/DoF per iteration at D = 4. One rank: the one-pass
# kernel (pb_cg_sr.hip, reads r, p_old, writes p, r': 32) on the 3 iterations of 4 that carry no
# x update, pass P + pass S on the 4th: (3 * 32 + 64 + 8) / 4 = 42 B/DoF
SR_BYTES = {"p": 32, "p_x4": 64, "s": 8, "sr1": 32}
SR_ITER_BYTES = SR_BYTES["p"] + SR_BYTES["s"] + (SR_BYTES["p_x4"] - SR_BYTES["p"]) / 4


def memory_clock():
    """The memory clock level in use per card (sysfs pp_dpm_mclk, the level marked '*'), read
    without starting a program (no rocm-smi: under rocprofv3 a child would re-exec), or None."""
    import glob
    import re
    res = {}
    for f in sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_mclk")):
        try:
            for line in open(f):
                if "*" in line:
                    m = re.search(r"(\d+)\s*Mhz", line, re.I)
                    res[f.split("/")[4]] = int(m.group(1)) if m else line.strip()
        except Exception:
            pass
    return res or None


def cg_iter_bytes(defer, pstore=1):
    """Algorithmic bytes per DoF of one CG iteration, averaged over a deferral cycle (56 at D = 4
    with p stored by pass B, 58 with p stored by pass A; SURVEY §8d's fused 2-pass lower bound
    without deferral is 80)."""
    pb_ = PASS_BYTES[pstore]
    if defer == 0:
        return pb_["a"] + pb_["b_x"][0]
    return pb_["a"] + ((defer - 1) * pb_["b_even"] + pb_["b_x"][defer]) / defer
SEED = 20231015
SECONDARY_TIMEOUT_STATUS = 3  # exit status when the secondary workloads' watchdog fires


def nloc_even(n):
    return n - (n % 2)


def sustained_median_ms(samples):
    return float(np.median(samples)) if len(samples) else None


def run_sr_variant(args, pb, ctx, A, P, b, da, dist, world):
    """The single-reduction iteration (-ksp_cg_single_reduction: one reduction per iteration; one
    pass on 3 of 4 iterations on one rank, 42 B/DoF; 2 passes, 48 B/DoF, on N ranks)
    on the same system, same protocol as the headline (W untimed, K timed between barriers, max
    over ranks), then 16 iterations with every pass timed. A stated variant line: the headline
    stays PETSc's default KSPSolve_CG."""
    x = pb.Vec(da)
    opts = pb.ksp_options(["-ksp_type", "cg", "-pc_type", "jacobi", "-ksp_cg_single_reduction"],
                          rtol=0.0, atol=0.0, dtol=1e300, max_it=args.warmup + args.steps + 32,
                          check_every=8)
    ksp = pb.KSP(A, P, opts)
    ksp.begin(b, x)
    ksp.iterate(args.warmup)
    ctx.barrier()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    ksp.iterate(args.steps)
    ctx.sync()
    elapsed = time.perf_counter() - t0
    ctx.barrier()
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ctx.set_timing(True)
    ctx.reset_timing()
    ksp.iterate(16)
    ctx.sync()
    passes = {}
    nloc = da.nlocal
    iter_bytes = 0.0  # bytes per DoF per iteration, from the passes the 16 iterations ran
    for nm, key in (("cg_sr1", "sr1"), ("cg_sr_p", "p"), ("cg_sr_p_x4", "p_x4"), ("cg_sr_s", "s")):
        ms, cnt = ctx.timing(nm)
        if cnt:
            t_ = ms / cnt / 1e3
            gb = SR_BYTES[key] * nloc / t_ / 1e9
            passes[nm] = {"avg_ms": t_ * 1e3, "GBps": gb, "frac": gb / HBM_PEAK_GBS,
                          "bytes_per_dof": SR_BYTES[key], "launches": cnt}
            iter_bytes += SR_BYTES[key] * cnt / 16
    iter_bytes = iter_bytes or SR_ITER_BYTES
    ctx.set_timing(False)
    reason, its, hist = ksp.end()
    ksp.destroy()
    x.destroy()
    N = int(np.prod(da.n))
    per_step = elapsed / args.steps
    return {"ksp": "-ksp_type cg -pc_type jacobi -ksp_cg_single_reduction (PETSc "
                   "KSPSolve_CG_SingleReduction: z'z, z'r, z'Az in one reduction)",
            "ms_per_step": per_step * 1e3, "iter_per_s": 1.0 / per_step,
            "value": (N * args.steps / elapsed) if N else None, "unit": "DoF-updates/s",
            "bytes_per_dof": iter_bytes,
            "achieved_GBps": iter_bytes * nloc / per_step / 1e9 if nloc else None,
            "passes": passes, "its": its, "rnorm_last": float(hist[-1])}


def global_grid(ngpus, base=512):
    n = [base, base, base]
    k = ngpus
    d = 2
    while k > 1 and k % 2 == 0:
        n[d] *= 2
        d = (d - 1) % 3
        k //= 2
    n[2] *= k  # non power-of-two remainder goes to z
    return tuple(n)


def host_info():
    """nproc / lscpu of the host the CPU baseline runs on (record both), and the
    cores this process may use: its CPU affinity, the cgroup quota and OMP_NUM_THREADS (the GPU
    box exports its per-GPU CPU share there) -- the machine's total is usually larger."""
    import subprocess
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = -(-int(q) // int(per))
    except Exception:
        pass
    info["cgroup_cpus"] = quota
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    for cmd, key in ((["nproc"], "nproc"), (["lscpu"], "lscpu")):
        try:
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=10).stdout
        except Exception:
            out = ""
        if key == "nproc":
            info["nproc"] = int(out.strip()) if out.strip().isdigit() else None
        else:
            keep = ("Model name", "CPU(s)", "Thread(s) per core", "Core(s) per socket",
                    "Socket(s)", "NUMA node(s)", "L3 cache", "CPU max MHz")
            info["lscpu"] = {k.strip(): v.strip() for k, v in
                             (l.split(":", 1) for l in out.splitlines() if ":" in l)
                             if k.strip() in keep}
    usable = [info["affinity"] or 1]
    if quota:
        usable.append(quota)
    if (info["omp_num_threads"] or "").isdigit():
        usable.append(int(info["omp_num_threads"]))
    info["usable_cores"] = max(1, min(usable))
    try:
        pv = subprocess.run(["pkg-config", "--modversion", "petsc"], capture_output=True,
                            text=True, timeout=10)
        info["petsc"] = pv.stdout.strip() if pv.returncode == 0 else "absent (pkg-config petsc fails)"
    except Exception:
        info["petsc"] = "absent (no pkg-config)"
    return info


def _cpu_row(O, n, rtol, max_it, threads):
    """One CPU-baseline row: the oracle's PETSc-sequence CG + Jacobi (constant null space) on the
    §8(d) synthetic system, to convergence (rtol > 0) or for a fixed max_it iterations."""
    N = n ** 3
    h = (1.0 / n,) * 3
    b = O.stencil(O.fill_random(N, SEED), (n, n, n), h, nthreads=threads)
    t0 = time.perf_counter()
    x, reason, its, hist = O.cg_solve(b, (n, n, n), h, rtol=rtol, atol=0.0 if rtol == 0 else 1e-50,
                                      dtol=1e300 if rtol == 0 else 1e5, max_it=max_it,
                                      nthreads=threads)
    el = time.perf_counter() - t0
    r = O.stencil(x, (n, n, n), h, nthreads=threads) - b
    row = {"grid": f"{n}^3", "cores": threads, "rtol": rtol, "its": its,
           "reason": reason, "seconds": el, "iter_per_s": its / el,
           "dofs_updates_per_s": N * its / el,
           "GBps_at_80B": 80 * N * its / el / 1e9, "GBps_at_176B": 176 * N * its / el / 1e9,
           "true_residual": float(np.linalg.norm(r)),
           "true_residual_rel": float(np.linalg.norm(r) / np.linalg.norm(b)),
           "rnorm_last": float(hist[-1])}
    del b, x, r
    return row


def cpu_variants(threads, iters=100):
    """SURVEY §8(d)'s other CPU rows, a few seconds each on 128^3: the optimised 7-point CG on
    one core, and the reference-faithful operator (27-term pointwise dot product per point, as
    src/poissbox.f90:128-148 evaluates it) on one core and on all of them. Fixed iteration
    count (rtol = atol = 0), the same PETSc scalar sequence."""
    from oracle import oracle as O
    n = (128, 128, 128)
    N = 128 ** 3
    h = (1 / 128,) * 3
    b = O.stencil(O.fill_random(N, SEED), n, h, nthreads=threads)
    out = []
    for faithful, nt in ((False, 1), (True, 1), (True, threads)):
        k = iters if not faithful or nt > 1 else iters // 4
        t0 = time.perf_counter()
        _, _, its, _ = O.cg_solve(b, n, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=k,
                                  faithful=faithful, nthreads=nt)
        el = time.perf_counter() - t0
        out.append({"op": "faithful 27-term" if faithful else "7-point", "cores": nt,
                    "value": N * its / el, "unit": "DoF-updates/s",
                    "sample": f"128^3 grid, {its} CG + Jacobi iterations (+setup) in {el:.2f} s"})
    return out


def cpu_baseline(mode="full"):
    """SURVEY.md §8(d) / BASELINE.md §4 CPU baseline, timed on this host: the oracle's C
    restatement of PETSc KSPCG + PCJacobi + MatNullSpace (7-point, OpenMP) -- PETSc itself is
    absent from the image -- on all usable cores and on 1 core: 64^3 to rtol 1e-5 and 1e-10,
    256^3 to rtol 1e-10, 512^3 for a fixed 50 iterations (the headline `value`, the same
    workload as the GPU line). mode "quick" keeps only the 512^3 rows (10 iterations on 1 core)."""
    from oracle import oracle as O
    info = host_info()
    T = int(os.environ.get("PB_CPU_THREADS", info["usable_cores"]))
    budget = float(os.environ.get("PB_CPU_BUDGET_S", "300"))
    rows, skipped = [], []
    # headline row first; then the rest, each skipped if its predicted time (from the measured
    # rate of the same core count) would overrun the budget
    plan = [(512, 0.0, 50, T)]
    if mode == "full":
        plan += [(64, 1e-5, 10000, T), (64, 1e-10, 10000, T), (64, 1e-5, 10000, 1),
                 (64, 1e-10, 10000, 1), (256, 1e-10, 10000, T), (512, 0.0, 50, 1),
                 (256, 1e-10, 10000, 1)]
    else:
        plan += [(512, 0.0, 10, 1)]
    t_start = time.perf_counter()
    for n, rtol, max_it, t in plan:
        rate = [r["dofs_updates_per_s"] for r in rows if r["cores"] == t]
        est_its = max_it if rtol == 0 else 2.8 * n  # ~2.8 n its to rtol 1e-10
        est = n ** 3 * est_its / min(rate) if rate else 0.0
        if time.perf_counter() - t_start + est > budget:
            skipped.append(f"{n}^3 rtol={rtol} cores={t} (predicted {est:.0f} s over the "
                           f"{budget:.0f} s budget)")
            continue
        rows.append(_cpu_row(O, n, rtol, max_it, t))
        print(f"cpu baseline row: {json.dumps(rows[-1])}", file=sys.stderr, flush=True)
    head = [r for r in rows if r["grid"] == "512^3" and r["cores"] == T][0]
    return {"value": head["dofs_updates_per_s"], "unit": "DoF-updates/s", "cores": T,
            "kind": "port", "iter_per_s": head["iter_per_s"],
            "sample": f"512^3 grid, {head['its']} CG + Jacobi iterations (fixed count) of "
                      f"oracle/pb_oracle.c (PETSc KSPCG+PCJacobi+MatNullSpace sequence, 7-point, "
                      f"OpenMP {T} threads) in {head['seconds']:.1f} s on the GPU box host; "
                      f"rows: 64^3 and 256^3 to convergence and 512^3 x 50 its, on {T} cores "
                      f"and on 1",
            "host": info, "rows": rows, "skipped_rows": skipped, "variants": cpu_variants(T)}


# Workloads measured by whole solves (--workload): a step is one KSPSolve to rtol 1e-10 from x0 = 0
# (the solves take 1-13 iterations, so a fixed-iteration step would run past convergence).
#   compact-fft: BASELINE config 5's operator -- the compact-scheme Laplacian as A = P
#     (src/compact_schemes.f90:17-37, A != 7-point as src/poissbox.f90:226-228,294) -- with the
#     spectral -pc_type fft that inverts its symbol (the substitute for the V-cycle of
#     config 5's text, which cannot precondition the compact operator's Nyquist null modes);
#     default strong scaling of 512^3 (config 5: 512^3 on 8 GPUs).
#   star7-mg: the README's recommended solver shape (README.md:40-45, CG + multigrid with SOR
#     smoothing) on the 7-point operator: -pc_type mg, geometric V(1,1) red-black SOR; weak scaling.
# roofline: the kernel, its algorithmic bytes per owned DoF (N = 1 / N > 1: on a split grid MG's
# post-smoothing runs as prolongation 17 + fused sweep 24) and a description.
SOLVE_WORKLOADS = {
    "compact-fft": {
        "ops": ("compact", "compact"),
        "argv": ["-ksp_type", "cg", "-pc_type", "fft", "-ksp_rtol", "1e-10"],
        "scaling": "strong",
        "roof": ("pc_fft_z", (16, 16),
                 "pc_fft_z (spectral PC Z pass: forward FFT of z-lines, 1/(N lambda) of the compact "
                 "symbol, inverse FFT; read + write 16 B/DoF; on N > 1 ranks on y-slabs)"),
        # (the PC's X passes also carry CG's x / r update and residual sums: no fixed bytes)
        "kernels": {"pc_fft_x": None, "pc_fft_y": 16, "pc_fft_z": 16, "compact_lines_x": None,
                    "compact_lines_y": None, "compact_lines_z": None, "pc_fft": None,
                    "alltoallv": None, "allreduce": None},
        "describe": "fp64 CG, compact-scheme Laplacian A = P (src/compact_schemes.f90:17-37), "
                    "spectral PC (-pc_type fft), rtol 1e-10",
    },
    "star7-mg": {
        "ops": ("star7", "assembled"),
        "argv": ["-ksp_type", "cg", "-pc_type", "mg", "-ksp_rtol", "1e-10"],
        "scaling": "weak",
        "roof": ("mg_fine_prolong_post", (25, 41),
                 "mg_fine_prolong_post (finest level: prolongation + correction + both red-black "
                 "SOR post-smoothing half-sweeps; 25 B/DoF fused on one rank, 17 + 24 on a split "
                 "grid)"),
        "kernels": {"mg_apply": None, "mg_fine_smooth_first": 17, "mg_fine_prolong_post": None,
                    "mg_coarse_levels": None, "cg_pass_a": None, "cg_pass_b": None,
                    "halo": None, "allreduce": None},
        "describe": "fp64 CG + geometric multigrid V(1,1), red-black SOR smoothing "
                    "(-pc_type mg), 7-pt periodic Laplacian, rtol 1e-10",
    },
}


def cpu_solve_baseline(workload, budget_s=None, m=128):
    """cpu_baseline of a solve workload: the oracle's restatement of the same KSPSolve (PETSc
    KSPCG sequence + the same preconditioner) on a grid it finishes in seconds (128^3), repeated
    for about budget_s (PB_CPU_BUDGET_S, default 20 s) on the GPU box's host cores."""
    from oracle import oracle as O
    info = host_info()
    T = int(os.environ.get("PB_CPU_THREADS", info["usable_cores"]))
    budget = budget_s or float(os.environ.get("PB_CPU_SOLVE_BUDGET_S", "20"))
    n3 = (m, m, m)
    N = m ** 3
    h = (1.0 / m,) * 3
    xt = O.fill_random(N, SEED)
    if workload == "compact-fft":
        b = O.lapl(xt, n3, h)
        kw = dict(pc="fft", op="compact")
        what = ("compact lapl in the reference's operation order (1 thread) + spectral PC "
                f"(naive Hartley sums, OpenMP {T} threads)")
    else:
        b = O.stencil(xt, n3, h, nthreads=T)
        kw = dict(pc="mg", nthreads=T)
        what = "7-point CG + geometric MG V(1,1) red-black SOR (the pb_mg.hip restatement)"
    kw.setdefault("nthreads", T)
    solves, its_total, el = 0, 0, 0.0
    reason = None
    while el < budget or solves == 0:
        t0 = time.perf_counter()
        _, reason, its, _ = O.cg_solve(b, n3, h, rtol=1e-10, **kw)
        el += time.perf_counter() - t0
        solves += 1
        its_total += its
    return {"value": N * its_total / el, "unit": "DoF-updates/s", "cores": T, "kind": "port",
            "solves_per_s": solves / el, "its_per_solve": its_total / solves,
            "reason": reason, "host": info,
            "sample": f"{m}^3 grid, {solves} solve(s) to rtol 1e-10 of oracle/pb_oracle.c "
                      f"({what}; PETSc KSPCG sequence, constant null space) in {el:.1f} s on the "
                      f"GPU box host"}


def dominant_kernel(kern, s_per_solve):
    """The phase with the largest time per solve among the timed kernels (the roofline kernel is
    the one with fixed algorithmic bytes; for config 5 the PC's X passes take more time but carry
    CG's x / r update and residual sums, so their bytes per launch vary)."""
    best = None
    for nm, row in kern.items():
        if nm in ("pc_fft", "mg_apply", "alltoallv", "allreduce", "halo", "halo_comm"):
            continue  # (wrappers of other phases, communication)
        t = row["avg_ms"] * row["launches_per_solve"]
        if best is None or t > best[1]:
            best = (nm, t, row)
    if best is None:
        return None
    nm, t, row = best
    return {"name": nm, "ms_per_solve": t, "share_of_solve": t / (s_per_solve * 1e3),
            "avg_launch_ms": row["avg_ms"], "launches_per_solve": row["launches_per_solve"],
            "frac": row.get("frac")}


def workload_grid(workload, scaling, world, base):
    return global_grid(world, base) if scaling == "weak" else (base,) * 3


def run_solve_workload(args, pb, ctx, workload, scaling, steps, warmup, rank, world, dist,
                       comm_transport, comm_nranks, cpu_budget_s=None):
    """One step = one KSPSolve to rtol 1e-10 (SOLVE_WORKLOADS). Timed region: K solves after W
    warm-up solves, barrier + device sync on both sides, max over ranks. HIP events bracket only
    the roofline kernel inside it; the other kernels are timed in one further solve. Returns the
    JSON object on rank 0 (None elsewhere)."""
    W = SOLVE_WORKLOADS[workload]
    n = args.grid_override or workload_grid(workload, scaling, world, args.base)
    da = pb.initialise_grid(ctx, n)
    h = da.spacing
    kinds = {"compact": pb.COMPACT, "star7": pb.STAR7, "assembled": pb.ASSEMBLED27}
    A = pb.Mat(da, kinds[W["ops"][0]], h)
    P = A if W["ops"][1] == W["ops"][0] else pb.Mat(da, kinds[W["ops"][1]], h)
    x, b, xt = pb.Vec(da), pb.Vec(da), pb.Vec(da)
    xt.set_random(SEED)      # synthetic x_true, decomposition independent
    A.mult(xt, b)            # b = A x_true (src/example.f90:70-72)
    ksp = pb.KSP(A, P, pb.ksp_options(W["argv"]))
    for _ in range(warmup):
        ksp.solve(b, x)
    roof, roof_bytes_np, roof_desc = W["roof"]
    roof_bytes = roof_bytes_np[0] if world == 1 else roof_bytes_np[1]
    ctx.sync()
    ctx.barrier()
    if dist:
        dist.barrier()
    ctx.set_timing(True, only=roof, every=1)
    ctx.reset_timing()
    its_seen = []
    t0 = time.perf_counter()
    for _ in range(steps):
        reason, its, hist = ksp.solve(b, x)
        its_seen.append(its)
    ctx.sync()
    t1 = time.perf_counter()
    ctx.barrier()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    ms_roof, cnt_roof = ctx.timing(roof)
    ctx.set_timing(False)
    # diagnostics: one more solve with every phase timed
    ctx.set_timing(True)
    ctx.reset_timing()
    ksp.solve(b, x)
    ctx.sync()
    nloc = da.nlocal
    kern = {}
    comm = {"rank": rank, "device": ctx_device(ctx), "transport": comm_transport,
            "comm_nranks": comm_nranks}
    for nm, bpd in W["kernels"].items():
        ms_, cnt_ = ctx.timing(nm)
        if cnt_ == 0:
            continue
        row = {"avg_ms": ms_ / cnt_, "launches_per_solve": cnt_}
        if bpd:
            t_ = ms_ / cnt_ / 1e3
            row.update(GBps=bpd * nloc / t_ / 1e9, frac=bpd * nloc / t_ / 1e9 / HBM_PEAK_GBS,
                       bytes_per_dof=bpd)
        kern[nm] = row
        if nm in ("alltoallv", "allreduce", "halo", "halo_comm"):
            comm[f"{nm}_ms_per_solve"] = ms_
            comm[f"{nm}_calls"] = cnt_
    ctx.set_timing(False)
    if roof in kern and "frac" not in kern[roof]:  # the roofline kernel's fixed bytes
        t_ = kern[roof]["avg_ms"] / 1e3
        roof_bpd = roof_bytes_np[0] if world == 1 else roof_bytes_np[1]
        kern[roof].update(GBps=roof_bpd * nloc / t_ / 1e9,
                          frac=roof_bpd * nloc / t_ / 1e9 / HBM_PEAK_GBS, bytes_per_dof=roof_bpd)
    if workload == "compact-fft" and "pc_fft_x" in kern:
        # the spectral PC's X passes carry CG's work, so their bytes differ by role, but each
        # solve's are fixed: per PC apply a forward X pass (16 B/DoF: r in,
        # z out) and an inverse one taking the residual sums (24: z, r in, z out); on the
        # iterations' applies (x / r update fused, pb_solver.cpp enqueue_pc_iteration, planes
        # 512 / 1024 wide) the forward pass also reads w, p and x (not on the first) and stores
        # r and x: 48 (first iteration, x0 = 0) or 56
        its_d = int(its_seen[-1]) if its_seen else 0
        fused = n[0] in (512, 1024) and n[1] % 2 == 0 and pb.tune_get("fft_rupd") != 0
        bpd_it = [(48 if i == 0 else 56) if fused else 16 for i in range(its_d)]
        bpd_solve = 16 + 24 + sum(b_ + 24 for b_ in bpd_it)
        row = kern["pc_fft_x"]
        if row["launches_per_solve"] == 2 + 2 * its_d:
            t_ = row["avg_ms"] * row["launches_per_solve"] / 1e3
            row.update(bytes_per_dof_per_solve=bpd_solve, GBps=bpd_solve * nloc / t_ / 1e9,
                       frac=bpd_solve * nloc / t_ / 1e9 / HBM_PEAK_GBS)
    # true residual of the last solve: ||b - A x|| / ||b||
    r = pb.Vec(da)
    A.mult(x, r)
    r.axpy(-1.0, b)
    rel = r.norm() / b.norm()
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, comm)
    else:
        per_rank = [comm]
    t_roof = ms_roof / max(cnt_roof, 1) / 1e3
    achieved = roof_bytes * nloc / t_roof / 1e9 if t_roof > 0 else 0.0
    N = n[0] * n[1] * n[2]
    its_total = int(sum(its_seen))
    out = None
    if rank == 0:
        out = {
            "metric": "CG iter/s and DoF-updates/s at 512^3; achieved HBM GB/s vs peak",
            "value": N * its_total / elapsed,
            "unit": "DoF-updates/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.grid_override else scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (x_true = SplitMix64 U[-1,1], b = A x_true, x0 = 0)",
            "config": {"workload": f"{W['describe']}, {n[0]}x{n[1]}x{n[2]} grid",
                       "workload_key": workload,
                       "step": "one KSPSolve to rtol 1e-10 from x0 = 0",
                       "grid": list(n), "global_dofs": N, "per_gpu_dofs": nloc,
                       "parallelism": f"z-slab x{world}" + (
                           f" ({'RCCL' if args.transport == 'rccl' else 'gloo host'})"
                           if world > 1 else ""),
                       "ksp": " ".join(W["argv"]) + ", constant null space"},
            "iter_per_s": its_total / elapsed,
            "solves_per_s": steps / elapsed,
            "its_per_solve": its_total / max(steps, 1),
            "roofline": {"bound": "hbm", "kernel": roof_desc, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None, "bytes_per_dof": roof_bytes,
                         "avg_launch_ms": t_roof * 1e3, "launches_timed": cnt_roof,
                         "dominant": dominant_kernel(kern, elapsed / max(steps, 1))},
            "kernels": kern,
            "launcher": os.environ.get("PB_BENCH_LAUNCHER",
                                       "torch.distributed.run" if dist else "none"),
            "transport": comm_transport,
            "rccl_nranks": comm_nranks if comm_transport == "rccl" else None,
            "per_rank_comm": per_rank if world > 1 else None,
            "ksp_state": {"reason": pb.REASONS.get(reason, reason), "its": its,
                          "rnorm0": float(hist[0]), "rnorm_last": float(hist[-1]),
                          "true_residual_rel": rel},
        }
        traffic_file = os.path.join(REPO, "profiles", "pmc_traffic.json")
        key = f"{n[0]}x{n[1]}x{n[2]}/{workload}"
        try:
            tr = json.load(open(traffic_file)) if world == 1 else {}
            if roof in tr.get(key, {}):  # PMC bytes per launch of the roofline kernel (one GPU)
                out["roofline"]["traffic"] = tr[key][roof]["bytes_per_launch"]
                out["roofline"]["traffic_source"] = tr[key][roof].get("source")
        except Exception:
            pass
        if world == 1 and not args.no_cpu_baseline and args.cpu_baseline != "none":
            out["cpu_baseline"] = cpu_solve_baseline(workload, cpu_budget_s)
    for o in (ksp, r, xt, x, b):
        o.destroy()
    if P is not A:
        P.destroy()
    A.destroy()
    da.destroy()
    return out


def run_secondary(args, pb, ctx, rank, world, dist, comm_transport, comm_nranks, holder, json_fd):
    """The default run (star7-jacobi headline) also measures the solve workloads -- config 5
    (compact-fft, 512^3 strong-scaled) and star7-mg -- so every N of a scaling run records them
    beside the headline, under "secondary". A watchdog bounds them (PB_BENCH_SECONDARY_TIMEOUT_S,
    default 240 s): if they do not finish, rank 0 prints the headline line with the error and the
    process exits with status SECONDARY_TIMEOUT_STATUS (3), so a secondary can never cost the
    headline measurement and a launcher still sees the failure."""
    import threading
    limit = float(os.environ.get("PB_BENCH_SECONDARY_TIMEOUT_S", "240"))
    done = threading.Event()

    def fire():
        if done.is_set():
            return
        if rank == 0 and holder.get("out") is not None:
            o = dict(holder["out"])
            o.setdefault("secondary", {})["error"] = f"timed out after {limit:.0f} s"
            os.write(json_fd, (json.dumps(o) + "\n").encode())
        print(f"bench: secondary workloads timed out after {limit:.0f} s; exiting with status "
              f"{SECONDARY_TIMEOUT_STATUS}", file=sys.stderr, flush=True)
        os._exit(SECONDARY_TIMEOUT_STATUS)  # (not 0; the headline line is out)

    timer = threading.Timer(limit, fire)
    timer.daemon = True
    timer.start()
    sec = {}
    for wl, steps, warmup in (("compact-fft", 10, 2), ("star7-mg", 3, 1)):
        try:
            res = run_solve_workload(args, pb, ctx, wl, SOLVE_WORKLOADS[wl]["scaling"], steps,
                                     warmup, rank, world, dist, comm_transport, comm_nranks,
                                     cpu_budget_s=10)
        except Exception as e:  # recorded, never fatal to the headline
            res = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            for k in ("metric", "higher_is_better", "vs_baseline", "dtype", "data", "launcher",
                      "transport", "rccl_nranks"):
                res.pop(k, None)
            if "cpu_baseline" in res:
                res["cpu_baseline"].pop("host", None)
            sec[wl] = res
            holder["out"].setdefault("secondary", {})[wl] = res
    done.set()
    timer.cancel()
    return sec


def ctx_device(ctx):
    return getattr(ctx, "device", None)


def sustained_row(samples, nloc, gbs):
    """The sustained matvec row from per-launch durations (ms): average, median, and the first /
    last ten launches' averages (drift under sustained load)."""
    if not len(samples):
        return None
    s = np.asarray(samples, dtype=np.float64)
    avg = float(s.mean())
    return {"launches": int(len(s)), "avg_ms": avg, "median_ms": float(np.median(s)),
            "first10_ms": float(s[:10].mean()), "last10_ms": float(s[-10:].mean()),
            "GBps": gbs(MATVEC_BYTES, avg / 1e3), "frac": gbs(MATVEC_BYTES, avg / 1e3) / HBM_PEAK_GBS,
            "bytes_per_dof": MATVEC_BYTES}


def self_launch(nranks, argv, timeout_s=None, cmd=None):
    """`bench.py --gpus N` with no launcher in the environment (no WORLD_SIZE): start the N rank
    processes here, one per GPU, as torch.distributed.run would (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / a free MASTER_PORT). They are plain child processes started before
    this process has touched the GPU -- it never does: no HIP call, no torch import, no exec.
    Rank 0's stdout (the one JSON line) is relayed; every other child output goes to stderr.
    If a rank fails, the others get PB_BENCH_GRACE_S (30) to finish before their process groups
    are killed; the whole run is bounded by PB_BENCH_TIMEOUT_S (1800). Returns the exit status:
    0 only if every rank exited 0 and rank 0 printed its line."""
    import signal
    import socket
    import subprocess
    import threading

    timeout_s = timeout_s or float(os.environ.get("PB_BENCH_TIMEOUT_S", "1800"))
    grace_s = float(os.environ.get("PB_BENCH_GRACE_S", "30"))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PB_BENCH_LAUNCHER="self")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
        procs.append(subprocess.Popen((cmd or [sys.executable, os.path.abspath(__file__)]) + list(argv),
                                      env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr,
                                      start_new_session=True))
    lines = []
    reader = threading.Thread(target=lambda: lines.extend(
        l.decode(errors="replace") for l in procs[0].stdout), daemon=True)
    reader.start()

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass

    t0 = time.monotonic()
    failed_at, first_fail = None, 0
    while any(p.poll() is None for p in procs):
        now = time.monotonic()
        bad = [p.poll() for p in procs if p.poll() not in (None, 0)]
        if failed_at is None and bad:
            failed_at, first_fail = now, bad[0]
        if now - t0 > timeout_s or (failed_at is not None and now - failed_at > grace_s):
            print(f"bench self-launch: {'timeout' if now - t0 > timeout_s else 'a rank failed'};"
                  f" killing the remaining ranks", file=sys.stderr, flush=True)
            kill_all()
            break
        time.sleep(0.2)
    codes = [p.wait() for p in procs]
    reader.join(timeout=10)
    json_lines = [l for l in lines if l.lstrip().startswith("{")]
    for l in json_lines[-1:]:
        sys.stdout.write(l if l.endswith("\n") else l + "\n")
        sys.stdout.flush()
    if any(codes):
        print(f"bench self-launch: rank exit codes {codes}", file=sys.stderr, flush=True)
        first = first_fail or next(c for c in codes if c)  # the rank that failed first
        return first if first > 0 else 128 - first  # killed by signal s: 128 + s, as a shell
    return 0 if json_lines else 1


def dry_run(args):
    """--dry-run: the launch and the control plane only (no GPU call, no library load): every
    rank joins the gloo group and rank 0 prints one JSON line with the grid it would run and the
    ranks that joined. Lets the CPU tier check the self-launch path end to end."""
    from poissbox_amd.dist import init_from_env
    rank, world, local_rank, dist = init_from_env("gloo")
    seen = [rank]
    if dist:
        seen = [None] * world
        dist.all_gather_object(seen, (rank, local_rank, os.getpid()))
    n = global_grid(world, args.base) if args.scaling == "weak" else (args.base,) * 3
    out = {"dry_run": True, "n_gpus": world, "grid": list(n), "ranks": seen,
           "workload": args.workload, "scaling": args.scaling_eff,
           "launcher": os.environ.get("PB_BENCH_LAUNCHER", "env" if dist else "none")}
    if dist:
        dist.destroy_process_group()
    return out if rank == 0 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--base", type=int, default=512, help="per-GPU cube edge (default 512)")
    ap.add_argument("--matvecs", type=int, default=20)
    ap.add_argument("--sustained", type=int, default=100,
                    help="back-to-back matvecs of the sustained-rate row (SURVEY §8(d) (i))")
    ap.add_argument("--grid", default=None,
                    help="nx,ny,nz global grid override (diagnostics; default: weak scaling)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="weak (star7-jacobi / star7-mg default): base^3 DoF per GPU; strong "
                         "(compact-fft default): the base^3 grid split over all GPUs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline", choices=("full", "quick", "none"), default="full",
                    help="SURVEY §8(d) CPU rows: full (default), quick (512^3 only) or none")
    ap.add_argument("--transport", choices=("rccl", "host"), default="rccl",
                    help="multi-rank transport: RCCL (default) or the gloo host transport "
                         "(lets several ranks share one GPU for testing)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and join the ranks, print the plan; no GPU work")
    ap.add_argument("--workload", choices=("star7-jacobi",) + tuple(SOLVE_WORKLOADS),
                    default="star7-jacobi",
                    help="star7-jacobi (default, BASELINE configs 2-4: fixed CG + Jacobi "
                         "iterations); compact-fft (config 5: compact A = P, spectral PC, whole "
                         "solves, strong scaling by default); star7-mg (CG + MG V-cycle solves)")
    ap.add_argument("--tune", default="",
                    help="A/B runs: name=value[,name=value] tuning settings (pb_tune_set, "
                         "INTEGRATION.md) applied before the run")
    ap.add_argument("--secondary", type=int, choices=(0, 1), default=1,
                    help="default run: also measure the compact-fft (config 5) and star7-mg "
                         "solve workloads after the headline, under \"secondary\" (1, default)")
    args = ap.parse_args()
    # --scaling defaults to the workload's own (config 5 is a strong-scaling case)
    if args.scaling is None:
        args.scaling = SOLVE_WORKLOADS[args.workload]["scaling"] \
            if args.workload in SOLVE_WORKLOADS else "weak"
    args.scaling_eff = "strong" if (args.scaling == "strong" and not args.grid) else "weak"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks here (child processes; this process never touches the GPU)
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    if world != args.gpus:
        sys.exit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")

    # stdout carries exactly one JSON line (rank 0): everything else any library prints on fd 1 --
    # gloo's connection messages, RCCL's version banner -- is sent to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    if args.dry_run:
        out = dry_run(args)
        if out:
            os.write(json_fd, (json.dumps(out) + "\n").encode())
        return

    import poissbox_amd as pb
    from poissbox_amd.dist import GlooTransport, broadcast_uid, init_from_env
    for kv in filter(None, args.tune.split(",")):
        k_, v_ = kv.split("=", 1)
        pb.tune_set(k_.strip(), int(v_))

    dx = pb.tune_get("cg_defer_x")  # the solver's deferral depth (pb_solver.cpp, default 4)
    defer = 0 if dx == 0 else (2 if dx == 2 else 4)
    rank, world, local_rank, dist = init_from_env("gloo")   # control plane only
    uid = None
    device = local_rank
    if dist and args.transport == "rccl":
        uid = broadcast_uid(dist, rank, pb.comm_unique_id)
    elif dist:
        import torch
        device = local_rank % max(1, torch.cuda.device_count())

    if args.grid:
        n = tuple(int(v) for v in args.grid.split(","))
    elif args.scaling == "strong":
        n = (args.base,) * 3
    else:
        n = global_grid(world, args.base)
    ctx = pb.Context(device, rank, world, uid)
    if dist and args.transport == "host":
        tr = GlooTransport(dist)
        ctx.set_host_transport(tr.sendrecv, tr.allreduce, tr.alltoallv)
    # what the transport itself reports (RCCL: ncclCommCount / ncclCommUserRank)
    comm_transport, comm_nranks, comm_rank = ctx.comm_info()
    args.grid_override = tuple(int(v) for v in args.grid.split(",")) if args.grid else None
    if args.workload in SOLVE_WORKLOADS:
        out = run_solve_workload(args, pb, ctx, args.workload, args.scaling, args.steps,
                                 args.warmup, rank, world, dist, comm_transport, comm_nranks)
        if out:
            os.write(json_fd, (json.dumps(out) + "\n").encode())
        ctx.destroy()
        if dist:
            dist.destroy_process_group()
        return
    da = pb.initialise_grid(ctx, n)
    h = da.spacing
    P, A, x, b = pb.initialise_linear_system(da, h)
    xt = pb.Vec(da)
    xt.set_random(SEED)          # synthetic x_true, decomposition independent
    A.mult(xt, b)                # b = A x_true (src/example.f90:70-72)
    diag_steps = 16  # per-kernel diagnostics, after the timed region
    opts = pb.ksp_options(["-ksp_type", "cg", "-pc_type", "jacobi"], rtol=0.0, atol=0.0,
                          dtol=1e300, max_it=args.warmup + args.steps + diag_steps + 16,
                          check_every=8)
    ksp = pb.KSP(A, P, opts)
    ksp.begin(b, x)
    ksp.iterate(args.warmup)
    ctx.barrier()
    if dist:
        dist.barrier()
    # timed region: HIP events around the roofline kernel only, on every 4th launch (events
    # around every launch add ~2 % of gaps to the measured step; around every pass A ~0.7 %).
    # The roofline kernel is the one with the largest share of the step: pass A when it stores p
    # (cg_pstore_b = 0), otherwise pass B without the x update (3 of 4 iterations at D = 4)
    pstore = 1  # pass B stores p
    roof = "cg_pass_b_even" if (pstore and defer == 4) else "cg_pass_a"
    ctx.set_timing(True, only=roof, every=4)
    ctx.reset_timing()
    t0 = time.perf_counter()
    ksp.iterate(args.steps)
    ctx.sync()
    t1 = time.perf_counter()
    ctx.barrier()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    ms_roof, cnt_roof = ctx.timing(roof)
    ctx.set_timing(False)
    # per-kernel diagnostics of the other passes: a few more iterations, every launch timed
    ctx.set_timing(True)
    ctx.reset_timing()
    ksp.iterate(diag_steps)
    ctx.sync()
    ms_b, cnt_b = ctx.timing(PASS_B_X_NAME[defer])
    for d_, nm in PASS_B_X_NAME.items():  # the library's deferral depth, from the pass it ran
        if cnt_b == 0 and ctx.timing(nm)[1] > 0:
            defer = d_
            ms_b, cnt_b = ctx.timing(nm)
    ms_be, cnt_be = ctx.timing("cg_pass_b_even")
    ms_a, cnt_a = ctx.timing("cg_pass_a")
    # per-rank communication in the diagnostic iterations: the halo exchange on the comm stream
    # (overlapped with pass A's interior planes), the two scalar allreduces per iteration, and
    # pass A including its wait for the halo
    comm = {"rank": rank, "iterations": diag_steps, "device": device,
            "transport": comm_transport, "comm_nranks": comm_nranks, "comm_rank": comm_rank}
    for nm in ("halo_comm", "allreduce", "cg_pass_a", "halo"):
        ms_, cnt_ = ctx.timing(nm)
        comm[f"{nm}_ms_per_iter"] = ms_ / diag_steps
        comm[f"{nm}_calls"] = cnt_
    ctx.set_timing(False)
    reason, its, hist = ksp.end()
    per_rank = [comm]
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, comm)

    # standalone matvec timing (north-star target kernel), outside the timed CG region
    y = pb.Vec(da)
    for _ in range(3):
        A.mult(x, y)
    ctx.sync()
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(args.matvecs):
        A.mult(x, y)
    ctx.sync()
    ms_mv, cnt_mv = ctx.timing("stencil")
    # sustained: SURVEY §8(d) (i)'s 100 back-to-back matvecs, HIP events around each launch; the
    # first and last ten show whether the rate drifts under sustained load (clocks, heat)
    ctx.reset_timing()
    for _ in range(args.sustained):
        A.mult(x, y)
    ctx.sync()
    mv_s = ctx.timing_samples("stencil")
    ctx.set_timing(False)
    # HBM calibration in this same process: a flat copy of the matvec's
    # bytes, so a slow-mode box shows up as a slow copy too
    try:
        cp_best, cp_med = ctx.copy_probe(n=nloc_even(da.nlocal), reps=10)
    except Exception:
        cp_best = cp_med = None
    sr_var = run_sr_variant(args, pb, ctx, A, P, b, da, dist, world)

    nloc = da.nlocal
    N = n[0] * n[1] * n[2]
    t_b = ms_b / max(cnt_b, 1) / 1e3
    t_be = ms_be / max(cnt_be, 1) / 1e3
    t_a = ms_a / max(cnt_a, 1) / 1e3
    t_roof = ms_roof / max(cnt_roof, 1) / 1e3  # inside the timed region
    if roof == "cg_pass_a":
        t_a = t_roof
    else:
        t_be = t_roof
    PB = PASS_BYTES[pstore]
    roof_bytes = PB["a"] if roof == "cg_pass_a" else PB["b_even"]
    t_mv = ms_mv / max(cnt_mv, 1) / 1e3
    gbs = lambda bytes_per_dof, t: bytes_per_dof * nloc / t / 1e9 if t > 0 else 0.0

    out = None
    if rank == 0:
        out = {
            "metric": "CG iter/s and DoF-updates/s at 512^3; achieved HBM GB/s vs peak",
            "value": N * args.steps / elapsed,
            "unit": "DoF-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling_eff,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (x_true = SplitMix64 U[-1,1], b = A x_true, x0 = 0)",
            "config": {"workload_key": "star7-jacobi",
                       "workload": f"fp64 CG + Jacobi, 7-pt periodic Laplacian, "
                                   f"{n[0]}x{n[1]}x{n[2]} grid ({args.base}^3 DoF per GPU)",
                       "grid": list(n), "global_dofs": N, "per_gpu_dofs": nloc,
                       "parallelism": f"z-slab x{world}" + (
                           f" ({'RCCL' if args.transport == 'rccl' else 'gloo host'} halo + allreduce)"
                           if world > 1 else ""),
                       "ksp": "-ksp_type cg -pc_type jacobi, constant null space, rtol=0 (fixed iterations)"},
            "iter_per_s": args.steps / elapsed,
            "achieved_GBps_cg": cg_iter_bytes(defer, pstore) * N / (elapsed / args.steps) / 1e9,
            "cg_bytes_per_dof": cg_iter_bytes(defer, pstore),
            "cg_pstore_b": pstore,
            # the dominant kernel (largest share of the step), timed with HIP events inside the
            # timed region
            "roofline": {"bound": "hbm",
                         "kernel": ("cg_pass_b_even (p = z + beta p_old re-formed on load, 7-point "
                                    "stencil of p, r -= alpha A p, store p and r, residual sums)"
                                    if roof == "cg_pass_b_even" else
                                    "cg_pass_a (p = z + beta p_old fused into the 7-point stencil "
                                    "of p, p.Ap sums" + (", store p)" if not pstore else ")")),
                         "achieved": gbs(roof_bytes, t_roof), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs(roof_bytes, t_roof) / HBM_PEAK_GBS,
                         "traffic": None, "bytes_per_dof": roof_bytes,
                         "avg_launch_ms": t_roof * 1e3,
                         # the north-star kernel (standalone 7-point matvec, 16 B/DoF) and this
                         # process's flat-copy calibration of the same bytes, in the roofline
                         # object (the driver keeps it)
                         "matvec_ms": t_mv * 1e3,
                         "matvec_frac": gbs(MATVEC_BYTES, t_mv) / HBM_PEAK_GBS,
                         "matvec_sustained_median_ms": sustained_median_ms(mv_s),
                         "copy_probe_GBps": cp_best, "copy_probe_median_GBps": cp_med,
                         "copy_probe_frac": (cp_best / HBM_PEAK_GBS) if cp_best else None,
                         "mclk_MHz": memory_clock()},
            "kernels": {
                "cg_pass_a": {"avg_ms": t_a * 1e3, "GBps": gbs(PB["a"], t_a),
                              "frac": gbs(PB["a"], t_a) / HBM_PEAK_GBS, "bytes_per_dof": PB["a"]},
                "cg_pass_b_even": {"avg_ms": t_be * 1e3, "GBps": gbs(PB["b_even"], t_be),
                                   "frac": gbs(PB["b_even"], t_be) / HBM_PEAK_GBS,
                                   "bytes_per_dof": PB["b_even"]},
                PASS_B_X_NAME[defer]: {"avg_ms": t_b * 1e3, "GBps": gbs(PB["b_x"][defer], t_b),
                                       "frac": gbs(PB["b_x"][defer], t_b) / HBM_PEAK_GBS,
                                       "bytes_per_dof": PB["b_x"][defer]},
                "matvec_star7": {"avg_ms": t_mv * 1e3, "GBps": gbs(MATVEC_BYTES, t_mv),
                                 "frac": gbs(MATVEC_BYTES, t_mv) / HBM_PEAK_GBS,
                                 "dofs_per_s": nloc / t_mv if t_mv > 0 else 0.0,
                                 "bytes_per_dof": MATVEC_BYTES},
            },
            "matvec_star7_sustained": sustained_row(mv_s, nloc, gbs),
            "variants": {"cg_single_reduction": sr_var},
            "cg_x_update_every": defer,
            "launcher": os.environ.get("PB_BENCH_LAUNCHER",
                                       "torch.distributed.run" if dist else "none"),
            "transport": comm_transport,
            "rccl_nranks": comm_nranks if comm_transport == "rccl" else None,
            "per_rank_comm": per_rank if world > 1 else None,
            "ksp_state": {"reason": pb.REASONS.get(reason, reason), "its": its,
                          "rnorm0": float(hist[0]), "rnorm_last": float(hist[-1])},
        }
        traffic_file = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(traffic_file):
            try:
                tr = json.load(open(traffic_file))
                # PMC traffic is keyed by grid and p-store mode (the kernels differ)
                key = f"{n[0]}x{n[1]}x{n[2]}" + ("" if not pstore else "/pstore_b")
                if key in tr and roof in tr[key]:
                    out["roofline"]["traffic"] = tr[key][roof]["bytes_per_launch"]
                    out["roofline"]["traffic_source"] = tr[key][roof].get("source")
                for role, kv in out["kernels"].items():
                    if role in tr.get(key, {}):
                        kv["traffic"] = tr[key][role]["bytes_per_launch"]
            except Exception:
                pass
        if world == 1 and not args.no_cpu_baseline and args.cpu_baseline != "none":
            out["cpu_baseline"] = cpu_baseline(args.cpu_baseline)
    for o in (ksp, y, xt, x, b, A, P):
        o.destroy()
    da.destroy()
    holder = {"out": out if rank == 0 else None}
    if args.secondary and not args.grid_override:
        run_secondary(args, pb, ctx, rank, world, dist, comm_transport, comm_nranks, holder,
                      json_fd)
    if rank == 0:
        os.write(json_fd, (json.dumps(holder["out"]) + "\n").encode())
    ctx.destroy()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
