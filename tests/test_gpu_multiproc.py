"""GPU tier, N processes on the one GPU: each rank is a separate process with its own context,
connected through the gloo host transport (RCCL refuses two ranks on one device). Exercises
the library's multi-rank path end to end (slab split, interior/boundary overlap split, halo,
allreduce, lagged rank-consistent stopping) against the single-rank oracle."""
import os
import subprocess
import sys

import numpy as np
import pytest

from parity_bars import check_history, check_x
from test_dist_cpu import REPO, SEED, _run

pytestmark = pytest.mark.gpu

N3 = (24, 20, 13)


def _gpu_rank(rank, world, tr):
    import poissbox_amd as pb
    ctx = pb.Context(0, rank, world)
    ctx.set_host_transport(tr.sendrecv, tr.allreduce, tr.alltoallv)
    da = pb.DA(ctx, N3)
    (_, _, k0), (_, _, nk) = da.get_corners()
    h = da.spacing
    P, A, x, b = pb.initialise_linear_system(da, h)
    xt = pb.Vec(da)
    xt.set_random(SEED)
    A.mult(xt, b)
    bl = b.get_values()
    reason, its, hist = pb.solve(P, A, x, b, ["-ksp_rtol", "1e-9"])
    out = (k0, nk, bl, reason, its, hist, x.get_values())
    ctx.destroy()
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_cg_on_one_gpu(world):
    from oracle import oracle as O
    h = tuple(1.0 / m for m in N3)
    b = O.stencil(O.fill_random(int(np.prod(N3)), SEED), N3, h)
    xo, ro, itso, ho = O.cg_solve(b, N3, h, rtol=1e-9)
    bz, xz = b.reshape(N3[2], -1), xo.reshape(N3[2], -1)
    for k0, nk, bl, reason, its, hist, xs in _run(world, _gpu_rank):
        assert np.array_equal(bl, bz[k0:k0 + nk].reshape(-1))      # bit-exact distributed A x
        assert (reason, its) == (ro, itso)
        check_history(hist, ho)
        check_x(xs, xz[k0:k0 + nk].reshape(-1), scale=np.max(np.abs(xo)))


def _gpu_rank_compact(rank, world, tr):
    import poissbox_amd as pb
    n = (64, 32, 64)
    ctx = pb.Context(0, rank, world)
    ctx.set_host_transport(tr.sendrecv, tr.allreduce, tr.alltoallv)
    da = pb.DA(ctx, n, (2 * np.pi,) * 3)
    (_, _, k0), (_, _, nk) = da.get_corners()
    from oracle import oracle as O
    f = O.fill_random(int(np.prod(n)), 5).reshape(n[2], -1)
    fv, out = pb.Vec(da), pb.Vec(da)
    fv.set_values(f[k0:k0 + nk])
    pb.compact_lapl_fast(da, da.spacing, fv, out)
    res = (k0, nk, out.get_values())
    ctx.destroy()
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_compact_lapl(world):
    """z-slab <-> y-slab transposes through the gloo alltoallv between processes."""
    from oracle import oracle as O
    n = (64, 32, 64)
    h = tuple(2 * np.pi / m for m in n)
    ref = O.lapl(O.fill_random(int(np.prod(n)), 5), n, h).reshape(n[2], -1)
    for k0, nk, y in _run(world, _gpu_rank_compact):
        assert np.max(np.abs(y - ref[k0:k0 + nk].reshape(-1))) <= 1e-12 * np.max(np.abs(ref))


N_CFG4 = (1024, 1024, 1024)
CFG4_ITS = 30  # (r04: 8 -> 30; the oracle runs ~1 s per 1024^3 iteration on 16 threads)


def _gpu_rank_cfg4(rank, world, tr):
    """One rank of BASELINE config 4's decomposition: a 1024x1024x128 slab of the 1024^3 grid."""
    import hashlib
    import poissbox_amd as pb
    ctx = pb.Context(0, rank, world)
    ctx.set_host_transport(tr.sendrecv, tr.allreduce, tr.alltoallv)
    da = pb.DA(ctx, N_CFG4)
    (_, _, k0), (_, _, nk) = da.get_corners()
    h = da.spacing
    P, A, x, b = pb.initialise_linear_system(da, h)
    xt = pb.Vec(da)
    xt.set_random(SEED)
    A.mult(xt, b)
    digest = hashlib.blake2b(b.get_values().tobytes()).hexdigest()
    opts = ["-ksp_type", "cg", "-pc_type", "jacobi", "-ksp_rtol", "0", "-ksp_atol", "0",
            "-ksp_max_it", str(CFG4_ITS), "-ksp_divtol", "1e300"]
    reason, its, hist = pb.solve(P, A, x, b, opts)
    out = (k0, nk, digest, reason, its, np.asarray(hist))
    ctx.destroy()
    return out


def test_config4_geometry_eight_ranks():
    """BASELINE config 4's decomposition (1024^3 over 8 ranks, 1024x1024x128 slabs, halo planes of
    8 MiB, two allreduces per iteration) as 8 processes on the one GPU through the host transport:
    every rank's b = A x_true slab bit-exact against the oracle's, and a fixed-iteration CG + Jacobi
    history against the oracle's whole-grid solve (src/poissbox.f90:269-298)."""
    import hashlib
    from oracle import oracle as O
    world = 8
    res = _run(world, _gpu_rank_cfg4)
    assert [(r[0], r[1]) for r in res] == [(128 * q, 128) for q in range(world)]
    n = N_CFG4
    h = tuple(1.0 / m for m in n)
    threads = min(16, os.cpu_count() or 1)
    xs = O.fill_random(int(np.prod(n)), SEED)
    bo = O.stencil(xs, n, h, nthreads=threads)
    del xs
    plane = n[0] * n[1]
    for k0, nk, digest, *_ in res:
        assert digest == hashlib.blake2b(bo[k0 * plane:(k0 + nk) * plane].tobytes()).hexdigest()
    _, ro, itso, ho = O.cg_solve(bo, n, h, rtol=0.0, atol=0.0, dtol=1e300, max_it=CFG4_ITS,
                                 nthreads=threads)
    del bo
    for *_, reason, its, hist in res:
        assert (reason, its) == (ro, itso) == (reason, CFG4_ITS)
        check_history(hist, ho)


@pytest.mark.parametrize("workload,extra", [("compact-fft", ["--base", "64"]),
                                            ("star7-mg", ["--base", "32"])])
def test_bench_solve_workload_self_launch(workload, extra):
    """bench.py --workload (whole KSPSolves) through the self-launch path with no
    launcher in the environment: 2 rank processes on the one GPU over the gloo host transport
    (config 5 strong-scaled: the compact operator's transposes run as host all-to-alls)."""
    import json
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = REPO
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--workload", workload, "--transport", "host"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["launcher"] == "self" and d["transport"] == "host"
    assert d["config"]["workload_key"] == workload
    assert d["ksp_state"]["reason"] == "CONVERGED_RTOL"
    assert d["ksp_state"]["true_residual_rel"] < 1e-8
    assert d["value"] > 0 and d["roofline"]["launches_timed"] > 0
    if workload == "compact-fft":
        assert d["scaling"] == "strong" and d["config"]["grid"] == [64, 64, 64]
        assert all("alltoallv_calls" in r for r in d["per_rank_comm"])
    else:
        assert d["scaling"] == "weak" and d["config"]["grid"] == [32, 32, 64]


def test_bench_two_ranks_host_transport():
    """bench.py's multi-rank orchestration (torch.distributed.run, barrier, max-over-ranks,
    weak-scaling grid) on one GPU through the host transport, at a small per-GPU size."""
    env = dict(os.environ, PYTHONPATH=REPO)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29531", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "6", "--warmup", "2", "--base", "48", "--matvecs", "2",
           "--transport", "host"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    import json
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["config"]["grid"] == [48, 48, 96] and d["value"] > 0
    # the default run also measures the solve workloads (config 5 strong-scaled, CG + MG)
    sec = d["secondary"]
    assert sec["compact-fft"]["config"]["grid"] == [48, 48, 48]
    assert sec["star7-mg"]["config"]["grid"] == [48, 48, 96]
    for wl in ("compact-fft", "star7-mg"):
        assert sec[wl]["ksp_state"]["reason"] == "CONVERGED_RTOL", sec[wl]
        assert sec[wl]["value"] > 0


def test_bench_eight_ranks_default_run_host_transport():
    """Rehearsal of the driver's N = 8 scaling run on one GPU: `bench.py --gpus 8` with no launcher
    (self-launch: 8 rank processes), the default workload plus its secondaries (config 5's compact
    operator with the spectral PC strong-scaled over 8 slabs -- all-to-all transposes on 8 ranks --
    and CG + MG), over the gloo host transport in place of RCCL (which refuses two ranks on one
    GPU). One JSON line; every workload converges and reports 8 ranks."""
    import json
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = REPO
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "4",
           "--warmup", "1", "--base", "32", "--matvecs", "2", "--sustained", "2",
           "--transport", "host"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 8 and d["launcher"] == "self" and d["config"]["grid"] == [64, 64, 64]
    assert len(d["per_rank_comm"]) == 8 and d["value"] > 0
    sec = d["secondary"]
    assert "error" not in sec, sec.get("error")
    assert sec["compact-fft"]["config"]["grid"] == [32, 32, 32]
    for wl in ("compact-fft", "star7-mg"):
        assert sec[wl]["n_gpus"] == 8
        assert sec[wl]["ksp_state"]["reason"] == "CONVERGED_RTOL", sec[wl]
        assert sec[wl]["ksp_state"]["true_residual_rel"] < 1e-8
    assert all(r["alltoallv_calls"] > 0 for r in sec["compact-fft"]["per_rank_comm"])
