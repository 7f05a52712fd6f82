"""CPU tier: bench.py's host-side pieces (the CPU-baseline leg and the weak-scaling grids) run
here without a GPU, so a broken helper cannot first show up in the driver's bench run."""
import bench


def test_global_grid_weak_scaling():
    assert bench.global_grid(1) == (512, 512, 512)
    assert bench.global_grid(2) == (512, 512, 1024)
    assert bench.global_grid(4) == (512, 1024, 1024)
    assert bench.global_grid(8) == (1024, 1024, 1024)


def test_cg_iter_bytes():
    # p stored by pass B (library default): 16 + (3 * 32 + 64) / 4
    assert bench.cg_iter_bytes(4) == 56
    assert bench.cg_iter_bytes(2) == 56
    assert bench.cg_iter_bytes(0) == 64


def test_host_info_fields():
    info = bench.host_info()
    for k in ("nproc", "lscpu", "usable_cores", "os_cpu_count", "petsc"):
        assert k in info
    assert info["usable_cores"] >= 1


def test_cpu_rows_and_variants_small():
    from oracle import oracle as O
    row = bench._cpu_row(O, 16, 1e-10, 10000, 2)
    assert row["reason"] == 2 and row["its"] > 10 and row["true_residual_rel"] < 1e-8
    v = bench.cpu_variants(2, iters=4)
    assert [r["op"] for r in v] == ["7-point", "faithful 27-term", "faithful 27-term"]
    assert all(r["value"] > 0 for r in v)


def test_self_launch_dry_run_two_and_four_ranks():
    """`bench.py --gpus N` with no launcher in the environment starts the N ranks itself (child
    processes, no GPU call in the parent) and relays rank 0's single JSON line."""
    import json
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    for n in (2, 4):
        p = subprocess.run([sys.executable, bench.__file__, "--gpus", str(n), "--dry-run"],
                           capture_output=True, text=True, env=env, timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        lines = [l for l in p.stdout.splitlines() if l.strip()]
        assert len(lines) == 1, p.stdout
        out = json.loads(lines[0])
        assert out["n_gpus"] == n and out["launcher"] == "self"
        assert [r[0] for r in out["ranks"]] == list(range(n))
        assert [r[1] for r in out["ranks"]] == list(range(n))  # LOCAL_RANK = device per rank
        assert len({r[2] for r in out["ranks"]}) == n          # n separate processes
        assert tuple(out["grid"]) == bench.global_grid(n)


def test_self_launch_failing_rank_is_an_error():
    """A rank that exits non-zero makes the launcher exit non-zero; a rank that hangs is killed
    after the grace period instead of hanging the run."""
    import sys
    fail = ["-c", "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)"]
    assert bench.self_launch(2, [], cmd=[sys.executable] + fail) == 3
    hang = ["-c", "import os, sys, time; print('{}'); sys.stdout.flush(); "
                  "os.environ['RANK'] == '1' and sys.exit(5); time.sleep(600)"]
    os_env = __import__("os").environ
    old = os_env.get("PB_BENCH_GRACE_S")
    os_env["PB_BENCH_GRACE_S"] = "1"
    try:
        import time
        t0 = time.monotonic()
        assert bench.self_launch(2, [], cmd=[sys.executable] + hang) == 5
        assert time.monotonic() - t0 < 60
    finally:
        if old is None:
            os_env.pop("PB_BENCH_GRACE_S")
        else:
            os_env["PB_BENCH_GRACE_S"] = old
    ok = ["-c", "import os; os.environ['RANK'] == '0' and print('{\"metric\": 1}')"]
    assert bench.self_launch(2, [], cmd=[sys.executable] + ok) == 0


def test_sustained_row():
    import numpy as np
    gbs = lambda b, t: b * 1000 / t / 1e9
    r = bench.sustained_row(np.r_[np.full(10, 1.0), np.full(80, 1.5), np.full(10, 2.0)], 1000, gbs)
    assert r["launches"] == 100 and r["first10_ms"] == 1.0 and r["last10_ms"] == 2.0
    assert abs(r["avg_ms"] - 1.5) < 1e-12 and r["median_ms"] == 1.5
    assert bench.sustained_row([], 1, gbs) is None


def test_solve_workload_dry_run_and_cpu_rows():
    """--workload compact-fft defaults to strong scaling (config 5: 512^3 over the GPUs); its CPU
    baseline (the oracle's compact CG + spectral PC) and star7-mg's run on small grids here."""
    import json
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--dry-run",
                        "--workload", "compact-fft"], capture_output=True, text=True, env=env,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["workload"] == "compact-fft" and out["scaling"] == "strong"
    assert out["grid"] == [512, 512, 512]
    for wl in ("compact-fft", "star7-mg"):
        cb = bench.cpu_solve_baseline(wl, budget_s=0.01, m=16)
        assert cb["reason"] == 2 and cb["value"] > 0 and cb["its_per_solve"] >= 1
        assert cb["kind"] == "port" and cb["cores"] >= 1


def test_dominant_kernel_and_sr_bytes():
    """The solve lines' dominant phase: largest time per solve among the timed kernels, wrappers
    and communication left out; the single-reduction variant's bytes per iteration on one rank
    (3 one-pass iterations of 32 B/DoF, one two-pass x-update iteration of 64 + 8)."""
    kern = {"pc_fft": {"avg_ms": 2.6, "launches_per_solve": 2},
            "pc_fft_x": {"avg_ms": 0.64, "launches_per_solve": 4},
            "pc_fft_z": {"avg_ms": 0.51, "launches_per_solve": 2, "frac": 0.52},
            "alltoallv": {"avg_ms": 5.0, "launches_per_solve": 7}}
    d = bench.dominant_kernel(kern, 7.7e-3)
    assert d["name"] == "pc_fft_x" and d["launches_per_solve"] == 4
    assert abs(d["ms_per_solve"] - 2.56) < 1e-9 and abs(d["share_of_solve"] - 2.56 / 7.7) < 1e-9
    assert bench.dominant_kernel({}, 1.0) is None
    b = bench.SR_BYTES
    assert (3 * b["sr1"] + b["p_x4"] + b["s"]) / 4 == 42
    assert bench.SR_ITER_BYTES == 48
