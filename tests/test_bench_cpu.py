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
    # p stored by pass A (PB_CG_PSTORE_B=0): 24 + (3 * 24 + 64) / 4
    assert bench.cg_iter_bytes(4, 0) == 58
    assert bench.cg_iter_bytes(0, 0) == 64


def test_pstore_mode_env(monkeypatch):
    monkeypatch.delenv("PB_CG_PSTORE_B", raising=False)
    assert bench.pstore_mode() == 1
    monkeypatch.setenv("PB_CG_PSTORE_B", "0")
    assert bench.pstore_mode() == 0


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
