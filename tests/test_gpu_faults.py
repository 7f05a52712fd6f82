"""GPU tier: communication failures on split (multi-rank) contexts surface as PB_ERR_COMM instead
of hangs (include/poissbox_gpu.h pb_ctx_comm_status). The reference's MPI path has no such
handling (src/poissbox.f90:104-105 DMGlobalToLocal blocks forever on a dead peer); here every host
wait is bounded and a failed context refuses further communication.

Both cases run one process as rank 0 of a 2-rank context over a loop-back host transport, so no
RCCL communicator is involved (aborting one with kernels still queued is left to real failures)."""
import os

import numpy as np
import pytest

import poissbox_amd as pb
from poissbox_amd._lib import PbError

PB_ERR_COMM = 3


def _split_ctx(sendrecv, allreduce):
    ctx = pb.Context(0, 0, 2)
    ctx.set_host_transport(sendrecv, allreduce)
    return ctx


@pytest.mark.gpu
def test_failing_host_callback_is_an_error_and_poisons_the_context():
    calls = {"n": 0}

    def bad_sendrecv(lo, hi):
        calls["n"] += 1
        raise ConnectionError("peer gone")

    ctx = _split_ctx(bad_sendrecv, lambda v: v)
    try:
        da = pb.initialise_grid(ctx, (32, 32, 16))
        x, y = pb.Vec(da), pb.Vec(da)
        A = pb.Mat(da, pb.STAR7)
        with pytest.raises(PbError) as e:
            A.mult(x, y)
        assert e.value.code == PB_ERR_COMM and "sendrecv" in str(e.value)
        assert ctx.comm_failed
        with pytest.raises(PbError) as e2:  # no further collective traffic on a failed context
            A.mult(x, y)
        assert e2.value.code == PB_ERR_COMM and calls["n"] == 1
        for o in (A, x, y, da):
            o.destroy()
    finally:
        ctx.destroy()


@pytest.mark.gpu
def test_long_local_work_is_not_a_comm_timeout(monkeypatch):
    """PB_COMM_TIMEOUT_MS bounds communication in flight, not local work: with a
    1 ms bound, waiting for ~1000 queued vector updates of a 512x512x256 slab (~0.3 ms each) on a
    split context completes, and the context stays usable."""
    monkeypatch.setenv("PB_COMM_TIMEOUT_MS", "1")
    loop = lambda lo, hi: (hi.copy(), lo.copy())  # noqa: E731 - loop-back halo
    ctx = _split_ctx(loop, lambda v: v)
    try:
        da = pb.initialise_grid(ctx, (512, 512, 256))
        x, y = pb.Vec(da), pb.Vec(da)
        y.set_random(1)
        for _ in range(1000):
            x.axpy(1e-3, y)
        ctx.sync()
        assert not ctx.comm_failed
        assert x.norm() > 0
        for o in (x, y, da):
            o.destroy()
    finally:
        ctx.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("forced", [True, False])
def test_stalled_peer_times_out(monkeypatch, tune, forced):
    """A communication that starts and never finishes -- the test hook comm_stall_test_ms puts a
    kernel that waits for a peer's data (a host-mapped flag) inside the allreduce's
    communication scope -- fails the wait with PB_ERR_COMM after PB_COMM_TIMEOUT_MS (200 ms), the
    failure releases the waiting kernel, and the failed context refuses further collectives.
    forced = False: the stall rides in a group without a progress mark of its own (marks only
    every 1000th group) -- the wait marks the unmarked groups before it polls."""
    import time
    monkeypatch.setenv("PB_COMM_TIMEOUT_MS", "200")
    loop = lambda lo, hi: (hi.copy(), lo.copy())  # noqa: E731 - loop-back halo
    ctx = _split_ctx(loop, lambda v: v)
    try:
        da = pb.initialise_grid(ctx, (64, 64, 32))
        x = pb.Vec(da)
        x.set_random(1)
        assert x.norm() > 0                        # the hook off: a normal allreduce
        if not forced:
            tune.set("comm_mark_every", 1000)
        tune.set("comm_stall_test_ms", 20000 if forced else -20000)  # (ends by itself after 20 s)
        t0 = time.monotonic()
        with pytest.raises(PbError) as e:
            x.norm()
        took = time.monotonic() - t0
        assert e.value.code == PB_ERR_COMM and "PB_COMM_TIMEOUT_MS" in str(e.value)
        assert 0.15 < took < 10.0, took            # the bound, not the kernel's own 20 s
        assert ctx.comm_failed
        tune.set("comm_stall_test_ms", 0)
        with pytest.raises(PbError) as e2:
            x.norm()
        assert e2.value.code == PB_ERR_COMM
        x.destroy()
        da.destroy()
    finally:
        ctx.destroy()
    # a fresh context is unaffected
    c2 = pb.Context(0)
    try:
        assert not c2.comm_failed
    finally:
        c2.destroy()


@pytest.mark.gpu
def test_out_of_memory_is_an_error_and_the_context_goes_on():
    """A vector that cannot be allocated (8192^3 doubles, 4 TiB) is PB_ERR_ALLOC (4), with nothing
    left behind; the same context then runs a matvec and a CG solve on a small grid (HIP's
    last-error state of the refused allocation does not resurface at their launch checks)."""
    from oracle import oracle as O
    ctx = pb.Context(0)
    big = pb.DA(ctx, (8192, 8192, 8192))
    with pytest.raises(PbError) as e:
        pb.Vec(big)
    assert e.value.code == 4
    big.destroy()
    n3 = (16, 12, 10)
    da = pb.DA(ctx, n3)
    h = tuple(1.0 / m for m in n3)
    x0 = O.fill_random(int(np.prod(n3)), 7)
    P, A, x, b = pb.initialise_linear_system(da, h)
    x.set_values(x0)
    A.mult(x, b)
    assert np.array_equal(b.get_values(), O.stencil(x0, n3, h))
    x.set(0.0)
    reason, its, hist = pb.solve(P, A, x, b, ["-ksp_rtol", "1e-8"])
    assert reason == 2 and its > 0
    ctx.destroy()
