"""CPU tier, world_size > 1 over gloo: the N>1 protocol of the library (z-slabs, remainder planes
on low ranks, one halo exchange of the first/last owned planes, SUM allreduce of scalars) driven
through poissbox_amd.dist.GlooTransport -- the host transport the GPU tests plug into the library --
with the oracle computing each rank's slab. Bit-exact stencil; CG history vs the single-rank
restatement within 1e-9 relative (only the allreduce summation order differs)."""
import multiprocessing as mp
import os
import socket
import traceback

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 20231015


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, fn, *args):
    ctx = mp.get_context("spawn")
    port = _free_port()
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(r, world, port, q, fn, args)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res = q.get(timeout=300)
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
    for r, res in out.items():
        if isinstance(res, str) and res.startswith("ERROR"):
            raise AssertionError(res)
    return [out[r] for r in range(world)]


def _entry(rank, world, port, q, fn, args):
    import sys
    sys.path.insert(0, REPO)
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from poissbox_amd.dist import GlooTransport
        res = fn(rank, world, GlooTransport(dist))
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:
        q.put((rank, "ERROR " + traceback.format_exc()))


def _partition(nz, world, rank):
    from poissbox_amd import slab_partition
    return slab_partition(nz, world, rank)


def _halo_protocol(rank, world, tr):
    lo = np.full(6, 100.0 * rank + 1)   # my first plane
    hi = np.full(6, 100.0 * rank + 2)   # my last plane
    r_lo, r_hi = tr.sendrecv(lo, hi)
    s = tr.allreduce(np.array([rank + 1.0, 2.0]))
    return r_lo[0], r_hi[0], list(s)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_halo_protocol(world):
    res = _run(world, _halo_protocol)
    for rank, (r_lo, r_hi, s) in enumerate(res):
        down, up = (rank - 1) % world, (rank + 1) % world
        assert r_lo == 100.0 * down + 2   # plane below me = last plane of rank-1
        assert r_hi == 100.0 * up + 1     # plane above me = first plane of rank+1
        assert s == [world * (world + 1) / 2, 2.0 * world]


N3 = (12, 10, 11)


def _slab_stencil(rank, world, tr):
    from oracle import oracle as O
    nx, ny, nz = N3
    k0, nk = _partition(nz, world, rank)
    x = O.fill_random(nx * ny * nz, SEED).reshape(nz, -1)[k0:k0 + nk].reshape(-1)
    plane = nx * ny
    glo, ghi = tr.sendrecv(x[:plane], x[-plane:])
    h = tuple(1.0 / m for m in N3)
    return k0, nk, O.stencil_slab(x, (nx, ny, nk), h, glo, ghi)


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_stencil_bit_exact(world):
    from oracle import oracle as O
    h = tuple(1.0 / m for m in N3)
    ref = O.stencil(O.fill_random(int(np.prod(N3)), SEED), N3, h).reshape(N3[2], -1)
    for k0, nk, y in _run(world, _slab_stencil):
        assert np.array_equal(y, ref[k0:k0 + nk].reshape(-1))


def _slab_cg(rank, world, tr):
    """KSPCG + PCJacobi + constant null space on this rank's slab; every
    global reduction goes through the transport's allreduce, the operator through sendrecv."""
    from oracle import oracle as O
    nx, ny, nz = N3
    k0, nk = _partition(nz, world, rank)
    plane = nx * ny
    h = tuple(1.0 / m for m in N3)
    N = nx * ny * nz
    xt = O.fill_random(N, SEED).reshape(nz, -1)[k0:k0 + nk].reshape(-1)

    def A(v):
        glo, ghi = tr.sendrecv(v[:plane], v[-plane:])
        return O.stencil_slab(v, (nx, ny, nk), h, glo, ghi)

    gsum = lambda *vals: tr.allreduce(np.array(vals, dtype=np.float64))
    dinv = 1.0 / O.diag(h)

    def pc(r):
        z = dinv * r
        return z + gsum(z.sum())[0] / (-1.0 * N)

    b = A(xt)
    x = np.zeros_like(b)
    r = b.copy()
    z = pc(r)
    dp = np.sqrt(gsum(np.dot(z, z))[0])
    hist = [dp]
    ttol = max(1e-8 * dp, 1e-50)
    beta = gsum(np.dot(z, r))[0]
    p = np.zeros_like(b)
    its, reason = 0, 0
    for i in range(500):
        its = i + 1
        p = z.copy() if i == 0 else z + (beta / betaold) * p
        w = A(p)
        dpi = gsum(np.dot(p, w))[0]
        betaold = beta
        a = beta / dpi
        x = x + a * p
        r = r + (-a) * w
        z = pc(r)
        dp = np.sqrt(gsum(np.dot(z, z))[0])
        hist.append(dp)
        if dp <= ttol:
            reason = 2
            break
        beta = gsum(np.dot(z, r))[0]
    return reason, its, hist


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_cg_matches_single_rank(world):
    from oracle import oracle as O
    h = tuple(1.0 / m for m in N3)
    b = O.stencil(O.fill_random(int(np.prod(N3)), SEED), N3, h)
    _, ro, itso, ho = O.cg_solve(b, N3, h, rtol=1e-8)
    for reason, its, hist in _run(world, _slab_cg):
        assert (reason, its) == (ro, itso)
        assert np.max(np.abs(np.array(hist) - ho) / ho) < 1e-9


def _a2a_protocol(rank, world, tr):
    blocks = [np.full(p + 1 + rank, 10.0 * rank + p) for p in range(world)]
    sizes = [rank + 1 + p for p in range(world)]   # rank p sends me rank + 1 + p doubles
    return [b.tolist() for b in tr.alltoallv(blocks, sizes)]


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_alltoallv_protocol(world):
    res = _run(world, _a2a_protocol)
    for rank, got in enumerate(res):
        for p in range(world):
            assert got[p] == [10.0 * p + rank] * (rank + 1 + p)


def _stalled_peer(rank, world, tr):
    """Rank 1 never joins the exchange (a dead or stalled peer); rank 0's transport calls must
    raise within their timeout, not hang. Both ranks meet again over the store afterwards."""
    import time
    import torch.distributed as dist
    from poissbox_amd.dist import GlooTransport
    res = "no error"
    if rank == 0:
        t = GlooTransport(dist, timeout_s=2.0)
        t0 = time.perf_counter()
        for op in (lambda: t.sendrecv(np.zeros(4), np.zeros(4)),
                   lambda: t.allreduce(np.ones(3))):
            try:
                op()
            except Exception as e:  # noqa: BLE001 - any transport error is the expected outcome
                res = f"raised after {time.perf_counter() - t0:.1f} s: {type(e).__name__}"
                break
    else:
        time.sleep(6.0)
    return res


def test_gloo_transport_times_out_on_stalled_peer():
    out = _run(2, _stalled_peer)
    assert out[0].startswith("raised"), out[0]
    assert float(out[0].split()[2]) < 10.0, out[0]
