"""Process-group plumbing for multi-GPU runs (one process per GPU).

* init_from_env(): reads RANK / WORLD_SIZE / LOCAL_RANK (torch.distributed.run), initialises a
  gloo process group (CPU-side control plane only) and broadcasts rank 0's RCCL unique id.
* GlooTransport: the host transport of pb_ctx_set_host_transport over a gloo group -- the same
  halo/allreduce protocol the RCCL path implements on the device (include/poissbox_gpu.h:
  send the first owned plane to rank-1 and the last to rank+1, receive the plane below / above).
  Used by tests to run N processes on one GPU (RCCL refuses two ranks on one device) and on CPU.
"""
import datetime
import os

import numpy as np


def comm_timeout_s():
    """Per-operation bound of the host transport (PB_COMM_TIMEOUT_MS, as the library's own
    waits): a peer that died or stalls surfaces as an exception, which the transport callback
    turns into PB_ERR_COMM, instead of a hang."""
    return int(os.environ.get("PB_COMM_TIMEOUT_MS", "180000")) / 1000.0


def env_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend="gloo"):
    """Returns (rank, world, local_rank, dist or None)."""
    rank, world, local = env_world()
    if world == 1:
        return rank, world, local, None
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group(backend)
    return rank, world, local, dist


def broadcast_uid(dist, rank, make_uid):
    obj = [make_uid() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


class GlooTransport:
    """sendrecv(lo, hi) -> (recv_lo, recv_hi); allreduce(vals) -> summed vals (float64)."""

    def __init__(self, dist, group=None, timeout_s=None):
        import torch
        self.torch = torch
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.timeout = datetime.timedelta(seconds=timeout_s if timeout_s else comm_timeout_s())

    def _wait(self, reqs):
        for q in reqs:
            q.wait(self.timeout)  # raises on timeout / peer failure

    def sendrecv(self, lo, hi):
        t = self.torch
        down, up = (self.rank - 1) % self.world, (self.rank + 1) % self.world
        if self.world == 1:
            return hi.copy(), lo.copy()
        r_lo = t.empty(lo.size, dtype=t.float64)
        r_hi = t.empty(hi.size, dtype=t.float64)
        # tags keep the two directions apart when down == up (2 ranks)
        reqs = [self.dist.isend(t.from_numpy(np.ascontiguousarray(lo)), down, self.group, tag=1),
                self.dist.isend(t.from_numpy(np.ascontiguousarray(hi)), up, self.group, tag=2),
                self.dist.irecv(r_hi, up, self.group, tag=1),
                self.dist.irecv(r_lo, down, self.group, tag=2)]
        self._wait(reqs)
        return r_lo.numpy(), r_hi.numpy()

    def allreduce(self, vals):
        v = self.torch.from_numpy(np.ascontiguousarray(vals, dtype=np.float64).copy())
        self._wait([self.dist.all_reduce(v, group=self.group, async_op=True)])
        return v.numpy()

    def alltoallv(self, blocks, recv_sizes):
        """blocks[p] goes to rank p; returns the blocks received from every rank
        (recv_sizes[p] doubles from rank p)."""
        t = self.torch
        out = [None] * self.world
        out[self.rank] = np.array(blocks[self.rank], copy=True)
        reqs, bufs = [], {}
        for p in range(self.world):
            if p == self.rank:
                continue
            bufs[p] = t.empty(int(recv_sizes[p]), dtype=t.float64)
            if recv_sizes[p]:
                reqs.append(self.dist.irecv(bufs[p], p, self.group, tag=3))
            if len(blocks[p]):
                reqs.append(self.dist.isend(t.from_numpy(np.ascontiguousarray(blocks[p])), p,
                                            self.group, tag=3))
        self._wait(reqs)
        for p, b in bufs.items():
            out[p] = b.numpy()
        return out
