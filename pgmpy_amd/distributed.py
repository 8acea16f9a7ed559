"""Multi-GPU evidence sharding: one process per GPU, rows split in contiguous blocks.

Rows are independent given a compiled plan, so the data path has no
collective: every rank runs the same plan on its own block of rows.  Results
leave a rank one of two ways:

* HostDelivery (default for C5): each rank DMAs its block's results into pinned
  host memory over its own host link, double-buffered so step k's copy overlaps
  step k + 1's launch — no collective, every GPU's link carries only its share;
* gather_rows: one gather of per-row results to rank 0 (torch.distributed
  `gather`; backend "nccl" is RCCL over xGMI on MI355X, "gloo" on CPU for the
  tests) — every row's bytes funnel into rank 0's links.

CPTs are replicated: each rank compiles its own plan (munin's CPTs are 787 KB).
"""
import ctypes

import numpy as np


def shard_bounds(n_rows, world, rank):
    """Contiguous block [lo, hi) of rank `rank` (sizes differ by at most one row)."""
    base, rem = divmod(int(n_rows), int(world))
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def gather_rows(local, n_rows, dist, dst=0):
    """Gather per-row results (tensor [..., rows_local], rows innermost) to rank `dst`.

    Returns the concatenated tensor [..., n_rows] on dst and None elsewhere.
    Uses one collective (torch.distributed.gather); rows are padded to the
    largest shard so every rank sends the same shape (a block already of that
    size is sent as it is, without a padded copy)."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    bounds = [shard_bounds(n_rows, world, r) for r in range(world)]
    max_rows = max(hi - lo for lo, hi in bounds)
    if local.shape[-1] == max_rows and local.is_contiguous():
        send = local
    else:
        send = torch.zeros(list(local.shape[:-1]) + [max_rows], dtype=local.dtype, device=local.device)
        send[..., :local.shape[-1]] = local
    recv = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, gather_list=recv, dst=dst)
    if rank != dst:
        return None
    parts = [recv[r][..., :hi - lo] for r, (lo, hi) in enumerate(bounds)]
    return torch.cat(parts, dim=-1)


def run_sharded(executor, codes_host, n_rows, dist, gather=True):
    """Run `executor(codes_block [n_cols, rows], row_offset) -> tensor [..., rows]` on this rank's
    block and (optionally) gather to rank 0."""
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = shard_bounds(n_rows, world, rank)
    local = executor(np.ascontiguousarray(codes_host[:, lo:hi]), lo)
    if not gather:
        return local
    return gather_rows(local, n_rows, dist)


class HostDelivery:
    """Results of consecutive launches delivered into pinned host buffers of this rank's node, with no
    collective (SURVEY.md §8(e)'s alternative to the gather): `depth` pinned buffers and one copy
    stream.  Step k: acquire(k, stream) before the launch that writes the step's device buffer (the
    launch stream then waits until slot k % depth's previous copy-out is done, so that device buffer
    and that host buffer are free), then deliver(k, device_tensor, stream) after it: a DMA on the copy
    stream, ordered after the launch, so the copy of step k overlaps the launch of step k + 1.
    Each GPU's copies use its own host link."""

    def __init__(self, shape, dtype, depth=2, device=None, same_stream=None):
        import os

        import torch

        self.depth = int(depth)
        self.hosts = [torch.empty(tuple(shape), dtype=dtype, pin_memory=True) for _ in range(self.depth)]
        # same_stream: the copy goes on the launch stream itself, right behind its launch (no overlap of
        # copy k with launch k + 1, no cross-stream events) — knob PGM_HOST_DELIVERY=same (A/B)
        if same_stream is None:
            same_stream = os.environ.get("PGM_HOST_DELIVERY", "separate") == "same"
        self.same_stream = bool(same_stream)
        self.stream = torch.cuda.Stream(device=device)
        self._copied = [torch.cuda.Event() for _ in range(self.depth)]
        self._ready = [torch.cuda.Event() for _ in range(self.depth)]
        self._used = [False] * self.depth

    def acquire(self, k, stream):
        i = k % self.depth
        if self._used[i]:
            stream.wait_event(self._copied[i])

    def deliver(self, k, src, stream):
        """Queue the copy of `src` (written by work already queued on `stream`) into host slot k %
        depth; returns that pinned host tensor (complete after wait(k))."""
        import torch

        from . import _native as N

        i = k % self.depth
        cs = stream if self.same_stream else self.stream
        if not self.same_stream:
            self._ready[i].record(stream)
            cs.wait_event(self._ready[i])
        if not src.is_contiguous():
            raise ValueError("HostDelivery: the device result must be contiguous")
        h = self.hosts[i]
        N.check(N.lib().pgm_memcpy_d2h_async(ctypes.c_void_p(h.data_ptr()), N.ptr(src), h.numel() * h.element_size(),
                                             N.stream_handle(cs)), "memcpy_d2h_async")
        self._copied[i].record(cs)
        self._used[i] = True
        return self.hosts[i]

    def wait(self, k=None):
        """Every queued copy (k None) or step k's copy has completed."""
        if k is None:
            for e in self._copied:
                e.synchronize()
        else:
            self._copied[k % self.depth].synchronize()
        return None if k is None else self.hosts[k % self.depth]
