"""Multi-GPU evidence sharding: one process per GPU, rows split in contiguous blocks.

Rows are independent given a compiled plan, so the data path has no
collective: every rank runs the same plan on its own block of rows.  Results
leave a rank one of two ways:

* HostDelivery (default for C5): each rank DMAs its block's results into pinned
  host memory over its own host link, double-buffered on two stream lanes so step
  k's copy overlaps step k + 1's launch — no collective, every GPU's link carries
  only its share;
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
    collective (SURVEY.md §8(e)'s alternative to the gather): `depth` pinned host buffers, one per
    device result buffer.  Step k: launch on launch_stream(k, stream), after acquire(k, stream) (slot
    k % depth's previous copy-out is done, so that device buffer and that host buffer are free), then
    deliver(k, device_tensor, stream) queues the DMA into host slot k % depth behind the launch.
    Each GPU's copies use its own host link.  Three orderings (`mode`, knob PGM_HOST_DELIVERY):

    * "lanes" (default): one stream per slot.  Step k launches and copies on lane k % depth, so the
      copy of step k overlaps the launch of step k + 1 on the other lane with no cross-stream event:
      a lane's next launch is ordered after its own previous copy by the stream itself.
    * "same": launch and copy on the caller's stream, one behind the other (no overlap).
    * "separate": copies on one copy stream, ordered after their launches by cross-stream events.
      Measured on MI355X (profiles/r04h/) those events cost more than the overlap gains: MAP rows
      1.9 G rows/s against 8.0 G for "same"."""

    MODES = ("lanes", "same", "separate")

    def __init__(self, shape, dtype, depth=2, device=None, mode=None, lanes=None):
        import os

        import torch

        self.depth = int(depth)
        self.mode = mode or os.environ.get("PGM_HOST_DELIVERY", "lanes")
        if self.mode not in self.MODES:
            raise ValueError(f"HostDelivery: mode {self.mode!r} is not one of {self.MODES}")
        self.hosts = [torch.empty(tuple(shape), dtype=dtype, pin_memory=True) for _ in range(self.depth)]
        self.stream = torch.cuda.Stream(device=device) if self.mode == "separate" else None
        # lanes: another HostDelivery's lanes may be shared (several results of one launch)
        self.lanes = None
        if self.mode == "lanes":
            self.lanes = list(lanes) if lanes is not None else [torch.cuda.Stream(device=device)
                                                                 for _ in range(self.depth)]
            if len(self.lanes) != self.depth:
                raise ValueError("HostDelivery: one lane per slot")
        self._copied = [torch.cuda.Event() for _ in range(self.depth)]
        self._ready = [torch.cuda.Event() for _ in range(self.depth)]
        self._used = [False] * self.depth

    def launch_stream(self, k, stream):
        """The stream step k's launch (and its deliver) must be queued on."""
        return self.lanes[k % self.depth] if self.lanes is not None else stream

    def acquire(self, k, stream):
        i = k % self.depth
        if self._used[i] and self.lanes is None:
            stream.wait_event(self._copied[i])

    def deliver(self, k, src, stream):
        """Queue the copy of `src` (written by work already queued on `stream`, which is
        launch_stream(k, ...)) into host slot k % depth; returns that pinned host tensor (complete
        after wait(k))."""
        from . import _native as N

        i = k % self.depth
        if self.lanes is not None and stream is not self.lanes[i]:
            raise ValueError("HostDelivery: step k's result must be produced on launch_stream(k)")
        cs = self.stream if self.mode == "separate" else stream
        if self.mode == "separate":
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
