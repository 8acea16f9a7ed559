"""Multi-GPU evidence sharding: one process per GPU, rows split in contiguous blocks.

Rows are independent given a compiled plan, so the data path has no
collective: every rank runs the same plan on its own block of rows.  The only
exchange is the optional final gather of per-row results to rank 0
(torch.distributed `gather`; backend "nccl" is RCCL over xGMI on MI355X, "gloo"
on CPU for the tests).  CPTs are replicated: each rank compiles its own plan
(munin's CPTs are 787 KB).
"""
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
    largest shard so every rank sends the same shape."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    bounds = [shard_bounds(n_rows, world, r) for r in range(world)]
    max_rows = max(hi - lo for lo, hi in bounds)
    pad_shape = list(local.shape[:-1]) + [max_rows]
    send = torch.zeros(pad_shape, dtype=local.dtype, device=local.device)
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
