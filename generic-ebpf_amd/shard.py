"""Multi-GPU sharding of a packet batch: packets are independent and array
maps are read-only during a batch, so the batch splits into contiguous per-rank shards with no
data-path collective.  The only exchange is the per-GPU verdict histogram (EBPF_HIST_BINS u64),
summed with one all-reduce (RCCL over xGMI on GPUs, gloo in CPU tests)."""


def shard_bounds(count, rank, world):
    """Contiguous [lo, hi) of ``count`` packets owned by ``rank`` of ``world``."""
    base, extra = divmod(count, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def reduce_hist(hist, group=None):
    """Sum a per-rank histogram tensor across ranks in place (no-op when not distributed)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    return hist
