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


class OverlappedHistReduce:
    """Per-step histogram all-reduce overlapped with the next step's launch.

    Step i accumulates into buffer ``i % 2``; its all-reduce is issued asynchronously (on the
    collective's own stream, after the step's kernel) and is only waited for before step i + 2
    zeroes that buffer again, so the all-reduce of step i runs under the kernel of step i + 1
    instead of between them.  ``finish()`` waits for every pending reduce and returns the
    buffer of the last step.  Without a process group the reduces are no-ops."""

    def __init__(self, bufs, group=None):
        import torch.distributed as dist
        self.bufs = bufs
        self.group = group
        self.work = [None] * len(bufs)
        self.last = None
        self.active = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1

    def acquire(self, i):
        """Buffer for step ``i`` (its previous reduce waited for)."""
        b = i % len(self.bufs)
        if self.work[b] is not None:
            self.work[b].wait()
            self.work[b] = None
        return b

    def issue(self, b):
        """Start the all-reduce of buffer ``b`` (after the step that filled it)."""
        import torch.distributed as dist
        if self.active:
            self.work[b] = dist.all_reduce(self.bufs[b], op=dist.ReduceOp.SUM, group=self.group,
                                           async_op=True)
        self.last = b

    def finish(self):
        for b, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[b] = None
        return None if self.last is None else self.bufs[self.last]
