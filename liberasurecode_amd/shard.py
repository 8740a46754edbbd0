"""Multi-GPU sharding of independent stripes (one process per GPU).

Stripes have no cross-stripe dependency (each liberasurecode_encode call is self-contained,
src/erasurecode.c:383-477), so a job of N GPUs is N independent shards: rank r owns stripes
[r*S, (r+1)*S) (weak scaling, S per GPU).  The process group carries no fragment data; it is used
for a start barrier and for reducing elapsed times / counters.
"""
import os


def stripe_range(rank: int, world: int, per_rank: int):
    """(first stripe id, count) owned by `rank` under weak scaling."""
    if not (0 <= rank < world) or per_rank < 0:
        raise ValueError("bad shard request")
    return rank * per_rank, per_rank


def split_range(rank: int, world: int, total: int):
    """(first, count) of a fixed total split as evenly as possible (strong scaling)."""
    if not (0 <= rank < world) or total < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


class Coordinator:
    """Launch coordination over torch.distributed (RCCL when on GPUs, gloo on CPU)."""

    def __init__(self, backend=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.on_gpu = False
        self.device = None
        if torch.cuda.is_available() and torch.cuda.device_count() > 0:
            # one GPU per rank; ranks beyond the visible GPUs share them (rehearsal only)
            self.device = self.local % torch.cuda.device_count()
            torch.cuda.set_device(self.device)
        if self.world > 1:
            backend = backend or os.environ.get("ECAMD_DIST_BACKEND")
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            self.on_gpu = backend == "nccl"
            if self.on_gpu:
                dist.init_process_group(backend=backend,
                                        device_id=torch.device("cuda", self.device or 0))
            else:
                dist.init_process_group(backend=backend)

    def _tensor(self, values):
        dev = "cuda" if self.on_gpu else "cpu"
        return self.torch.tensor(values, dtype=self.torch.float64, device=dev)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def reduce(self, values, op="max"):
        """All-reduce a list of floats (max or sum); identity when world == 1."""
        values = list(values)
        if self.world == 1:
            return values
        t = self._tensor(values)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(v) for v in t.cpu().tolist()]

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()
