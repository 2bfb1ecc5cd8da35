"""Connection sharding across GPUs: one process per GPU,
connections dealt round-robin (`conn_id % world == rank`), no collective on
the data path.  torch.distributed (gloo, CPU tensors) is used only for the
start/stop barriers and the max-over-ranks / sum-over-ranks of the timing
numbers -- plumbing, not the product."""
import os

import numpy as np


def shard_indices(n, rank, world):
    """Connections owned by `rank`: round-robin, so every rank gets the same
    count +-1 and the byte load is balanced for equal-size connections."""
    return np.arange(rank, n, world, dtype=np.int64)


class ShardGroup:
    def __init__(self, backend="gloo"):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.dist = None
        if self.world > 1:
            import sys
            import torch.distributed as dist
            if not dist.is_initialized():
                # gloo prints connection banners on fd 1; keep stdout for the
                # bench's single JSON line
                sys.stdout.flush()
                saved = os.dup(1)
                os.dup2(2, 1)
                try:
                    dist.init_process_group(backend)
                finally:
                    sys.stdout.flush()
                    os.dup2(saved, 1)
                    os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def _reduce(self, x, op):
        if not self.dist:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return self._reduce(x, self.dist.ReduceOp.MAX if self.dist else None)

    def sum(self, x):
        return self._reduce(x, self.dist.ReduceOp.SUM if self.dist else None)

    def gather_bytes(self, b):
        """All ranks' byte strings (rank order); for checks only."""
        if not self.dist:
            return [bytes(b)]
        out = [None] * self.world
        self.dist.all_gather_object(out, bytes(b))
        return out

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()
            self.dist = None
