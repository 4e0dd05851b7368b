"""Per-rank sample sharding for data-parallel training (one process per GPU,
each rank its own share of every batch).

The reference trains on one device: its paired loader draws `len(pairs)` indices with
replacement from a WeightedRandomSampler (train_multimodal_fusion.py:266-275, weights 1 / count
of the pair's class) and walks the val / test sets in order (:279-280).  Under data
parallelism every rank must see a disjoint share of ONE such draw, and every rank must run the
same number of batches (the gradient all-reduce pairs collectives across ranks), so:

  * ShardedWeightedSampler: every rank makes the SAME weighted draw (a generator seeded with
    seed + epoch, so it changes per epoch as the reference's global-RNG draw does), pads it
    by wrapping to a multiple of world_size, and keeps positions rank, rank + world, ...  The
    union of the shards is the single-rank draw (plus the wrapped padding).
  * ShardedSequentialSampler: the val / test order (0 .. n-1) split by whole batches, no
    padding (every sample once; evaluate() restores the reference's order).

`set_epoch(e)` mirrors torch.utils.data.DistributedSampler.
"""
import math

import torch


def _shard(indices, rank, world):
    n = len(indices)
    per = math.ceil(n / world) if n else 0
    padded = indices + indices[:per * world - n] if n else []
    return padded[rank:per * world:world]


class ShardedWeightedSampler(torch.utils.data.Sampler):
    """WeightedRandomSampler(weights, num_samples, replacement=True) drawn identically on every
    rank and sharded: rank r yields draws r, r + world, ... (wrap-padded to equal length)."""

    def __init__(self, weights, num_samples=None, rank=0, world_size=1, seed=42):
        self.weights = torch.as_tensor(weights, dtype=torch.double)
        self.num_samples = len(self.weights) if num_samples is None else int(num_samples)
        if world_size < 1 or not 0 <= rank < world_size:
            raise ValueError(f"rank {rank} of world {world_size}")
        self.rank, self.world = rank, world_size
        self.seed = seed
        self.epoch = 0

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def full_draw(self):
        """The draw every rank shares (what a single-rank WeightedRandomSampler with this
        generator would yield)."""
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        return torch.multinomial(self.weights, self.num_samples, True, generator=g).tolist()

    def __iter__(self):
        return iter(_shard(self.full_draw(), self.rank, self.world))

    def __len__(self):
        return math.ceil(self.num_samples / self.world)


class ShardedSequentialSampler(torch.utils.data.Sampler):
    """0 .. n-1 sharded over ranks by whole batches, without padding: the val / test loaders.

    The single-process loader walks batches [0, B), [B, 2B), ... (the last one possibly short);
    rank r takes batches r, r + world, ...  So every sample is evaluated exactly once, every
    rank's batches are batches of the single-process run (the union of the ranks' batch losses
    and confusion counts is the single-process one, with batch_size = the loader's), and
    ``global_indices()`` tells evaluate() how to put the gathered per-rank rows back in the
    reference's order.  Ranks may run different numbers of batches (eval has no per-batch
    collective).  ``batch_size`` is required and must equal the loader's (training.loop checks
    it): a sampler split by one batch size under a loader batching by another would form
    batches the single-process run never forms."""

    def __init__(self, n, rank=0, world_size=1, *, batch_size):
        if world_size < 1 or not 0 <= rank < world_size:
            raise ValueError(f"rank {rank} of world {world_size}")
        if batch_size < 1:
            raise ValueError(f"batch_size {batch_size}")
        self.n, self.rank, self.world, self.batch_size = int(n), rank, world_size, int(batch_size)

    def set_epoch(self, epoch):
        pass

    def indices_of(self, rank):
        B = self.batch_size
        nb = (self.n + B - 1) // B
        return [i for j in range(rank, nb, self.world) for i in range(j * B, min(self.n, (j + 1) * B))]

    def global_indices(self):
        """The sample index of every row of the rank-order concatenation of all shards."""
        return [i for r in range(self.world) for i in self.indices_of(r)]

    def __iter__(self):
        return iter(self.indices_of(self.rank))

    def __len__(self):
        return len(self.indices_of(self.rank))


def dp_rank_world(group=None):
    """(rank, world) of the default process group, (0, 1) without one."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1
