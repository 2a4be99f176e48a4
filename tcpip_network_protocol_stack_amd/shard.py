"""Multi-GPU sharding of a segment batch.

Segments are independent and no segment spans GPUs, so the batch splits into
contiguous index ranges, one per rank (one process per GPU), with no data-path
collective: every GPU reads only its own HBM shard and writes its own outputs.
The only cross-rank traffic is timing (barrier + max, over gloo on the host)
and, in the tests, the gather of the u16 outputs.  Fixed-stride batches split by segment count;
mixed-length batches split by bytes (cut at the prefix sums of the lengths) so
every GPU streams about the same number of bytes.
"""
from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class Shard:
    rank: int
    index0: int  # first global segment index
    n: int  # segments in this shard
    byte0: int  # first global byte offset
    nbytes: int  # bytes spanned


def shard_range(n_total, rank, world):
    """Contiguous [i0, i1) segment range of `rank` (sizes differ by <= 1)."""
    return n_total * rank // world, n_total * (rank + 1) // world


def fixed_stride_shard(n_total, stride, seg_len, rank, world):
    i0, i1 = shard_range(n_total, rank, world)
    n = i1 - i0
    return Shard(rank, i0, n, i0 * stride, (n - 1) * stride + seg_len if n else 0)


def byte_balanced_cuts(offsets, world):
    """Segment cut points [c_0=0, ..., c_world=n] splitting packed offsets
    (n+1 entries) into `world` ranges of ~equal bytes."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    total = int(offsets[-1] - offsets[0])
    targets = offsets[0] + np.array([total * r // world for r in range(world + 1)], dtype=np.uint64)
    cuts = np.searchsorted(offsets, targets, side="left").astype(np.int64)
    cuts[0], cuts[-1] = 0, n
    return np.maximum.accumulate(np.clip(cuts, 0, n))


def offsets_shard(offsets, rank, world):
    cuts = byte_balanced_cuts(offsets, world)
    i0, i1 = int(cuts[rank]), int(cuts[rank + 1])
    b0 = int(offsets[i0])
    return Shard(rank, i0, i1 - i0, b0, int(offsets[i1]) - b0)


def max_over_ranks(value, dist=None):
    """MAX of a float over all ranks (the timing reduction bench.py reports),
    over the process group's own backend on a host tensor (bench.py's group
    is gloo: timing needs no device collective)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
