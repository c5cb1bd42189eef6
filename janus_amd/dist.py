"""Multi-GPU layer: report sharding and the cross-rank aggregate-share combine.

One process per GPU (``torch.distributed``; backend ``nccl`` is RCCL on ROCm).  Reports are
independent, so each rank prepares a contiguous range of the batch with no collective on the
data path.  The only exchange is the per-rank partial aggregate share
(``n_segments x agg_share_len`` bytes plus ``u64`` counts per segment): it is all-gathered over
xGMI and summed mod p by ``prio3_device_combine`` -- RCCL's integer reduction is mod 2^64, not
mod p, so an ``all_reduce(SUM)`` would be wrong.

The analogue in Janus is merging per-shard ``batch_aggregations`` rows at collection time
(``/root/reference/aggregator/src/aggregator/aggregate_share.rs:55-96``), which is also a
mod-p element-wise sum of encoded aggregate shares.

This module is the code bench.py runs for N > 1; tests/test_dist.py drives it with ``gloo`` on
CPU tensors, where the combine callable is the test's own mod-p sum.
"""
from __future__ import annotations

from typing import Callable, Tuple


def shard_bounds(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) report range of ``rank``; sizes differ by at most one report."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class AggregateCombiner:
    """Gathers every rank's partial aggregate share and reduces them mod p.

    ``combine(k, gathered_agg, gathered_counts, out_agg, out_counts)`` does the mod-p sum of
    the k gathered partials (on the GPU: ``HelperEngine.combine_device``).  Buffers are
    preallocated once, so a step issues exactly two all-gathers and one combine launch.
    """

    def __init__(self, dist, agg, counts, combine: Callable):
        import torch
        self.dist = dist
        self.world = dist.get_world_size()
        self.combine = combine
        self.g_agg = torch.empty((self.world,) + tuple(agg.shape), dtype=agg.dtype,
                                 device=agg.device)
        self.g_cnt = torch.empty((self.world,) + tuple(counts.shape), dtype=counts.dtype,
                                 device=counts.device)
        self.out_agg = torch.empty_like(agg)
        self.out_cnt = torch.empty_like(counts)

    def __call__(self, agg, counts):
        self.dist.all_gather_into_tensor(self.g_agg.view(-1), agg.contiguous().view(-1))
        self.dist.all_gather_into_tensor(self.g_cnt.view(-1), counts.contiguous().view(-1))
        self.combine(self.world, self.g_agg, self.g_cnt, self.out_agg, self.out_cnt)
        return self.out_agg, self.out_cnt
