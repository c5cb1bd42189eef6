"""Multi-GPU layer: report sharding and the cross-rank aggregate-share combine.

One process per GPU (``torch.distributed``; backend ``nccl`` is RCCL on ROCm).  Reports are
independent, so each rank prepares a contiguous range of the batch with no collective on the
data path.  The only exchange is the per-rank partial aggregate share
(``n_segments x agg_share_len`` bytes plus ``u64`` counts, the 32-byte report-ID checksum and
the client-timestamp interval per segment): it is all-gathered over xGMI in one packed
collective and summed mod p by ``prio3_device_combine`` (checksums XORed, intervals merged by
``prio3_device_combine_metadata``) -- RCCL's integer reduction is mod 2^64, not
mod p, so an ``all_reduce(SUM)`` would be wrong.

The analogue in Janus is merging per-shard ``batch_aggregations`` rows at collection time
(``/root/reference/aggregator/src/aggregator/aggregate_share.rs:55-96``), which is also a
mod-p element-wise sum of encoded aggregate shares.

This module is the code bench.py runs for N > 1.  tests/test_dist.py drives it with ``gloo`` on
CPU tensors (the combine callable is the test's own mod-p sum); tests/test_gpu_dist.py runs two
ranks whose partials come from the HIP engine and whose combine is the HIP kernel, with the
collective staged through host memory for gloo.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple


def shard_bounds(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) report range of ``rank``; sizes differ by at most one report."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class AggregateCombiner:
    """Gathers every rank's partial batch aggregation and reduces it.

    The per-rank partials -- aggregate shares [S, agg_len] (uint8), counts [S] (int64) and,
    optionally, the batch metadata (ReportIdChecksum [S, 32] uint8, interval [S, 2] int64) --
    are packed into one byte row, so a step issues exactly ONE all-gather over xGMI (the
    payload is a few KiB: latency-bound, so one collective instead of four).  Then
    ``combine(k, gathered_agg, gathered_counts, out_agg, out_counts)`` does the mod-p sum
    (on the GPU: ``HelperEngine.combine_device``) and ``combine_meta(k, gathered_checksums,
    gathered_intervals, out_checksums, out_intervals)`` the XOR / Interval::merge
    (``HelperEngine.combine_metadata_device``).  Buffers are preallocated once.
    """

    def __init__(self, dist, agg, counts, combine: Callable, checksums=None, intervals=None,
                 combine_meta: Optional[Callable] = None, stage_device=None):
        """stage_device: where the collective's buffers live when it differs from the partials'
        device (e.g. "cpu" for a gloo group whose partials come from a GPU engine); the gathered
        rows are copied back to the partials' device for the combine kernels."""
        import torch
        self.dist = dist
        self.world = dist.get_world_size()
        self.combine = combine
        self.combine_meta = combine_meta
        self.meta = checksums is not None
        dev = agg.device
        self.shapes = [tuple(agg.shape), tuple(counts.shape)]
        self.dtypes = [agg.dtype, counts.dtype]
        if self.meta:
            self.shapes += [tuple(checksums.shape), tuple(intervals.shape)]
            self.dtypes += [checksums.dtype, intervals.dtype]
        self.nbytes = [int(torch.empty(sh, dtype=dt, device="meta").numel()) *
                       torch.empty((), dtype=dt).element_size()
                       for sh, dt in zip(self.shapes, self.dtypes)]
        self.row = sum(self.nbytes)
        self.dev = dev
        cdev = torch.device(stage_device) if stage_device is not None else dev
        self.send = torch.empty(self.row, dtype=torch.uint8, device=cdev)
        self.gathered = torch.empty((self.world, self.row), dtype=torch.uint8, device=cdev)
        self.gathered_dev = (self.gathered if cdev == dev else
                             torch.empty((self.world, self.row), dtype=torch.uint8, device=dev))
        self.outs = [torch.empty(sh, dtype=dt, device=dev)
                     for sh, dt in zip(self.shapes, self.dtypes)]
        self.out_agg, self.out_cnt = self.outs[0], self.outs[1]
        if self.meta:
            self.out_checksums, self.out_intervals = self.outs[2], self.outs[3]

    def _gathered(self, idx):
        import torch
        off = sum(self.nbytes[:idx])
        g = self.gathered_dev[:, off:off + self.nbytes[idx]].contiguous()
        return g.view(self.dtypes[idx]).view((self.world,) + self.shapes[idx]) \
            if self.dtypes[idx] != torch.uint8 else g.view((self.world,) + self.shapes[idx])

    def __call__(self, agg, counts, checksums=None, intervals=None):
        import torch
        parts = [agg, counts] + ([checksums, intervals] if self.meta else [])
        flat = [t.contiguous().view(-1).view(torch.uint8) for t in parts]
        if self.send.device == self.dev:
            torch.cat(flat, out=self.send)
        else:
            self.send.copy_(torch.cat(flat))
        self.dist.all_gather_into_tensor(self.gathered.view(-1), self.send)
        if self.gathered_dev is not self.gathered:
            self.gathered_dev.copy_(self.gathered)
        self.combine(self.world, self._gathered(0), self._gathered(1), self.out_agg, self.out_cnt)
        if self.meta:
            self.combine_meta(self.world, self._gathered(2), self._gathered(3),
                              self.out_checksums, self.out_intervals)
            return self.out_agg, self.out_cnt, self.out_checksums, self.out_intervals
        return self.out_agg, self.out_cnt
