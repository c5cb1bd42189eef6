"""Multi-rank path (janus_amd/dist.py) on CPU with the gloo backend, world size 2.

Each rank prepares its contiguous shard of one report batch and produces a partial
per-segment aggregate share; AggregateCombiner all-gathers the partials and sums them mod p.
The result must equal the single-process aggregate of the whole batch -- the same property
Janus relies on when it merges per-shard batch aggregations at collection time
(aggregator/src/aggregator/aggregate_share.rs:55-96).  On CPU the oracle stands in for the
per-rank device engine and a numpy mod-p sum for prio3_device_combine; on a GPU box bench.py
runs the same code with RCCL and the HIP combine kernel.
"""
import os
import socket

import numpy as np
import pytest

from janus_amd.dist import shard_bounds

VK = bytes(range(16))
CFG = dict(kind="histogram", length=10, chunk_length=3)
N, NSEG = 300, 3


def test_shard_bounds_cover_exactly_once():
    for n in (0, 1, 7, 64, 1000):
        for world in (1, 2, 3, 8):
            got = [shard_bounds(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            sizes = [hi - lo for lo, hi in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _modp_combine(p, es):
    import torch

    def combine(k, g_agg, g_cnt, out_agg, out_cnt):
        a = g_agg.numpy().reshape(k, -1, es)
        tot = []
        for j in range(a.shape[1]):
            tot.append(sum(int.from_bytes(a[i, j].tobytes(), "little") for i in range(k)) % p)
        out = b"".join(v.to_bytes(es, "little") for v in tot)
        out_agg.copy_(torch.frombuffer(bytearray(out), dtype=torch.uint8).view(out_agg.shape))
        out_cnt.copy_(g_cnt.sum(dim=0))
    return combine


def _meta_combine(k, g_ck, g_iv, out_ck, out_iv):
    """numpy stand-in for prio3_device_combine_metadata: XOR, Interval::merge."""
    import torch
    ck = np.bitwise_xor.reduce(g_ck.numpy(), axis=0)
    iv = g_iv.numpy().view(np.uint64)
    res = np.zeros(iv.shape[1:], np.uint64)
    for s in range(iv.shape[1]):
        spans = [(a, a + d) for a, d in iv[:, s] if d]
        if spans:
            lo, hi = min(a for a, _ in spans), max(b for _, b in spans)
            res[s] = (lo, hi - lo)
    out_ck.copy_(torch.from_numpy(ck))
    out_iv.copy_(torch.from_numpy(res.view(np.int64)))


def _times():
    return (1_700_000_000 + (np.arange(N) * 7919) % 5000).astype(np.uint64)


def _rank(rank, world, port, result_path):
    import torch
    import torch.distributed as dist
    from janus_amd.dist import AggregateCombiner
    from oracle.oracle import Oracle, batch_metadata, field_modulus
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = Oracle(**CFG)
    d = o.gen_reports(VK, N, seed=77, n_threads=2)  # identical batch on every rank
    seg = (np.arange(N) * NSEG // N).astype(np.uint32)
    lo, hi = shard_bounds(N, rank, world)
    sl = slice(lo, hi)
    _, _, agg, cnt = o.helper_batch(VK, d["nonces"][sl], d["public_shares"][sl],
                                    d["helper_shares"][sl], d["leader_prep_shares"][sl],
                                    segment_ids=seg[sl], n_segments=NSEG, n_threads=2)
    st = o.helper_batch(VK, d["nonces"][sl], d["public_shares"][sl], d["helper_shares"][sl],
                        d["leader_prep_shares"][sl], n_threads=2)[1]
    ck, iv = batch_metadata(d["nonces"][sl], _times()[sl], st, None, seg[sl], NSEG)
    agg_t = torch.from_numpy(agg.copy())
    cnt_t = torch.from_numpy(cnt.astype(np.int64))
    ck_t = torch.from_numpy(ck)
    iv_t = torch.from_numpy(iv.view(np.int64).copy())
    comb = AggregateCombiner(dist, agg_t, cnt_t, _modp_combine(field_modulus("histogram"), 16),
                             ck_t, iv_t, _meta_combine)
    out_agg, out_cnt, out_ck, out_iv = comb(agg_t, cnt_t, ck_t, iv_t)
    if rank == 0:
        np.savez(result_path, agg=out_agg.numpy(), cnt=out_cnt.numpy(), ck=out_ck.numpy(),
                 iv=out_iv.numpy())
    dist.destroy_process_group()


def test_two_rank_combine_equals_single_process(tmp_path):
    import torch.multiprocessing as mp
    from oracle.oracle import Oracle, batch_metadata
    res = str(tmp_path / "r.npz")
    mp.spawn(_rank, args=(2, _free_port(), res), nprocs=2, join=True)
    got = np.load(res)
    o = Oracle(**CFG)
    d = o.gen_reports(VK, N, seed=77, n_threads=2)
    seg = (np.arange(N) * NSEG // N).astype(np.uint32)
    _, _, agg, cnt = o.helper_batch(VK, d["nonces"], d["public_shares"], d["helper_shares"],
                                    d["leader_prep_shares"], segment_ids=seg, n_segments=NSEG,
                                    n_threads=2)
    np.testing.assert_array_equal(got["agg"], agg)
    np.testing.assert_array_equal(got["cnt"].astype(np.uint64), cnt)
    st = o.helper_batch(VK, d["nonces"], d["public_shares"], d["helper_shares"],
                        d["leader_prep_shares"], n_threads=2)[1]
    ck, iv = batch_metadata(d["nonces"], _times(), st, None, seg, NSEG)
    np.testing.assert_array_equal(got["ck"], ck)
    np.testing.assert_array_equal(got["iv"].view(np.uint64), iv)
