"""GPU, every BASELINE.json config at its benchmark size, against the oracle.

Collected first among the `-m gpu` tests (alphabetical order of tests/), so a driver run pins
the configs before anything else.  Each case drives the exact chain `bench.py` times --
prio3_device_prepare_aggregate (the fused XOF + query kernel and the fused wave-partial
accumulate) -> prio3_device_aggregate_finish (k_agg_*) -> prio3_device_batch_metadata -- on
device-generated reports with a sprinkling of tampered ones, and compares with the C
restatement's Janus job driver (oracle.helper_batch, the per-report loop of
aggregator.rs:2020-2042 plus the merge of aggregation_job_writer.rs:591-695) and the
checksum / interval oracle (report_id.rs:18-42, time.rs:294-317), as the reference's
transcript tests compare with prio (core/src/test_util/mod.rs:86-232).

  C1 Prio3Count, 100k reports                        full oracle parity
  C2 Prio3Histogram(256, 16), 1,048,576 reports      full oracle parity, 1 and 8 segments
  C3 Prio3SumVec(8, 1000, 63), 125k (one GPU's 1/8)  oracle parity on an 8,192-report subset;
                                                     the whole batch by unshard (test_gpu_fullsize)
  C4 Prio3Sum(32), 1.25M (one GPU's 1/8)             full oracle parity
  C5 FixedPointBoundedL2VecSum(10000), 100k          tests/test_fpvec_client.py: 100k distinct
                                                     device-generated reports, unshard over all
                                                     of them and the C restatement on a subset
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VK = bytes.fromhex("4a414e55532d414d442d42454e434821")  # bench.py's verify key
SEED = 0x4A414E5553000001                                # bench.py's report seed


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _tamper(d, es, jr, stride):
    """Flip a few reports on the device: decide (verifier bit), decode (element >= p),
    joint-rand mismatch (leader part) and wrong public share; returns the tampered indices."""
    import torch
    n = d["nonces"].shape[0]
    lps = d["leader_prep_shares"]
    dec = torch.arange(1, n, stride, device=lps.device)
    lps[dec, es] ^= 1
    bad = torch.arange(3, n, 3 * stride, device=lps.device)
    lps[bad, :es] = 0xFF
    if jr:
        j = torch.arange(5, n, 2 * stride, device=lps.device)
        lps[j, -1] ^= 0x80
        p = torch.arange(7, n, 5 * stride, device=lps.device)
        d["public_shares"][p, 3] ^= 0x10


def _chain(eng, d, seg, n_segments, times):
    """bench.py's step: prepare + fused aggregate, finish, batch metadata."""
    import torch
    sz = eng.sz
    n = d["nonces"].shape[0]
    dev = d["nonces"].device
    msgs = torch.empty((n, max(sz.prep_msg_len, 1)), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    agg = torch.zeros((n_segments, sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(n_segments, dtype=torch.int64, device=dev)
    cks = torch.zeros((n_segments, 32), dtype=torch.uint8, device=dev)
    ivs = torch.zeros((n_segments, 2), dtype=torch.int64, device=dev)
    pub = d["public_shares"] if sz.public_share_len else None
    eng.prepare_aggregate_device(d["nonces"], pub, d["helper_shares"], d["leader_prep_shares"],
                                 seg, n_segments, msgs, status)
    eng.aggregate_finish_device(status, None, agg, cnt)
    eng.batch_metadata_device(d["nonces"], times, status, None, seg, n_segments, cks, ivs)
    torch.cuda.synchronize()
    return msgs, status, agg, cnt, cks, ivs


def _host(d, m=None):
    sl = slice(None) if m is None else slice(0, m)
    return {k: d[k][sl].cpu().numpy() for k in
            ("nonces", "public_shares", "helper_shares", "leader_prep_shares")}


def _fullsize(vdaf, okw, n, stride, segment_sets=(1,)):
    import torch
    from janus_amd import prio3 as J
    from oracle.oracle import Oracle, batch_metadata
    eng = J.HelperEngine(vdaf, VK, device=0)
    sz = eng.sz
    d = eng.generate_reports_device(n, seed=SEED)
    _tamper(d, 8 if okw["kind"] == "count" else 16, sz.public_share_len > 0, stride)
    dev = d["nonces"].device
    g = torch.Generator(device=dev).manual_seed(0x4A414E55)
    times = 1_700_000_000 + torch.randint(0, 3600, (n,), generator=g, device=dev,
                                          dtype=torch.int64)
    h = _host(d)
    o = Oracle(**okw)
    S = max(segment_sets)
    seg_np = np.sort(np.random.default_rng(5).integers(0, S, n)).astype(np.uint32)
    rm, rs, ra, rc = o.helper_batch(VK, h["nonces"], h["public_shares"], h["helper_shares"],
                                    h["leader_prep_shares"], segment_ids=seg_np, n_segments=S,
                                    n_threads=_threads(), job_size=500)
    assert set(np.unique(rs).tolist()) >= {0, 2, 3}
    p = o.p
    P = 2**64 - 2**32 + 1 if okw["kind"] == "count" else 2**128 - 28 * 2**64 + 1
    es = p.es
    t_np = times.cpu().numpy()
    for n_seg in segment_sets:
        if n_seg == 1:
            seg = torch.zeros(n, dtype=torch.int32, device=dev)
            ra_s = np.zeros((1, ra.shape[1]), np.uint8)
            tot = [0] * (ra.shape[1] // es)
            for s in range(S):
                row = np.ascontiguousarray(ra[s]).reshape(-1, es)
                for e in range(len(tot)):
                    tot[e] = (tot[e] + int.from_bytes(row[e].tobytes(), "little")) % P
            ra_s[0] = np.frombuffer(b"".join(v.to_bytes(es, "little") for v in tot), np.uint8)
            rc_s = np.array([int(rc.sum())], np.uint64)
            seg_h = None
        else:
            seg = torch.from_numpy(seg_np.astype(np.int32)).to(dev)
            ra_s, rc_s, seg_h = ra, rc, seg_np
        msgs, status, agg, cnt, cks, ivs = _chain(eng, d, seg, n_seg, times)
        np.testing.assert_array_equal(status.cpu().numpy(), rs)
        np.testing.assert_array_equal(msgs[:, :rm.shape[1]].cpu().numpy(), rm)
        np.testing.assert_array_equal(cnt.cpu().numpy().astype(np.uint64), rc_s)
        np.testing.assert_array_equal(agg.cpu().numpy(), ra_s)
        eck, eiv = batch_metadata(h["nonces"], t_np, rs, None, seg_h, n_seg)
        np.testing.assert_array_equal(cks.cpu().numpy(), eck)
        np.testing.assert_array_equal(ivs.cpu().numpy().view(np.uint64), eiv)


def test_c2_histogram_1mi_bench_chain_vs_oracle():
    """configs[1], the headline: 1,048,576 Histogram(256,16) reports through bench.py's chain
    (fused k_prep_h + k_agg_* + k_meta), one segment as timed and eight segments."""
    from janus_amd import prio3 as J
    _fullsize(J.Prio3Histogram(256, 16), dict(kind="histogram", length=256, chunk_length=16),
              1 << 20, 4099, segment_sets=(1, 8))


def test_c1_count_100k_vs_oracle():
    from janus_amd import prio3 as J
    _fullsize(J.Prio3Count(), dict(kind="count"), 100_000, 997, segment_sets=(1, 3))


def test_c4_sum32_shard_vs_oracle():
    from janus_amd import prio3 as J
    _fullsize(J.Prio3Sum(32), dict(kind="sum", bits=32), 10_000_000 // 8, 4099,
              segment_sets=(1, 4))


def test_c3_sumvec_shard_subset_vs_oracle():
    """configs[2] at one GPU's share (125k): the whole batch on the device, the first 8,192
    reports against the oracle -- statuses, prepare messages, and their aggregate share and
    count (the device run finished again with an accept mask selecting the subset)."""
    import torch
    from janus_amd import prio3 as J
    from oracle.oracle import Oracle
    n, m = 1_000_000 // 8, 8192
    eng = J.HelperEngine(J.Prio3SumVec(8, 1000, 63), VK, device=0)
    d = eng.generate_reports_device(n, seed=SEED)
    _tamper(d, 16, True, 211)
    dev = d["nonces"].device
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    times = torch.full((n,), 1_700_000_000, dtype=torch.int64, device=dev)
    msgs, status, agg, cnt, _, _ = _chain(eng, d, seg, 1, times)
    h = _host(d, m)
    o = Oracle(kind="sumvec", bits=8, length=1000, chunk_length=63)
    rm, rs, ra, rc = o.helper_batch(VK, h["nonces"], h["public_shares"], h["helper_shares"],
                                    h["leader_prep_shares"], n_threads=_threads(), job_size=500)
    assert set(np.unique(rs).tolist()) >= {0, 2, 3, 4}
    np.testing.assert_array_equal(status[:m].cpu().numpy(), rs)
    np.testing.assert_array_equal(msgs[:m].cpu().numpy(), rm)
    accept = torch.zeros(n, dtype=torch.uint8, device=dev)
    accept[:m] = 1
    agg_s = torch.zeros_like(agg)
    cnt_s = torch.zeros_like(cnt)
    eng.aggregate_finish_device(status, accept, agg_s, cnt_s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(agg_s.cpu().numpy(), ra)
    assert int(cnt_s[0]) == int(rc[0])
    # the whole batch: every untampered report finishes
    assert int(cnt[0]) == int((status == 0).sum())
