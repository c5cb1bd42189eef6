"""GPU, BASELINE.json config sizes (per-GPU shard), through size-independent properties.

The oracle is too slow at these sizes, so each case checks what must hold for any correct
engine (the semantic known answer of integration_tests/tests/integration/common.rs:332-554):
every honest report finishes, the count is n, and the leader aggregate (summed from the
on-device client's leader output shares) plus the helper aggregate unshards to the plaintext
sum of the measurements.  Bit-exactness at small sizes is test_gpu_parity.py's job.

  C1 Prio3Count, 100k reports                       (configs[0], plumbing size)
  C3 Prio3SumVec bits=8 length=1000, 1M/8 reports   (configs[2], one GPU's shard)
  C4 Prio3Sum bits=32, 10M/8 reports                 (configs[3], one GPU's shard)
  C3 at its whole 1M and C4 at its whole 10M on ONE GPU: the 8-GPU totals
  fit one MI355X's HBM (C3's leader output shares are 16 GB), so the same properties hold
  over the whole configured workload, not only a shard
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VK = bytes(range(0x60, 0x70))


def _decode(buf, es):
    b = np.ascontiguousarray(buf, np.uint8).reshape(-1, es)
    return [int.from_bytes(r.tobytes(), "little") for r in b]


def _run(vdaf, n, field_p, es):
    import torch
    from janus_amd import prio3 as J
    eng = J.HelperEngine(vdaf, VK, device=0)
    sz = eng.sz
    d = eng.generate_reports_device(n, seed=4242, with_checks=True)
    assert int(d["flags"].sum()) == 0
    dev = d["nonces"].device
    msgs = torch.empty((n, max(sz.prep_msg_len, 1)), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    agg = torch.zeros((1, sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    pub = d["public_shares"] if sz.public_share_len else None
    eng.prepare_aggregate_device(d["nonces"], pub, d["helper_shares"], d["leader_prep_shares"],
                                 seg, 1, msgs, status)
    eng.aggregate_finish_device(status, None, agg, cnt)
    # leader aggregate: mod-p sum of the n leader output shares (the multi-GPU combine kernel
    # with one "rank" per report), in two levels so no work-item loops over millions of rows:
    # k1 rows of k2 "segments", then the k2 partial sums
    k1 = next(k for k in (1000, 500, 100, 10, 1) if n % k == 0)
    k2 = n // k1
    part = torch.zeros((k2, sz.agg_share_len), dtype=torch.uint8, device=dev)
    pcnt = torch.zeros(k2, dtype=torch.int64, device=dev)
    eng.combine_device(k1, k2, d["leader_out_shares"],
                       torch.zeros(n, dtype=torch.int64, device=dev), part, pcnt)
    lagg = torch.zeros((1, sz.agg_share_len), dtype=torch.uint8, device=dev)
    lcnt = torch.zeros(1, dtype=torch.int64, device=dev)
    eng.combine_device(k2, 1, part, pcnt, lagg, lcnt)
    meas_sum = d["measurements"].sum(dim=0).cpu().numpy()
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert int(cnt[0]) == n
    h = _decode(agg.cpu().numpy(), es)
    lo = _decode(lagg.cpu().numpy(), es)
    tot = [(a + b) % field_p for a, b in zip(h, lo)]
    return tot, [int(x) for x in meas_sum]


def test_c1_count_100k():
    from janus_amd import prio3 as J
    tot, exp = _run(J.Prio3Count(), 100_000, 2**64 - 2**32 + 1, 8)
    assert tot == exp


def test_c4_sum32_shard_of_10m():
    from janus_amd import prio3 as J
    tot, exp = _run(J.Prio3Sum(32), 10_000_000 // 8, 2**128 - 28 * 2**64 + 1, 16)
    assert tot == exp


def test_c3_sumvec_8x1000_shard_of_1m():
    from janus_amd import prio3 as J
    tot, exp = _run(J.Prio3SumVec(8, 1000, 63), 1_000_000 // 8, 2**128 - 28 * 2**64 + 1, 16)
    assert tot == exp


def test_c4_sum32_whole_10m_one_gpu():
    from janus_amd import prio3 as J
    tot, exp = _run(J.Prio3Sum(32), 10_000_000, 2**128 - 28 * 2**64 + 1, 16)
    assert tot == exp


def test_c3_sumvec_8x1000_whole_1m_one_gpu():
    import torch
    from janus_amd import prio3 as J
    tot, exp = _run(J.Prio3SumVec(8, 1000, 63), 1_000_000, 2**128 - 28 * 2**64 + 1, 16)
    torch.cuda.empty_cache()
    assert tot == exp
