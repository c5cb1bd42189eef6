"""Per-segment batch metadata: ReportIdChecksum and client-timestamp
interval, GPU (prio3_device_batch_metadata / prio3_batch_metadata) against the oracle.

The checksum semantics follow core/src/report_id.rs:18-42 (SHA-256 of the report ID, XOR
combine) as folded in aggregation_job_writer.rs:637-690; the XOR-combine property is the one
aggregator/src/aggregator/http_handlers/tests/aggregate_share.rs:183-200,333-418 rely on
(checksum of a union = XOR of the parts).  Interval semantics: core/src/time.rs:294-317.
"""
import hashlib

import numpy as np
import pytest

from oracle.oracle import batch_metadata

VK = bytes(range(16))


def test_sha256_fips180_kat():
    # FIPS 180-4 example "abc" -- the digest the oracle (hashlib) and ring both compute
    assert hashlib.sha256(b"abc").hexdigest() == \
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"


def test_oracle_checksum_is_xor_of_digests_and_unions_combine():
    rng = np.random.default_rng(1)
    ids = rng.integers(0, 256, (50, 16), dtype=np.uint8)
    st = np.zeros(50, np.uint8)
    st[[3, 9]] = 3                      # failed reports are not in the checksum / count
    ck, _ = batch_metadata(ids, None, st)
    exp = np.zeros(32, np.uint8)
    for r in range(50):
        if st[r] == 0:
            exp ^= np.frombuffer(hashlib.sha256(ids[r].tobytes()).digest(), np.uint8)
    np.testing.assert_array_equal(ck[0], exp)
    # two segments' checksums XOR to the single-segment one (merge of batch aggregations)
    seg = (np.arange(50) >= 20).astype(np.uint32)
    ck2, _ = batch_metadata(ids, None, st, segment_ids=seg, n_segments=2)
    np.testing.assert_array_equal(ck2[0] ^ ck2[1], ck[0])


def test_oracle_interval_semantics():
    ids = np.zeros((4, 16), np.uint8)
    t = np.array([10, 5, 7, 100], np.uint64)
    st = np.array([0, 3, 0, 0], np.uint8)   # a failed report still widens the interval
    seg = np.array([0, 0, 0, 2], np.uint32)
    _, iv = batch_metadata(ids, t, st, segment_ids=seg, n_segments=3)
    assert iv[0].tolist() == [5, 6]          # [5, 11)
    assert iv[1].tolist() == [0, 0]          # Interval::EMPTY
    assert iv[2].tolist() == [100, 1]        # from_time: one second


def _case(n, n_segments, mode, seed):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    t = (1_700_000_000 + rng.integers(0, 7200, n)).astype(np.uint64)
    st = np.where(rng.random(n) < 0.05, rng.integers(1, 6, n), 0).astype(np.uint8)
    mask = (rng.random(n) < 0.95).astype(np.uint8)
    if mode == "runs":
        seg = np.sort(rng.integers(0, n_segments, n)).astype(np.uint32)
    else:
        seg = rng.integers(0, n_segments, n).astype(np.uint32)
    return ids, t, st, mask, seg


@pytest.mark.gpu
@pytest.mark.parametrize("n,n_segments,mode", [(1, 1, "runs"), (255, 1, "runs"),
                                               (5000, 7, "runs"), (3000, 5, "random"),
                                               (70000, 3, "runs")])
def test_gpu_batch_metadata_matches_oracle(n, n_segments, mode):
    import torch
    from janus_amd import prio3 as J
    ids, t, st, mask, seg = _case(n, n_segments, mode, seed=n + n_segments)
    eng = J.HelperEngine(J.Prio3Histogram(10, 3), VK, device=0)
    exp_ck, exp_iv = batch_metadata(ids, t, st, mask, seg, n_segments)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ck = torch.full((n_segments, 32), 0xAB, dtype=torch.uint8, device=dev)  # overwritten
    iv = torch.full((n_segments, 2), 7, dtype=torch.int64, device=dev)
    eng.batch_metadata_device(T(ids), T(t.view(np.int64)), T(st), T(mask), T(seg), n_segments,
                              ck, iv)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ck.cpu().numpy(), exp_ck)
    np.testing.assert_array_equal(iv.cpu().numpy().view(np.uint64), exp_iv)
    # host-buffer form, no mask / no times
    hck, hiv = eng.batch_metadata(ids, None, st, None, seg, n_segments)
    eck, eiv = batch_metadata(ids, None, st, None, seg, n_segments)
    np.testing.assert_array_equal(hck, eck)
    np.testing.assert_array_equal(hiv, eiv)


@pytest.mark.gpu
def test_gpu_batch_metadata_empty_batch():
    from janus_amd import prio3 as J
    eng = J.HelperEngine(J.Prio3Count(), VK, device=0)
    ck, iv = eng.batch_metadata(np.zeros((0, 16), np.uint8), np.zeros(0, np.uint64),
                                np.zeros(0, np.uint8), n_segments=2)
    assert not ck.any() and not iv.any()
