"""GPU parity of the leader side against the CPU restatement.

prio3_leader_prepare_init_batch is prio's Prio3::prepare_init with agg_id 0 (Janus's
leader_initialized, aggregation_job_driver.rs:397-415) and prio3_leader_prepare_next_batch is
prepare_next on the helper's prepare message (leader_continued, :677-691).  Reports are sharded
by the oracle's client (orc_shard) from seeded randomness; prepare shares, statuses, output
shares and aggregates must equal the oracle's bit for bit.  The last test runs a whole
aggregation job through both roles on the device and unshards it to the plaintext.
"""
import numpy as np
import pytest

from tests.conftest import CONFIGS
from tests.test_gpu_parity import VK, _engine, _oracle

pytestmark = pytest.mark.gpu


def _measurement(cfg, rng):
    k = cfg["kind"]
    if k == "count":
        return int(rng.integers(0, 2))
    if k == "sum":  # up to 64 bits (beyond numpy's int64 bounds)
        return int.from_bytes(rng.bytes(8), "little") >> (64 - cfg["bits"])
    if k == "sumvec":
        return [int(x) for x in rng.integers(0, 1 << cfg["bits"], cfg["length"])]
    return int(rng.integers(0, cfg["length"]))


def _reports(o, cfg, n, seed):
    rng = np.random.default_rng(seed)
    nonces, pubs, ls, hs, meas = [], [], [], [], []
    for _ in range(n):
        m = _measurement(cfg, rng)
        nonce = rng.bytes(16)
        pub, l, h = o.shard(m, nonce, rng.bytes(o.rand_size))
        nonces.append(nonce), pubs.append(pub), ls.append(l), hs.append(h), meas.append(m)
    arr = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(n, -1).copy() if xs[0] else \
        np.zeros((n, 0), np.uint8)
    return dict(nonces=arr(nonces), public_shares=arr(pubs), leader_shares=arr(ls),
                helper_shares=arr(hs), measurements=meas)


@pytest.mark.parametrize("fast", [1, 0])
@pytest.mark.parametrize("name", ["count", "sum8", "sumvec_8x10_c9", "hist_256_c16", "hist_10_c3",
                                  "hist_100_c10", "sum15", "sum17", "sum32", "sum64"])
def test_leader_parity_vs_oracle(name, fast):
    cfg = CONFIGS[name]
    o, eng = _oracle(cfg), _engine(cfg)
    eng.set_option("leader_fast", fast)
    n = 150
    d = _reports(o, cfg, n, seed=31)
    # corrupt: a non-canonical leader measurement-share element in one report
    d["leader_shares"][9, :o.es] = 0xFF
    ps, st, batch = eng.leader_prepare_init_batch(d["nonces"], d["public_shares"], d["leader_shares"])
    ref_ps, states, msgs, ref_out = [], [], [], []
    for i in range(n):
        rc, state, lps = o.prepare_init(VK, 0, d["nonces"][i].tobytes(), d["public_shares"][i].tobytes(),
                                        d["leader_shares"][i].tobytes())
        ref_ps.append(lps if rc == 0 else None)
        states.append(state)
        rc2, _, hps = o.prepare_init(VK, 1, d["nonces"][i].tobytes(), d["public_shares"][i].tobytes(),
                                     d["helper_shares"][i].tobytes())
        msg = b""
        if rc == 0 and rc2 == 0:
            rc3, msg = o.prep_shares_to_prep_msg(lps, hps)
        msgs.append(msg)
    assert st[9] == 6  # PRIO3_STATUS_INPUT_SHARE_DECODE
    for i in range(n):
        if i == 9:
            continue
        assert st[i] == 0
        assert ps[i].tobytes() == ref_ps[i], i
    # prepare_next with the prepare messages; corrupt one (joint-rand mismatch)
    msg_arr = np.zeros((n, eng.sz.prep_msg_len), np.uint8)
    for i in range(n):
        if msgs[i]:
            msg_arr[i] = np.frombuffer(msgs[i], np.uint8)
    if eng.sz.prep_msg_len:
        msg_arr[17, 0] ^= 1
    st2 = batch.leader_prepare_next(msg_arr, st)
    want = st.copy()
    if eng.sz.prep_msg_len:
        want[17] = 4  # PRIO3_STATUS_PREP_NEXT
    np.testing.assert_array_equal(st2, want)
    outs = batch.output_shares()
    ref_sum = None
    for i in range(n):
        if want[i] != 0:
            continue
        rc, out = o.prepare_next(states[i], msgs[i])
        assert rc == 0 and outs[i].tobytes() == out, i
    # aggregate into two segments with a host mask
    seg = (np.arange(n) % 2).astype(np.uint32)
    accept = np.ones(n, np.uint8)
    accept[3] = 0
    agg, cnt = batch.accumulate(seg, accept, 2)
    from oracle.oracle import field_modulus
    p = field_modulus(cfg["kind"])
    es = o.es
    for s in range(2):
        idx = [i for i in range(n) if seg[i] == s and want[i] == 0 and accept[i]]
        assert int(cnt[s]) == len(idx)
        tot = [0] * (eng.sz.agg_share_len // es)
        for i in idx:
            row = outs[i].tobytes()
            for e in range(len(tot)):
                tot[e] = (tot[e] + int.from_bytes(row[e * es:(e + 1) * es], "little")) % p
        assert agg[s].tobytes() == b"".join(v.to_bytes(es, "little") for v in tot)


@pytest.mark.parametrize("name", ["hist_10_c3", "hist_256_c16", "sum32"])
def test_leader_slow_path(name):
    cfg = CONFIGS[name]
    o, eng = _oracle(cfg), _engine(cfg)
    eng.set_option("force_slow_path", 1)
    d = _reports(o, cfg, 70, seed=5)
    ps, st, _ = eng.leader_prepare_init_batch(d["nonces"], d["public_shares"], d["leader_shares"])
    assert not st.any()
    for i in range(70):
        rc, _, lps = o.prepare_init(VK, 0, d["nonces"][i].tobytes(), d["public_shares"][i].tobytes(),
                                    d["leader_shares"][i].tobytes())
        assert rc == 0 and ps[i].tobytes() == lps


@pytest.mark.parametrize("name", ["hist_256_c16", "sum8", "count", "sum32"])
def test_full_job_both_roles_unshard(name):
    """Leader init (GPU) -> helper init+finish (GPU) -> leader continue (GPU) -> both
    aggregates unshard to the plaintext sum (integration_tests/.../common.rs:332-554)."""
    from oracle.oracle import field_modulus
    cfg = CONFIGS[name]
    o = _oracle(cfg)
    leader, helper = _engine(cfg), _engine(cfg)
    n = 300
    d = _reports(o, cfg, n, seed=8)
    lps, lst, lbatch = leader.leader_prepare_init_batch(d["nonces"], d["public_shares"],
                                                        d["leader_shares"])
    msgs, hst, hbatch = helper.prepare_batch(d["nonces"], d["public_shares"], d["helper_shares"], lps)
    assert not lst.any() and not hst.any()
    lst2 = lbatch.leader_prepare_next(msgs, lst)
    assert not lst2.any()
    la, lc = lbatch.accumulate()
    ha, hc = hbatch.accumulate()
    assert int(lc[0]) == int(hc[0]) == n
    p, es = field_modulus(cfg["kind"]), o.es
    dec = lambda b: [int.from_bytes(b[i:i + es], "little") for i in range(0, len(b), es)]
    tot = [(a + b) % p for a, b in zip(dec(la[0].tobytes()), dec(ha[0].tobytes()))]
    if cfg["kind"] == "histogram":
        exp = np.bincount(d["measurements"], minlength=cfg["length"]).tolist()
    else:
        exp = [sum(d["measurements"])]
    assert tot == exp


@pytest.mark.parametrize("fuse", [1, 0])
@pytest.mark.parametrize("name", ["hist_256_c16", "hist_10_c3", "hist_100_c10"])
def test_device_leader_fused_accumulate(name, fuse):
    """The device-resident leader step (bench.py --role leader): init -> next -> accumulate, the
    accumulate fused into k_jrpart's wave partials (option leader_fuse_acc = 1) or the separate
    segmented pass, against the host-batch leader path (pinned to the oracle above).  A
    non-canonical leader share, a tampered prepare message, a ragged batch, a host mask,
    out-of-range segment ids with one segment (fused + fix-ups) and three segments (the
    separate pass)."""
    import torch
    cfg = CONFIGS[name]
    o = _oracle(cfg)
    ref, helper, eng = _engine(cfg), _engine(cfg), _engine(cfg)
    eng.set_option("leader_fuse_acc", fuse)
    n = 300
    d = _reports(o, cfg, n, seed=77)
    d["leader_shares"][9, :o.es] = 0xFF
    lps, lst, lbatch = ref.leader_prepare_init_batch(d["nonces"], d["public_shares"],
                                                     d["leader_shares"])
    msgs, _, _ = helper.prepare_batch(d["nonces"], d["public_shares"], d["helper_shares"], lps)
    msgs = msgs.copy()
    msgs[17, -1] ^= 1
    lst2 = lbatch.leader_prepare_next(msgs, lst.copy())
    assert lst[9] != 0 and lst2[17] != 0 and (lst2 == 0).sum() > n - 5
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda")
    ps_d = torch.zeros(lps.shape, dtype=torch.uint8, device="cuda")
    st_d = torch.zeros(n, dtype=torch.uint8, device="cuda")
    eng.leader_prepare_init_device(t(d["nonces"]), t(d["public_shares"]), t(d["leader_shares"]),
                                   ps_d, st_d)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st_d.cpu().numpy(), lst)
    ok = lst == 0
    np.testing.assert_array_equal(ps_d.cpu().numpy()[ok], lps[ok])
    eng.leader_prepare_next_device(n, t(msgs), st_d)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st_d.cpu().numpy(), lst2)
    rng = np.random.default_rng(3)
    accept = (rng.random(n) > 0.1).astype(np.uint8)
    seg1 = np.where(rng.random(n) > 0.05, 0, 5).astype(np.uint32)
    seg3 = rng.integers(0, 3, n).astype(np.uint32)
    for seg, acc, S in [(None, None, 1), (seg1, accept, 1), (None, accept, 1), (seg3, accept, 3)]:
        ra, rc = lbatch.accumulate(seg, acc, S)
        agg = torch.zeros(ra.shape, dtype=torch.uint8, device="cuda")
        cnt = torch.zeros(S, dtype=torch.int64, device="cuda")
        eng.accumulate_device(n, st_d, None if seg is None else t(seg),
                              None if acc is None else t(acc), S, agg, cnt)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(agg.cpu().numpy(), ra)
        np.testing.assert_array_equal(cnt.cpu().numpy().astype(np.uint64), rc)
