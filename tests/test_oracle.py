"""CPU tests of the oracle (the parity checker): known-answer tests, field constants,
agreement of the two independent restatements, golden fixtures, completeness/soundness
and the end-to-end semantic known answer (unshard == plaintext sum,
/root/reference/integration_tests/tests/integration/common.rs:332-554)."""
import glob
import hashlib
import json
import os
import random

import numpy as np
import pytest

from tests.conftest import CONFIGS

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_shake128_matches_hashlib(oracle_lib):
    from oracle import prio3_py as py
    for m in [b"", b"abc", bytes(range(167)), bytes(168), bytes(169), bytes(range(256)) * 3]:
        exp = hashlib.shake_128(m).digest(400)
        assert oracle_lib.shake128(m, 400) == exp
        assert py.shake128_24(m, 400) == exp


def test_turboshake128_rfc9861_kat(oracle_lib):
    from oracle import prio3_py as py
    exp = "1e415f1c5983aff2169217277d17bb538cd945a397ddec541f1ce41af2c1b74c"
    assert oracle_lib.turboshake128(b"", 0x1F, 32).hex() == exp
    assert py.turboshake128(b"", 0x1F, 32).hex() == exp
    for m in [b"x" * 200, bytes(range(100))]:
        for d in (0x01, 0x06, 0x1F):
            assert oracle_lib.turboshake128(m, d, 300) == py.turboshake128(m, d, 300)


def test_field_constants():
    from oracle import prio3_py as py
    for F, order in [(py.Field64, 32), (py.Field128, 66)]:
        assert pow(F.gen, 2 ** order, F.p) == 1
        assert pow(F.gen, 2 ** (order - 1), F.p) != 1
        assert F.gen == pow(7, (F.p - 1) >> order, F.p)
    assert py.Field128.p == 340282366920938462946865773367900766209
    assert py.Field64.p == 0xFFFFFFFF00000001


def _meas(rnd, cfg):
    k = cfg["kind"]
    if k == "count":
        return rnd.randrange(2)
    if k == "sum":
        return rnd.randrange(2 ** cfg["bits"])
    if k == "sumvec":
        return [rnd.randrange(2 ** cfg["bits"]) for _ in range(cfg["length"])]
    return rnd.randrange(cfg["length"])


SMALL = ["count", "sum8", "sum1", "sumvec_8x10_c9", "sumvec_1x1_c1", "hist_10_c3", "hist_1_c1",
         "hist_256_c16"]


@pytest.mark.parametrize("name", SMALL)
def test_c_and_python_restatements_agree(oracle_lib, name):
    from oracle import prio3_py as py
    cfg = CONFIGS[name]
    o = oracle_lib.Oracle(**cfg)
    t = py.Prio3Type(cfg["kind"], **{k: v for k, v in cfg.items() if k != "kind"})
    vdaf = py.Prio3(t)
    rnd = random.Random(name)
    for _ in range(2):
        m = _meas(rnd, cfg)
        nonce, vk = bytes(rnd.randrange(256) for _ in range(16)), bytes(16)
        rand = bytes(rnd.randrange(256) for _ in range(o.rand_size))
        pub, ls, hs = o.shard(m, nonce, rand)
        assert (pub, ls, hs) == vdaf.shard(m, nonce, rand)
        rc0, st0, ps0 = o.prepare_init(vk, 0, nonce, pub, ls)
        rc1, st1, ps1 = o.prepare_init(vk, 1, nonce, pub, hs)
        _, pps0, _ = vdaf.prepare_init(vk, 0, nonce, pub, ls)
        s1, pps1, _ = vdaf.prepare_init(vk, 1, nonce, pub, hs)
        assert (rc0, rc1) == (0, 0) and ps0 == pps0 and ps1 == pps1
        rc, msg = o.prep_shares_to_prep_msg(ps0, ps1)
        assert rc == 0 and msg == vdaf.prep_shares_to_prep_msg(pps0, pps1)
        rc, out = o.prepare_next(st1, msg)
        assert rc == 0 and out == b"".join(t.F.enc(x) for x in vdaf.prepare_next(s1, msg))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "prio3_*.json"))))
def test_golden_fixtures(oracle_lib, path):
    doc = json.load(open(path))
    cfg = doc["vdaf"]
    o = oracle_lib.Oracle(**cfg)
    vk = bytes.fromhex(doc["verify_key"])
    h = lambda s: bytes.fromhex(s)
    outs = []
    for r in doc["reports"]:
        rc, tr = o.helper_trace(vk, h(r["nonce"]), h(r["public_share"]), h(r["helper_share"]))
        assert rc == 0
        assert tr["meas"].hex() == r["helper_meas_share"]
        assert tr["proofs"].hex() == r["helper_proofs_share"]
        assert tr["part"].hex() == r["joint_rand_part"]
        assert tr["corrected"].hex() == r["corrected_joint_rand_seed"]
        assert tr["jr"].hex() == r["joint_rands"]
        assert tr["qr"].hex() == r["query_rands"]
        assert tr["verifiers"].hex() == r["helper_verifier"]
        rc, st, ps = o.prepare_init(vk, 1, h(r["nonce"]), h(r["public_share"]), h(r["helper_share"]))
        assert ps.hex() == r["helper_prep_share"]
        rc, msg = o.prep_shares_to_prep_msg(h(r["leader_prep_share"]), ps)
        assert rc == 0 and msg.hex() == r["prep_msg"]
        rc, out = o.prepare_next(st, msg)
        assert out.hex() == r["helper_output_share"]
        outs.append(r)
    # batch path over the same reports reproduces statuses, messages and the aggregate
    n = len(doc["reports"])
    col = lambda k, L: np.array([np.frombuffer(h(r[k]), np.uint8) for r in doc["reports"]]).reshape(n, L)
    pub_len = o.public_share_len
    msgs, status, agg, cnt = o.helper_batch(
        vk, col("nonce", 16), col("public_share", pub_len) if pub_len else np.zeros((n, 0), np.uint8),
        col("helper_share", o.helper_share_len), col("leader_prep_share", o.prep_share_len))
    assert not status.any() and int(cnt[0]) == n
    assert agg[0].tobytes().hex() == doc["helper_aggregate_share"]
    # negative cases
    for neg in doc["negative"]:
        r = dict(doc["reports"][neg["base"]])
        r[neg["field"]] = neg["value"]
        rc, st, ps = o.prepare_init(vk, 1, h(r["nonce"]), h(r["public_share"]), h(r["helper_share"]))
        rc, msg = o.prep_shares_to_prep_msg(h(r["leader_prep_share"]), ps)
        if rc == 0:
            rc, _ = o.prepare_next(st, msg)
        assert rc == neg["status"], neg


@pytest.mark.parametrize("name", ["count", "sum8", "sumvec_8x10_c9", "hist_256_c16"])
def test_batch_unshard_equals_plaintext(oracle_lib, name):
    cfg = CONFIGS[name]
    o = oracle_lib.Oracle(**cfg)
    vk = bytes(range(16))
    n = 300
    d = o.gen_reports(vk, n, seed=3, n_threads=4)
    msgs, status, agg, cnt = o.helper_batch(vk, d["nonces"], d["public_shares"], d["helper_shares"],
                                            d["leader_prep_shares"], n_threads=4)
    assert not status.any() and int(cnt[0]) == n
    p = oracle_lib.field_modulus(cfg["kind"])
    tot = [(a + b) % p for a, b in zip(oracle_lib.sum_mod(d["leader_out_shares"], o.es, p),
                                       oracle_lib.decode_elems(agg[0], o.es))]
    m = d["measurements"].astype(object)
    if cfg["kind"] == "histogram":
        exp = np.bincount(d["measurements"][:, 0].astype(np.int64), minlength=cfg["length"]).tolist()
    elif cfg["kind"] == "sumvec":
        exp = [int(x) for x in m.sum(axis=0)]
    else:
        exp = [int(m.sum())]
    assert tot == exp


@pytest.mark.parametrize("name", ["count", "sumvec_8x10_c9", "hist_256_c16"])
def test_leader_batch_matches_python(oracle_lib, name):
    """orc_leader_batch (the leader line's CPU baseline) against the Python restatement's
    prepare_init(agg 0) / prepare_next: prep shares, statuses (non-canonical share element ->
    1, tampered prepare message -> 4) and the leader aggregate share."""
    from oracle import prio3_py as py
    cfg = CONFIGS[name]
    o = oracle_lib.Oracle(**cfg)
    t = py.Prio3Type(cfg["kind"], **{k: v for k, v in cfg.items() if k != "kind"})
    v = py.Prio3(t)
    rnd = random.Random(name + "leader")
    vk = bytes(range(16))
    reps = []
    for i in range(12):
        m = _meas(rnd, cfg)
        nonce = bytes(rnd.randrange(256) for _ in range(16))
        pub, ls, hs = v.shard(m, nonce, bytes(rnd.randrange(256) for _ in range(o.rand_size)))
        reps.append(dict(nonce=nonce, pub=pub, ls=bytearray(ls), hs=hs))
    reps[2]["ls"][0:o.es] = b"\xff" * o.es                 # non-canonical element
    exp_ps, exp_st, msgs, tot = [], [], [], [0] * t.out_len
    for i, r in enumerate(reps):
        try:
            st0, ps0, _ = v.prepare_init(vk, 0, r["nonce"], r["pub"], bytes(r["ls"]))
        except ValueError:
            exp_ps.append(bytes(o.prep_share_len)), exp_st.append(1), msgs.append(bytes(16))
            continue
        st1, ps1, _ = v.prepare_init(vk, 1, r["nonce"], r["pub"], r["hs"])
        msg = bytearray(v.prep_shares_to_prep_msg(ps0, ps1))
        if i == 5 and msg:
            msg[0] ^= 1
        exp_ps.append(ps0), msgs.append(bytes(msg) or bytes(16))
        if i == 5 and msg:
            exp_st.append(4)
            continue
        exp_st.append(0)
        tot = [(a + b) % t.F.p for a, b in zip(tot, v.prepare_next(st0, bytes(msg)))]
    n = len(reps)
    A = lambda k, w: np.array([np.frombuffer(bytes(r[k]), np.uint8) for r in reps]).reshape(n, w)
    ps, st, agg, cnt = o.leader_batch(
        vk, A("nonce", 16), A("pub", o.public_share_len) if o.public_share_len else None,
        A("ls", o.leader_share_len), np.array([np.frombuffer(m, np.uint8) for m in msgs]),
        n_threads=3, job_size=4)
    assert st.tolist() == exp_st
    assert [bytes(x) for x in ps] == exp_ps
    assert oracle_lib.decode_elems(agg[0], o.es) == tot and int(cnt[0]) == exp_st.count(0)


def test_invalid_measurements_rejected(oracle_lib):
    """Soundness smoke: a two-hot histogram and a bucket value of 2, proven honestly over the
    invalid encoding, fail decide (status 3)."""
    from oracle import prio3_py as py
    t = py.Prio3Type("histogram", length=8, chunk_length=3)
    vdaf = py.Prio3(t)
    o = oracle_lib.Oracle("histogram", length=8, chunk_length=3)
    rnd = random.Random(5)
    for bad in ([1, 1, 0, 0, 0, 0, 0, 0], [2, 0, 0, 0, 0, 0, 0, 0], [0] * 8):
        t.encode = lambda m, bad=bad: list(bad)  # malicious client bypasses encode checks
        nonce = bytes(rnd.randrange(256) for _ in range(16))
        rand = bytes(rnd.randrange(256) for _ in range(80))
        vk = bytes(16)
        pub, ls, hs = vdaf.shard(0, nonce, rand)
        _, lps, _ = vdaf.prepare_init(vk, 0, nonce, pub, ls)
        rc, st, hps = o.prepare_init(vk, 1, nonce, pub, hs)
        rc, msg = o.prep_shares_to_prep_msg(lps, hps)
        assert rc == 3
