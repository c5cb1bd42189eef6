"""Prio3SumVecField64MultiproofHmacSha256Aes128 (core/src/vdaf.rs:173-195):
SumVec over Field64 with XofHmacSha256Aes128 (32-byte seeds) and >= 2 proofs.

CPU: the Python restatement (oracle/prio3_py.py, XofHmacSha256Aes128 restated over hashlib's
HMAC-SHA256 and an OpenSSL AES-128 Ctr64BE keystream) is internally consistent -- shard, both
aggregators' prepare, decide, unshard == plaintext sum; an out-of-range measurement is rejected
-- the semantic known answer of the reference's end-to-end test for this VDAF
(integration_tests/tests/integration/janus.rs:378-400, common.rs:458).  Byte parity with prio's
XofHmacSha256Aes128 is UNPINNED (the crate is not vendored).  GPU: k_mp64_prepare is bit-exact
against the restatement (prepare messages, statuses, aggregate), with tampered reports."""
import os

import numpy as np
import pytest

from oracle import prio3_py as P

VK = bytes(range(0x40, 0x60))


def _vdaf(proofs, bits, length, chunk):
    return P.Prio3(P.Prio3Type("sumvec_f64_mp", bits=bits, length=length, chunk_length=chunk,
                               num_proofs=proofs))


def _reports(v, n, seed):
    rng = np.random.default_rng(seed)
    t = v.t
    out = []
    for _ in range(n):
        m = [int(x) for x in rng.integers(0, 2 ** t.bits, t.length)]
        nonce = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        rand = bytes(rng.integers(0, 256, 32 * 5, dtype=np.uint8))
        pub, leader, helper = v.shard(m, nonce, rand)
        _, lps, _ = v.prepare_init(VK, 0, nonce, pub, leader)
        out.append(dict(m=m, nonce=nonce, pub=pub, helper=helper, lps=bytearray(lps)))
    return out


def test_oracle_rejects_tampered_verifier_share():
    v = _vdaf(3, 2, 5, 3)
    nonce = os.urandom(16)
    pub, leader, helper = v.shard([1] * v.t.length, nonce, os.urandom(160))
    _, lps, _ = v.prepare_init(VK, 0, nonce, pub, leader)
    _, hps, _ = v.prepare_init(VK, 1, nonce, pub, helper)
    assert len(v.prep_shares_to_prep_msg(lps, hps)) == 32
    for pos in (8, 8 * v.t.verifier_len + 8):  # a wire value of proof 0, then of proof 1
        bad = bytearray(lps)
        bad[pos] ^= 1
        with pytest.raises(ValueError):
            v.prep_shares_to_prep_msg(bytes(bad), hps)


def test_oracle_unshard_equals_sum():
    v = _vdaf(2, 3, 4, 5)
    rng = np.random.default_rng(2)
    meas = [[int(x) for x in rng.integers(0, 8, 4)] for _ in range(5)]
    agg = [[0] * 4, [0] * 4]
    for m in meas:
        nonce = os.urandom(16)
        pub, leader, helper = v.shard(m, nonce, os.urandom(160))
        st0, lps, _ = v.prepare_init(VK, 0, nonce, pub, leader)
        st1, hps, _ = v.prepare_init(VK, 1, nonce, pub, helper)
        msg = v.prep_shares_to_prep_msg(lps, hps)
        for i, st in enumerate((st0, st1)):
            agg[i] = [(a + b) % P.Field64.p for a, b in zip(agg[i], v.prepare_next(st, msg))]
    assert v.unshard(agg) == [sum(col) for col in zip(*meas)]


def _expected(v, reps):
    msgs, status, outs = [], [], []
    for r in reps:
        st1, hps, _ = v.prepare_init(VK, 1, r["nonce"], r["pub"], r["helper"])
        try:
            msg = v.prep_shares_to_prep_msg(bytes(r["lps"]), hps)
        except ValueError as e:
            code = 2 if "range" in str(e) else 3
            msgs.append(bytes(32)), status.append(code), outs.append(None)
            continue
        try:
            out = v.prepare_next(st1, msg)
        except ValueError:
            msgs.append(bytes(32)), status.append(4), outs.append(None)
            continue
        msgs.append(msg), status.append(0), outs.append(out)
    return msgs, status, outs


@pytest.mark.gpu
@pytest.mark.parametrize("proofs,bits,length,chunk,n", [(2, 1, 10, 3, 70), (3, 2, 5, 3, 40),
                                                        (2, 8, 20, 7, 33),
                                                        # the reference's own end-to-end config
                                                        # (integration janus.rs:387-392)
                                                        (2, 16, 15, 16, 24)])
def test_gpu_mp64_matches_oracle(proofs, bits, length, chunk, n):
    from janus_amd import prio3 as J
    v = _vdaf(proofs, bits, length, chunk)
    reps = _reports(v, n, seed=proofs * 100 + bits)
    rng = np.random.default_rng(7)
    nv = v.t.verifier_len * proofs
    for i in rng.choice(n, n // 4, replace=False):
        kind = int(rng.integers(0, 3))
        if kind == 0:
            reps[i]["lps"][8 * int(rng.integers(0, nv))] ^= 1        # verifier value
        elif kind == 1:
            reps[i]["lps"][8 * nv + 3] ^= 0x20                       # leader joint-rand part
        else:
            reps[i]["lps"][8 * int(rng.integers(0, nv)) + 7] = 0xff  # out of range: decode
    exp_msgs, exp_st, exp_out = _expected(v, reps)
    eng = J.HelperEngine(J.Prio3SumVecField64MultiproofHmacSha256Aes128(proofs, bits, length,
                                                                         chunk), VK)
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    msgs, status, batch = eng.prepare_batch(A("nonce"), A("pub"), A("helper"), A("lps"))
    assert status.tolist() == exp_st
    np.testing.assert_array_equal(msgs, np.array([list(m) for m in exp_msgs], np.uint8))
    agg, cnt = batch.accumulate()
    tot = [0] * length
    for o in exp_out:
        if o is not None:
            tot = [(a + b) % P.Field64.p for a, b in zip(tot, o)]
    got = [int.from_bytes(agg[0, 8 * e:8 * e + 8].tobytes(), "little") for e in range(length)]
    assert got == tot and int(cnt[0]) == sum(1 for s in exp_st if s == 0)


@pytest.mark.parametrize("proofs,bits,length,chunk", [(2, 16, 15, 16), (3, 2, 5, 3), (2, 1, 10, 3)])
def test_c_restatement_matches_python(proofs, bits, length, chunk):
    """The compiled C restatement (oracle/prio3_oracle.c ORC_SUMVEC_F64_MP: XofHmacSha256Aes128
    on OpenSSL's SHA-256 / AES-128, 32-byte seeds; the CPU baseline of bench.py --role mp64)
    against the Python restatement, tampered reports included."""
    from oracle.oracle import Oracle, build
    build()
    v = _vdaf(proofs, bits, length, chunk)
    reps = _reports(v, 9, seed=proofs * 10 + bits)
    reps[2]["lps"][8] ^= 1                                  # a wire value: decide fails
    reps[5]["lps"][-1] ^= 0x40                              # leader joint-rand part
    reps[7]["lps"][0:8] = b"\xff" * 8                       # verifier element >= p
    exp_msgs, exp_st, exp_out = _expected(v, reps)
    o = Oracle("sumvec_f64_mp", bits=bits, length=length, chunk_length=chunk, num_proofs=proofs)
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    msgs, st, agg, cnt = o.helper_batch(VK, A("nonce"), A("pub"), A("helper"), A("lps"),
                                        n_threads=3)
    assert st.tolist() == exp_st
    np.testing.assert_array_equal(msgs, np.array([list(m) for m in exp_msgs], np.uint8))
    tot = [0] * length
    for o_ in exp_out:
        if o_ is not None:
            tot = [(a + b) % P.Field64.p for a, b in zip(tot, o_)]
    assert [int.from_bytes(agg[0, 8 * e:8 * e + 8].tobytes(), "little") for e in range(length)] == tot
    assert int(cnt[0]) == exp_st.count(0)


@pytest.mark.gpu
@pytest.mark.parametrize("proofs,bits,length,chunk,n", [(2, 16, 15, 16, 40), (3, 2, 5, 3, 300)])
def test_gpu_mp64_leader_role(proofs, bits, length, chunk, n):
    """the mp64 leader (prepare_init agg_id 0 + prepare_next) on the device.
    The leader prep shares (verifier shares || joint-rand part) must equal the restatement's;
    both roles on the device then decide, and the two aggregate shares unshard to the plaintext
    sum.  A non-canonical element in one leader input share gives status 6 (the helper's decide
    on that report then fails); a tampered prepare message gives VdafPrepareNext (4)."""
    from janus_amd import prio3 as J
    v = _vdaf(proofs, bits, length, chunk)
    rng = np.random.default_rng(proofs * 7 + bits)
    reps, leaders = [], []
    for i in range(n):
        if i >= 16:  # tile 16 distinct reports
            reps.append(reps[i % 16]), leaders.append(bytearray(leaders[i % 16]))
            continue
        m = [int(x) for x in rng.integers(0, 2 ** bits, length)]
        nonce = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        pub, leader, helper = v.shard(m, nonce, bytes(rng.integers(0, 256, 160, dtype=np.uint8)))
        _, lps, _ = v.prepare_init(VK, 0, nonce, pub, leader)
        reps.append(dict(m=m, nonce=nonce, pub=pub, helper=helper, lps=lps))
        leaders.append(bytearray(leader))
    leaders[3][8 * 2:8 * 3] = b"\xff" * 8          # a non-canonical measurement-share element
    ml = v.t.meas_len
    leaders[5][8 * (ml + 1):8 * (ml + 2)] = b"\xff" * 8  # a non-canonical proof-share element
    eng = J.HelperEngine(J.Prio3SumVecField64MultiproofHmacSha256Aes128(proofs, bits, length,
                                                                         chunk), VK)
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    lps, lst, lbatch = eng.leader_prepare_init_batch(
        A("nonce"), A("pub"), np.array([list(x) for x in leaders], np.uint8))
    bad = {3, 5}
    assert [i for i in range(n) if lst[i]] == sorted(bad) and set(lst[list(bad)]) == {6}
    for i in range(n):
        if i not in bad:
            assert lps[i].tobytes() == bytes(reps[i]["lps"]), i
    msgs, hst, hbatch = eng.prepare_batch(A("nonce"), A("pub"), A("helper"), lps)
    assert [i for i in range(n) if hst[i]] == sorted(bad)
    sent = msgs.copy()
    sent[7, 0] ^= 1                               # the leader must reject this prepare message
    st = lbatch.leader_prepare_next(sent, lst.copy())
    assert st[7] == 4 and [i for i in range(n) if st[i] and i != 7] == sorted(bad)
    lagg, lcnt = lbatch.accumulate()
    hagg, hcnt = hbatch.accumulate()
    assert int(lcnt[0]) == n - 3 and int(hcnt[0]) == n - 2
    tot = [(int.from_bytes(lagg[0, 8 * e:8 * e + 8].tobytes(), "little") +
            int.from_bytes(hagg[0, 8 * e:8 * e + 8].tobytes(), "little")) % P.Field64.p
           for e in range(length)]
    # the helper aggregated report 7, which the leader rejected: the sum is every other good
    # report's measurement plus the helper's own output share of report 7
    st7, _, _ = v.prepare_init(VK, 1, reps[7]["nonce"], reps[7]["pub"], reps[7]["helper"])
    h7 = v.prepare_next(st7, msgs[7].tobytes())
    expect = [(sum(reps[i]["m"][e] for i in range(n) if i not in bad and i != 7) + h7[e])
              % P.Field64.p for e in range(length)]
    assert tot == expect
