"""Prio3FixedPointBoundedL2VecSum (BASELINE.json config C5; SURVEY 8(a) rows a3-a8 for the
FixedPoint L2 circuit; core/src/vdaf.rs:292-335).

prio's fixedpoint_l2.rs is not in the reference and SURVEY A.11(3) records its circuit as
approximate, so the circuit is the reconstruction documented in oracle/fpvec_py.py: parity with
prio is UNPINNED and the GPU is pinned to that restatement.

CPU: the restatement is internally consistent -- shard, both aggregators' prepare, decide,
unshard == the sum of the encoded entries; a vector of norm >= 1 cannot be encoded; a client
that claims a wrong norm, a non-bit entry bit, or a tampered share is rejected -- and the C
engine's sizes (prio3_sizes, host code) equal the restatement's.  GPU: k_xof + k_query_fp are
bit-exact against the restatement (prepare messages, statuses, output shares, aggregate), with
tampered reports, across sub-batches of the per-report scratch."""
import os

import numpy as np
import pytest

from oracle import prio3_py as P
from oracle.fpvec_py import FpVecType, optimal_chunk_length

VK = bytes(range(0x20, 0x30))


def _vdaf(length, bits=16):
    return P.Prio3(FpVecType(length, bits))


def _vector(rng, length, bits):
    """Random raw fixed-point entries with ||x||^2 < 1 (x_i = X_i / 2^(bits-1))."""
    half = 1 << (bits - 1)
    lim = max(1, int(half / np.sqrt(length)) - 1)
    return [int(x) for x in rng.integers(-lim, lim, length)]


def _prep_all(v, xs, nonce, rand):
    pub, leader, helper = v.shard(xs, nonce, rand)
    st0, lps, _ = v.prepare_init(VK, 0, nonce, pub, leader)
    st1, hps, _ = v.prepare_init(VK, 1, nonce, pub, helper)
    return pub, leader, helper, st0, lps, st1, hps


def test_optimal_chunk_length_known_values():
    # optimal_chunk_length(8000) = 63 (SumVec 8x1000); A.10 C5: ~314 / ~79
    assert optimal_chunk_length(8000) == 63
    assert optimal_chunk_length(160030) == 314
    assert optimal_chunk_length(10000) == 79
    assert optimal_chunk_length(1) == 1


@pytest.mark.parametrize("length,bits", [(1, 16), (7, 16), (10000, 16), (3, 32), (1000, 32)])
def test_engine_sizes_match_restatement(length, bits):
    from janus_amd import prio3 as J
    t = FpVecType(length, bits)
    sz = J.Prio3FixedPointBoundedL2VecSum(length, bits).sizes()
    assert (sz.field_bytes, sz.meas_len, sz.out_len, sz.proof_len, sz.verifier_len,
            sz.joint_rand_len) == (16, t.meas_len, t.out_len, t.proof_len, t.verifier_len, 2)
    assert sz.prep_share_len == 16 * t.verifier_len + 16
    assert sz.helper_share_len == 48 and sz.public_share_len == 32 and sz.prep_msg_len == 16
    assert sz.leader_input_share_len == 16 * (t.meas_len + t.proof_len) + 16


def test_engine_rejects_bad_bitsize():
    from janus_amd import prio3 as J
    with pytest.raises(ValueError):
        J.Prio3FixedPointBoundedL2VecSum(4, 8)
    with pytest.raises(ValueError):
        J.Prio3(J.PRIO3_FPVEC_BOUNDED_L2, bits=64, length=4).sizes()


@pytest.mark.parametrize("length,bits", [(1, 16), (5, 16), (3, 32), (24, 16)])
def test_oracle_unshard_equals_sum(length, bits):
    v = _vdaf(length, bits)
    rng = np.random.default_rng(length * bits)
    half = 1 << (bits - 1)
    agg = [[0] * length, [0] * length]
    xs_all = []
    for _ in range(4):
        xs = _vector(rng, length, bits)
        xs_all.append(xs)
        _, _, _, st0, lps, st1, hps = _prep_all(v, xs, os.urandom(16), os.urandom(80))
        msg = v.prep_shares_to_prep_msg(lps, hps)
        for i, st in enumerate((st0, st1)):
            agg[i] = [(a + b) % P.Field128.p for a, b in zip(agg[i], v.prepare_next(st, msg))]
    tot = v.unshard(agg)
    assert tot == [sum(x[e] + half for x in xs_all) for e in range(length)]
    assert v.t.decode_result(tot, 4) == [sum(x[e] for x in xs_all) / half for e in range(length)]


def test_oracle_norm_bound():
    t = FpVecType(2, 16)
    t.encode([23170, 23170])  # 2 * 23170^2 < 2^30
    with pytest.raises(ValueError):
        t.encode([23171, 23171])


def test_oracle_rejects_dishonest_clients():
    v = _vdaf(4)
    t = v.t
    xs = [1000, -2000, 300, 0]
    good = t.encode(xs)
    nb = t.bits * t.length
    cases = []
    wrong_norm = list(good)
    wrong_norm[nb + 3] ^= 1  # claims another norm (still a bit vector)
    cases.append(wrong_norm)
    not_bit = list(good)
    not_bit[5] = 2  # an entry "bit" of 2
    cases.append(not_bit)
    orig = t.encode
    try:
        for meas in cases:
            t.encode = lambda _m, meas=meas: meas
            nonce = os.urandom(16)
            _, _, _, _, lps, _, hps = _prep_all(v, xs, nonce, os.urandom(80))
            with pytest.raises(ValueError):
                v.prep_shares_to_prep_msg(lps, hps)
    finally:
        t.encode = orig
    # an honest report passes; a tampered wire value of either gadget fails
    _, _, _, _, lps, _, hps = _prep_all(v, xs, os.urandom(16), os.urandom(80))
    v.prep_shares_to_prep_msg(lps, hps)
    for e in (1, 1 + t.A0 + 1):
        bad = bytearray(lps)
        bad[16 * e] ^= 1
        with pytest.raises(ValueError):
            v.prep_shares_to_prep_msg(bytes(bad), hps)


# ------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------
def _reports(v, n, seed, distinct=None):
    rng = np.random.default_rng(seed)
    t = v.t
    out = []
    for i in range(n):
        if distinct and i >= distinct:  # tile the first `distinct` reports
            out.append(dict(out[i % distinct], lps=bytearray(out[i % distinct]["lps"])))
            continue
        xs = _vector(rng, t.length, t.bits)
        nonce = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        rand = bytes(rng.integers(0, 256, 80, dtype=np.uint8))
        pub, leader, helper = v.shard(xs, nonce, rand)
        _, lps, _ = v.prepare_init(VK, 0, nonce, pub, leader)
        out.append(dict(nonce=nonce, pub=pub, helper=helper, lps=bytearray(lps)))
    return out


def _expected(v, reps):
    msgs, status, outs = [], [], []
    cache = {}
    for r in reps:
        key = (r["nonce"], r["helper"])
        if key not in cache:
            cache[key] = v.prepare_init(VK, 1, r["nonce"], r["pub"], r["helper"])
        st1, hps, _ = cache[key]
        try:
            msg = v.prep_shares_to_prep_msg(bytes(r["lps"]), hps)
        except ValueError as e:
            code = 2 if "range" in str(e) else 3
            msgs.append(bytes(16)), status.append(code), outs.append(None)
            continue
        try:
            out = v.prepare_next(st1, msg)
        except ValueError:
            msgs.append(bytes(16)), status.append(4), outs.append(None)
            continue
        msgs.append(msg), status.append(0), outs.append(out)
    return msgs, status, outs


def _tamper(v, reps, frac, seed):
    rng = np.random.default_rng(seed)
    n, nv = len(reps), v.t.verifier_len
    for i in rng.choice(n, max(1, int(n * frac)), replace=False):
        kind = int(rng.integers(0, 4))
        if kind == 0:
            reps[i]["lps"][16 * int(rng.integers(0, nv))] ^= 1         # a verifier value
        elif kind == 1:
            reps[i]["lps"][16 * nv + 5] ^= 0x40                         # leader joint-rand part
        elif kind == 2:
            reps[i]["lps"][16 * int(rng.integers(0, nv)) + 15] = 0xff   # out of range: decode
        else:
            reps[i]["lps"][16 * (2 + v.t.A0)] ^= 2                      # a gadget-1 wire


def _run(v, reps, sub_bytes=None, opts=None):
    from janus_amd import prio3 as J
    t = v.t
    eng = J.HelperEngine(J.Prio3FixedPointBoundedL2VecSum(t.length, t.bits), VK, allow_unpinned=True)
    if sub_bytes:
        eng.set_option("fp_sub_bytes", sub_bytes)
    for k, val in (opts or {}).items():
        eng.set_option(k, val)
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    msgs, status, batch = eng.prepare_batch(A("nonce"), A("pub"), A("helper"), A("lps"))
    outs = batch.output_shares()
    agg, cnt = batch.accumulate()
    return msgs, status, outs, agg, cnt


def _check(v, reps, got):
    msgs, status, outs, agg, cnt = got
    exp_msgs, exp_st, exp_out = _expected(v, reps)
    assert status.tolist() == exp_st
    np.testing.assert_array_equal(msgs, np.array([list(m) for m in exp_msgs], np.uint8))
    L = v.t.length
    tot = [0] * L
    for i, o in enumerate(exp_out):
        if o is None:
            continue
        row = outs[i].reshape(L, 16)
        assert [int.from_bytes(row[e].tobytes(), "little") for e in range(L)] == o
        tot = [(a + b) % P.Field128.p for a, b in zip(tot, o)]
    got_agg = [int.from_bytes(agg[0, 16 * e:16 * e + 16].tobytes(), "little") for e in range(L)]
    assert got_agg == tot and int(cnt[0]) == sum(1 for s in exp_st if s == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("length,bits,n", [(1, 16, 40), (5, 16, 70), (3, 32, 33), (24, 16, 65)])
def test_gpu_fpvec_matches_oracle(length, bits, n):
    v = _vdaf(length, bits)
    reps = _reports(v, n, seed=length * 7 + bits)
    _tamper(v, reps, 0.25, seed=length)
    _check(v, reps, _run(v, reps))


@pytest.mark.gpu
def test_gpu_fpvec_sub_batches():
    """A per-report scratch budget of one 256-report column block forces 3 sub-batches; the
    output shares of every sub-batch land in their own columns and the aggregate covers all."""
    v = _vdaf(6)
    reps = _reports(v, 600, seed=11, distinct=150)
    _tamper(v, reps, 0.05, seed=3)
    _check(v, reps, _run(v, reps, sub_bytes=1))


@pytest.mark.gpu
@pytest.mark.parametrize("fp_round", [1, 0])
def test_gpu_fpvec_sub_batches_rounded_to_query_rounds(fp_round):
    """40,000 reports in scratch of 24,576 columns: two sub-batches, which fp_sub_sizes cuts at
    whole eight-lane query rounds (16,384 + 23,616 on a 256-CU part) instead of 2 x 20,000.
    Statuses, messages, output shares and the aggregate must not depend on the cut, for the
    helper and for the leader."""
    from janus_amd import prio3 as J
    v = _vdaf(1)
    t = v.t
    n, distinct = 40000, 16
    reps = _reports(v, n, seed=29, distinct=distinct)
    reps[5]["lps"][16 * t.verifier_len + 5] ^= 0x40  # one tampered leader joint-rand part
    per = 16 * (t.meas_len + t.proof_len + 2 + 2 + 2 * (t.P0 + t.P1) + t.K0) + 33
    msgs, status, outs, agg, cnt = _run(v, reps, sub_bytes=per * 24576 + 1,
                                        opts={"fp_round": fp_round})
    # expectations of the distinct reports, plus a clean copy of the tampered one (its tiles
    # keep the original prep share)
    exp = _expected(v, reps[:distinct] + [reps[distinct + 5]])
    src = lambda i: i if i < distinct else (distinct if i % distinct == 5 else i % distinct)
    want_st = [exp[1][src(i)] for i in range(n)]
    assert status.tolist() == want_st and want_st[5] != 0
    tot = 0
    for i in range(n):
        assert msgs[i].tobytes() == exp[0][src(i)], i
        o = exp[2][src(i)]
        if o is not None:
            assert int.from_bytes(outs[i].tobytes(), "little") == o[0], i
            tot = (tot + o[0]) % P.Field128.p
    assert int.from_bytes(agg[0, :16].tobytes(), "little") == tot
    assert int(cnt[0]) == sum(1 for x in want_st if x == 0)
    # the leader over the same cut
    eng = J.HelperEngine(J.Prio3FixedPointBoundedL2VecSum(t.length, t.bits), VK,
                         allow_unpinned=True)
    eng.set_option("fp_sub_bytes", per * 24576 + 1)
    eng.set_option("fp_round", fp_round)
    leaders = []
    rng = np.random.default_rng(29)
    for i in range(distinct):  # the leader shares of the same distinct reports
        xs = _vector(rng, t.length, t.bits)
        nonce = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        rand = bytes(rng.integers(0, 256, 80, dtype=np.uint8))
        _, leader, _ = v.shard(xs, nonce, rand)
        assert nonce == reps[i]["nonce"]
        leaders.append(list(leader))
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    lps, lst, _ = eng.leader_prepare_init_batch(
        A("nonce"), A("pub"), np.array([leaders[i % distinct] for i in range(n)], np.uint8))
    assert not lst.any()
    clean = [bytes(v.prepare_init(VK, 0, reps[i]["nonce"], reps[i]["pub"], bytes(leaders[i]))[1])
             for i in range(distinct)]
    for i in range(n):
        assert lps[i].tobytes() == clean[i % distinct], i


@pytest.mark.gpu
def test_gpu_fpvec_1000_entries():
    """1000 entries (MEAS_LEN 16,030; gadget 0: C0 127, P0 128; gadget 1: C1 33, P1 32): 3
    distinct reports tiled to 130 lanes."""
    v = _vdaf(1000)
    reps = _reports(v, 130, seed=5, distinct=3)
    reps[1]["lps"][16 * 7] ^= 1
    _check(v, reps, _run(v, reps))


GOLDEN_C5 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fpvec_l10000.npz")


def test_c5_fixture_shapes_match_engine_sizes():
    """The full-size fixtures (gen_fpvec_l10000.py) have the wire sizes the engine expects."""
    from janus_amd import prio3 as J
    g = np.load(GOLDEN_C5)
    sz = J.Prio3FixedPointBoundedL2VecSum(10000, 16).sizes()
    assert g["helper"].shape[1] == sz.helper_share_len
    assert g["lps"].shape[1] == sz.prep_share_len
    assert g["pub"].shape[1] == sz.public_share_len
    assert g["out_shares"].shape == (2, sz.agg_share_len)
    assert g["status"].tolist() == [0, 0, 3]


@pytest.mark.gpu
def test_gpu_fpvec_c5_full_size():
    """Config C5 at its full length (10000 entries, MEAS_LEN ~160k Field128 elements): two
    honest reports and a tampered one, tiled to 384 lanes, against the committed fixtures --
    statuses, prepare messages, sampled output shares and the whole aggregate share."""
    from janus_amd import prio3 as J
    g = np.load(GOLDEN_C5)
    n = 384
    idx = np.arange(n) % 3
    eng = J.HelperEngine(J.Prio3FixedPointBoundedL2VecSum(10000, 16), bytes(g["verify_key"]),
                         allow_unpinned=True)
    msgs, status, batch = eng.prepare_batch(g["nonce"][idx], g["pub"][idx], g["helper"][idx],
                                            g["lps"][idx])
    assert status.tolist() == g["status"][idx].tolist()
    np.testing.assert_array_equal(msgs, g["prep_msg"][idx])
    outs = batch.output_shares()
    for r in (0, 1, 3, 4, n - 3, n - 2):
        np.testing.assert_array_equal(outs[r].reshape(-1), g["out_shares"][idx[r]])
    agg, cnt = batch.accumulate()
    assert int(cnt[0]) == 2 * n // 3
    o = [np.frombuffer(g["out_shares"][k].tobytes(), "<u8").reshape(-1, 2) for k in (0, 1)]
    c = [int((idx == k).sum()) for k in (0, 1)]
    want = b"".join(((c[0] * (int(o[0][e, 0]) | int(o[0][e, 1]) << 64) +
                      c[1] * (int(o[1][e, 0]) | int(o[1][e, 1]) << 64)) % P.Field128.p)
                    .to_bytes(16, "little") for e in range(10000))
    assert agg[0].tobytes() == want


@pytest.mark.gpu
def test_gpu_fpvec_three_sub_batches():
    """1300 reports through a scratch budget of 512 columns: sub-batches 512 + 512 + 276, each
    one's shares, statuses and the aggregate equal to the restatement's."""
    v = _vdaf(6)
    t = v.t
    reps = _reports(v, 1300, seed=21, distinct=130)
    _tamper(v, reps, 0.05, seed=4)
    per = 16 * (t.meas_len + t.proof_len + 2 + 2 + 2 * (t.P0 + t.P1) + t.K0) + 33
    _check(v, reps, _run(v, reps, sub_bytes=per * 512 + 1, opts={"fp_round": 0}))


@pytest.mark.gpu
def test_gpu_fpvec_scratch_wider_than_sub_batch():
    """the r01u fault geometry -- the scratch leading dimension (ld) wider
    than the equal sub-batches it is cut into, and both narrower than the output-share columns
    (ld_out).  A budget of 768 scratch columns over 1000 reports gives ld 768, two sub-batches
    of 512 + 488, ld_out 1024."""
    from janus_amd import prio3 as J
    v = _vdaf(6)
    t = v.t
    reps = _reports(v, 1000, seed=41, distinct=100)
    _tamper(v, reps, 0.05, seed=5)
    per = 16 * (t.meas_len + t.proof_len + 2 + 2 + 2 * (t.P0 + t.P1) + t.K0) + 33
    eng = J.HelperEngine(J.Prio3FixedPointBoundedL2VecSum(t.length, t.bits), VK, allow_unpinned=True)
    eng.set_option("fp_sub_bytes", per * 768 + per // 2)
    eng.set_option("timing", 1)
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    msgs, status, batch = eng.prepare_batch(A("nonce"), A("pub"), A("helper"), A("lps"))
    tm = eng.timing()
    assert tm.get("k_query_fpw", tm.get("k_query_fp"))[1] == 2  # two sub-batches
    outs = batch.output_shares()
    agg, cnt = batch.accumulate()
    _check(v, reps, (msgs, status, outs, agg, cnt))


@pytest.mark.gpu
def test_gpu_fpvec_requires_explicit_opt_in():
    """the reconstructed (parity-unpinned) FPVec circuit prepares only after the
    experimental_fpvec opt-in; without it every prepare entry point returns EUNSUPPORTED."""
    from janus_amd import prio3 as J
    v = _vdaf(3)
    reps = _reports(v, 4, seed=3)
    eng = J.HelperEngine(J.Prio3FixedPointBoundedL2VecSum(3, 16), VK)
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    with pytest.raises(RuntimeError, match="rc=-3"):
        eng.prepare_batch(A("nonce"), A("pub"), A("helper"), A("lps"))


@pytest.mark.gpu
def test_gpu_fpvec_xof_lane_pairs():
    """The FPVec share phase on the lane-pair XOF (k_xof_pair, the entries decoded as the share
    is squeezed) across two sub-batches."""
    v = _vdaf(24)
    reps = _reports(v, 300, seed=23, distinct=60)
    _tamper(v, reps, 0.05, seed=6)
    t = v.t
    per = 16 * (t.meas_len + t.proof_len + 2 + 2 + 2 * (t.P0 + t.P1) + t.K0) + 33
    _check(v, reps, _run(v, reps, sub_bytes=per * 256 + 1))


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [16, 32])
def test_gpu_fpvec_slow_path_decodes_entries(bits):
    """Every report through the rejection-sampling XOF (force_slow_path): its entry decode must
    give the same output shares as the fast kernels'."""
    v = _vdaf(5, bits)
    reps = _reports(v, 70, seed=31 + bits)
    _tamper(v, reps, 0.1, seed=7)
    _check(v, reps, _run(v, reps, opts={"force_slow_path": 1}))


@pytest.mark.gpu
@pytest.mark.parametrize("length,opts", [
    (24, {}), (24, {"force_generic_query": 1}), (200, {}), (1000, {}),
])
def test_gpu_fpvec_query_variants(length, opts):
    """The eight-lane FPVec query (k_query_fpw) against the restatement, and the one-lane
    k_query_fp that takes the domains beyond its four-step split (test hook
    force_generic_query); 1000 entries exercises the two-level Lagrange split
    (P0 = 128 -> 8 x 16)."""
    v = _vdaf(length)
    n = 130 if length >= 1000 else 200
    reps = _reports(v, n, seed=43 + length, distinct=5 if length >= 1000 else 40)
    _tamper(v, reps, 0.1, seed=9)
    _check(v, reps, _run(v, reps, opts=opts))


def _c_oracle(length, bits):
    from oracle.oracle import Oracle, build
    build()
    return Oracle("fpvec", bits=bits, length=length)


@pytest.mark.parametrize("length,bits", [(1, 16), (3, 32), (24, 16), (200, 16)])
def test_c_restatement_matches_python(length, bits):
    """The compiled C restatement of the FPVec helper path (oracle/prio3_oracle.c ORC_FPVEC: the
    CPU baseline of bench.py --role fpvec) against the Python restatement, tampered reports
    included: statuses, prepare messages, aggregate share and count."""
    v = _vdaf(length, bits)
    reps = _reports(v, 12, seed=51 + length)
    _tamper(v, reps, 0.3, seed=13)
    exp_msgs, exp_st, exp_out = _expected(v, reps)
    o = _c_oracle(length, bits)
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    msgs, st, agg, cnt = o.helper_batch(VK, A("nonce"), A("pub"), A("helper"), A("lps"),
                                        n_threads=4)
    assert st.tolist() == exp_st
    np.testing.assert_array_equal(msgs, np.array([list(m) for m in exp_msgs], np.uint8))
    tot = [0] * length
    for o_ in exp_out:
        if o_ is not None:
            tot = [(a + b) % P.Field128.p for a, b in zip(tot, o_)]
    assert [int.from_bytes(agg[0, 16 * e:16 * e + 16].tobytes(), "little")
            for e in range(length)] == tot
    assert int(cnt[0]) == exp_st.count(0)


def test_c_restatement_reproduces_c5_fixture():
    """Full size (10^4 entries, 160,030-element shares): the C restatement reproduces the
    committed fixtures the Python restatement generated (tests/golden/fpvec_l10000.npz)."""
    g = np.load(GOLDEN_C5)
    o = _c_oracle(10000, 16)
    msgs, st, agg, cnt = o.helper_batch(bytes(g["verify_key"]), g["nonce"], g["pub"], g["helper"],
                                        g["lps"], n_threads=3)
    assert st.tolist() == g["status"].tolist()
    np.testing.assert_array_equal(msgs, g["prep_msg"])
    want = b"".join(((int.from_bytes(g["out_shares"][0][16 * e:16 * e + 16].tobytes(), "little") +
                      int.from_bytes(g["out_shares"][1][16 * e:16 * e + 16].tobytes(), "little"))
                     % P.Field128.p).to_bytes(16, "little") for e in range(10000))
    assert agg[0].tobytes() == want and int(cnt[0]) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("length,bits,n,sub", [(5, 16, 70, None), (24, 32, 90, None),
                                               (1000, 16, 40, None), (24, 16, 600, 256)])
def test_gpu_fpvec_leader_role(length, bits, n, sub):
    """the FPVec leader (prepare_init agg_id 0 + prepare_next) on the device.
    The leader prep shares must equal the restatement's; both roles on the device then decide,
    and the two aggregate shares unshard to the sum of the encoded entries.  A non-canonical
    element in one leader input share gives status 6; `sub` forces scratch sub-batches."""
    from janus_amd import prio3 as J
    v = _vdaf(length, bits)
    t = v.t
    rng = np.random.default_rng(61 + length)
    reps, leaders, xs_all = [], [], []
    for i in range(n):
        if i >= 8:  # tile 8 distinct reports
            reps.append(reps[i % 8]), leaders.append(leaders[i % 8]), xs_all.append(xs_all[i % 8])
            continue
        xs = _vector(rng, length, bits)
        nonce = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        pub, leader, helper = v.shard(xs, nonce, bytes(rng.integers(0, 256, 80, dtype=np.uint8)))
        _, lps, _ = v.prepare_init(VK, 0, nonce, pub, leader)
        reps.append(dict(nonce=nonce, pub=pub, helper=helper, lps=lps))
        leaders.append(bytearray(leader))
        xs_all.append(xs)
    leaders = [bytearray(x) for x in leaders]
    leaders[3][16 * 2:16 * 3] = b"\xff" * 16  # a non-canonical measurement-share element
    eng = J.HelperEngine(J.Prio3FixedPointBoundedL2VecSum(length, bits), VK, allow_unpinned=True)
    if sub:
        per = 16 * (t.meas_len + t.proof_len + 2 + 2 + 2 * (t.P0 + t.P1) + t.K0) + 33
        eng.set_option("fp_sub_bytes", per * sub + 1)
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    lps, lst, lbatch = eng.leader_prepare_init_batch(
        A("nonce"), A("pub"), np.array([list(x) for x in leaders], np.uint8))
    want = [0] * n
    want[3] = 6
    assert lst.tolist() == want
    for i in range(n):
        if i != 3:
            assert lps[i].tobytes() == bytes(reps[i]["lps"]), i
    msgs, hst, hbatch = eng.prepare_batch(A("nonce"), A("pub"), A("helper"), lps)
    assert [int(x) for x in hst if x] == [3]  # the decode-failed leader share: decide fails
    st = lbatch.leader_prepare_next(msgs, lst.copy())
    assert st.tolist() == want
    lagg, lcnt = lbatch.accumulate()
    hagg, hcnt = hbatch.accumulate()
    assert int(lcnt[0]) == int(hcnt[0]) == n - 1
    tot = [(int.from_bytes(lagg[0, 16 * e:16 * e + 16].tobytes(), "little") +
            int.from_bytes(hagg[0, 16 * e:16 * e + 16].tobytes(), "little")) % P.Field128.p
           for e in range(length)]
    half = 1 << (bits - 1)
    expect = [sum(xs_all[i][e] + half for i in range(n) if i != 3) for e in range(length)]
    assert tot == expect
