"""The reference's own end-to-end measurement sets (interop_binaries/tests/end_to_end.rs:582-841),
run through shard -> leader prepare -> helper prepare -> aggregate -> unshard -> decode.

These are the only known answers the reference holds for Prio3 aggregation semantics:
  e2e_prio3_count          Prio3Count, 18 measurements                         (:582-611)
  e2e_prio3_sum            Prio3Sum bits 64                                    (:613-632)
  e2e_prio3_sum_vec        Prio3SumVec bits 64, length 4, chunk_length 18      (:634-657)
  e2e_prio3_histogram      Prio3Histogram length 6, chunk_length 2             (:659-686)
  e2e_prio3_fixed16vec     FixedPointBoundedL2VecSum BitSize16, length 3  -> ["0.5","0.5","0.6875"]
  e2e_prio3_fixed32vec     FixedPointBoundedL2VecSum BitSize32, length 3  -> ["0.5","0.5","0.6875"]
                                                                               (:688-764)
  janus_in_process_customized_sum_vec
                           Prio3SumVecField64MultiproofHmacSha256Aes128 proofs 2, bits 16,
                           length 15, chunk 16, random 16-bit entries
                           (integration_tests/tests/integration/janus.rs:378-400, common.rs:458-490)
The reference asserts the fixed-point result literally and the others by type; here the
others are checked against the plaintext sums they must decode to (the semantic known answer of
integration_tests/tests/integration/common.rs:332-554).  The client shard is the Python
restatement; the CPU test runs both aggregators on the restatement, the GPU test runs the helper
(and the leader, for the instances whose leader role is on the device) on the HIP engine.
"""
import numpy as np
import pytest

from oracle import prio3_py as P
from oracle.fpvec_py import FpVecType

COUNT = [0, 1, 1, 0, 1, 0, 1, 0, 1, 1, 0, 1, 0, 1, 0, 0, 0, 0]
SUM = [0, 10, 9, 21, 8, 12, 14]
SUMVEC = [[0, 0, 0, 10], [0, 0, 10, 0], [0, 10, 0, 0], [10, 0, 0, 0]]
HIST = [0, 1, 2, 3, 4, 5]
# fixed!(0.25 / 0.125 / 0.0625) as I1F15 / I1F31 raw values, end_to_end.rs:700-719, 739-758
FIXED = [[0.25, 0.125, 0.125], [0.0625, 0.125, 0.0625], [0.125, 0.125, 0.25],
         [0.0625, 0.125, 0.25]]

CASES = {
    "e2e_prio3_count": (P.Prio3Type("count"), COUNT),
    "e2e_prio3_sum": (P.Prio3Type("sum", bits=64), SUM),
    "e2e_prio3_sum_vec": (P.Prio3Type("sumvec", bits=64, length=4, chunk_length=18), SUMVEC),
    "e2e_prio3_histogram": (P.Prio3Type("histogram", length=6, chunk_length=2), HIST),
    "e2e_prio3_fixed16vec": (FpVecType(3, 16), [[int(x * (1 << 15)) for x in v] for v in FIXED]),
    "e2e_prio3_fixed32vec": (FpVecType(3, 32), [[int(x * (1 << 31)) for x in v] for v in FIXED]),
    "janus_in_process_customized_sum_vec": (
        P.Prio3Type("sumvec_f64_mp", bits=16, length=15, chunk_length=16, num_proofs=2),
        [[int(x) for x in row] for row in np.random.default_rng(458).integers(0, 1 << 16, (20, 15))]),
}
VK16 = bytes(range(0x70, 0x80))
VK32 = bytes(range(0x70, 0x90))


def _vk(t):
    return VK32 if getattr(t, "seed_size", 16) == 32 else VK16


def _expected(name, meas):
    if name == "e2e_prio3_count" or name == "e2e_prio3_sum":
        return sum(meas)
    if name == "e2e_prio3_sum_vec":
        return [sum(m[e] for m in meas) for e in range(4)]
    if name == "janus_in_process_customized_sum_vec":
        return [sum(m[e] for m in meas) for e in range(15)]
    if name == "e2e_prio3_histogram":
        return [meas.count(b) for b in range(6)]
    return ["0.5", "0.5", "0.6875"]  # end_to_end.rs:724, 763


def _decode(name, t, agg, count):
    if isinstance(t, FpVecType):
        return [str(x) for x in t.decode_result(agg, count)]  # Rust f64 Display of the result
    return t.decode_agg(agg)


def _shard_all(v, meas, seed):
    rng = np.random.default_rng(seed)
    rand_len = v.S * (5 if v.t.jr_len else 3)
    out = []
    for m in meas:
        nonce = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        pub, leader, helper = v.shard(m, nonce, bytes(rng.integers(0, 256, rand_len, dtype=np.uint8)))
        out.append(dict(nonce=nonce, pub=pub, leader=leader, helper=helper))
    return out


@pytest.mark.parametrize("name", list(CASES))
def test_reference_e2e_restatement(name):
    """CPU: the restatement alone reproduces each reference end-to-end result."""
    t, meas = CASES[name]
    v = P.Prio3(t)
    VK = _vk(t)
    aggs = [[0] * t.out_len, [0] * t.out_len]
    for r in _shard_all(v, meas, seed=len(name)):
        st0, lps, _ = v.prepare_init(VK, 0, r["nonce"], r["pub"], r["leader"])
        st1, hps, _ = v.prepare_init(VK, 1, r["nonce"], r["pub"], r["helper"])
        msg = v.prep_shares_to_prep_msg(lps, hps)
        for i, st in enumerate((st0, st1)):
            aggs[i] = [(a + b) % v.F.p for a, b in zip(aggs[i], v.prepare_next(st, msg))]
    agg = v.aggregate(aggs)
    assert _decode(name, t, agg, len(meas)) == _expected(name, meas)


def _engine_vdaf(t):
    from janus_amd import prio3 as J
    if isinstance(t, FpVecType):
        return J.Prio3FixedPointBoundedL2VecSum(t.length, t.bits)
    return {"count": lambda: J.Prio3Count(), "sum": lambda: J.Prio3Sum(t.bits),
            "sumvec": lambda: J.Prio3SumVec(t.bits, t.length, t.chunk_length),
            "histogram": lambda: J.Prio3Histogram(t.length, t.chunk_length),
            "sumvec_f64_mp": lambda: J.Prio3SumVecField64MultiproofHmacSha256Aes128(
                t.num_proofs, t.bits, t.length, t.chunk_length)}[
                "sumvec_f64_mp" if t.seed_size == 32 else t.kind]()


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_reference_e2e_on_device(name):
    """GPU: both aggregators' prepare on the HIP engine (the leader's prep shares also checked
    against the restatement's), aggregate shares from the engine, unshard, decode."""
    from janus_amd import prio3 as J
    t, meas = CASES[name]
    v = P.Prio3(t)
    reps = _shard_all(v, meas, seed=len(name))
    VK = _vk(t)
    eng = J.HelperEngine(_engine_vdaf(t), VK, allow_unpinned=True)
    sz = eng.sz
    n = len(reps)
    A = lambda k, w: np.array([np.frombuffer(r[k], np.uint8) for r in reps], np.uint8).reshape(n, w)
    nonces = A("nonce", 16)
    pub = A("pub", sz.public_share_len) if sz.public_share_len else None
    # every instance here has its leader role on the device (FPVec and mp64 since round 2)
    lps, lst, lbatch = eng.leader_prepare_init_batch(nonces, pub,
                                                     A("leader", sz.leader_input_share_len))
    assert not lst.any()
    assert lps.tobytes() == b"".join(
        v.prepare_init(VK, 0, r["nonce"], r["pub"], r["leader"])[1] for r in reps)
    msgs, status, hbatch = eng.prepare_batch(nonces, pub, A("helper", sz.helper_share_len), lps)
    assert not status.any()
    hagg, hcnt = hbatch.accumulate()
    st = lbatch.leader_prepare_next(msgs if sz.prep_msg_len else None, np.zeros(n, np.uint8))
    assert not st.any()
    lagg, _ = lbatch.accumulate()
    leader_agg = [int.from_bytes(lagg[0, i:i + sz.field_bytes].tobytes(), "little")
                  for i in range(0, sz.agg_share_len, sz.field_bytes)]
    helper_agg = [int.from_bytes(hagg[0, i:i + sz.field_bytes].tobytes(), "little")
                  for i in range(0, sz.agg_share_len, sz.field_bytes)]
    assert int(hcnt[0]) == n
    agg = v.aggregate([leader_agg, helper_agg])
    assert _decode(name, t, agg, n) == _expected(name, meas)
