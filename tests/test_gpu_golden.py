"""GPU against the COMMITTED golden bytes (tests/golden/prio3_*.json), not a live oracle run.

The fixtures were written once by tests/golden/gen_golden.py (Python restatement, asserted equal
to the C restatement when generated).  Here the HIP engine's helper and leader roles are run on
the fixture inputs through the C-ABI and compared byte-for-byte with the stored transcript:
prepare messages, statuses of the stored negative cases, helper output shares, the helper
aggregate share and the leader prepare shares.  An oracle regression can therefore no longer
move both sides of a GPU parity test together.  Prio-byte parity is
still unpinned (no prio vectors exist in the reference: core/src/test_util/mod.rs:86-232).
"""
import glob
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "prio3_*.json")))


def _vdaf(cfg):
    from janus_amd import prio3 as J
    k = cfg["kind"]
    if k == "count":
        return J.Prio3Count()
    if k == "sum":
        return J.Prio3Sum(cfg["bits"])
    if k == "sumvec":
        return J.Prio3SumVec(cfg["bits"], cfg["length"], cfg["chunk_length"])
    return J.Prio3Histogram(cfg["length"], cfg["chunk_length"])


def _col(rows, key, width):
    a = np.array([np.frombuffer(bytes.fromhex(r[key]), np.uint8) for r in rows], np.uint8)
    return a.reshape(len(rows), width)


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_helper_matches_committed_transcript(path):
    from janus_amd import prio3 as J
    doc = json.load(open(path))
    vk = bytes.fromhex(doc["verify_key"])
    eng = J.HelperEngine(_vdaf(doc["vdaf"]), vk)
    sz = eng.sz
    reps = list(doc["reports"])
    # the stored negative cases ride along as extra reports of the same batch
    for ng in doc["negative"]:
        r = dict(reps[ng["base"]])
        r[ng["field"]] = ng["value"]
        reps.append(r)
    n, nh = len(reps), len(doc["reports"])
    pub = _col(reps, "public_share", sz.public_share_len) if sz.public_share_len else None
    msgs, status, batch = eng.prepare_batch(_col(reps, "nonce", 16), pub,
                                            _col(reps, "helper_share", sz.helper_share_len),
                                            _col(reps, "leader_prep_share", sz.prep_share_len))
    want_status = [r["status"] for r in doc["reports"]] + [ng["status"] for ng in doc["negative"]]
    assert status.tolist() == want_status
    for i in range(nh):
        assert msgs[i].tobytes().hex() == doc["reports"][i]["prep_msg"]
    outs = batch.output_shares()
    for i in range(nh):
        assert outs[i].tobytes().hex() == doc["reports"][i]["helper_output_share"]
    accept = np.array([1] * nh + [0] * (n - nh), np.uint8)
    agg, cnt = batch.accumulate(None, accept, 1)
    assert agg[0].tobytes().hex() == doc["helper_aggregate_share"] and int(cnt[0]) == nh


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_leader_matches_committed_transcript(path):
    """Leader prepare_init (agg_id 0) on the stored leader input shares reproduces the stored
    leader prepare shares; prepare_next on the stored prepare messages finishes every report."""
    from janus_amd import prio3 as J
    doc = json.load(open(path))
    vk = bytes.fromhex(doc["verify_key"])
    eng = J.HelperEngine(_vdaf(doc["vdaf"]), vk)
    sz = eng.sz
    reps = doc["reports"]
    pub = _col(reps, "public_share", sz.public_share_len) if sz.public_share_len else None
    ps, status, batch = eng.leader_prepare_init_batch(
        _col(reps, "nonce", 16), pub, _col(reps, "leader_share", sz.leader_input_share_len))
    assert not status.any()
    for i, r in enumerate(reps):
        assert ps[i].tobytes().hex() == r["leader_prep_share"]
    msgs = _col(reps, "prep_msg", sz.prep_msg_len) if sz.prep_msg_len else None
    st = batch.leader_prepare_next(msgs, status)
    assert not st.any()
