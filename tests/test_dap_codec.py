"""DAP-09 wire format <-> SoA marshaling, pinned by the reference codec's
own roundtrip fixtures (messages/src/tests/aggregation.rs, extracted to
tests/golden/dap_fixtures.json by tests/golden/gen_dap_fixtures.py).

CPU: the oracle codec (oracle/dap_codec.py) decodes and re-encodes the fixtures byte-exactly;
the library's host parser and response encoder agree with it.  GPU: the speculative device
unpack and the device response encoder agree with the host forms, and the whole device-resident
helper init (request body -> unpack -> HPKE open -> prepare+aggregate -> response body) agrees
with the CPU oracles end to end."""
import json
import os
import struct

import numpy as np
import pytest

from oracle import dap_codec as D

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dap_fixtures.json")))
RID1 = bytes(range(1, 17))
RID2 = bytes(range(16, 0, -1))


def test_oracle_decodes_reference_init_req_fixtures():
    for key, qt in (("agg_init_req_time_interval", 1), ("agg_init_req_fixed_size", 2)):
        b = bytes.fromhex(FX[key])
        d = D.decode_agg_init_req(b)
        assert d["aggregation_parameter"] == b"012345" and d["query_type"] == qt
        assert d["batch_id"] == (None if qt == 1 else bytes([2] * 32))
        p0, p1 = d["prepare_inits"]
        assert (p0["report_id"], p0["time"], p0["public_share"], p0["config_id"], p0["enc"],
                p0["payload"]) == (RID1, 54321, b"", 42, b"012345", b"543210")
        assert p0["message"] == dict(type="initialize", prep_share=b"012345")
        assert (p1["report_id"], p1["time"], p1["public_share"], p1["config_id"], p1["enc"],
                p1["payload"]) == (RID2, 73542, b"0123", 13, b"abce", b"abfd")
        assert p1["message"] == dict(type="finish", prep_msg=b"")
        assert D.encode_agg_init_req(d["aggregation_parameter"], qt, d["batch_id"],
                                     d["prepare_inits"]) == b


def test_oracle_encodes_reference_resp_fixtures():
    resp = D.encode_agg_job_resp([
        (RID1, ("continue", dict(type="continue", prep_msg=b"01234", prep_share=b"56789"))),
        (RID2, ("finished",))])
    assert resp == bytes.fromhex(FX["agg_job_resp"])
    # the Reject(VdafPrepError) PrepareResp: what the helper sends for a failed report
    assert D.encode_prepare_resp(bytes([255] * 16), ("reject", 5)) == \
        bytes.fromhex(FX["prepare_resps"])[-18:]


def test_host_scan_and_unpack_match_the_fixture():
    from janus_amd import dap as J
    for key in ("agg_init_req_time_interval", "agg_init_req_fixed_size"):
        b = bytes.fromhex(FX[key])
        lay = J.scan(b)
        assert lay.query_type == (1 if "time" in key else 2)
        assert lay.record_len == 16 + 8 + 4 + 0 + 1 + 2 + 6 + 4 + 6 + 4 + 11
        assert not lay.uniform  # the second record is shorter: host path
        out = J.unpack_host(b, lay, 8, 16)
        assert len(out["times"]) == 2
        assert out["report_ids"][0].tobytes() == RID1 and out["report_ids"][1].tobytes() == RID2
        assert out["times"].tolist() == [54321, 73542]
        assert out["config_ids"].tolist() == [42, 13]
        assert out["ct"][0, :6].tobytes() == b"543210" and out["ct_len"][0] == 6
        assert out["ct_len"][1] == 0  # enc of another length than the first record's
        assert out["prep_shares"][0].tobytes() == b"012345"
        # record 2: a public share of another length than the first record's does not decode
        # (InvalidMessage, aggregator.rs:1985-1999) -- before its Finish message would matter
        assert out["msg_status"].tolist() == [0, 6]
    with pytest.raises(ValueError):
        J.scan(bytes.fromhex(FX["agg_init_req_time_interval"]) + b"\0")  # trailing byte


def _body(records):
    return D.encode_agg_init_req(b"", 1, None, [
        dict(report_id=bytes([i] * 16), time=1000 + i, public_share=ps, config_id=1,
             enc=b"e" * 32, payload=b"p" * 40, message=msg)
        for i, (ps, msg) in enumerate(records)])


def test_host_unpack_message_and_public_share_errors():
    """ADVICE r1 (dap_codec host unpack): per-report statuses follow Janus's order -- public
    share decode (6 -> InvalidMessage) before the ping-pong message (5 PeerMessageMismatch,
    2 CodecPrepShare); an unknown PingPongMessage type or bad framing rejects the request."""
    from janus_amd import dap as J
    init = lambda n: dict(type="initialize", prep_share=b"s" * n)
    body = _body([(b"P" * 32, init(48)), (b"P" * 31, init(48)), (b"P" * 32, init(47)),
                  (b"P" * 32, dict(type="continue", prep_msg=b"m", prep_share=b"s" * 48)),
                  (b"P" * 32, dict(type="finish", prep_msg=b"m" * 16)), (b"", init(48))])
    lay = J.scan(body)
    out = J.unpack_host(body, lay, 8, J.ct_stride_for(lay))
    assert out["msg_status"].tolist() == [0, 6, 2, 5, 5, 6]
    assert not out["public_shares"][1].any() and out["public_shares"][0].tobytes() == b"P" * 32
    hs = np.array([0, 0, 0, 0, 4, 4], np.uint8)  # HPKE errors win over the public share's
    assert J.prepare_error(hs, out["msg_status"]).tolist() == [0xFF, 8, 0xFF, 0xFF, 4, 4]
    good = bytearray(_body([(b"P" * 32, init(48))]))
    for mutate in (lambda b: b.__setitem__(len(b) - 53, 3),   # message type 3: not a type
                   lambda b: b.__setitem__(len(b) - 49, 40)):  # prep_share length 40 of 48 bytes
        bad = bytearray(good)
        mutate(bad)
        with pytest.raises(ValueError):
            J.unpack_host(bytes(bad), J.scan(bytes(bad)), 8, 64)


def test_scan_with_expected_lengths_fails_only_the_malformed_first_record():
    """ADVICE r2 (dap_codec.hip scan): only record 0 has a public share of the wrong length (and,
    in a second body, an enc of the wrong length and a short prep share).  With the task's
    expected lengths (scan_ex) the layout keeps those lengths, the body goes to the host unpack,
    and only record 0 fails -- the reference fails just the report whose share does not decode
    (aggregator.rs:1967-1999); taking the first record's lengths would fail all the others."""
    from janus_amd import dap as J
    init = lambda n: dict(type="initialize", prep_share=b"s" * n)
    body = _body([(b"P" * 31, init(48))] + [(b"P" * 32, init(48))] * 4)
    naive = J.unpack_host(body, J.scan(body), 8, 64)
    assert naive["msg_status"].tolist() == [0, 6, 6, 6, 6]  # what first-record lengths give
    lay = J.scan(body, public_share_len=32, enc_len=32, prep_share_len=48)
    assert (lay.public_share_len, lay.enc_len, lay.prep_share_len, lay.uniform) == (32, 32, 48, 0)
    out = J.unpack_host(body, lay, 8, J.ct_stride_for(lay))
    assert out["msg_status"].tolist() == [6, 0, 0, 0, 0]
    assert not out["public_shares"][0].any() and out["public_shares"][1].tobytes() == b"P" * 32
    assert out["ct_len"].tolist() == [40] * 5
    # a wrong-length enc in record 0 is that report's HPKE decrypt error; a short prep share
    # its CodecPrepShare
    recs = [dict(report_id=bytes([i] * 16), time=1000 + i, public_share=b"P" * 32, config_id=1,
                 enc=b"e" * (31 if i == 0 else 32), payload=b"p" * 40,
                 message=init(47 if i == 0 else 48)) for i in range(4)]
    body2 = D.encode_agg_init_req(b"", 1, None, recs)
    lay2 = J.scan(body2, public_share_len=32, enc_len=32, prep_share_len=48)
    assert not lay2.uniform
    out2 = J.unpack_host(body2, lay2, 8, J.ct_stride_for(lay2))
    assert out2["msg_status"].tolist() == [2, 0, 0, 0]
    assert out2["ct_len"].tolist() == [0, 40, 40, 40]
    # a uniform body with the expected lengths keeps the device path
    ok = J.scan(_body([(b"P" * 32, init(48))] * 3), public_share_len=32, enc_len=32,
                prep_share_len=48)
    assert ok.uniform and ok.n == 3


def test_host_resp_encoder_matches_oracle():
    from janus_amd import dap as J
    rng = np.random.default_rng(3)
    n, pml = 500, 16
    ids = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    pe = np.where(rng.random(n) < 0.1, rng.integers(0, 10, n), 0xFF).astype(np.uint8)
    st = np.where(rng.random(n) < 0.1, rng.integers(1, 6, n), 0).astype(np.uint8)
    pm = rng.integers(0, 256, (n, pml), dtype=np.uint8)
    got = J.encode_resp_host(ids, pe, st, pm, pml)
    assert got == D.helper_init_resp(ids, pe, st, pm)
    assert J.encode_resp_host(ids[:0], pe[:0], st[:0], pm[:0], pml) == b"\0\0\0\0"


def _uniform_body(n, psl, ps_len, seed, bad_type=()):
    rng = np.random.default_rng(seed)
    inits = []
    for r in range(n):
        msg = (dict(type="finish", prep_msg=bytes(rng.integers(0, 256, ps_len, dtype=np.uint8)))
               if r in bad_type else
               dict(type="initialize", prep_share=bytes(rng.integers(0, 256, ps_len, dtype=np.uint8))))
        inits.append(dict(report_id=bytes(rng.integers(0, 256, 16, dtype=np.uint8)),
                          time=1_700_000_000 + int(rng.integers(0, 3600)),
                          public_share=bytes(rng.integers(0, 256, psl, dtype=np.uint8)),
                          config_id=7, enc=bytes(rng.integers(0, 256, 32, dtype=np.uint8)),
                          payload=bytes(rng.integers(0, 256, 70, dtype=np.uint8)), message=msg))
    return D.encode_agg_init_req(b"", 1, None, inits)


@pytest.mark.gpu
@pytest.mark.parametrize("n,psl", [(1, 32), (1000, 32), (777, 0)])
def test_gpu_unpack_matches_host(n, psl):
    import torch
    from janus_amd import dap as J
    body = _uniform_body(n, psl, 560, seed=n + psl, bad_type={3, 50})
    lay = J.scan(body)
    assert lay.uniform and lay.n == n
    stride = J.ct_stride_for(lay)
    d_body = torch.zeros(len(body) + 8, dtype=torch.uint8, device="cuda")
    d_body[:len(body)] = torch.frombuffer(bytearray(body), dtype=torch.uint8).cuda()
    out, mism = J.unpack_device(lay, d_body, stride)
    torch.cuda.synchronize()
    assert int(mism[0]) == 0
    ref = J.unpack_host(body, lay, n, stride)
    for k, v in ref.items():
        g = out[k].cpu().numpy()
        if k == "times":
            g = g.view(np.uint64)
        if k == "ct_len":
            g = g.view(np.uint32)
        if k == "public_shares" and psl == 0:
            continue
        if k == "prep_shares":  # rows with a message error are not written on the device
            ok = ref["msg_status"] == 0
            np.testing.assert_array_equal(g[ok], v[ok])
            continue
        np.testing.assert_array_equal(g.reshape(v.shape), v, err_msg=k)
    assert sorted(np.nonzero(ref["msg_status"])[0].tolist()) == ([3, 50] if n > 50 else [])


@pytest.mark.gpu
def test_gpu_unpack_reports_nonuniform_records():
    import torch
    from janus_amd import dap as J
    body = bytes.fromhex(FX["agg_init_req_time_interval"])
    # two copies of the first record of the fixture + the shorter second one: not uniform
    lay = J.scan(body)
    assert not lay.uniform
    # a uniform-length body where one record hides a different field split
    b2 = bytearray(_uniform_body(10, 32, 560, seed=1))
    lay2 = J.scan(bytes(b2))
    off = lay2.list_off + 4 * lay2.record_len + 24
    b2[off:off + 4] = struct.pack(">I", 31)  # public share 31 bytes -> enc misplaced
    d_body = torch.zeros(len(b2) + 8, dtype=torch.uint8, device="cuda")
    d_body[:len(b2)] = torch.frombuffer(b2, dtype=torch.uint8).cuda()
    out, mism = J.unpack_device(lay2, d_body, J.ct_stride_for(lay2))
    torch.cuda.synchronize()
    assert int(mism[0]) == 1


@pytest.mark.gpu
def test_gpu_resp_encoder_matches_host():
    import torch
    from janus_amd import dap as J
    rng = np.random.default_rng(5)
    for n, pml in ((1, 16), (300, 16), (70000, 16), (513, 0)):
        ids = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        pe = np.where(rng.random(n) < 0.1, rng.integers(0, 10, n), 0xFF).astype(np.uint8)
        st = np.where(rng.random(n) < 0.2, rng.integers(1, 6, n), 0).astype(np.uint8)
        pm = rng.integers(0, 256, (n, max(pml, 1)), dtype=np.uint8)
        T = lambda a: torch.from_numpy(a).cuda()
        out, ln = J.encode_resp_device(T(ids), T(pe), T(st), T(pm), pml)
        torch.cuda.synchronize()
        got = out[:int(ln[0])].cpu().numpy().tobytes()
        assert got == J.encode_resp_host(ids, pe, st, pm[:, :pml], pml)
