"""The device-resident helper aggregation-job init, request bytes to response bytes:
AggregationJobInitializeReq body -> janus_dap unpack -> janus_hpke open of the helper input
shares -> prio3 prepare + aggregate (+ batch metadata) -> AggregationJobResp body, against the
CPU oracles of each stage (oracle/dap_codec.py, oracle/hpke_oracle.c, oracle/prio3_oracle.c),
with HPKE, message-type and decide failures mixed in.  Mirrors aggregator.rs:1720-2096."""
import numpy as np
import pytest

from oracle import dap_codec as D
from oracle import hpke as H

pytestmark = pytest.mark.gpu
VK = bytes(range(0x20, 0x30))


def _job(n, seed):
    from oracle.oracle import Oracle
    rng = np.random.default_rng(seed)
    o = Oracle("histogram", length=256, chunk_length=16)
    d = o.gen_reports(VK, n, seed=seed, n_threads=8)
    skR = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    pkR = H.x25519_public(skR)
    task = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    times = (1_700_000_000 + rng.integers(0, 3600, n)).astype(np.uint64)
    lps = d["leader_prep_shares"].copy()
    bad_hpke = set(rng.choice(n, max(1, n // 20), replace=False).tolist())
    bad_msg = set(rng.choice(n, max(1, n // 30), replace=False).tolist()) - bad_hpke
    bad_decide = set(rng.choice(n, max(1, n // 25), replace=False).tolist())
    for r in bad_decide:
        lps[r, 20] ^= 1
    inits = []
    for r in range(n):
        aad = H.input_share_aad(task, d["nonces"][r].tobytes(), int(times[r]),
                                d["public_shares"][r].tobytes())
        enc, ct = H.seal(pkR, bytes(rng.integers(0, 256, 32, dtype=np.uint8)),
                         H.INFO_INPUT_SHARE_HELPER, aad,
                         H.plaintext_input_share(d["helper_shares"][r].tobytes()))
        if r in bad_hpke:
            ct = ct[:-1] + bytes([ct[-1] ^ 1])
        msg = (dict(type="finish", prep_msg=lps[r].tobytes()) if r in bad_msg else
               dict(type="initialize", prep_share=lps[r].tobytes()))
        inits.append(dict(report_id=d["nonces"][r].tobytes(), time=int(times[r]),
                          public_share=d["public_shares"][r].tobytes(), config_id=1, enc=enc,
                          payload=ct, message=msg))
    body = D.encode_agg_init_req(b"", 1, None, inits)
    return o, skR, pkR, task, body


def _expected(o, skR, pkR, task, body):
    req = D.decode_agg_init_req(body)
    P = req["prepare_inits"]
    n = len(P)
    ids = np.array([list(p["report_id"]) for p in P], np.uint8)
    times = np.array([p["time"] for p in P], np.uint64)
    pubs = np.array([list(p["public_share"]) for p in P], np.uint8)
    enc = np.array([list(p["enc"]) for p in P], np.uint8)
    stride = -(-max(len(p["payload"]) for p in P) // 16) * 16
    ct = np.zeros((n, stride), np.uint8)
    cl = np.zeros(n, np.uint32)
    for r, p in enumerate(P):
        ct[r, :len(p["payload"])] = np.frombuffer(p["payload"], np.uint8)
        cl[r] = len(p["payload"])
    shares, hs = H.open_input_shares(skR, pkR, task, enc, ct, cl, ids, times, pubs, 48)
    msg_st = np.array([0 if p["message"]["type"] == "initialize" else 5 for p in P], np.uint8)
    lps = np.array([list(p["message"].get("prep_share", p["message"].get("prep_msg"))) for p in P],
                   np.uint8)
    msgs, st, agg, cnt = o.helper_batch(VK, ids, pubs, shares, lps,
                                        accept_mask=((hs == 0) & (msg_st == 0)).astype(np.uint8),
                                        n_threads=8)
    pe = np.where(hs == 0, 0xFF, hs).astype(np.uint8)
    resp = D.helper_init_resp(ids, pe, st | msg_st, msgs)
    return resp, agg, cnt


@pytest.mark.parametrize("n", [64, 700])
def test_device_helper_init_request_to_response(n):
    import torch
    from janus_amd import dap as DJ
    from janus_amd import hpke as G
    from janus_amd import prio3 as J
    o, skR, pkR, task, body = _job(n, seed=n)
    exp_resp, exp_agg, exp_cnt = _expected(o, skR, pkR, task, body)
    dev = torch.device("cuda", 0)
    lay = DJ.scan(body)
    assert lay.uniform and lay.n == n
    d_body = torch.zeros(len(body) + 8, dtype=torch.uint8, device=dev)
    d_body[:len(body)] = torch.frombuffer(bytearray(body), dtype=torch.uint8).to(dev)
    u, mism = DJ.unpack_device(lay, d_body, DJ.ct_stride_for(lay))
    op = G.HpkeOpener(skR, pkR)
    shares = torch.empty((n, 48), dtype=torch.uint8, device=dev)
    hs = torch.empty(n, dtype=torch.uint8, device=dev)
    op.open_input_shares_device(task, u["enc"], u["ct"], u["ct_len"], u["report_ids"],
                                u["times"], u["public_shares"], shares, hs)
    eng = J.HelperEngine(J.Prio3Histogram(256, 16), VK, device=0)
    msgs = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    eng.prepare_aggregate_device(u["report_ids"], u["public_shares"], shares, u["prep_shares"],
                                 seg, 1, msgs, st)
    accept = ((hs == 0) & (u["msg_status"] == 0)).to(torch.uint8)
    agg = torch.zeros((1, eng.sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    eng.aggregate_finish_device(st, accept, agg, cnt)
    pe = DJ.prepare_error(hs, u["msg_status"])
    out, ln = DJ.encode_resp_device(u["report_ids"], pe, st | u["msg_status"], msgs, 16)
    torch.cuda.synchronize()
    assert int(mism[0]) == 0
    got = out[:int(ln[0])].cpu().numpy().tobytes()
    assert got == exp_resp
    np.testing.assert_array_equal(agg.cpu().numpy(), exp_agg)
    assert int(cnt[0]) == int(exp_cnt[0])
