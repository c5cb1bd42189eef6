"""The on-device client of Prio3SumVecField64MultiproofHmacSha256Aes128:
prio3_client_generate_device shards the multiproof VDAF on the GPU -- XofHmacSha256Aes128
shares (prio3_mp64_xof.h), both joint-rand parts, num_proofs SumVec proofs over Field64 (the
per-lane prover of the other single-gadget kinds) -- and runs the engine's device leader
prepare_init.  Pinned byte for byte against oracle/prio3_py.py gen_report_mp64 (the Python
restatement's shard + prepare_init on the same derivation; prio-byte parity of the XOF itself
is unpinned, as for every mp64 test)."""
import numpy as np
import pytest

from oracle import prio3_py as P

VK = bytes(range(0x40, 0x60))


def test_python_generator_reports_decide():
    v = P.Prio3(P.Prio3Type("sumvec_f64_mp", bits=16, length=15, chunk_length=16, num_proofs=2))
    for idx in range(2):
        d = P.gen_report_mp64(VK, 16, 15, 16, 2, seed=5, idx=idx)
        st, hps, _ = v.prepare_init(VK, 1, d["nonce"], d["public"], d["helper"])
        msg = v.prep_shares_to_prep_msg(d["lps"], hps)
        hout = v.prepare_next(st, msg)
        lout = [int.from_bytes(d["leader_out"][8 * e:8 * e + 8], "little") for e in range(15)]
        assert [(a + b) % v.F.p for a, b in zip(lout, hout)] == d["m"]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(2, 16, 15, 16), (3, 8, 10, 9), (2, 1, 4, 2)])
def test_device_generator_matches_python(cfg):
    from janus_amd import prio3 as J
    proofs, bits, length, chunk = cfg
    eng = J.HelperEngine(J.Prio3SumVecField64MultiproofHmacSha256Aes128(*cfg), VK, device=0)
    d = eng.generate_reports_device(4, seed=0x4A414E55, first_index=3, with_checks=True,
                                    with_leader_inputs=True)
    assert int(d["flags"].sum()) == 0
    for row in range(4):
        ref = P.gen_report_mp64(VK, bits, length, chunk, proofs, seed=0x4A414E55, idx=3 + row)
        got = lambda k: d[k][row].cpu().numpy().tobytes()
        assert got("nonces") == ref["nonce"]
        assert got("public_shares") == ref["public"]
        assert got("helper_shares") == ref["helper"]
        assert got("leader_input_shares") == ref["leader"]
        assert got("leader_prep_shares") == ref["lps"]
        assert [int(x) for x in d["measurements"][row].cpu().tolist()] == ref["m"]
        assert got("leader_out_shares") == ref["leader_out"]


@pytest.mark.gpu
def test_device_reports_prepare_and_unshard():
    """200k device-generated reports at the reference's configuration through the helper
    prepare + aggregate: all finish; helper + leader aggregates unshard to the measurements'
    sum."""
    import torch
    from janus_amd import prio3 as J
    n = 200_000
    eng = J.HelperEngine(J.Prio3SumVecField64MultiproofHmacSha256Aes128(2, 16, 15, 16), VK,
                         device=0)
    d = eng.generate_reports_device(n, seed=9, with_checks=True)
    assert int(d["flags"].sum()) == 0
    dev = d["nonces"].device
    sz = eng.sz
    msgs = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    agg = torch.zeros((1, sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    eng.prepare_aggregate_device(d["nonces"], d["public_shares"], d["helper_shares"],
                                 d["leader_prep_shares"], seg, 1, msgs, status)
    eng.aggregate_finish_device(status, None, agg, cnt)
    k1, k2 = 1000, n // 1000
    part = torch.zeros((k2, sz.agg_share_len), dtype=torch.uint8, device=dev)
    pc = torch.zeros(k2, dtype=torch.int64, device=dev)
    eng.combine_device(k1, k2, d["leader_out_shares"], torch.zeros(n, dtype=torch.int64,
                                                                   device=dev), part, pc)
    lagg = torch.zeros_like(agg)
    eng.combine_device(k2, 1, part, pc, lagg, torch.zeros_like(cnt))
    msum = d["measurements"].sum(dim=0).cpu().tolist()
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0 and int(cnt[0]) == n
    p = 2**64 - 2**32 + 1
    dec = lambda t: [int.from_bytes(t.cpu().numpy().tobytes()[8 * e:8 * e + 8], "little")
                     for e in range(15)]
    assert [(a + b) % p for a, b in zip(dec(agg), dec(lagg))] == msum
