"""The on-device FixedPointBoundedL2VecSum client.

prio3_client_generate_device now shards FPVec reports on the GPU -- entries from the seeded
stream, the measurement share, both joint-rand parts, the two-gadget FLP proof (NTTs in LDS,
janus_amd/csrc/prio3_client.hip k_fg_*), the leader's proofs share -- and runs the engine's own
device leader prepare_init on them.  Pinned against oracle/fpvec_py.py gen_report (the Python
restatement's shard + prepare_init on the same derivation), byte for byte: nonce, public share,
helper share, leader input share, leader prepare share, the entries and the leader output
share.  The circuit itself is the reconstruction oracle/fpvec_py.py documents (prio-byte parity
unpinned, as for every FPVec test).

  * CPU: the Python generator's reports decide at the helper and unshard to their entries;
  * GPU: the device generator equals the Python one at small sizes (P = 4 .. 64 NTTs) and at
    the full C5 size (length 10000, P = 512 and 128) for one report;
  * GPU: C5 on 100k distinct device-generated reports -- every report finishes, the helper
    aggregate plus the leader aggregate unshards to the sum of all 100k entry vectors, and the
    C restatement agrees on a subset (statuses, prepare messages, aggregate share, count).
"""
import numpy as np
import pytest

VK = bytes(range(0x50, 0x60))
P128 = 2**128 - 28 * 2**64 + 1


def _dec(buf):
    b = np.ascontiguousarray(buf, np.uint8).reshape(-1, 16)
    return [int.from_bytes(r.tobytes(), "little") for r in b]


@pytest.mark.parametrize("length,bits", [(4, 16), (30, 16), (7, 32)])
def test_python_generator_reports_decide_and_unshard(length, bits):
    from oracle.fpvec_py import FpVecType, gen_report
    from oracle.prio3_py import Prio3
    typ = FpVecType(length, bits)
    P = Prio3(typ)
    for idx in range(2):
        d = gen_report(VK, length, bits, seed=91, idx=idx)
        st, hps, _ = P.prepare_init(VK, 1, d["nonce"], d["public"], d["helper"])
        msg = P.prep_shares_to_prep_msg(d["lps"], hps)
        hout = P.prepare_next(st, msg)
        lout = _dec(np.frombuffer(d["leader_out"], np.uint8))
        half = 1 << (bits - 1)
        assert [(a + b) % P128 for a, b in zip(lout, hout)] == [x + half for x in d["X"]]
        assert sum(x * x for x in d["X"]) < 2 ** (2 * bits - 2)


def _device(length, bits, n, first, seed, leader_inputs=True):
    from janus_amd import prio3 as J
    eng = J.HelperEngine(J.Prio3FixedPointBoundedL2VecSum(length, bits), VK, device=0,
                         allow_unpinned=True)
    d = eng.generate_reports_device(n, seed=seed, first_index=first, with_checks=True,
                                    with_leader_inputs=leader_inputs)
    return eng, d


def _check_against_python(d, length, bits, seed, idxs, rows):
    from oracle.fpvec_py import gen_report
    assert int(d["flags"][rows].sum()) == 0
    for row, idx in zip(rows, idxs):
        ref = gen_report(VK, length, bits, seed=seed, idx=idx)
        got = lambda k: d[k][row].cpu().numpy().tobytes()
        assert got("nonces") == ref["nonce"]
        assert got("public_shares") == ref["public"]
        assert got("helper_shares") == ref["helper"]
        assert got("leader_input_shares") == ref["leader"]
        assert got("leader_prep_shares") == ref["lps"]
        assert d["measurements"][row].cpu().tolist() == ref["X"]
        assert got("leader_out_shares") == ref["leader_out"]


@pytest.mark.gpu
@pytest.mark.parametrize("length,bits", [(4, 16), (30, 16), (100, 16), (7, 32), (60, 32)])
def test_device_generator_matches_python(length, bits):
    _, d = _device(length, bits, 3, first=5, seed=77)
    _check_against_python(d, length, bits, 77, [5, 6, 7], [0, 1, 2])


@pytest.mark.gpu
def test_device_generator_matches_python_full_size():
    """Length 10000 (C5): gadget 0 on P = 512, gadget 1 on P = 128 -- report 1 of a chunk of
    two against the Python restatement (about a minute of CPU)."""
    _, d = _device(10000, 16, 2, first=0, seed=0x4A414E5553000005)
    _check_against_python(d, 10000, 16, 0x4A414E5553000005, [1], [1])


@pytest.mark.gpu
def test_c5_100k_distinct_device_reports():
    """configs[4] on 100k distinct device-generated reports: all finish; helper + leader
    aggregates unshard to the entries' sum; the C restatement agrees on the first reports."""
    import torch
    from oracle.oracle import Oracle
    n, m, L = 100_000, 32, 10000
    eng, d = _device(L, 16, n, first=0, seed=0x4A414E5553000006, leader_inputs=False)
    assert int(d["flags"].sum()) == 0
    dev = d["nonces"].device
    msgs = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    seg = torch.zeros(n, dtype=torch.int32, device=dev)
    agg = torch.zeros((1, eng.sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    eng.prepare_device(d["nonces"], d["public_shares"], d["helper_shares"],
                       d["leader_prep_shares"], msgs, status)
    eng.accumulate_device(n, status, seg, None, 1, agg, cnt)
    # leader aggregate: mod-p sum of the leader output shares, two combine levels
    k1, k2 = 1000, n // 1000
    part = torch.zeros((k2, eng.sz.agg_share_len), dtype=torch.uint8, device=dev)
    pc = torch.zeros(k2, dtype=torch.int64, device=dev)
    eng.combine_device(k1, k2, d["leader_out_shares"], torch.zeros(n, dtype=torch.int64,
                                                                   device=dev), part, pc)
    lagg = torch.zeros_like(agg)
    lc = torch.zeros_like(cnt)
    eng.combine_device(k2, 1, part, pc, lagg, lc)
    esum = d["measurements"].sum(dim=0).cpu().tolist()
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0 and int(cnt[0]) == n
    tot = [(a + b) % P128 for a, b in zip(_dec(agg.cpu().numpy()), _dec(lagg.cpu().numpy()))]
    assert tot == [x + n * (1 << 15) for x in esum]
    # the C restatement on the first m reports (accept mask selecting them on the device)
    h = {k: d[k][:m].cpu().numpy() for k in
         ("nonces", "public_shares", "helper_shares", "leader_prep_shares")}
    o = Oracle("fpvec", bits=16, length=L)
    rm, rs, ra, rc = o.helper_batch(VK, h["nonces"], h["public_shares"], h["helper_shares"],
                                    h["leader_prep_shares"], n_threads=16)
    np.testing.assert_array_equal(status[:m].cpu().numpy(), rs)
    np.testing.assert_array_equal(msgs[:m].cpu().numpy(), rm)
    acc = torch.zeros(n, dtype=torch.uint8, device=dev)
    acc[:m] = 1
    agg_s = torch.zeros_like(agg)
    cnt_s = torch.zeros_like(cnt)
    eng.accumulate_device(n, status, seg, acc, 1, agg_s, cnt_s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(agg_s.cpu().numpy().reshape(-1), np.asarray(ra).reshape(-1))
    assert int(cnt_s[0]) == int(np.asarray(rc).reshape(-1)[0]) == m
    # the engine gone, its ~225 GB run goes back to the pool, and the
    # pool frees it -- it is above the pool's budget (1/8 of HBM) -- without prio3_device_trim
    eng.close()
    del d, msgs, status, seg, agg, cnt, part, pc, lagg, lc, acc, agg_s, cnt_s
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, total = torch.cuda.mem_get_info(0)
    held = torch.cuda.memory_reserved(0)
    assert total - free <= total // 8 + held + (6 << 30), \
        f"{(total - free) / 2**30:.1f} GiB in use of {total / 2**30:.0f} after the C5 batch"
