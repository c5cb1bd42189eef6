"""The helper's whole per-report loop body in ONE host-buffer call:
prio3_helper_aggregate_init_batch = the HPKE open of each report's sealed input share, the
PlaintextInputShare decode and extension checks, helper_initialized + evaluate and the accumulate
(VdafOps::handle_aggregate_init_generic, /root/reference/aggregator/src/aggregator.rs:1794-2096),
coalesced by the executor across jobs of several tasks, with the decrypted shares kept on the GPU.

Expected values: the OpenSSL-composed HPKE oracle (oracle/hpke_oracle.c, pinned by RFC 9180's
vectors) opens the same ciphertexts, then the C restatement of prio prepares and aggregates what it
opened with the open's rejections excluded; the merged status is 0x80 | PrepareError for a report
the open rejected (the order of aggregator.rs), else the VDAF status."""
import threading

import numpy as np
import pytest

from tests.conftest import CONFIGS
from tests.test_gpu_executor import _Held, _engine
from tests.test_gpu_parity import _tamper

pytestmark = pytest.mark.gpu

TASKPROV = 0xFF00


def _sealed_job(o, vk, n, seed, pkR, task_id, rng, tamper=True, share_len=None):
    """n reports of the instance, sealed to pkR under task_id, with VDAF failures (decide, decode,
    joint-rand, wrong helper seed), HPKE failures (flipped tag) and InvalidMessage rejections (an
    unexpected taskprov extension; a payload of the wrong length) mixed in."""
    from oracle import hpke as H
    d = o.gen_reports(vk, n, seed=seed, n_threads=4)
    if tamper:
        d = _tamper(o, d, rng)
    times = (1_700_000_000 + rng.integers(0, 3600, n)).astype(np.uint64)
    pubs = d["public_shares"] if d["public_shares"].shape[1] else None
    enc, ct, cl, stride = H.seal_input_shares(pkR, task_id, d["nonces"], times, pubs,
                                              d["helper_shares"], seed=seed, n_threads=4)
    stride += 16  # room for the resealed plaintexts below (extension / longer payload)
    ct = np.concatenate([ct, np.zeros((n, 16), np.uint8)], axis=1)
    if tamper:
        for r in rng.choice(n, max(1, n // 20), replace=False):
            ct[r, cl[r] - 1] ^= 0x01  # the AEAD tag
        bad = rng.choice(n, max(2, n // 25), replace=False)
        for i, r in enumerate(bad):
            share = d["helper_shares"][r].tobytes()
            pt = (H.plaintext_input_share(share, [(TASKPROV, b"")]) if i % 2 == 0 else
                  H.plaintext_input_share(share + b"\x00"))
            aad = H.input_share_aad(task_id, d["nonces"][r].tobytes(), int(times[r]),
                                    b"" if pubs is None else pubs[r].tobytes())
            e, c = H.seal(pkR, bytes(rng.integers(0, 256, 32, dtype=np.uint8)),
                          H.INFO_INPUT_SHARE_HELPER, aad, pt)
            enc[r] = np.frombuffer(e, np.uint8)
            ct[r] = 0
            ct[r, :len(c)] = np.frombuffer(c, np.uint8)
            cl[r] = len(c)
    d.update(times=times, enc=enc, ct=ct, ct_len=cl)
    return d


def _expected(o, vk, d, skR, pkR, task_id, seg=None, accept=None, n_segments=1):
    from oracle import hpke as H
    n = d["nonces"].shape[0]
    pubs = d["public_shares"] if d["public_shares"].shape[1] else None
    shares, hs = H.open_input_shares(skR, pkR, task_id, d["enc"], d["ct"], d["ct_len"],
                                     d["nonces"], d["times"], pubs, o.helper_share_len,
                                     n_threads=4)
    acc = (hs == 0).astype(np.uint8)
    if accept is not None:
        acc &= accept
    msgs, st, agg, cnt = o.helper_batch(vk, d["nonces"], d["public_shares"], shares,
                                        d["leader_prep_shares"], segment_ids=seg, accept_mask=acc,
                                        n_segments=n_segments, n_threads=4)
    merged = np.where(hs != 0, 0x80 | hs, st).astype(np.uint8)
    return msgs, merged, agg, cnt, hs


def _check(got, exp):
    msgs, st, agg, cnt = got
    emsgs, est, eagg, ecnt, hs = exp
    np.testing.assert_array_equal(st, est)
    ok = hs == 0  # the prepare message of a report the open rejected is not defined
    np.testing.assert_array_equal(msgs[ok], emsgs[ok])
    np.testing.assert_array_equal(agg, eagg)
    np.testing.assert_array_equal(cnt, ecnt)


@pytest.mark.parametrize("name", ["hist_256_c16", "count", "sum32"])
def test_one_job_matches_open_then_prepare(name):
    """One job per instance (pub share 32 / 0 bytes, helper share 48 / 32 bytes; fused and
    unfused accumulate), three segments and an accept mask, every failure kind present."""
    from janus_amd import hpke as G
    from janus_amd import prio3 as J
    from oracle import hpke as H
    from oracle.oracle import Oracle
    cfg = CONFIGS[name]
    o = Oracle(**cfg)
    rng = np.random.default_rng(41)
    vk = bytes(range(0x40, 0x50))
    skR = H.kem_private(rng)
    pkR = H.kem_public(skR)
    task = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    n = 437
    d = _sealed_job(o, vk, n, 7, pkR, task, rng)
    seg = rng.integers(0, 3, n).astype(np.uint32)
    accept = (rng.random(n) < 0.9).astype(np.uint8)
    eng = _engine(cfg, vk)
    op = G.HpkeOpener(skR, pkR, device=0)
    got = eng.aggregate_init_batch(op, task, d["nonces"], d["times"], d["public_shares"],
                                   d["enc"], d["ct"], d["ct_len"], d["leader_prep_shares"],
                                   seg, accept, 3)
    exp = _expected(o, vk, d, skR, pkR, task, seg, accept, 3)
    _check(got, exp)
    st = got[1]
    for code in (J.STATUS_HPKE_DECRYPT, J.STATUS_INVALID_MESSAGE, J.STATUS_PREP_MSG,
                 J.STATUS_FINISHED):
        assert (st == code).any(), (name, code)


def test_concurrent_jobs_of_several_tasks_and_keypairs():
    """18 jobs of 3 tasks (verify keys, task IDs) under two HPKE keypairs, queued behind the
    executor's hold from 18 threads: every job equals the oracles', and the jobs of one keypair
    share launches (fewer prepare groups than jobs)."""
    from janus_amd import hpke as G
    from oracle import hpke as H
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_256_c16"]
    o = Oracle(**cfg)
    rng = np.random.default_rng(43)
    vks = [bytes([0x71 + t]) * 16 for t in range(3)]
    tasks = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(3)]
    keys = [H.kem_private(rng) for _ in range(2)]
    pks = [H.kem_public(k) for k in keys]
    engines = [_engine(cfg, vk) for vk in vks]
    openers = [G.HpkeOpener(k, p, device=0) for k, p in zip(keys, pks)]
    jobs = []
    for j in range(18):
        t, k = j % 3, (j // 3) % 2
        n = int(rng.integers(100, 501))
        d = _sealed_job(o, vks[t], n, 200 + j, pks[k], tasks[t], rng, tamper=j % 2 == 0)
        seg = rng.integers(0, 2, n).astype(np.uint32)
        jobs.append((t, k, d, seg))
    out = [None] * len(jobs)

    def run(j):
        t, k, d, seg = jobs[j]
        out[j] = engines[t].aggregate_init_batch(openers[k], tasks[t], d["nonces"], d["times"],
                                                 d["public_shares"], d["enc"], d["ct"],
                                                 d["ct_len"], d["leader_prep_shares"], seg, None,
                                                 2)

    g0 = engines[0].executor_stats(0)["groups"]
    with _Held(engines[0], len(jobs)) as h:
        th = [threading.Thread(target=run, args=(j,)) for j in range(len(jobs))]
        for x in th:
            x.start()
        h.wait()
        for x in th:
            x.join()
    launches = engines[0].executor_stats(0)["groups"] - g0
    assert 2 <= launches < len(jobs), launches
    for j, (t, k, d, seg) in enumerate(jobs):
        _check(out[j], _expected(o, vks[t], d, keys[k], pks[k], tasks[t], seg, None, 2))


def test_taskprov_task_and_wide_segment_fallback():
    """require_taskprov (aggregator.rs:1929-1949: the taskprov extension must be present and
    empty) and a job with more segments than one group carries (the open and the prepare then
    run as two host calls): both equal the oracles'."""
    from janus_amd import hpke as G
    from oracle import hpke as H
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_256_c16"]
    o = Oracle(**cfg)
    rng = np.random.default_rng(47)
    vk = bytes([0x5A]) * 16
    skR = H.kem_private(rng)
    pkR = H.kem_public(skR)
    task = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    eng = _engine(cfg, vk)
    op = G.HpkeOpener(skR, pkR, device=0)
    # taskprov: half the reports carry the extension, so half are rejected as InvalidMessage
    n = 300
    d = o.gen_reports(vk, n, seed=5, n_threads=4)
    times = (1_700_000_000 + rng.integers(0, 3600, n)).astype(np.uint64)
    enc = np.zeros((n, 32), np.uint8)
    ct = np.zeros((n, 96), np.uint8)
    cl = np.zeros(n, np.uint32)
    for r in range(n):
        ext = [(TASKPROV, b"")] if r % 2 == 0 else []
        aad = H.input_share_aad(task, d["nonces"][r].tobytes(), int(times[r]),
                                d["public_shares"][r].tobytes())
        e, c = H.seal(pkR, bytes(rng.integers(0, 256, 32, dtype=np.uint8)),
                      H.INFO_INPUT_SHARE_HELPER, aad,
                      H.plaintext_input_share(d["helper_shares"][r].tobytes(), ext))
        enc[r] = np.frombuffer(e, np.uint8)
        ct[r, :len(c)] = np.frombuffer(c, np.uint8)
        cl[r] = len(c)
    got = eng.aggregate_init_batch(op, task, d["nonces"], times, d["public_shares"], enc, ct, cl,
                                   d["leader_prep_shares"], require_taskprov=True)
    shares, hs = H.open_input_shares(skR, pkR, task, enc, ct, cl, d["nonces"], times,
                                     d["public_shares"], 48, require_taskprov=True, n_threads=4)
    assert (hs[1::2] == 8).all() and (hs[0::2] == 0).all()
    msgs, st, agg, cnt = o.helper_batch(vk, d["nonces"], d["public_shares"], shares,
                                        d["leader_prep_shares"], accept_mask=(hs == 0).astype(
                                            np.uint8), n_threads=4)
    _check(got, (msgs, np.where(hs != 0, 0x80 | hs, st).astype(np.uint8), agg, cnt, hs))
    assert int(got[3][0]) == n // 2
    # 1025 segments (one more than a group takes): the two-call form inside the library
    d2 = _sealed_job(o, vk, 500, 9, pkR, task, rng)
    seg = rng.integers(0, 1025, 500).astype(np.uint32)
    got = eng.aggregate_init_batch(op, task, d2["nonces"], d2["times"], d2["public_shares"],
                                   d2["enc"], d2["ct"], d2["ct_len"], d2["leader_prep_shares"],
                                   seg, None, 1025)
    _check(got, _expected(o, vk, d2, skR, pkR, task, seg, None, 1025))


def test_sealed_jobs_on_an_engine_over_two_executors():
    """The one-call helper init on an engine over the device list [0, 0] (two executors standing
    in for two GPUs, prio3_engine_create_devices): 16 concurrent sealed-input jobs are placed on
    both members, each opens its input shares on the member that runs it (the opener is bound to
    GPU 0 only for its own stream), and every job equals OpenSSL + the restatement."""
    from concurrent.futures import ThreadPoolExecutor

    from janus_amd import hpke as G
    from janus_amd import prio3 as J
    from oracle import hpke as H
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_256_c16"]
    o = Oracle(**cfg)
    rng = np.random.default_rng(61)
    vk = bytes([0x3C]) * 16
    skR = H.kem_private(rng)
    pkR = H.kem_public(skR)
    task = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    eng = J.HelperEngine(J.Prio3Histogram(256, 16), vk, devices=[0, 0])
    op = G.HpkeOpener(skR, pkR, device=0)
    m0 = eng.members()
    jobs = [_sealed_job(o, vk, int(rng.integers(100, 400)), 1500 + j, pkR, task, rng,
                        tamper=j % 2 == 0) for j in range(16)]

    def run(d):
        return eng.aggregate_init_batch(op, task, d["nonces"], d["times"], d["public_shares"],
                                        d["enc"], d["ct"], d["ct_len"], d["leader_prep_shares"])

    with ThreadPoolExecutor(16) as ex:
        got = list(ex.map(run, jobs))
    m1 = eng.members()
    placed = [m["jobs"] - a["jobs"] for m, a in zip(m1, m0)]
    assert sum(placed) == 16 and min(placed) > 0, placed
    for d, g in zip(jobs, got):
        _check(g, _expected(o, vk, d, skR, pkR, task))
