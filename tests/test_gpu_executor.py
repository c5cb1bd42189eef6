"""The host runtime under the C ABI: per-batch device state and the coalescing executor.

* Janus prepares concurrent aggregation jobs of one task on one VdafOps (one engine), each in
  its own rayon::spawn (/root/reference/aggregator/src/aggregator.rs:2100-2123), and merges each
  job's output shares later (aggregation_job_writer.rs:591-695).  A batch handle must therefore
  keep its own output shares and verdicts however many other batches were prepared since
  (ADVICE r1, high).
* Concurrent jobs of engines with the same VDAF instance -- different tasks, different verify
  keys -- are merged into one launch by the executor (per-report verify-key slots); every job
  must still get exactly its own bytes back.
Expected values come from the CPU restatement (oracle/), Janus job structure.
"""
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from tests.conftest import CONFIGS
from tests.test_gpu_parity import _tamper

pytestmark = pytest.mark.gpu


def _engine(cfg, vk):
    from janus_amd import prio3 as J
    k = cfg["kind"]
    v = {"count": lambda: J.Prio3Count(), "sum": lambda: J.Prio3Sum(cfg["bits"]),
         "sumvec": lambda: J.Prio3SumVec(cfg["bits"], cfg["length"], cfg["chunk_length"]),
         "histogram": lambda: J.Prio3Histogram(cfg["length"], cfg["chunk_length"])}[k]()
    return J.HelperEngine(v, vk, device=0)


def _ref(o, vk, d, seg=None, accept=None, n_segments=1):
    return o.helper_batch(vk, d["nonces"], d["public_shares"], d["helper_shares"],
                          d["leader_prep_shares"], segment_ids=seg, accept_mask=accept,
                          n_segments=n_segments, n_threads=4)


def test_interleaved_batches_keep_their_own_outputs():
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_256_c16"]
    vk = bytes(range(0x10, 0x20))
    o = Oracle(**cfg)
    eng = _engine(cfg, vk)
    rng = np.random.default_rng(5)
    dA = _tamper(o, o.gen_reports(vk, 300, seed=1, n_threads=4), rng)
    dB = o.gen_reports(vk, 517, seed=2, n_threads=4)
    mA, sA, bA = eng.prepare_batch(dA["nonces"], dA["public_shares"], dA["helper_shares"],
                                   dA["leader_prep_shares"])
    mB, sB, bB = eng.prepare_batch(dB["nonces"], dB["public_shares"], dB["helper_shares"],
                                   dB["leader_prep_shares"])
    # a leader batch on the same engine in between as well (the device client derives report i
    # from (seed, i) exactly as the oracle's generator, so these are dB's leader input shares)
    gB = eng.generate_reports_device(517, seed=2, with_leader_inputs=True)
    ps, lst, lb = eng.leader_prepare_init_batch(dB["nonces"], dB["public_shares"],
                                                gB["leader_input_shares"].cpu().numpy())
    segA = rng.integers(0, 3, 300).astype(np.uint32)
    accA = (rng.random(300) < 0.9).astype(np.uint8)
    rm, rs, ra, rc = _ref(o, vk, dA, segA, accA, 3)
    np.testing.assert_array_equal(sA, rs)
    np.testing.assert_array_equal(mA, rm)
    agg, cnt = bA.accumulate(segA, accA, 3)
    np.testing.assert_array_equal(agg, ra)
    np.testing.assert_array_equal(cnt, rc)
    rm, rs, ra, rc = _ref(o, vk, dB)
    agg, cnt = bB.accumulate()
    np.testing.assert_array_equal(agg, ra)
    assert int(cnt[0]) == 517
    np.testing.assert_array_equal(ps, dB["leader_prep_shares"])
    # output shares of A are still A's
    outs = bA.output_shares()
    assert outs.shape == (300, 4096)
    fin = np.flatnonzero(sA == 0)
    from oracle.oracle import sum_mod, decode_elems, field_modulus
    p = field_modulus("histogram")
    tot = sum_mod(outs[fin], 16, p)
    ref_tot = decode_elems(_ref(o, vk, dA)[2][0], 16)
    assert tot == ref_tot
    for b in (bA, bB, lb):
        b.free()


class _Held:
    """Holds the executors of `eng` (prio3_executor_control "hold") until `n` jobs have entered
    them, then releases them: the jobs are queued before the launcher can take any, so whether
    they are coalesced no longer depends on thread timing.  Always released on exit
    -- the executors are process-wide."""

    def __init__(self, eng, n, kind=0):
        self.eng, self.n, self.kind = eng, n, kind

    def _entered(self):
        return sum(self.eng.executor_stats(self.kind, i)["jobs"]
                   for i in range(len(self.eng.members())))

    def __enter__(self):
        self.base = self._entered()
        self.eng.executor_control("hold", 1, self.kind)
        return self

    def wait(self, timeout=60.0):
        import time
        t0 = time.monotonic()
        while self._entered() - self.base < self.n:
            if time.monotonic() - t0 > timeout:
                raise AssertionError(f"only {self._entered() - self.base} of {self.n} jobs queued")
            time.sleep(0.005)
        time.sleep(0.05)  # their staging copies (the launcher waits for writers anyway)
        self.eng.executor_control("hold", 0, self.kind)

    def __exit__(self, *exc):
        self.eng.executor_control("hold", 0, self.kind)


@pytest.mark.parametrize("name", ["hist_256_c16", "sumvec_8x10_c9", "count", "sum32"])
def test_concurrent_jobs_of_several_tasks_are_coalesced(name):
    """24 jobs of 100-500 reports for 4 tasks (verify keys) of one VDAF instance, queued behind
    the executor's hold from 24 threads and then released: every job's prepare messages,
    statuses and aggregate equal the restatement's, and the executor merged them into fewer
    launches than jobs (one group holds them all)."""
    from oracle.oracle import Oracle
    cfg = CONFIGS[name]
    o = Oracle(**cfg)
    vks = [bytes([k]) * 16 for k in (0x31, 0x32, 0x33, 0x34)]
    engines = [_engine(cfg, vk) for vk in vks]
    for e in engines:
        e.set_option("timing", 1)
        e.timing_reset()
    rng = np.random.default_rng(9)
    jobs = []
    for j in range(24):
        t = j % 4
        n = int(rng.integers(100, 501))
        d = o.gen_reports(vks[t], n, seed=100 + j, n_threads=4)
        if j % 3 == 0:
            d = _tamper(o, d, rng)
        jobs.append((t, d))

    def run(j):
        t, d = jobs[j]
        msgs, status, batch = engines[t].prepare_batch(d["nonces"], d["public_shares"],
                                                       d["helper_shares"],
                                                       d["leader_prep_shares"])
        agg, cnt = batch.accumulate()
        batch.free()
        return msgs, status, agg, cnt

    with _Held(engines[0], 24) as held, ThreadPoolExecutor(24) as ex:
        futs = [ex.submit(run, j) for j in range(24)]
        held.wait()
        got = [f.result(timeout=120) for f in futs]
    for (t, d), (msgs, status, agg, cnt) in zip(jobs, got):
        rm, rs, ra, rc = _ref(o, vks[t], d)
        np.testing.assert_array_equal(status, rs)
        np.testing.assert_array_equal(msgs, rm)
        np.testing.assert_array_equal(agg, ra)
        np.testing.assert_array_equal(cnt, rc)
    # the prepare launch of each instance (one kernel per group: the fused XOF + query, or the
    # XOF of the two-kernel chains)
    kern = {"count": ("k_prep_gen",), "hist_256_c16": ("k_prep_h", "k_prep_hp"),
            "sum32": ("k_prep_sum",)}.get(name, ("k_xofd",))
    launches = sum(e.timing().get(k, (0, 0))[1] for e in engines for k in kern)
    assert 0 < launches < 24, launches


@pytest.mark.parametrize("name", ["hist_256_c16", "hist_100_c10", "sumvec_8x10_c9", "count",
                                  "sum32", "hist_256_c16/one_lane", "hist_256_c16/heavy",
                                  "count/heavy", "sumvec_8x10_c9/heavy", "hist_100_c10/heavy"])
def test_combined_prepare_aggregate_jobs(name):
    """prio3_helper_prepare_aggregate_batch from 32 threads: 32 jobs of 100-500 reports for 4
    tasks, each with its own segments (1-4, ids past n_segments included) and accept mask, some
    tampered, and every fourth job a plain prepare_batch + accumulate in the same groups.  Each
    job's messages, statuses, per-segment aggregates and counts equal the restatement's.
    Default: the jobs are queued behind the executor's hold, so the groups mix them into fewer
    launches than jobs.  /heavy: no hold, and the executor's heavy-load launcher from the first
    job (prio3_executor_control "heavy" 1) -- its sleep predictor and its issue of the next group
    behind the running one's prepare kernels, the path the 128-thread load runs on.
    /one_lane runs the groups on the one-lane k_prep_h."""
    from oracle.oracle import Oracle
    name, _, variant = name.partition("/")
    cfg = CONFIGS[name]
    o = Oracle(**cfg)
    vks = [bytes([k]) * 16 for k in (0x41, 0x42, 0x43, 0x44)]
    engines = [_engine(cfg, vk) for vk in vks]
    for e in engines:
        e.set_option("timing", 1)
        if variant == "one_lane":  # groups on the one-lane k_prep_h, not k_prep_hp
            e.set_option("pair_max", 0)
        e.timing_reset()
    rng = np.random.default_rng(19)
    jobs = []
    for j in range(32):
        t = j % 4
        n = int(rng.integers(100, 501))
        d = o.gen_reports(vks[t], n, seed=300 + j, n_threads=4)
        if j % 3 == 1:
            d = _tamper(o, d, rng)
        S = int(rng.integers(1, 5))
        seg = rng.integers(0, S + 1, n).astype(np.uint32)  # id S: out of range, excluded
        acc = (rng.random(n) < 0.9).astype(np.uint8)
        jobs.append((t, d, S, seg, acc))

    def run(j):
        t, d, S, seg, acc = jobs[j]
        args = (d["nonces"], d["public_shares"], d["helper_shares"], d["leader_prep_shares"])
        if j % 4 == 3:
            msgs, status, batch = engines[t].prepare_batch(*args)
            agg, cnt = batch.accumulate(seg, acc, S)
            batch.free()
            return msgs, status, agg, cnt
        return engines[t].prepare_aggregate_batch(*args, segment_ids=seg, accept_mask=acc,
                                                  n_segments=S)

    if variant == "heavy":
        engines[0].executor_control("heavy", 1)
        try:
            start = threading.Barrier(8)

            def run8(j):
                if j < 8:
                    start.wait()
                return run(j)

            with ThreadPoolExecutor(8) as ex:
                got = list(ex.map(run8, range(32)))
        finally:
            engines[0].executor_control("heavy", 0)
    else:
        with _Held(engines[0], 32) as held, ThreadPoolExecutor(32) as ex:
            futs = [ex.submit(run, j) for j in range(32)]
            held.wait()
            got = [f.result(timeout=120) for f in futs]
    for (t, d, S, seg, acc), (msgs, status, agg, cnt) in zip(jobs, got):
        ref_seg = np.where(seg < S, seg, 0).astype(np.uint32)
        ref_acc = np.where(seg < S, acc, 0).astype(np.uint8)
        rm, rs, ra, rc = _ref(o, vks[t], d, ref_seg, ref_acc, S)
        np.testing.assert_array_equal(status, rs)
        np.testing.assert_array_equal(msgs, rm)
        np.testing.assert_array_equal(agg, ra)
        np.testing.assert_array_equal(cnt, rc)
    kern = {"count": ("k_prep_gen",), "hist_256_c16": ("k_prep_h", "k_prep_hp"),
            "sum32": ("k_prep_sum",), "hist_100_c10": ("k_xofd", "k_prep_h")}.get(name, ("k_xofd",))
    launches = sum(e.timing().get(k, (0, 0))[1] for e in engines for k in kern)
    if variant == "heavy":
        assert 0 < launches <= 32, launches
    else:
        assert 0 < launches < 32, launches


def test_heavy_load_group_takes_at_most_half_the_jobs():
    """Under heavy load a group takes at most about half the jobs inside the executor
    (Exec::cohort_full), so the two cohorts of a closed loop of callers stay balanced (DESIGN.md
    11: 41 / 87 jobs of the 128-thread line ran at 33.5 M reports/s, 58 / 68 at 37.6).  32 jobs
    queued behind the hold with the heavy-load launcher on from the first job land in at least two
    groups -- one group would hold them all without the cap -- and every job matches the
    restatement."""
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_256_c16"]
    o = Oracle(**cfg)
    vk = bytes([0x4d]) * 16
    eng = _engine(cfg, vk)
    eng.set_option("timing", 1)
    eng.timing_reset()
    jobs = [o.gen_reports(vk, 200, seed=700 + j, n_threads=4) for j in range(32)]

    def run(j):
        d = jobs[j]
        return eng.prepare_aggregate_batch(d["nonces"], d["public_shares"], d["helper_shares"],
                                           d["leader_prep_shares"])

    eng.executor_control("heavy", 1)
    try:
        with _Held(eng, 32) as held, ThreadPoolExecutor(32) as ex:
            futs = [ex.submit(run, j) for j in range(32)]
            held.wait()
            got = [f.result(timeout=120) for f in futs]
    finally:
        eng.executor_control("heavy", 0)
    for d, (msgs, status, agg, cnt) in zip(jobs, got):
        rm, rs, ra, rc = _ref(o, vk, d)
        np.testing.assert_array_equal(status, rs)
        np.testing.assert_array_equal(msgs, rm)
        np.testing.assert_array_equal(agg, ra)
        np.testing.assert_array_equal(cnt, rc)
    launches = sum(eng.timing().get(k, (0, 0))[1] for k in ("k_prep_h", "k_prep_hp"))
    assert 2 <= launches < 32, launches


def test_jobs_after_a_subprocess_still_match():
    """The executor's pinned staging (2 MB pages registered with the GPU, MADV_DONTFORK) is not
    shared copy-on-write with a child process: jobs before and after a subprocess started by
    this process, on the same pooled staging, all match the restatement."""
    import subprocess
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_256_c16"]
    o = Oracle(**cfg)
    vk = bytes([0x5a]) * 16
    eng = _engine(cfg, vk)
    for rnd in range(3):
        d = o.gen_reports(vk, 300, seed=900 + rnd, n_threads=4)
        with ThreadPoolExecutor(4) as ex:
            got = list(ex.map(lambda _: eng.prepare_aggregate_batch(
                d["nonces"], d["public_shares"], d["helper_shares"], d["leader_prep_shares"]),
                range(4)))
        rm, rs, ra, rc = _ref(o, vk, d)
        for msgs, status, agg, cnt in got:
            np.testing.assert_array_equal(status, rs)
            np.testing.assert_array_equal(msgs, rm)
            np.testing.assert_array_equal(agg, ra)
            np.testing.assert_array_equal(cnt, rc)
        subprocess.run(["true"], check=True)


def test_combined_prepare_aggregate_single_job_and_empty():
    """One combined call alone (the executor launches a lone job at once), with coalescing off
    (the two-call fallback), and an empty job."""
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_256_c16"]
    vk = bytes(range(0x50, 0x60))
    o = Oracle(**cfg)
    eng = _engine(cfg, vk)
    d = _tamper(o, o.gen_reports(vk, 777, seed=8, n_threads=4), np.random.default_rng(8))
    seg = (np.arange(777) % 3).astype(np.uint32)
    rm, rs, ra, rc = _ref(o, vk, d, seg, None, 3)
    for coalesce in (1, 0):
        eng.set_option("coalesce", coalesce)
        msgs, status, agg, cnt = eng.prepare_aggregate_batch(
            d["nonces"], d["public_shares"], d["helper_shares"], d["leader_prep_shares"],
            segment_ids=seg, n_segments=3)
        np.testing.assert_array_equal(status, rs)
        np.testing.assert_array_equal(msgs, rm)
        np.testing.assert_array_equal(agg, ra)
        np.testing.assert_array_equal(cnt, rc)
    z = lambda k: np.zeros((0, k), np.uint8)
    sz = eng.sz
    msgs, status, agg, cnt = eng.prepare_aggregate_batch(
        z(16), z(sz.public_share_len), z(sz.helper_share_len), z(sz.prep_share_len), n_segments=2)
    assert status.shape == (0,) and cnt.tolist() == [0, 0] and not agg.any()


def test_coalescing_off_matches():
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_10_c3"]
    vk = bytes(range(16))
    o = Oracle(**cfg)
    eng = _engine(cfg, vk)
    eng.set_option("coalesce", 0)
    d = o.gen_reports(vk, 333, seed=4, n_threads=4)
    msgs, status, batch = eng.prepare_batch(d["nonces"], d["public_shares"], d["helper_shares"],
                                            d["leader_prep_shares"])
    rm, rs, ra, rc = _ref(o, vk, d)
    np.testing.assert_array_equal(msgs, rm)
    agg, cnt = batch.accumulate()
    np.testing.assert_array_equal(agg, ra)


def test_roctx_ranges_on_request(tmp_path):
    """JANUS_ROCTX=1: the library loads roctx and wraps its entry points in ranges named after
    Janus's spans; a prepare + accumulate still gives the oracle's bytes (child process: the
    switch is read once per process)."""
    import subprocess
    import sys
    code = (
        "import numpy as np\n"
        "from janus_amd import prio3 as J\n"
        "from oracle.oracle import Oracle\n"
        "assert J.load_library().prio3_trace_enabled() == 1\n"
        "VK = bytes(range(16))\n"
        "o = Oracle('histogram', length=256, chunk_length=16)\n"
        "d = o.gen_reports(VK, 300, seed=3, n_threads=4)\n"
        "m, s, a, c = o.helper_batch(VK, d['nonces'], d['public_shares'], d['helper_shares'],\n"
        "                            d['leader_prep_shares'], n_threads=4)\n"
        "e = J.HelperEngine(J.Prio3Histogram(256, 16), VK)\n"
        "gm, gs, b = e.prepare_batch(d['nonces'], d['public_shares'], d['helper_shares'],\n"
        "                            d['leader_prep_shares'])\n"
        "ga, gc = b.accumulate()\n"
        "assert (gm == m).all() and (gs == s).all() and (ga == a).all()\n"
        "print('ok')\n")
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                       env=dict(os.environ, JANUS_ROCTX="1", PYTHONPATH=root), timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_engine_over_two_executors_places_jobs_and_matches():
    """VERDICT r4 item 1 on the one-GPU box: an engine over the device list [0, 0] has two
    executors (lanes 0 and 1 of GPU 0) standing in for two GPUs of a node.  Jobs submitted one
    at a time (equal load) alternate between them; concurrent jobs from 16 threads spread over
    both by load; every job -- prepare_aggregate, prepare + accumulate, leader prepare_init +
    prepare_next -- equals the restatement's bytes, whichever member ran it."""
    from janus_amd import prio3 as J
    from oracle.oracle import Oracle
    cfg = CONFIGS["hist_256_c16"]
    vk = bytes(range(0x60, 0x70))
    o = Oracle(**cfg)
    eng = J.HelperEngine(J.Prio3Histogram(256, 16), vk, devices=[0, 0])
    m0 = eng.members()
    assert [(m["device"], m["lane"]) for m in m0] == [(0, 0), (0, 1)]
    rng = np.random.default_rng(23)
    # sequential: equal load every time, so the members alternate
    for j in range(6):
        d = o.gen_reports(vk, 200 + j, seed=700 + j, n_threads=4)
        msgs, status, agg, cnt = eng.prepare_aggregate_batch(
            d["nonces"], d["public_shares"], d["helper_shares"], d["leader_prep_shares"])
        rm, rs, ra, rc = _ref(o, vk, d)
        np.testing.assert_array_equal(status, rs)
        np.testing.assert_array_equal(msgs, rm)
        np.testing.assert_array_equal(agg, ra)
    m1 = eng.members()
    assert [m["jobs"] - a["jobs"] for m, a in zip(m1, m0)] == [3, 3], m1
    assert all(m["exec_groups"] > a["exec_groups"] for m, a in zip(m1, m0)), m1
    # concurrent: 32 jobs from 16 threads, mixed entry points, every job checked
    jobs = []
    for j in range(32):
        n = int(rng.integers(100, 501))
        d = o.gen_reports(vk, n, seed=800 + j, n_threads=4)
        if j % 3 == 0:
            d = _tamper(o, d, rng)
        S = int(rng.integers(1, 4))
        seg = rng.integers(0, S, n).astype(np.uint32)
        jobs.append((d, S, seg))

    def run(j):
        d, S, seg = jobs[j]
        args = (d["nonces"], d["public_shares"], d["helper_shares"], d["leader_prep_shares"])
        if j % 2:
            msgs, status, b = eng.prepare_batch(*args)
            agg, cnt = b.accumulate(seg, None, S)
            b.free()
            return msgs, status, agg, cnt
        return eng.prepare_aggregate_batch(*args, segment_ids=seg, n_segments=S)

    with ThreadPoolExecutor(16) as ex:
        got = list(ex.map(run, range(32)))
    for (d, S, seg), (msgs, status, agg, cnt) in zip(jobs, got):
        rm, rs, ra, rc = _ref(o, vk, d, seg, None, S)
        np.testing.assert_array_equal(status, rs)
        np.testing.assert_array_equal(msgs, rm)
        np.testing.assert_array_equal(agg, ra)
        np.testing.assert_array_equal(cnt, rc)
    m2 = eng.members()
    placed = [m["jobs"] - a["jobs"] for m, a in zip(m2, m1)]
    assert sum(placed) == 32 and min(placed) > 0, placed
    # the leader role on the same engine: the batch handle stays with the member that ran it
    gen = eng.generate_reports_device(300, seed=31, with_leader_inputs=True)
    d = o.gen_reports(vk, 300, seed=31, n_threads=4)
    for _ in range(2):
        ps, lst, lb = eng.leader_prepare_init_batch(d["nonces"], d["public_shares"],
                                                    gen["leader_input_shares"].cpu().numpy())
        np.testing.assert_array_equal(ps, d["leader_prep_shares"])
        rm, rs, ra, rc = _ref(o, vk, d)
        st = lb.leader_prepare_next(rm, lst)
        assert (st == 0).all()
        lagg, lcnt = lb.accumulate()
        assert int(lcnt[0]) == 300
        lb.free()
    eng.close()


@pytest.mark.parametrize("name", ["hist_256_c16", "sum32", "count", "sumvec_8x10_c9"])
def test_concurrent_leader_jobs_are_coalesced(name):
    """the leader's prepare_init (leader_initialized,
    aggregation_job_driver.rs:397-415) and prepare_next (leader_continued, :677-691) of 24
    concurrent 100-500-report jobs of 4 tasks, each queued behind its executor's hold: one
    prepare_init launch and one prepare_next launch serve them all, and every job's prepare
    shares, statuses (one tampered prepare message per third job) and aggregate equal the
    restatement's leader path (orc_leader_batch)."""
    from janus_amd import prio3 as J
    from oracle.oracle import Oracle
    cfg = CONFIGS[name]
    o = Oracle(**cfg)
    vks = [bytes([k]) * 16 for k in (0x71, 0x72, 0x73, 0x74)]
    engines = [_engine(cfg, vk) for vk in vks]
    rng = np.random.default_rng(41)
    jobs = []
    for j in range(24):
        t = j % 4
        n = int(rng.integers(100, 501))
        d = o.gen_reports(vks[t], n, seed=900 + j, n_threads=4)
        lin = engines[t].generate_reports_device(n, seed=900 + j, with_leader_inputs=True)
        lin = lin["leader_input_shares"].cpu().numpy()
        msgs = _ref(o, vks[t], d)[0].copy()
        if j % 3 == 0 and msgs.shape[1]:
            msgs[int(rng.integers(0, n)), 0] ^= 1  # the leader's prepare_next rejects it
        jobs.append((t, d, lin, msgs))
    g0 = [engines[0].executor_stats(k)["groups"] for k in (J.EXEC_LEADER_INIT, J.EXEC_LEADER_NEXT)]
    barrier = threading.Barrier(24)

    def run(j):
        t, d, lin, msgs = jobs[j]
        ps, st, b = engines[t].leader_prepare_init_batch(d["nonces"], d["public_shares"], lin)
        barrier.wait()  # every prepare_init is back before the first prepare_next is queued
        st2 = b.leader_prepare_next(msgs, st)
        agg, cnt = b.accumulate()
        b.free()
        return ps, st, st2, agg, cnt

    with ThreadPoolExecutor(24) as ex, _Held(engines[0], 24, J.EXEC_LEADER_NEXT) as held_next:
        with _Held(engines[0], 24, J.EXEC_LEADER_INIT) as held_init:
            futs = [ex.submit(run, j) for j in range(24)]
            held_init.wait()
        held_next.wait()
        got = [f.result(timeout=120) for f in futs]
    for (t, d, lin, msgs), (ps, st, st2, agg, cnt) in zip(jobs, got):
        rps, rst, ragg, rcnt = o.leader_batch(vks[t], d["nonces"], d["public_shares"], lin, msgs,
                                              n_threads=4)
        np.testing.assert_array_equal(ps, rps)
        np.testing.assert_array_equal(ps, d["leader_prep_shares"])
        assert (st == 0).all()
        np.testing.assert_array_equal(st2, rst)
        np.testing.assert_array_equal(agg, ragg)
        np.testing.assert_array_equal(cnt, rcnt)
    g1 = [engines[0].executor_stats(k)["groups"] for k in (J.EXEC_LEADER_INIT, J.EXEC_LEADER_NEXT)]
    assert [b - a for a, b in zip(g0, g1)] == [1, 1], (g0, g1)


@pytest.mark.parametrize("name", ["hist_256_c16", "sum32", "sumvec_8x10_c9"])
def test_leader_next_uncoalesced_on_shared_runs(name):
    """leader batches of one coalesced prepare_init group start at non-zero columns c0
    of a shared run; with coalescing switched off before prepare_next, each batch takes the
    direct prepare_next path (the SoA offsets es * c0 with stride ld into the measurement and
    output shares) and then the accumulate with segments and a mask -- every job equal to the
    restatement's leader path."""
    from oracle.oracle import Oracle
    cfg = CONFIGS[name]
    o = Oracle(**cfg)
    vks = [bytes([k]) * 16 for k in (0x61, 0x62)]
    engines = [_engine(cfg, vk) for vk in vks]
    rng = np.random.default_rng(53)
    jobs = []
    for j in range(8):
        t = j % 2
        n = int(rng.integers(60, 300))
        d = o.gen_reports(vks[t], n, seed=700 + j, n_threads=4)
        lin = engines[t].generate_reports_device(n, seed=700 + j, with_leader_inputs=True)
        lin = lin["leader_input_shares"].cpu().numpy()
        msgs = _ref(o, vks[t], d)[0].copy()
        if msgs.shape[1]:
            msgs[int(rng.integers(0, n)), 0] ^= 1
        seg = rng.integers(0, 3, n).astype(np.uint32)
        acc = (rng.random(n) < 0.85).astype(np.uint8)
        jobs.append((t, d, lin, msgs, seg, acc))
    from janus_amd import prio3 as J
    g0 = engines[0].executor_stats(J.EXEC_LEADER_INIT)["groups"]
    with ThreadPoolExecutor(8) as ex, _Held(engines[0], 8, J.EXEC_LEADER_INIT) as held:
        futs = [ex.submit(engines[t].leader_prepare_init_batch, d["nonces"], d["public_shares"],
                          lin) for (t, d, lin, _, _, _) in jobs]
        held.wait()
        inits = [f.result(timeout=120) for f in futs]
    assert engines[0].executor_stats(J.EXEC_LEADER_INIT)["groups"] - g0 == 1  # one shared run
    for e in engines:
        e.set_option("coalesce", 0)
    for (t, d, lin, msgs, seg, acc), (ps, st, b) in zip(jobs, inits):
        st2 = b.leader_prepare_next(msgs, st)
        agg, cnt = b.accumulate(seg, acc, 3)
        b.free()
        rps, rst, _, _ = o.leader_batch(vks[t], d["nonces"], d["public_shares"], lin, msgs,
                                        n_threads=4)
        np.testing.assert_array_equal(ps, rps)
        np.testing.assert_array_equal(st2, rst)
        _, _, ragg, rcnt = o.leader_batch(vks[t], d["nonces"], d["public_shares"], lin, msgs,
                                          n_threads=4, segment_ids=np.where(acc, seg, 3),
                                          n_segments=3)
        np.testing.assert_array_equal(agg, ragg)
        np.testing.assert_array_equal(cnt, rcnt)


@pytest.mark.parametrize("name", ["hist_256_c16", "sumvec_8x10_c9", "sum32", "count"])
def test_concurrent_leader_next_aggregate_jobs(name):
    """prio3_leader_prepare_next_aggregate_batch: 16 jobs of 4 tasks queued behind the prepare_next
    executor's hold share ONE launch that checks every job's prepare messages (a tampered message
    per third job) and sums its kept output shares per segment under a mask; statuses,
    aggregates and counts equal the restatement's leader path, and the batches can still be
    accumulated again afterwards (the same aggregates)."""
    from janus_amd import prio3 as J
    from oracle.oracle import Oracle
    cfg = CONFIGS[name]
    o = Oracle(**cfg)
    vks = [bytes([k]) * 16 for k in (0x91, 0x92, 0x93, 0x94)]
    engines = [_engine(cfg, vk) for vk in vks]
    rng = np.random.default_rng(59)
    jobs = []
    for j in range(16):
        t = j % 4
        n = int(rng.integers(80, 400))
        d = o.gen_reports(vks[t], n, seed=1300 + j, n_threads=4)
        lin = engines[t].generate_reports_device(n, seed=1300 + j, with_leader_inputs=True)
        lin = lin["leader_input_shares"].cpu().numpy()
        msgs = _ref(o, vks[t], d)[0].copy()
        if j % 3 == 0 and msgs.shape[1]:
            msgs[int(rng.integers(0, n)), 0] ^= 1
        seg = rng.integers(0, 3, n).astype(np.uint32)
        acc = (rng.random(n) < 0.9).astype(np.uint8)
        jobs.append((t, d, lin, msgs, seg, acc))
    inits = [engines[t].leader_prepare_init_batch(d["nonces"], d["public_shares"], lin)
             for (t, d, lin, _, _, _) in jobs]
    g0 = engines[0].executor_stats(J.EXEC_LEADER_NEXT)["groups"]
    with ThreadPoolExecutor(16) as ex, _Held(engines[0], 16, J.EXEC_LEADER_NEXT) as held:
        futs = [ex.submit(b.leader_prepare_next_aggregate, msgs, st, seg, acc, 3)
                for (_, _, _, msgs, seg, acc), (_, st, b) in zip(jobs, inits)]
        held.wait()
        got = [f.result(timeout=120) for f in futs]
    assert engines[0].executor_stats(J.EXEC_LEADER_NEXT)["groups"] - g0 == 1
    for (t, d, lin, msgs, seg, acc), (ps, st, b), (st2, agg, cnt) in zip(jobs, inits, got):
        _, rst, ragg, rcnt = o.leader_batch(vks[t], d["nonces"], d["public_shares"], lin, msgs,
                                            n_threads=4, segment_ids=np.where(acc, seg, 3),
                                            n_segments=3)
        np.testing.assert_array_equal(st2, rst)
        np.testing.assert_array_equal(agg, ragg)
        np.testing.assert_array_equal(cnt, rcnt)
        agg2, cnt2 = b.accumulate(seg, acc, 3)
        np.testing.assert_array_equal(agg2, ragg)
        np.testing.assert_array_equal(cnt2, rcnt)
        b.free()
