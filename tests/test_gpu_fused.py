"""GPU parity of the one-pass prepare + aggregate entry points
(prio3_device_prepare_aggregate / prio3_device_aggregate_finish) against the CPU restatement.

The Histogram path sums the output shares inside the joint-randomness kernel, one wave of 64
reports at a time, and then fixes up every report it must not have counted (decide failures,
host-rejected reports, flagged slow-path reports) and every report it could not fuse (waves
spanning two segments, the ragged last wave).  These cases are exercised here; the expected
aggregate is the oracle's Janus-structured batch aggregate (aggregation_job_writer.rs:591-695).
"""
import numpy as np
import pytest

from tests.conftest import CONFIGS
from tests.test_gpu_parity import VK, _engine, _oracle, _tamper

pytestmark = pytest.mark.gpu


def _run(cfg, n, seed, n_segments=1, seg_mode="runs", tamper=True, accept_frac=0.9,
         force_slow=False, fuse=True, chunks=None, oob_frac=0.0, opts=None, oob_waves=()):
    import torch
    o = _oracle(cfg)
    eng = _engine(cfg)
    eng.set_option("fuse_acc", int(fuse))
    if force_slow:
        eng.set_option("force_slow_path", 1)
    if chunks is not None:
        eng.set_option("chunks", chunks)
    for k, v in (opts or {}).items():
        eng.set_option(k, v)
    d = o.gen_reports(VK, n, seed=seed, n_threads=8)
    rng = np.random.default_rng(seed)
    if tamper:
        d = _tamper(o, d, rng)
    if seg_mode == "runs":  # contiguous batches whose boundaries fall inside waves
        cuts = np.sort(rng.choice(np.arange(1, n), n_segments - 1, replace=False)) if n_segments > 1 else []
        seg = np.zeros(n, np.uint32)
        for c in cuts:
            seg[c:] += 1
    else:
        seg = rng.integers(0, n_segments, n).astype(np.uint32)
    accept = (rng.random(n) < accept_frac).astype(np.uint8)
    # segment ids >= n_segments: the report is excluded from every aggregate and count, as if
    # its accept-mask byte were 0 (include/janus_prio3.h); the oracle sees exactly that
    oob = rng.random(n) < oob_frac
    for w in oob_waves:  # every report of these waves out of range (no lane left to fuse)
        oob[64 * w:64 * w + 64] = True
    dev_seg = np.where(oob, n_segments + 5 + (np.arange(n) % 3), seg).astype(np.uint32)
    ref_seg = np.where(oob, 0, seg).astype(np.uint32)
    ref_accept = np.where(oob, 0, accept).astype(np.uint8)
    ref_msgs, ref_status, ref_agg, ref_cnt = o.helper_batch(
        VK, d["nonces"], d["public_shares"], d["helper_shares"], d["leader_prep_shares"],
        segment_ids=ref_seg, accept_mask=ref_accept, n_segments=n_segments, n_threads=8)
    seg = dev_seg
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    sz = eng.sz
    msgs = torch.zeros((n, max(sz.prep_msg_len, 1)), dtype=torch.uint8, device=dev)
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    agg = torch.zeros((n_segments, sz.agg_share_len), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(n_segments, dtype=torch.int64, device=dev)
    pub = t(d["public_shares"]) if sz.public_share_len else None
    eng.prepare_aggregate_device(t(d["nonces"]), pub, t(d["helper_shares"]),
                                 t(d["leader_prep_shares"]), t(seg), n_segments, msgs, status)
    eng.aggregate_finish_device(status, t(accept), agg, cnt)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(status.cpu().numpy(), ref_status)
    np.testing.assert_array_equal(msgs.cpu().numpy()[:, :sz.prep_msg_len], ref_msgs)
    np.testing.assert_array_equal(cnt.cpu().numpy().astype(np.uint64), ref_cnt)
    np.testing.assert_array_equal(agg.cpu().numpy(), ref_agg)
    return ref_status


def test_fused_single_segment_all_accepted():
    _run(CONFIGS["hist_256_c16"], 1024, seed=1, tamper=False, accept_frac=1.0)


def test_fused_tampered_and_masked():
    st = _run(CONFIGS["hist_256_c16"], 1000, seed=2)
    assert (st != 0).any()


def test_fused_segment_runs_inside_waves():
    _run(CONFIGS["hist_256_c16"], 1500, seed=3, n_segments=7, seg_mode="runs")


def test_fused_random_segments():
    """Every wave spans several segments: nothing fuses, all goes through the fix-up pass."""
    _run(CONFIGS["hist_256_c16"], 600, seed=4, n_segments=4, seg_mode="random")


def test_fused_ragged_tail_and_small_histogram():
    _run(CONFIGS["hist_10_c3"], 200, seed=5, n_segments=2)
    _run(CONFIGS["hist_100_c10"], 131, seed=6)


@pytest.mark.parametrize("chunks", [None, 2])
def test_fused_slow_path_flags(chunks):
    """Every report flagged: the query skips flagged reports and the run ends with one deferred
    redo launch (k_slow_redo: the byte-level XOF, then the query); with 2 chunks both side
    streams carry flags."""
    _run(CONFIGS["hist_256_c16"], 192 if chunks is None else 700, seed=7 + (chunks or 0),
         force_slow=True, chunks=chunks)


@pytest.mark.parametrize("name", ["count", "sum8", "sumvec_8x10_c9"])
def test_prepare_aggregate_other_instances(name):
    """Instances without the fused kernel take the deferred masked reduction."""
    _run(CONFIGS[name], 700, seed=8, n_segments=3)


def test_fused_off_matches():
    _run(CONFIGS["hist_256_c16"], 700, seed=9, n_segments=2, fuse=False)


@pytest.mark.parametrize("case", ["runs", "random", "slow", "chunks", "tampered_masked"])
def test_fused_accumulate_fixups(case):
    """Every fix-up path of the fused aggregate (wave partials taken in the XOF, k_agg_fix /
    k_agg_final): segment runs inside waves, random segments (no wave fuses), the slow path,
    stream-overlapped chunks with out-of-range segment ids, tampered and host-masked reports."""
    cfg = CONFIGS["hist_256_c16"]
    if case == "runs":
        _run(cfg, 1500, seed=81, n_segments=7, seg_mode="runs")
    elif case == "random":
        _run(cfg, 600, seed=82, n_segments=4, seg_mode="random")
    elif case == "slow":
        _run(cfg, 192, seed=83, force_slow=True)
    elif case == "chunks":
        _run(cfg, 1500, seed=84, n_segments=5, chunks=3, oob_frac=0.02)
    else:
        st = _run(cfg, 1000, seed=85, accept_frac=0.8)
        assert (st != 0).any()


@pytest.mark.parametrize("chunks", [2, 3, 5])
def test_fused_stream_overlapped_chunks(chunks):
    """The batch cut into column chunks on two side streams (the engine's default above 192Ki
    reports): chunk boundaries fall inside segments and the wave partials stay aligned."""
    _run(CONFIGS["hist_256_c16"], 1500, seed=10 + chunks, n_segments=5, chunks=chunks)


def test_chunks_unfused_instance():
    _run(CONFIGS["sumvec_8x10_c9"], 1100, seed=20, n_segments=2, chunks=3)


@pytest.mark.parametrize("name,fuse", [("hist_256_c16", True), ("hist_256_c16", False),
                                       ("sum8", True)])
def test_out_of_range_segment_ids_are_excluded(name, fuse):
    """a segment id >= n_segments never reaches the aggregate or the counts (fused
    Histogram path, its unfused fallback, and the deferred masked reduction alike)."""
    _run(CONFIGS[name], 900, seed=31, n_segments=3, oob_frac=0.05, fuse=fuse)


@pytest.mark.parametrize("n_segments,oob_frac", [(1, 0.3), (3, 0.1), (1, 0.9)])
def test_out_of_range_lanes_fuse_with_their_wave(n_segments, oob_frac):
    """Lanes with a segment id >= n_segments (the executor's pad columns, excluded reports) are
    masked out of the fused XOF's wave partials, so the wave's other reports still fuse; a wave
    with no in-range lane is not fused.  Tampered reports, the host mask and segment runs inside
    waves on top."""
    _run(CONFIGS["hist_256_c16"], 2048, seed=41 + n_segments, n_segments=n_segments,
         oob_frac=oob_frac, oob_waves=(3, 17))


@pytest.mark.parametrize("opts", [{}, {"chunks": 3}])
def test_fused_accumulate_on_fused_prepare_variants(opts):
    """The fused accumulate (wave partials in the XOF) under the fused XOF + query kernel, in one
    launch or three stream-overlapped chunks: segment runs inside waves, tampered reports, the
    host mask, every report on the deferred slow path."""
    _run(CONFIGS["hist_256_c16"], 3000, seed=91, n_segments=4, opts=opts)
    _run(CONFIGS["hist_256_c16"], 256, seed=92, force_slow=True, opts=opts)


@pytest.mark.parametrize("name", ["hist_100_c10", "hist_10_c3"])
def test_fused_segment_runs_partial_waves(name):
    """for M % 32 != 0 the last k_agg_waves wave has lanes past the slot
    range; with many segment runs per 32-wave chunk (the mixed path, as the executor's one
    segment per job) those lanes must stay alive through the readlane of the wave segments."""
    _run(CONFIGS[name], 4100, seed=51, n_segments=9, seg_mode="runs", accept_frac=0.95)
    _run(CONFIGS[name], 2600, seed=52, n_segments=5, seg_mode="runs", oob_frac=0.03)


@pytest.mark.parametrize("pair_max", [196608, 0])
@pytest.mark.parametrize("case", ["runs", "oob", "slow", "masked"])
def test_fused_accumulate_pair_and_one_lane(case, pair_max):
    """The fused accumulate on both Histogram(256, 16) kernels: the lane-pair k_prep_hp (32-report
    waves, wshift 5 in k_agg_fix) and the one-lane k_prep_h (64-report waves): segment runs inside
    waves, out-of-range lanes and whole out-of-range waves, the forced slow path, tampered and
    host-masked reports."""
    cfg = CONFIGS["hist_256_c16"]
    o = {"pair_max": pair_max}
    if case == "runs":
        _run(cfg, 2500, seed=61, n_segments=9, seg_mode="runs", opts=o)
    elif case == "oob":
        _run(cfg, 2048, seed=62, n_segments=3, oob_frac=0.2, oob_waves=(1, 6, 21), opts=o)
    elif case == "slow":
        _run(cfg, 200, seed=63, force_slow=True, n_segments=2, opts=o)
    else:
        st = _run(cfg, 1100, seed=64, accept_frac=0.7, opts=o)
        assert (st != 0).any()
