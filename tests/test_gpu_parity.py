"""GPU parity: the HIP engine (through the C-ABI) against the CPU restatement (oracle/).

Mirrors the reference's transcript pattern (core/src/test_util/mod.rs:86-232, used by
taskprov_tests.rs:1268-1369): every helper output -- prepare message, per-report status,
output share and aggregate share -- must equal the oracle's bit-for-bit.  Error paths use
tampered inputs, mirroring FakeFailsPrepInit/FakeFailsPrepStep (core/src/vdaf.rs:354-385).
"""
import numpy as np
import pytest

from tests.conftest import CONFIGS

pytestmark = pytest.mark.gpu

VK = bytes(range(0x40, 0x50))


def _engine(cfg):
    from janus_amd import prio3 as J
    kind = cfg["kind"]
    if kind == "count":
        v = J.Prio3Count()
    elif kind == "sum":
        v = J.Prio3Sum(cfg["bits"])
    elif kind == "sumvec":
        v = J.Prio3SumVec(cfg["bits"], cfg["length"], cfg["chunk_length"])
    else:
        v = J.Prio3Histogram(cfg["length"], cfg["chunk_length"])
    return J.HelperEngine(v, VK, device=0)


def _oracle(cfg):
    from oracle.oracle import Oracle
    return Oracle(**cfg)


def _tamper(o, d, rng):
    """Corrupt a few reports to hit each status code; returns the modified copy."""
    d = {k: v.copy() for k, v in d.items()}
    n = d["nonces"].shape[0]
    es = o.es
    # decide failure: flip a bit in the leader verifier share (element 1)
    for i in range(1, n, 17):
        d["leader_prep_shares"][i, es] ^= 0x01
    # decode failure: leader verifier element 0 set to 0xff.. (>= p)
    for i in range(3, n, 29):
        d["leader_prep_shares"][i, :es] = 0xFF
    if o.jr_len:
        # joint-rand mismatch: corrupt the leader's joint-rand part in its prep share
        for i in range(5, n, 23):
            d["leader_prep_shares"][i, -1] ^= 0x80
        # wrong public share (helper's corrected seed differs)
        for i in range(7, n, 31):
            d["public_shares"][i, 3] ^= 0x10
    # corrupt a helper seed (share no longer matches the proof)
    for i in range(11, n, 37):
        d["helper_shares"][i, 0] ^= 0x01
    return d


def _check_against_oracle(cfg, n, seed, tamper=True, force_slow=False, n_segments=1, opts=None):
    from oracle.oracle import decode_elems
    o = _oracle(cfg)
    eng = _engine(cfg)
    if force_slow:
        eng.set_option("force_slow_path", 1)
    for k, v in (opts or {}).items():
        eng.set_option(k, v)
    d = o.gen_reports(VK, n, seed=seed, n_threads=8)
    rng = np.random.default_rng(seed)
    if tamper:
        d = _tamper(o, d, rng)
    seg = rng.integers(0, n_segments, n).astype(np.uint32)
    accept = (rng.random(n) > 0.1).astype(np.uint8)
    ref_msgs, ref_status, ref_agg, ref_cnt = o.helper_batch(
        VK, d["nonces"], d["public_shares"], d["helper_shares"], d["leader_prep_shares"],
        segment_ids=seg, accept_mask=accept, n_segments=n_segments, n_threads=8)
    msgs, status, batch = eng.prepare_batch(d["nonces"], d["public_shares"], d["helper_shares"],
                                            d["leader_prep_shares"])
    np.testing.assert_array_equal(status, ref_status)
    np.testing.assert_array_equal(msgs, ref_msgs)
    agg, cnt = batch.accumulate(seg, accept, n_segments)
    np.testing.assert_array_equal(cnt, ref_cnt)
    np.testing.assert_array_equal(agg, ref_agg)
    if tamper:
        assert set(np.unique(status)) >= {0, 3}
    return o, d, status, batch


@pytest.mark.parametrize("name", list(CONFIGS))
def test_parity_vs_oracle(name):
    cfg = CONFIGS[name]
    n = 64 if "1000" in name else 700
    _check_against_oracle(cfg, n, seed=11)


@pytest.mark.parametrize("name", ["count", "sum8", "sumvec_8x10_c9", "hist_256_c16"])
def test_slow_path_parity(name):
    """The general rejection-sampling kernel must give the same bytes as the fast path."""
    _check_against_oracle(CONFIGS[name], 130, seed=5, force_slow=True)


@pytest.mark.parametrize("name", ["hist_256_c16", "hist_10_c3"])
def test_slow_path_over_chunks(name):
    """Every report on the slow path with the batch cut into three stream-overlapped chunks: the
    deferred redo launch runs once after the last chunk."""
    _check_against_oracle(CONFIGS[name], 130, seed=6, force_slow=True, opts={"chunks": 3})


@pytest.mark.parametrize("name", ["count", "hist_256_c16", "sumvec_8x10_c9"])
def test_segments_and_accept_mask(name):
    _check_against_oracle(CONFIGS[name], 900, seed=3, n_segments=5)


@pytest.mark.parametrize("name", ["count", "sum8", "sumvec_8x10_c9", "hist_10_c3"])
def test_output_shares_match_prepare_next(name):
    """Per-report output shares equal the oracle's prepare_next (truncate) output."""
    from oracle.oracle import Oracle
    cfg = CONFIGS[name]
    o, d, status, batch = _check_against_oracle(cfg, 40, seed=9, tamper=False)
    outs = batch.output_shares()
    for i in range(0, 40, 7):
        rc, st, ps = o.prepare_init(VK, 1, d["nonces"][i].tobytes(), d["public_shares"][i].tobytes(),
                                    d["helper_shares"][i].tobytes())
        assert rc == 0
        rc, msg = o.prep_shares_to_prep_msg(d["leader_prep_shares"][i].tobytes(), ps)
        assert rc == 0
        rc, out = o.prepare_next(st, msg)
        assert rc == 0 and out == outs[i].tobytes()


def test_empty_batch():
    eng = _engine(CONFIGS["hist_10_c3"])
    z = lambda k: np.zeros((0, k), np.uint8)
    sz = eng.sz
    msgs, status, batch = eng.prepare_batch(z(16), z(sz.public_share_len), z(sz.helper_share_len),
                                            z(sz.prep_share_len))
    assert status.shape == (0,)
    agg, cnt = batch.accumulate(None, None, 2)
    assert cnt.tolist() == [0, 0] and not agg.any()


def test_unshard_equals_plaintext_histogram():
    """Semantic known answer (integration_tests/.../common.rs:513-526): leader + helper
    aggregate shares unshard to the plaintext histogram."""
    from oracle.oracle import Oracle, sum_mod, decode_elems, field_modulus
    cfg = CONFIGS["hist_256_c16"]
    o = Oracle(**cfg)
    eng = _engine(cfg)
    n = 5000
    d = o.gen_reports(VK, n, seed=21, n_threads=8)
    msgs, status, batch = eng.prepare_batch(d["nonces"], d["public_shares"], d["helper_shares"],
                                            d["leader_prep_shares"])
    assert not status.any()
    agg, cnt = batch.accumulate()
    p = field_modulus("histogram")
    la = sum_mod(d["leader_out_shares"], 16, p)
    ha = decode_elems(agg[0], 16)
    tot = [(a + b) % p for a, b in zip(la, ha)]
    exp = np.bincount(d["measurements"][:, 0].astype(np.int64), minlength=256)
    assert tot == [int(x) for x in exp]
    assert int(cnt[0]) == n


GEN_CASES = ["count", "sum8", "sum32", "sumvec_8x10_c9", "sumvec_1x1_c1", "hist_256_c16",
             "hist_10_c3", "hist_1_c1"]


@pytest.mark.parametrize("name", GEN_CASES)
def test_device_generator_matches_oracle_generator(name):
    """The on-device client (shard + leader prepare_init) is bit-exact with the oracle's."""
    cfg = CONFIGS[name]
    eng = _engine(cfg)
    o = _oracle(cfg)
    first, n = 5, 70
    d = eng.generate_reports_device(n, seed=99, first_index=first, with_checks=True)
    ref = o.gen_reports(VK, first + n, seed=99, n_threads=8)
    assert not d["flags"].any()
    for k in ("nonces", "public_shares", "helper_shares", "leader_prep_shares",
              "leader_out_shares"):
        np.testing.assert_array_equal(d[k].cpu().numpy(), ref[k][first:], err_msg=k)
    np.testing.assert_array_equal(d["measurements"].cpu().numpy().astype(np.uint64),
                                  ref["measurements"][first:])


def test_full_size_histogram_unshard_property():
    """BASELINE configs[1] size (1M reports): leader agg (from the generator's leader output
    shares) + helper agg (engine) unshards to the plaintext histogram; every report finishes."""
    import torch
    from oracle.oracle import sum_mod, decode_elems, field_modulus
    from janus_amd import prio3 as J
    eng = J.HelperEngine(J.Prio3Histogram(256, 16), VK, device=0)
    n = 1 << 20
    d = eng.generate_reports_device(n, seed=2024, with_checks=True)
    assert int(d["flags"].sum()) == 0
    dev = d["nonces"].device
    msgs = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    agg = torch.zeros((1, 4096), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    eng.prepare_device(d["nonces"], d["public_shares"], d["helper_shares"],
                       d["leader_prep_shares"], msgs, status)
    eng.accumulate_device(n, status, None, None, 1, agg, cnt)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0 and int(cnt[0]) == n
    p = field_modulus("histogram")
    la = [0] * 256
    step = 1 << 16
    for i in range(0, n, step):
        part = sum_mod(d["leader_out_shares"][i:i + step].cpu().numpy(), 16, p)
        la = [(a + b) % p for a, b in zip(la, part)]
    ha = decode_elems(agg[0].cpu().numpy(), 16)
    tot = [(a + b) % p for a, b in zip(la, ha)]
    exp = torch.bincount(d["measurements"][:, 0], minlength=256).cpu().tolist()
    assert tot == exp


WIDE = ["sumvec_8x1000_c63", "sumvec_4x100_c10", "sumvec_32x20_c7", "hist_500_c8",
        "hist_1000_c10"]


@pytest.mark.parametrize("name", WIDE)
def test_query_wide_parity(name):
    """P = 64/128 ParallelSum query on eight lanes per report (k_query_w, three columns per lane
    and sweep): tampered reports, a batch that is not a multiple of the 32 reports of a block;
    then every report through the slow path (the rejection-sampling XOF feeds k_query_w)."""
    n = 101 if "1000" in name else 333
    _check_against_oracle(CONFIGS[name], n, seed=21, opts={})
    _check_against_oracle(CONFIGS[name], 70 if "1000" in name else 200, seed=29, force_slow=True)


@pytest.mark.parametrize("name", ["sum8", "sum15", "sum17", "sum32", "sum50", "sum64"])
def test_query_sum_parity(name):
    """Prio3Sum on k_query_sum (P = 16..128 as NPH phases of an in-register DFT16; the
    validity weights with 16 | bits applied per phase, else per element): tampered reports and
    the slow path."""
    _check_against_oracle(CONFIGS[name], 700, seed=61)
    _check_against_oracle(CONFIGS[name], 130, seed=67, force_slow=True)


@pytest.mark.parametrize("name", ["sumvec_8x1000_c63", "sumvec_32x20_c7"])
def test_truncate_in_xof_chunked(name):
    """SumVec under k_query_w truncates inside the XOF: over stream-overlapped chunks (the
    output-share columns of every chunk)."""
    n = 600 if "1000" in name else 1500
    _check_against_oracle(CONFIGS[name], n, seed=37, opts={"coalesce": 0, "chunks": 3})


HIST_ROWS = {"hist_256_c16": CONFIGS["hist_256_c16"],
             "hist_250_c16": dict(kind="histogram", length=250, chunk_length=16),
             "hist_241_c16": dict(kind="histogram", length=241, chunk_length=16)}


@pytest.mark.parametrize("pair_max", [196608, 0])
@pytest.mark.parametrize("n", [1, 127, 700])
@pytest.mark.parametrize("name", list(HIST_ROWS))
def test_query_h_shapes(name, n, pair_max):
    """Histogram with 16 calls of chunk 16 (P = 32) on the lane-pair k_prep_hp (runs of at most
    pair_max reports) and on the one-lane k_prep_h (pair_max 0): tampered reports (decide,
    decode, joint-rand and public-share failures), a share shorter than K x C (masked rows),
    odd and sub-block batch sizes."""
    _check_against_oracle(HIST_ROWS[name], n, seed=71 + n, tamper=n > 100,
                          opts={"pair_max": pair_max})


@pytest.mark.parametrize("opts", [{}, {"chunks": 3}, {"pair_max": 0}])
@pytest.mark.parametrize("name", ["hist_256_c16", "sumvec_2x100_c10", "hist_100_c4"])
def test_fused_prepare_kernel_parity(name, opts):
    """P = 32 ParallelSum(Mul) (Histogram with 16 and 25 calls, SumVec with 20): the XOF and the
    query in one launch (k_prep_h; one chunk or three stream-overlapped ones), on tampered ragged
    batches, with and without the fused accumulate, and every report on the deferred slow path."""
    _check_against_oracle(CONFIGS[name], 777, seed=83, opts=opts)
    _check_against_oracle(CONFIGS[name], 300, seed=53, opts=dict(opts, fuse_acc=0))
    _check_against_oracle(CONFIGS[name], 97, seed=47, force_slow=True, opts=opts)


@pytest.mark.parametrize("name", ["sum8", "sum15", "sum32", "sum50", "sum64"])
def test_fused_sum_prepare_chunked(name):
    """Prio3Sum (P = 16..128; k_prep_sum from 19 bits, where the share spans two joint-rand
    blocks) in three stream-overlapped chunks, on tampered ragged batches; every report through
    the deferred slow path (k_slow_redo_sum) once after the last chunk."""
    _check_against_oracle(CONFIGS[name], 555, seed=89, opts={"chunks": 3})
    _check_against_oracle(CONFIGS[name], 130, seed=90, force_slow=True, opts={"chunks": 3})


@pytest.mark.parametrize("name", ["sumvec_8x1000_c63", "sumvec_4x100_c10", "sumvec_32x20_c7"])
def test_sumvec_wide_prepare_chunked(name):
    """SumVec on the eight-lane query (P = 64 / 128): the two-kernel chain (its XOF truncating on
    the fly) in three chunks, with every report through the slow path."""
    n = 101 if "1000" in name else 333
    _check_against_oracle(CONFIGS[name], n, seed=93, opts={"chunks": 3})
    _check_against_oracle(CONFIGS[name], 70, seed=94, force_slow=True, opts={"chunks": 3})


@pytest.mark.parametrize("opts", [{}, {"chunks": 3}])
def test_fused_count_prepare_parity(opts):
    """Prio3Count (Field64) with the generic XOF and query in one launch (k_prep_gen) on a
    tampered ragged batch and with every report on the slow path (its redo in one
    k_slow_redo_gen launch)."""
    _check_against_oracle(CONFIGS["count"], 999, seed=95, opts=opts)
    _check_against_oracle(CONFIGS["count"], 130, seed=96, force_slow=True, opts=opts)


@pytest.mark.parametrize("name", ["hist_256_c16", "hist_10_c3", "sum32", "sum8",
                                  "sumvec_4x100_c10", "sumvec_8x1000_c63"])
def test_generic_fallback_queries(name):
    """The one-lane fallback queries (k_query_ps for ParallelSum at any P, the generic k_query for
    Prio3Sum) that take the shapes the specialised kernels do not, forced on through the test
    hook force_generic_query: tampered ragged batches and every report on the slow path."""
    n = 70 if "1000" in name else 300
    _check_against_oracle(CONFIGS[name], n, seed=97, opts={"force_generic_query": 1})
    _check_against_oracle(CONFIGS[name], 64, seed=98, force_slow=True,
                          opts={"force_generic_query": 1})
