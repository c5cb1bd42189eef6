"""Edge sizes at the C ABI (the reference's tests cover empty and ragged
jobs): an empty batch, a single report, and sizes that end inside a wave, a 256-report block
and an eight-lane report group, for every kernel family -- one-lane (Count), k_query_sum (Sum),
k_query_h (Histogram), k_query_w (SumVec P = 128) -- against the restatement."""
import numpy as np
import pytest

from tests.conftest import CONFIGS
from tests.test_gpu_parity import VK, _check_against_oracle, _engine, _oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["count", "sum32", "hist_256_c16", "sumvec_8x1000_c63"])
def test_empty_batch(name):
    """n = 0: every entry point succeeds, the aggregate share is zero and the count 0."""
    cfg = CONFIGS[name]
    o, eng = _oracle(cfg), _engine(cfg)
    sz = eng.sz
    z = lambda w: np.zeros((0, w), np.uint8)
    msgs, status, batch = eng.prepare_batch(z(16), z(sz.public_share_len) if sz.public_share_len
                                            else None, z(sz.helper_share_len),
                                            z(sz.prep_share_len))
    assert msgs.shape[0] == 0 and status.shape == (0,)
    agg, cnt = batch.accumulate()
    assert not agg.any() and int(cnt[0]) == 0
    batch.free()
    lps, lst, lbatch = eng.leader_prepare_init_batch(
        z(16), z(sz.public_share_len) if sz.public_share_len else None,
        z(sz.leader_input_share_len))
    assert lps.shape[0] == 0 and lst.shape == (0,)
    lbatch.free()


@pytest.mark.parametrize("n", [1, 2, 63, 65, 255, 257, 519])
@pytest.mark.parametrize("name", ["count", "sum32", "hist_256_c16"])
def test_ragged_sizes(name, n):
    _check_against_oracle(CONFIGS[name], n, seed=n, tamper=n >= 63)


@pytest.mark.parametrize("n", [1, 7, 9, 33])
def test_ragged_sizes_eight_lane_query(n):
    """k_query_w: groups of eight lanes per report, blocks of 32 reports."""
    _check_against_oracle(CONFIGS["sumvec_8x1000_c63"], n, seed=n, tamper=False)
