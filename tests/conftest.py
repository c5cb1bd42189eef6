import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle


# Configurations exercised by the parity tests (BASELINE.json configs at test sizes plus
# edge shapes: partial last chunk, single-bucket histogram, 1-bit sum, ...).
CONFIGS = {
    "count": dict(kind="count"),
    "sum8": dict(kind="sum", bits=8),
    "sum32": dict(kind="sum", bits=32),
    "sum1": dict(kind="sum", bits=1),
    # k_query_sum domains: P = 16 (b = 15), 32 (b = 1), 64 (b = 0 and 2), 128 (b = 0)
    "sum15": dict(kind="sum", bits=15),
    "sum17": dict(kind="sum", bits=17),
    "sum32": dict(kind="sum", bits=32),
    "sum50": dict(kind="sum", bits=50),
    "sum64": dict(kind="sum", bits=64),
    "sumvec_8x10_c9": dict(kind="sumvec", bits=8, length=10, chunk_length=9),
    "sumvec_1x1_c1": dict(kind="sumvec", bits=1, length=1, chunk_length=1),
    "sumvec_8x1000_c63": dict(kind="sumvec", bits=8, length=1000, chunk_length=63),
    "hist_256_c16": dict(kind="histogram", length=256, chunk_length=16),
    "hist_10_c3": dict(kind="histogram", length=10, chunk_length=3),
    "hist_1_c1": dict(kind="histogram", length=1, chunk_length=1),
    "hist_100_c10": dict(kind="histogram", length=100, chunk_length=10),
    # 64- and 128-point wire domains (k_query_w, eight lanes per report)
    "sumvec_4x100_c10": dict(kind="sumvec", bits=4, length=100, chunk_length=10),
    "sumvec_32x20_c7": dict(kind="sumvec", bits=32, length=20, chunk_length=7),
    "hist_500_c8": dict(kind="histogram", length=500, chunk_length=8),
    "hist_1000_c10": dict(kind="histogram", length=1000, chunk_length=10),
    # P = 32 with 20 and 25 gadget calls (k_prep_h with partially filled wire domains)
    "sumvec_2x100_c10": dict(kind="sumvec", bits=2, length=100, chunk_length=10),
    "hist_100_c4": dict(kind="histogram", length=100, chunk_length=4),
}
