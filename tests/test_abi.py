"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every symbol
include/janus_prio3.h declares, reports the right per-instance sizes, and fails loudly
(no CPU fallback) when no GPU is available."""
import ctypes as C
import os
import re

import pytest

from tests.conftest import CONFIGS, ROOT

HEADER = os.path.join(ROOT, "include", "janus_prio3.h")


def _declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|void)\s+(prio3_\w+)\s*\(", src, re.M)))


def test_header_declares_the_exported_set():
    from janus_amd import prio3 as J
    assert _declared_symbols() == sorted(J.EXPORTED_SYMBOLS)


def _declared_hpke_symbols():
    src = open(os.path.join(ROOT, "include", "janus_hpke.h")).read()
    return sorted(set(re.findall(r"^(?:int|void)\s+(janus_hpke_\w+)\s*\(", src, re.M)))


def test_hpke_header_declares_the_exported_set():
    from janus_amd import prio3 as J
    assert _declared_hpke_symbols() == sorted(J.HPKE_EXPORTED_SYMBOLS)
    L = J.load_library()
    for name in _declared_hpke_symbols():
        assert hasattr(L, name), name


def test_dap_header_declares_the_exported_set():
    from janus_amd import dap as J
    src = open(os.path.join(ROOT, "include", "janus_dap.h")).read()
    declared = sorted(set(re.findall(r"^(?:int|void|int64_t|size_t)\s+(janus_dap_\w+)\s*\(",
                                     src, re.M)))
    assert declared == sorted(J.DAP_EXPORTED_SYMBOLS)
    L = J._lib()
    for name in declared:
        assert hasattr(L, name), name


def test_hpke_unsupported_suite_is_refused():
    """Unknown KEM / KDF / AEAD ids stay on the host path: creation says EUNSUPPORTED before any
    GPU call; a NIST-curve key outside [1, n) or a key of the wrong length is EINVAL (no GPU
    call).  (P-384, 0x0011, opens on the device since r05: tests/test_hpke.py.)"""
    from janus_amd import hpke as H
    with pytest.raises(NotImplementedError):
        H.HpkeOpener(bytes(48), bytes(97), kem_id=0x0013)   # no such KEM
    with pytest.raises(RuntimeError, match="rc=-1"):
        H.HpkeOpener(bytes(48), b"\x04" + bytes(96), kem_id=0x0011)  # P-384 sk = 0
    with pytest.raises(NotImplementedError):
        H.HpkeOpener(bytes(32), bytes(32), kdf_id=0x0004)   # no such KDF
    with pytest.raises(NotImplementedError):
        H.HpkeOpener(bytes(32), bytes(32), aead_id=0xFFFF)  # export-only
    with pytest.raises(RuntimeError, match="rc=-1"):
        H.HpkeOpener(bytes(32), b"\x04" + bytes(64), kem_id=0x0010)  # sk = 0
    with pytest.raises(RuntimeError, match="rc=-1"):
        H.HpkeOpener(b"\xff" * 66, b"\x04" + bytes(132), kem_id=0x0012)  # P-521 sk >= n
    with pytest.raises(RuntimeError, match="rc=-1"):
        H.HpkeOpener(bytes(32), bytes(32), kem_id=0x0021)   # X448 takes 56-byte keys
    with pytest.raises(RuntimeError, match="rc=-1"):
        H.HpkeOpener(b"\xff" * 32, b"\x04" + bytes(64), kem_id=0x0010)  # sk >= n


def test_library_exports_every_declared_symbol():
    from janus_amd import prio3 as J
    L = J.load_library()
    for name in _declared_symbols():
        assert hasattr(L, name), name


@pytest.mark.parametrize("name", list(CONFIGS))
def test_sizes_match_oracle(name, oracle_lib):
    from janus_amd import prio3 as J
    cfg = CONFIGS[name]
    o = oracle_lib.Oracle(**cfg)
    v = J.Prio3({"count": 0, "sum": 1, "sumvec": 2, "histogram": 3}[cfg["kind"]],
                cfg.get("bits", 0), cfg.get("length", 0), cfg.get("chunk_length", 0))
    s = v.sizes()
    assert s.field_bytes == o.es
    assert s.meas_len == o.meas_len and s.out_len == o.out_len
    assert s.proof_len == o.proof_len and s.verifier_len == o.verifier_len
    assert s.public_share_len == o.public_share_len
    assert s.helper_share_len == o.helper_share_len
    assert s.prep_share_len == o.prep_share_len
    assert s.prep_msg_len == o.prep_msg_len
    assert s.agg_share_len == o.out_share_bytes
    assert s.leader_input_share_len == o.leader_share_len


def test_histogram_256_sizes_match_survey():
    """PROOF_LEN 95, VERIFIER_LEN 34, leader prep 560 B."""
    from janus_amd import prio3 as J
    s = J.Prio3Histogram(256, 16).sizes()
    assert (s.proof_len, s.verifier_len, s.prep_share_len, s.helper_share_len) == (95, 34, 560, 48)


def test_invalid_parameters_rejected():
    from janus_amd import prio3 as J
    for v in (J.Prio3Sum(0), J.Prio3Histogram(0, 1), J.Prio3SumVec(8, 10, 0), J.Prio3(9)):
        with pytest.raises(ValueError):
            v.sizes()
    with pytest.raises(ValueError):
        J.Prio3(J.PRIO3_COUNT, num_proofs=2).sizes()


def test_engine_requires_gpu_or_fails_loudly():
    import torch
    from janus_amd import prio3 as J
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        J.HelperEngine(J.Prio3Count(), bytes(16), device=0)


def test_set_device_only_inside_the_guard():
    """every entry point and runtime helper makes its GPU current through
    DeviceGuard (prio3_runtime.h), which gives the calling thread its own device back; no other
    hipSetDevice may appear in the library's sources, or a Janus worker whose job a multi-GPU
    engine placed on GPU k would come back bound to GPU k."""
    csrc = os.path.join(ROOT, "janus_amd", "csrc")
    hits = []
    for fn in sorted(os.listdir(csrc)):
        if not fn.endswith((".hip", ".h", ".cpp")):
            continue
        for i, line in enumerate(open(os.path.join(csrc, fn)), 1):
            code = line.split("//")[0]
            if "hipSetDevice(" in code:
                hits.append((fn, i, line.strip()))
    guard = [h for h in hits if h[0] == "prio3_runtime.h"]
    assert len(guard) == 2, hits  # the guard's set and its restore
    assert [h for h in hits if h[0] != "prio3_runtime.h"] == []
