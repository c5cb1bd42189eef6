"""Generates tests/golden/fpvec_l10000.npz: full-size config C5 (Prio3FixedPointBoundedL2VecSum,
length 10000, BitSize 16) fixtures from the Python restatement (oracle/fpvec_py.py, itself pinned
as documented there; parity with prio UNPINNED).

Two honest reports plus one copy of report 0 whose leader verifier share is tampered.  Stored per
report: nonce, public share, helper input share, leader prep share, and the expected helper
prepare message, status and output share (honest reports only).  ~80 s on one core.

    python tests/golden/gen_fpvec_l10000.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_fpvec import VK, _expected, _reports, _vdaf  # noqa: E402


def main():
    v = _vdaf(10000, 16)
    reps = _reports(v, 2, seed=10000)
    bad = dict(reps[0], lps=bytearray(reps[0]["lps"]))
    bad["lps"][16 * 3] ^= 1  # a leader verifier value: decide fails
    reps.append(bad)
    msgs, status, outs = _expected(v, reps)
    assert status == [0, 0, 3], status
    A = lambda k: np.array([list(r[k]) for r in reps], np.uint8)
    out_bytes = np.array([[b for e in o for b in e.to_bytes(16, "little")] for o in outs[:2]],
                         np.uint8)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "fpvec_l10000.npz"),
                        verify_key=np.frombuffer(VK, np.uint8), nonce=A("nonce"), pub=A("pub"),
                        helper=A("helper"), lps=A("lps"),
                        prep_msg=np.array([list(m) for m in msgs], np.uint8),
                        status=np.array(status, np.uint8), out_shares=out_bytes)


if __name__ == "__main__":
    main()
