"""SURVEY.md 5 "ASan host build": the DAP request parser (the host code that reads untrusted
bytes) built with AddressSanitizer and driven by tools/fuzz_dap.cpp over mutated
AggregationJobInitializeReq bodies (bit flips, truncations, length-field extremes, splices).
CPU only; any heap over-read / over-write aborts the harness with an ASan report."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not present")
def test_dap_host_parser_under_asan():
    mk = subprocess.run(["make", "-C", os.path.join(ROOT, "janus_amd"), "build_asan/fuzz_dap"],
                        capture_output=True, text=True, timeout=600)
    assert mk.returncode == 0, mk.stdout + mk.stderr
    r = subprocess.run([os.path.join(ROOT, "janus_amd", "build_asan", "fuzz_dap"), "6000", "7"],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1"))
    assert r.returncode == 0 and "no ASan report" in r.stdout, r.stdout + r.stderr
