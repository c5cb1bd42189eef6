"""The generated inline-asm headers are what their generators print (no hand edits drift)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gen,header", [("gen_fe25519_asm.py", "fe25519_asm.h"),
                                        ("gen_p256_asm.py", "p256_asm.h")])
def test_generated_header_matches_generator(gen, header):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", gen)], check=True,
                         capture_output=True, text=True).stdout
    with open(os.path.join(ROOT, "janus_amd", "csrc", header)) as f:
        assert f.read() == out
