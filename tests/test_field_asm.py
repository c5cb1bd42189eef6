"""GPU: the device Field128 primitives (compiler-built and hand-scheduled asm) against Python
integers, on random and edge-case canonical operands.  The hand-written blocks keep their
VCC carry chains back to back and keep scratch in fixed VGPRs, so they get their own test
next to the end-to-end parity suite (tests/test_gpu_parity.py)."""
import random

import numpy as np
import pytest

from janus_amd import prio3 as J

pytestmark = pytest.mark.gpu

P = 2**128 - 28 * 2**64 + 1
EDGE = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, 2**127, 2**64 - 1, 2**64, 28 * 2**64,
        2**96 - 1, 2**128 - 28 * 2**64 - 2**32, P - 2**64]


def enc(xs):
    return np.frombuffer(b"".join(x.to_bytes(16, "little") for x in xs), np.uint8).reshape(-1, 16)


def dec(arr):
    return [int.from_bytes(r.tobytes(), "little") for r in arr]


def operands(n, seed):
    rnd = random.Random(seed)
    a = [rnd.choice(EDGE) if rnd.random() < 0.15 else rnd.randrange(P) for _ in range(n)]
    b = [rnd.choice(EDGE) if rnd.random() < 0.15 else rnd.randrange(P) for _ in range(n)]
    a[:len(EDGE)] = EDGE
    b[:len(EDGE)] = EDGE[::-1]
    return a, b


@pytest.mark.parametrize("op,fn", [(0, lambda x, y: x * y % P), (1, lambda x, y: x * y % P),
                                   (2, lambda x, y: (x + y) % P), (3, lambda x, y: (x - y) % P)])
def test_binary_ops(op, fn):
    a, b = operands(1 << 16, op)
    got = dec(J.selftest_field(op, enc(a), enc(b)))
    want = [fn(x, y) for x, y in zip(a, b)]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, f"op {op}: {len(bad)} mismatches, first at {bad[0]}"


@pytest.mark.parametrize("op", [4, 5])
def test_mac_reduce(op):
    n = 1 << 13
    a, b = operands(16 * n, 10 + op)
    # all-(p-1) rows maximise every column and overflow word
    a[16:32] = [P - 1] * 16
    b[16:32] = [P - 1] * 16
    got = dec(J.selftest_field(op, enc(a), enc(b)))
    want = [sum(a[16 * i + k] * b[16 * i + k] for k in range(16)) % P for i in range(n)]
    assert got == want
