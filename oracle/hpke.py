"""ctypes binding of oracle/hpke_oracle.c -- TEST INFRASTRUCTURE (checker + CPU baseline).

HPKE base mode (RFC 9180) with KEM DHKEM(X25519 / P-256, HKDF-SHA256) or DHKEM(X448 / P-521,
HKDF-SHA512), KDF HKDF-SHA256 / -SHA384 / -SHA512 and AEAD AES-128-GCM, AES-256-GCM or
ChaCha20Poly1305, composed over OpenSSL 3.0 primitives, plus Janus's helper input-share layer (aggregator.rs:1796-1990).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "libhpke_oracle.so")
INFO_INPUT_SHARE_HELPER = b"dap-09 input share" + bytes([1, 3])  # Role::Client, Role::Helper
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB) or \
                os.path.getmtime(_LIB) < os.path.getmtime(os.path.join(_HERE, "hpke_oracle.c")):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        _lib = C.CDLL(_LIB)
        vp = C.c_void_p
        _lib.hpke_open.argtypes = [vp, vp, vp, vp, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, vp]
        _lib.hpke_seal.argtypes = [vp, vp, vp, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, vp, vp]
        _lib.hpke_x25519_public.argtypes = [vp, vp]
        _lib.hpke_input_share_aad.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint32, vp]
        _lib.hpke_input_share_aad.restype = C.c_size_t
        _lib.hpke_open_input_shares.argtypes = [vp, vp, vp, C.c_uint32, vp, vp, vp, C.c_uint32,
                                                vp, vp, vp, C.c_uint32, C.c_uint32, C.c_int, vp,
                                                vp, C.c_int]
        _lib.hpke_make_input_shares.argtypes = [vp, vp, C.c_uint32, C.c_uint64, C.c_uint32,
                                                C.c_uint32, C.c_int, C.c_uint32, vp, vp, vp, vp,
                                                vp, vp, vp, C.c_int]
        _lib.hpke_seal_input_shares.argtypes = [vp, vp, C.c_uint32, C.c_uint64, vp, vp, vp,
                                                C.c_uint32, vp, C.c_uint32, C.c_uint32, vp, vp,
                                                vp, C.c_int]
        _lib.aes128_ctr64_keystream.argtypes = [vp, vp, vp, C.c_size_t]
        # the AEAD-selecting forms (aead 1 AES-128-GCM, 2 AES-256-GCM, 3 ChaCha20Poly1305)
        u16 = C.c_uint16
        _lib.hpke_open_ex.argtypes = [u16] + _lib.hpke_open.argtypes
        _lib.hpke_seal_ex.argtypes = [u16] + _lib.hpke_seal.argtypes
        _lib.hpke_open_input_shares_ex.argtypes = [u16] + _lib.hpke_open_input_shares.argtypes
        _lib.hpke_make_input_shares_ex.argtypes = [u16] + _lib.hpke_make_input_shares.argtypes
        # and the KEM-selecting forms (kem 0x20 X25519, 0x10 P-256)
        _lib.hpke_p256_public.argtypes = [vp, vp]
        _lib.hpke_open_kem.argtypes = [u16] + _lib.hpke_open_ex.argtypes
        _lib.hpke_seal_kem.argtypes = [u16] + _lib.hpke_seal_ex.argtypes
        _lib.hpke_open_input_shares_kem.argtypes = [u16] + _lib.hpke_open_input_shares_ex.argtypes
        _lib.hpke_make_input_shares_kem.argtypes = [u16] + _lib.hpke_make_input_shares_ex.argtypes
        # and the suite forms (kem, kdf, aead): every KEM of KEMS, KDF 1 / 2 / 3
        _lib.hpke_kem_public.argtypes = [u16, vp, vp]
        _lib.hpke_open_suite.argtypes = [u16, u16, u16] + _lib.hpke_open.argtypes
        _lib.hpke_seal_suite.argtypes = [u16, u16, u16] + _lib.hpke_seal.argtypes
        _lib.hpke_open_input_shares_suite.argtypes = [u16, u16, u16] + \
            _lib.hpke_open_input_shares.argtypes
        _lib.hpke_make_input_shares_suite.argtypes = [u16, u16, u16] + \
            _lib.hpke_make_input_shares.argtypes
    return _lib


def _p(b):
    if b is None:
        return None
    if isinstance(b, np.ndarray):
        return b.ctypes.data_as(C.c_void_p)
    return C.cast(C.c_char_p(bytes(b)), C.c_void_p)


KEM_X25519, KEM_P256, KEM_X448, KEM_P521, KEM_P384 = 0x20, 0x10, 0x21, 0x12, 0x11
KDF_SHA256, KDF_SHA384, KDF_SHA512 = 1, 2, 3
# RFC 9180 7.1: Nsk, Nenc (= Npk; the NIST curves' uncompressed points)
NSK = {KEM_X25519: 32, KEM_P256: 32, KEM_X448: 56, KEM_P521: 66, KEM_P384: 48}
NENC = {KEM_X25519: 32, KEM_P256: 65, KEM_X448: 56, KEM_P521: 133, KEM_P384: 97}


def nenc(kem: int) -> int:
    """Nenc = Npk of the KEM."""
    return NENC[kem]


def x25519_public(sk: bytes) -> bytes:
    return kem_public(sk, KEM_X25519)


def kem_public(sk: bytes, kem=KEM_X25519) -> bytes:
    out = C.create_string_buffer(NENC[kem])
    assert lib().hpke_kem_public(kem, _p(sk), out) == 0
    return out.raw


def kem_private(rng, kem=KEM_X25519) -> bytes:
    """A random private key (P-256 / P-384: below 2^255 / 2^383, P-521: below 2^520, hence below
    the order)."""
    sk = bytearray(rng.integers(0, 256, NSK[kem], dtype=np.uint8).tobytes())
    if kem in (KEM_P256, KEM_P384):
        sk[0] &= 0x7F
    if kem == KEM_P521:
        sk[0] = 0
    return bytes(sk)


def open_(skR: bytes, pkR: bytes, enc: bytes, info: bytes, aad: bytes, ct: bytes, aead=1,
          kem=KEM_X25519, kdf=KDF_SHA256):
    pt = C.create_string_buffer(max(len(ct), 1))
    n = lib().hpke_open_suite(kem, kdf, aead, _p(skR), _p(pkR), _p(enc), _p(info), len(info),
                              _p(aad), len(aad), _p(ct), len(ct), pt)
    return None if n < 0 else pt.raw[:n]


def seal(pkR: bytes, skE: bytes, info: bytes, aad: bytes, pt: bytes, aead=1, kem=KEM_X25519,
         kdf=KDF_SHA256):
    enc = C.create_string_buffer(nenc(kem))
    ct = C.create_string_buffer(len(pt) + 16)
    assert lib().hpke_seal_suite(kem, kdf, aead, _p(pkR), _p(skE), _p(info), len(info), _p(aad),
                                 len(aad), _p(pt), len(pt), enc, ct) == 0
    return enc.raw, ct.raw


def input_share_aad(task_id: bytes, report_id: bytes, time: int, public_share: bytes) -> bytes:
    out = C.create_string_buffer(64 + 4 + len(public_share))
    n = lib().hpke_input_share_aad(_p(task_id), _p(report_id), time, _p(public_share),
                                   len(public_share), out)
    return out.raw[:n]


def plaintext_input_share(payload: bytes, extensions=()) -> bytes:
    """PlaintextInputShare encoding (messages/src/lib.rs:1326-1341)."""
    ext = b"".join(t.to_bytes(2, "big") + len(d).to_bytes(2, "big") + d for t, d in extensions)
    return len(ext).to_bytes(2, "big") + ext + len(payload).to_bytes(4, "big") + payload


def open_input_shares(skR, pkR, task_id, enc, ct, ct_len, report_ids, times, pubs, share_len,
                      require_taskprov=False, n_threads=8, aead=1, kem=KEM_X25519, kdf=KDF_SHA256):
    """Batched helper input-share open: (shares [n, share_len], status [n] in {0, 4, 8})."""
    n = enc.shape[0]
    enc = np.ascontiguousarray(enc, np.uint8)
    ct = np.ascontiguousarray(ct, np.uint8)
    ct_len = np.ascontiguousarray(ct_len, np.uint32)
    ids = np.ascontiguousarray(report_ids, np.uint8)
    times = np.ascontiguousarray(times, np.uint64)
    publen = 0 if pubs is None else pubs.shape[1]
    pubs = None if pubs is None else np.ascontiguousarray(pubs, np.uint8)
    shares = np.zeros((n, share_len), np.uint8)
    status = np.zeros(n, np.uint8)
    lib().hpke_open_input_shares_suite(kem, kdf, aead, _p(skR), _p(pkR), _p(task_id), n, _p(enc),
                                       _p(ct), _p(ct_len), ct.shape[1], _p(ids), _p(times),
                                       _p(pubs), publen, share_len, int(require_taskprov),
                                       _p(shares), _p(status), n_threads)
    return shares, status


def make_batch(n, share_len, pub_len, seed=1, skR=None, extensions=(), tamper=0.0, aead=1,
               kem=KEM_X25519, kdf=KDF_SHA256):
    """Synthetic Janus-shaped encrypted helper input shares (test/bench data), sealed by the
    oracle with deterministic ephemeral keys.  Returns a dict of numpy arrays."""
    rng = np.random.default_rng(seed)
    skR = kem_private(rng, kem) if skR is None else skR
    pkR = kem_public(skR, kem)
    task_id = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    ids = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    times = (1_700_000_000 + rng.integers(0, 3600, n)).astype(np.uint64)
    pubs = rng.integers(0, 256, (n, pub_len), dtype=np.uint8) if pub_len else None
    shares = rng.integers(0, 256, (n, share_len), dtype=np.uint8)
    pt_len = len(plaintext_input_share(bytes(share_len), extensions))
    stride = pt_len + 16
    enc = np.zeros((n, nenc(kem)), np.uint8)
    ct = np.zeros((n, stride), np.uint8)
    ct_len = np.full(n, stride, np.uint32)
    for r in range(n):
        aad = input_share_aad(task_id, ids[r].tobytes(), int(times[r]),
                              b"" if pubs is None else pubs[r].tobytes())
        skE = kem_private(rng, kem)
        e, c = seal(pkR, skE, INFO_INPUT_SHARE_HELPER, aad,
                    plaintext_input_share(shares[r].tobytes(), extensions), aead=aead, kem=kem,
                    kdf=kdf)
        enc[r] = np.frombuffer(e, np.uint8)
        ct[r] = np.frombuffer(c, np.uint8)
    return dict(skR=skR, pkR=pkR, task_id=task_id, report_ids=ids, times=times, pubs=pubs,
                shares=shares, enc=enc, ct=ct, ct_len=ct_len)


def make_batch_fast(n, share_len, pub_len, seed=1, taskprov=False, n_threads=8, skR=None, aead=1,
                    kem=KEM_X25519, kdf=KDF_SHA256):
    """make_batch in C with threads (bench-size batches); every report distinct."""
    rng = np.random.default_rng(seed)
    skR = kem_private(rng, kem) if skR is None else skR
    pkR = kem_public(skR, kem)
    task_id = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    stride = -(-((10 if taskprov else 6) + share_len + 16) // 16) * 16
    enc = np.zeros((n, nenc(kem)), np.uint8)
    ct = np.zeros((n, stride), np.uint8)
    ct_len = np.zeros(n, np.uint32)
    ids = np.zeros((n, 16), np.uint8)
    times = np.zeros(n, np.uint64)
    pubs = np.zeros((n, pub_len), np.uint8) if pub_len else None
    shares = np.zeros((n, share_len), np.uint8)
    rc = lib().hpke_make_input_shares_suite(kem, kdf, aead, _p(pkR), _p(task_id), n, seed,
                                            share_len, pub_len, int(taskprov), stride, _p(enc),
                                            _p(ct), _p(ct_len), _p(ids), _p(times), _p(pubs),
                                            _p(shares), n_threads)
    assert rc == 0
    return dict(skR=skR, pkR=pkR, task_id=task_id, report_ids=ids, times=times, pubs=pubs,
                shares=shares, enc=enc, ct=ct, ct_len=ct_len)


def seal_input_shares(pkR, task_id, ids, times, pubs, shares, seed=1, n_threads=8):
    """Seals the given helper input shares (no extensions) -> (enc, ct, ct_len, stride)."""
    n, share_len = shares.shape
    stride = -(-(6 + share_len + 16) // 16) * 16
    enc = np.zeros((n, 32), np.uint8)
    ct = np.zeros((n, stride), np.uint8)
    ct_len = np.zeros(n, np.uint32)
    publen = 0 if pubs is None else pubs.shape[1]
    rc = lib().hpke_seal_input_shares(
        _p(pkR), _p(task_id), n, seed, _p(np.ascontiguousarray(ids, np.uint8)),
        _p(np.ascontiguousarray(times, np.uint64)),
        None if pubs is None else _p(np.ascontiguousarray(pubs, np.uint8)), publen,
        _p(np.ascontiguousarray(shares, np.uint8)), share_len, stride, _p(enc), _p(ct),
        _p(ct_len), n_threads)
    assert rc == 0
    return enc, ct, ct_len, stride


def aes128_ctr64_keystream(key: bytes, iv: bytes, n: int) -> bytes:
    """AES-128-CTR keystream, 64-bit BE counter in the IV's low half (prio SeedStreamAes128)."""
    out = C.create_string_buffer(n)
    assert lib().aes128_ctr64_keystream(_p(key), _p(iv), out, n) == 0
    return out.raw
