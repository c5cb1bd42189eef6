"""Python mirror of the batched HPKE opener (include/janus_hpke.h), SURVEY 8(f) row 2.

``HpkeOpener`` corresponds to one Janus ``HpkeKeypair`` + ``HpkeApplicationInfo``
(/root/reference/core/src/hpke.rs:70-85, 186-203, 283-305); ``open_input_shares`` is the
decrypt + PlaintextInputShare decode + extension checks of the helper's aggregate-init loop
(aggregator.rs:1796-1990) for a whole batch, producing the helper input shares that
``HelperEngine.prepare_*`` consumes.  No CPU fallback: the HIP library must be built.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .prio3 import _np_ptr, _stream, _tptr, load_library

KEM_X25519_HKDF_SHA256 = 0x0020
KEM_P256_HKDF_SHA256 = 0x0010
KEM_X448_HKDF_SHA512 = 0x0021
KEM_P521_HKDF_SHA512 = 0x0012
KEM_P384_HKDF_SHA384 = 0x0011
KDF_HKDF_SHA256 = 0x0001
KDF_HKDF_SHA384 = 0x0002
KDF_HKDF_SHA512 = 0x0003
# Nenc (= Npk) per KEM (RFC 9180 7.1)
NENC = {KEM_X25519_HKDF_SHA256: 32, KEM_P256_HKDF_SHA256: 65, KEM_X448_HKDF_SHA512: 56,
        KEM_P521_HKDF_SHA512: 133, KEM_P384_HKDF_SHA384: 97}
AEAD_AES_128_GCM = 0x0001
AEAD_AES_256_GCM = 0x0002
AEAD_CHACHA20_POLY1305 = 0x0003
OK, DECRYPT_ERROR, INVALID_MESSAGE = 0, 4, 8
INFO_INPUT_SHARE_HELPER = b"dap-09 input share" + bytes([1, 3])  # Label::InputShare, Client->Helper

_bound = False


def _lib():
    global _bound
    L = load_library()
    if not _bound:
        vp, u32 = C.c_void_p, C.c_uint32
        L.janus_hpke_opener_create.argtypes = [C.c_uint16, C.c_uint16, C.c_uint16, vp, C.c_size_t,
                                               vp, C.c_size_t, vp, C.c_size_t, C.c_int,
                                               C.POINTER(vp)]
        L.janus_hpke_opener_destroy.argtypes = [vp]
        L.janus_hpke_open_input_shares_device.argtypes = [vp, u32, vp, vp, vp, vp, u32, vp, vp, vp,
                                                          u32, u32, C.c_int, vp, vp, vp]
        L.janus_hpke_open_input_shares.argtypes = [vp, u32, vp, vp, vp, vp, u32, vp, vp, vp, u32,
                                                   u32, C.c_int, vp, vp]
        L.janus_hpke_open_device.argtypes = [vp, u32, vp, vp, vp, u32, vp, vp, u32, vp, vp, vp]
        L.janus_hpke_open.argtypes = [vp, u32, vp, vp, vp, u32, vp, vp, u32, vp, vp]
        L.janus_hpke_set_timing.argtypes = [vp, C.c_int]
        L.janus_hpke_timing.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]
        L.janus_hpke_executor_stats_get.argtypes = [vp, C.POINTER(C.c_uint64 * 5)]
        L.janus_hpke_executor_control.argtypes = [vp, C.c_char_p, C.c_int64]
        L.janus_hpke_selftest_p256.argtypes = [C.c_int, u32, vp, vp, vp]
        L.janus_hpke_selftest_field.argtypes = [C.c_int, C.c_int, u32, vp, vp, vp]
        _bound = True
    return L


def _b(x: bytes):
    return C.cast(C.c_char_p(bytes(x)), C.c_void_p)


class HpkeOpener:
    def __init__(self, private_key: bytes, public_key: bytes, info: bytes = INFO_INPUT_SHARE_HELPER,
                 device: int = 0, kem_id=KEM_X25519_HKDF_SHA256, kdf_id=KDF_HKDF_SHA256,
                 aead_id=AEAD_AES_128_GCM):
        self.device = device
        self.nenc = NENC.get(kem_id, 0)  # enc bytes per report
        self._keep = (bytes(private_key), bytes(public_key), bytes(info))
        h = C.c_void_p()
        rc = _lib().janus_hpke_opener_create(kem_id, kdf_id, aead_id, _b(private_key),
                                             len(private_key), _b(public_key), len(public_key),
                                             _b(info) if info else None, len(info), device,
                                             C.byref(h))
        if rc == -3:
            raise NotImplementedError("HPKE suite not supported by the GPU opener")
        if rc:
            raise RuntimeError(f"janus_hpke_opener_create failed (rc={rc})")
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            _lib().janus_hpke_opener_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- DAP helper input shares ----------------------------------------------------
    def open_input_shares(self, task_id: bytes, enc, ct, ct_len, report_ids, times,
                          public_shares, helper_share_len: int, require_taskprov=False):
        """Host arrays -> (helper_shares [n, helper_share_len], status [n])."""
        enc = np.ascontiguousarray(enc, np.uint8)
        n = enc.shape[0]
        ct = np.ascontiguousarray(ct, np.uint8)
        if ct.shape[1] % 16:
            ct = np.pad(ct, ((0, 0), (0, 16 - ct.shape[1] % 16)))
        ct_len = np.ascontiguousarray(ct_len, np.uint32)
        ids = np.ascontiguousarray(report_ids, np.uint8)
        times = np.ascontiguousarray(times, np.uint64)
        pub = None if public_shares is None else np.ascontiguousarray(public_shares, np.uint8)
        publen = 0 if pub is None else pub.shape[1]
        shares = np.zeros((n, helper_share_len), np.uint8)
        status = np.zeros(n, np.uint8)
        rc = _lib().janus_hpke_open_input_shares(
            self.handle, n, _b(task_id), _np_ptr(enc), _np_ptr(ct), _np_ptr(ct_len), ct.shape[1],
            _np_ptr(ids), _np_ptr(times), _np_ptr(pub), publen, helper_share_len,
            int(require_taskprov), _np_ptr(shares), _np_ptr(status))
        if rc:
            raise RuntimeError(f"janus_hpke_open_input_shares failed (rc={rc})")
        return shares, status

    def open_input_shares_device(self, task_id: bytes, enc, ct, ct_len, report_ids, times,
                                 public_shares, helper_shares, status, require_taskprov=False,
                                 stream=None):
        """torch tensors on this opener's GPU; ct is [n, stride] with stride % 16 == 0."""
        rc = _lib().janus_hpke_open_input_shares_device(
            self.handle, enc.shape[0], _b(task_id), _tptr(enc), _tptr(ct), _tptr(ct_len),
            ct.shape[1], _tptr(report_ids), _tptr(times), _tptr(public_shares),
            0 if public_shares is None else public_shares.shape[1], helper_shares.shape[1],
            int(require_taskprov), _tptr(helper_shares), _tptr(status),
            _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"janus_hpke_open_input_shares_device failed (rc={rc})")

    # ---- generic single-shot open ----------------------------------------------------
    def open(self, enc, ct_list, aad_list):
        """Lists of byte strings -> list of plaintexts (None where the open failed)."""
        n = len(ct_list)
        cs = max(16, -(-max(len(c) for c in ct_list) // 16) * 16)
        as_ = -(-max([len(a) for a in aad_list] + [1]) // 16) * 16
        encs = np.zeros((n, self.nenc), np.uint8)
        ct = np.zeros((n, cs), np.uint8)
        aad = np.zeros((n, as_), np.uint8)
        cl = np.zeros(n, np.uint32)
        al = np.zeros(n, np.uint32)
        for i in range(n):
            encs[i] = np.frombuffer(bytes(enc[i]), np.uint8)
            ct[i, :len(ct_list[i])] = np.frombuffer(ct_list[i], np.uint8)
            aad[i, :len(aad_list[i])] = np.frombuffer(aad_list[i], np.uint8)
            cl[i], al[i] = len(ct_list[i]), len(aad_list[i])
        pt = np.zeros((n, cs), np.uint8)
        st = np.zeros(n, np.uint8)
        rc = _lib().janus_hpke_open(self.handle, n, _np_ptr(encs), _np_ptr(ct), _np_ptr(cl), cs,
                                    _np_ptr(aad), _np_ptr(al), as_, _np_ptr(pt), _np_ptr(st))
        if rc:
            raise RuntimeError(f"janus_hpke_open failed (rc={rc})")
        return [None if st[i] else pt[i, :cl[i] - 16].tobytes() for i in range(n)]

    def executor_stats(self) -> dict:
        """Counters of the GPU's HPKE executor (janus_hpke_executor_stats_get)."""
        v = (C.c_uint64 * 5)()
        rc = _lib().janus_hpke_executor_stats_get(self.handle, C.byref(v))
        if rc:
            raise RuntimeError(f"janus_hpke_executor_stats_get failed (rc={rc})")
        return dict(zip(("jobs", "reports", "groups", "active_jobs", "active_reports"), v))

    def executor_control(self, key: str, value: int):
        """janus_hpke_executor_control: "hold", "heavy", "coalesce"."""
        rc = _lib().janus_hpke_executor_control(self.handle, key.encode(), int(value))
        if rc:
            raise ValueError(f"executor control {key} failed (rc={rc})")

    def set_timing(self, on: bool):
        _lib().janus_hpke_set_timing(self.handle, int(on))

    def timing(self):
        ms, k = C.c_double(), C.c_uint32()
        _lib().janus_hpke_timing(self.handle, C.byref(ms), C.byref(k))
        return ms.value, k.value
