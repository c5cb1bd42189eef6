"""Python mirror of the DAP-09 marshaling around the device calls (include/janus_dap.h),
SURVEY 8(f) row 3: AggregationJobInitializeReq body -> SoA buffers for the HPKE opener and the
prio3 engine, and their outputs -> the AggregationJobResp body (helper init step)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from .prio3 import _np_ptr, _stream, _tptr, load_library

DAP_EXPORTED_SYMBOLS = (
    "janus_dap_agg_init_scan", "janus_dap_agg_init_scan_ex", "janus_dap_agg_init_unpack_device",
    "janus_dap_agg_init_unpack_host", "janus_dap_agg_job_resp_max_len",
    "janus_dap_agg_job_resp_encode_device", "janus_dap_agg_job_resp_encode_host",
)
NO_ERROR = 0xFF  # prepare_error value meaning "no DAP-level error for this report"


class Layout(C.Structure):
    _fields_ = [("n", C.c_uint32), ("query_type", C.c_uint8), ("batch_id", C.c_uint8 * 32),
                ("agg_param_off", C.c_uint64), ("agg_param_len", C.c_uint64),
                ("list_off", C.c_uint64), ("list_len", C.c_uint64), ("record_len", C.c_uint32),
                ("public_share_len", C.c_uint32), ("enc_len", C.c_uint32),
                ("payload_len", C.c_uint32), ("message_len", C.c_uint32),
                ("prep_share_len", C.c_uint32), ("uniform", C.c_int)]


_bound = False


def _lib():
    global _bound
    L = load_library()
    if not _bound:
        vp, u32 = C.c_void_p, C.c_uint32
        L.janus_dap_agg_init_scan.argtypes = [vp, C.c_size_t, C.POINTER(Layout)]
        L.janus_dap_agg_init_scan_ex.argtypes = [vp, C.c_size_t, u32, u32, u32, C.POINTER(Layout)]
        L.janus_dap_agg_init_unpack_device.argtypes = [C.POINTER(Layout), vp, vp, vp, vp, vp, vp,
                                                       vp, vp, u32, vp, vp, vp, vp]
        L.janus_dap_agg_init_unpack_host.argtypes = [vp, C.c_size_t, C.POINTER(Layout), u32, vp,
                                                     vp, vp, vp, vp, vp, vp, u32, vp, vp]
        L.janus_dap_agg_init_unpack_host.restype = C.c_int64
        L.janus_dap_agg_job_resp_max_len.argtypes = [u32, u32]
        L.janus_dap_agg_job_resp_max_len.restype = C.c_size_t
        L.janus_dap_agg_job_resp_encode_device.argtypes = [u32, vp, vp, vp, vp, u32, vp, vp, vp,
                                                           vp]
        L.janus_dap_agg_job_resp_encode_host.argtypes = [u32, vp, vp, vp, vp, u32, vp]
        L.janus_dap_agg_job_resp_encode_host.restype = C.c_int64
        _bound = True
    return L


LEN_ANY = 0xFFFFFFFF


def scan(body: bytes, public_share_len=None, enc_len=None, prep_share_len=None) -> Layout:
    """Layout of an AggregationJobInitializeReq body.  With the task's expected lengths (VDAF
    public share, KEM Nenc, VDAF leader prep share) every record is checked against those, so a
    malformed first record fails alone (janus_dap_agg_init_scan_ex); without them the first
    record's lengths are taken."""
    lay = Layout()
    buf = np.frombuffer(body, np.uint8)
    if public_share_len is None and enc_len is None and prep_share_len is None:
        rc = _lib().janus_dap_agg_init_scan(_np_ptr(buf), len(body), C.byref(lay))
    else:
        v = lambda x: LEN_ANY if x is None else int(x)
        rc = _lib().janus_dap_agg_init_scan_ex(_np_ptr(buf), len(body), v(public_share_len),
                                               v(enc_len), v(prep_share_len), C.byref(lay))
    if rc:
        raise ValueError("AggregationJobInitializeReq does not decode")
    return lay


INVALID_MESSAGE = 8  # DAP PrepareError::InvalidMessage


def prepare_error(hpke_status, msg_status):
    """Per-report DAP PrepareError for the response encoder: the HPKE opener's error first, then
    a public share that does not decode (msg_status 6 -> InvalidMessage, aggregator.rs:1985-1999),
    else NO_ERROR (the prio3 status decides).  numpy arrays or torch tensors."""
    try:
        import torch
        if isinstance(hpke_status, torch.Tensor):
            pe = torch.where(msg_status == 6, torch.full_like(hpke_status, INVALID_MESSAGE),
                             torch.full_like(hpke_status, NO_ERROR))
            return torch.where(hpke_status != 0, hpke_status, pe)
    except ImportError:
        pass
    hs = np.asarray(hpke_status, np.uint8)
    pe = np.where(np.asarray(msg_status) == 6, INVALID_MESSAGE, NO_ERROR).astype(np.uint8)
    return np.where(hs != 0, hs, pe).astype(np.uint8)


def ct_stride_for(lay: Layout, slack: int = 0) -> int:
    return max(16, -(-(lay.payload_len + slack) // 16) * 16)


def unpack_host(body: bytes, lay: Layout, cap: int, ct_stride: int):
    buf = np.frombuffer(body, np.uint8)
    out = dict(report_ids=np.zeros((cap, 16), np.uint8), times=np.zeros(cap, np.uint64),
               public_shares=np.zeros((cap, lay.public_share_len), np.uint8),
               config_ids=np.zeros(cap, np.uint8), enc=np.zeros((cap, lay.enc_len), np.uint8),
               ct=np.zeros((cap, ct_stride), np.uint8), ct_len=np.zeros(cap, np.uint32),
               prep_shares=np.zeros((cap, lay.prep_share_len), np.uint8),
               msg_status=np.zeros(cap, np.uint8))
    n = _lib().janus_dap_agg_init_unpack_host(
        _np_ptr(buf), len(body), C.byref(lay), cap, _np_ptr(out["report_ids"]),
        _np_ptr(out["times"]), _np_ptr(out["public_shares"]), _np_ptr(out["config_ids"]),
        _np_ptr(out["enc"]), _np_ptr(out["ct"]), _np_ptr(out["ct_len"]), ct_stride,
        _np_ptr(out["prep_shares"]), _np_ptr(out["msg_status"]))
    if n < 0:
        raise ValueError("AggregationJobInitializeReq does not decode")
    return {k: v[:n] for k, v in out.items()}


def unpack_device(lay: Layout, d_body, ct_stride: int, stream=None):
    """d_body: uint8 torch tensor (padded by >= 4 bytes) on the GPU. Returns (dict of tensors,
    mismatch count); mismatch > 0 means the body is not uniform -> use unpack_host."""
    import torch
    dev = d_body.device
    n = lay.n
    u8 = dict(dtype=torch.uint8, device=dev)
    out = dict(report_ids=torch.empty((n, 16), **u8),
               times=torch.empty(n, dtype=torch.int64, device=dev),
               public_shares=torch.empty((n, max(lay.public_share_len, 1)), **u8),
               config_ids=torch.empty(n, **u8), enc=torch.empty((n, max(lay.enc_len, 1)), **u8),
               ct=torch.zeros((n, ct_stride), **u8),
               ct_len=torch.empty(n, dtype=torch.int32, device=dev),
               prep_shares=torch.empty((n, max(lay.prep_share_len, 1)), **u8),
               msg_status=torch.empty(n, **u8))
    mism = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = _lib().janus_dap_agg_init_unpack_device(
        C.byref(lay), _tptr(d_body), _tptr(out["report_ids"]), _tptr(out["times"]),
        _tptr(out["public_shares"]) if lay.public_share_len else None, _tptr(out["config_ids"]),
        _tptr(out["enc"]), _tptr(out["ct"]), _tptr(out["ct_len"]), ct_stride,
        _tptr(out["prep_shares"]), _tptr(out["msg_status"]), _tptr(mism),
        _stream(stream, dev.index or 0))
    if rc:
        raise RuntimeError(f"janus_dap_agg_init_unpack_device failed (rc={rc})")
    return out, mism


def encode_resp_host(report_ids, prepare_error, prio3_status, prep_msgs, prep_msg_len: int):
    ids = np.ascontiguousarray(report_ids, np.uint8)
    n = ids.shape[0]
    pe = np.ascontiguousarray(prepare_error, np.uint8)
    st = np.ascontiguousarray(prio3_status, np.uint8)
    pm = np.ascontiguousarray(prep_msgs, np.uint8) if prep_msg_len else None
    out = np.zeros(_lib().janus_dap_agg_job_resp_max_len(n, prep_msg_len), np.uint8)
    ln = _lib().janus_dap_agg_job_resp_encode_host(n, _np_ptr(ids), _np_ptr(pe), _np_ptr(st),
                                                   _np_ptr(pm), prep_msg_len, _np_ptr(out))
    return out[:ln].tobytes()


def encode_resp_device(report_ids, prepare_error, prio3_status, prep_msgs, prep_msg_len: int,
                       stream=None):
    """torch tensors on the GPU -> (out tensor, length tensor)."""
    import torch
    dev = report_ids.device
    n = report_ids.shape[0]
    out = torch.empty(_lib().janus_dap_agg_job_resp_max_len(n, prep_msg_len), dtype=torch.uint8,
                      device=dev)
    ln = torch.zeros(1, dtype=torch.int64, device=dev)
    scratch = torch.empty(n // 256 + 2, dtype=torch.int32, device=dev)
    rc = _lib().janus_dap_agg_job_resp_encode_device(
        n, _tptr(report_ids), _tptr(prepare_error), _tptr(prio3_status),
        _tptr(prep_msgs) if prep_msg_len else None, prep_msg_len, _tptr(out), _tptr(ln),
        _tptr(scratch), _stream(stream, dev.index or 0))
    if rc:
        raise RuntimeError(f"janus_dap_agg_job_resp_encode_device failed (rc={rc})")
    return out, ln
