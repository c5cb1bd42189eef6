"""Host-side mirror of the prio 0.16.2 ``Prio3`` aggregator surface that Janus uses on the
helper's aggregate-init hot path, backed by the gfx950 HIP engine (``libjanus_prio3.so``).

Reference surface being mirrored:
  * instance constructors ``Prio3::new_count / new_sum / new_sum_vec_multithreaded /
    new_histogram`` as dispatched by ``vdaf_dispatch!`` (/root/reference/core/src/vdaf.rs:198-300);
  * the per-report ``helper_initialized(..) + evaluate(..)`` call inside
    ``handle_aggregate_init_generic`` (/root/reference/aggregator/src/aggregator.rs:2020-2042),
    here batched over the whole job;
  * ``AggregateShare::merge`` accumulation performed by ``AggregationJobWriter``
    (/root/reference/aggregator/src/aggregator/aggregation_job_writer.rs:591-695).

There is no CPU fallback: if the HIP library is missing or no GPU is present, engine
creation raises.  (The CPU restatement under ``oracle/`` is test infrastructure only.)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# JANUS_PRIO3_LIB selects an alternative build of the same sources (A/B experiments,
# tools/build_variant.sh); the default is the in-tree library built by `make -C janus_amd`.
LIB_PATH = os.environ.get("JANUS_PRIO3_LIB") or os.path.join(_HERE, "libjanus_prio3.so")

PRIO3_COUNT, PRIO3_SUM, PRIO3_SUMVEC, PRIO3_HISTOGRAM, PRIO3_SUMVEC_F64_MP = 0, 1, 2, 3, 4
PRIO3_FPVEC_BOUNDED_L2 = 5

STATUS_FINISHED = 0
STATUS_PREP_INIT = 1
STATUS_PREP_SHARE_DECODE = 2
STATUS_PREP_MSG = 3
STATUS_PREP_NEXT = 4
STATUS_PEER_MISMATCH = 5
STATUS_INPUT_SHARE_DECODE = 6
#: merged statuses of prio3_helper_aggregate_init_batch: 0x80 | the DAP PrepareError of a report
#: the input-share open rejected before its VDAF ran (aggregator.rs:1847-1983)
STATUS_HPKE_DECRYPT = 0x84
STATUS_INVALID_MESSAGE = 0x88

#: prio ``PingPongError`` variant for each status (error.rs:365-428 maps these to labels).
STATUS_PINGPONG_ERROR = {
    STATUS_PREP_INIT: "VdafPrepareInit",
    STATUS_PREP_SHARE_DECODE: "CodecPrepShare",
    STATUS_PREP_MSG: "VdafPrepareSharesToPrepareMessage",
    STATUS_PREP_NEXT: "VdafPrepareNext",
    STATUS_PEER_MISMATCH: "PeerMessageMismatch",
    STATUS_INPUT_SHARE_DECODE: "InvalidMessage",
}

#: ``janus_step_failures{type=...}`` metric label per status, helper role
#: (handle_ping_pong_error, /root/reference/aggregator/src/aggregator/error.rs:379-411).
STATUS_METRIC_LABEL = {
    STATUS_PREP_INIT: "prepare_init_failure",
    STATUS_PREP_SHARE_DECODE: "leader_prep_share_decode_failure",
    STATUS_PREP_MSG: "prepare_message_failure",
    STATUS_PREP_NEXT: "prepare_next_failure",
    STATUS_PEER_MISMATCH: "leader_ping_pong_message_mismatch",
}


class Prio3Params(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("bits", C.c_uint32), ("length", C.c_uint32),
                ("chunk_length", C.c_uint32), ("num_proofs", C.c_uint32)]


class Prio3MemberInfo(C.Structure):
    _fields_ = [("device", C.c_int32), ("lane", C.c_uint32), ("jobs", C.c_uint64),
                ("reports", C.c_uint64), ("exec_jobs", C.c_uint64), ("exec_groups", C.c_uint64)]


class Prio3ExecutorStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("jobs", "reports", "groups", "active_jobs",
                                          "active_reports")]


#: executor kinds of prio3_executor_stats_get
EXEC_PREPARE, EXEC_ACCUMULATE, EXEC_LEADER_INIT, EXEC_LEADER_NEXT = 0, 1, 2, 3


class Prio3Sizes(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "field_bytes", "meas_len", "out_len", "proof_len", "verifier_len", "joint_rand_len",
        "nonce_len", "public_share_len", "helper_share_len", "prep_share_len", "prep_msg_len",
        "agg_share_len", "leader_input_share_len")]


#: Every symbol include/janus_prio3.h declares.
EXPORTED_SYMBOLS = (
    "prio3_sizes", "prio3_engine_create", "prio3_engine_destroy", "prio3_helper_prepare_batch",
    "prio3_helper_prepare_aggregate_batch",
    "prio3_accumulate", "prio3_debug_output_shares", "prio3_batch_free", "prio3_device_prepare",
    "prio3_device_accumulate", "prio3_device_output_shares", "prio3_device_combine",
    "prio3_engine_set_option", "prio3_engine_timing", "prio3_engine_timing_reset",
    "prio3_client_generate_device", "prio3_selftest_field", "prio3_trace_enabled", "prio3_device_prepare_aggregate",
    "prio3_device_trim",
    "prio3_device_aggregate_finish", "prio3_leader_prepare_init_batch",
    "prio3_leader_prepare_next_batch", "prio3_device_leader_prepare_init",
    "prio3_device_leader_prepare_next", "prio3_device_batch_metadata", "prio3_batch_metadata",
    "prio3_device_combine_metadata", "prio3_engine_create_ex", "prio3_engine_create_mask",
    "prio3_engine_create_devices", "prio3_engine_members", "prio3_executor_control",
    "prio3_executor_stats_get", "prio3_helper_aggregate_init_batch",
    "prio3_leader_prepare_next_aggregate_batch",
)
# include/janus_hpke.h (the batched HPKE opener, janus_amd/hpke.py)
HPKE_EXPORTED_SYMBOLS = (
    "janus_hpke_opener_create", "janus_hpke_opener_destroy",
    "janus_hpke_open_input_shares_device", "janus_hpke_open_input_shares",
    "janus_hpke_open_device", "janus_hpke_open", "janus_hpke_set_timing", "janus_hpke_timing",
    "janus_hpke_selftest_p256", "janus_hpke_selftest_field", "janus_hpke_executor_stats_get",
    "janus_hpke_executor_control",
)

_lib = None


def load_library() -> C.CDLL:
    """Load the in-tree HIP engine; raise loudly if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"janus_amd HIP engine not built: {LIB_PATH} is missing "
                          "(run `make -C janus_amd` or __graft_entry__.build())")
    # One HIP runtime per process: when PyTorch-ROCm is present its bundled libamdhip64
    # (SONAME libamdhip64.so.7) must be the copy our NEEDED entry binds to, otherwise two HSA
    # runtimes coexist and the second one sees no GPU.  Importing torch first makes the
    # dynamic linker reuse torch's runtime for libjanus_prio3.so.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    # RTLD_GLOBAL: the native jobs harness (libjanus_jobs.so, linked against libjanus_prio3.so)
    # then binds to this same copy, also when JANUS_PRIO3_LIB selects an A/B build -- one engine
    # library (one set of executors) per process
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    P, u8p, vp = C.POINTER, C.POINTER(C.c_uint8), C.c_void_p
    L.prio3_sizes.argtypes = [P(Prio3Params), P(Prio3Sizes)]
    L.prio3_engine_create.argtypes = [P(Prio3Params), u8p, C.c_int, P(vp)]
    L.prio3_engine_create_ex.argtypes = [P(Prio3Params), u8p, C.c_size_t, C.c_int, P(vp)]
    L.prio3_engine_create_mask.argtypes = [P(Prio3Params), u8p, C.c_size_t, C.c_int, P(vp)]
    L.prio3_engine_create_devices.argtypes = [P(Prio3Params), u8p, C.c_size_t, P(C.c_int),
                                              C.c_uint32, P(vp)]
    L.prio3_engine_members.argtypes = [vp, P(Prio3MemberInfo), C.c_uint32]
    L.prio3_executor_control.argtypes = [vp, C.c_int, C.c_char_p, C.c_int64]
    L.prio3_executor_stats_get.argtypes = [vp, C.c_uint32, C.c_int, P(Prio3ExecutorStats)]
    L.prio3_engine_destroy.argtypes = [vp]
    L.prio3_engine_destroy.restype = None
    L.prio3_helper_prepare_batch.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, vp, vp, P(vp)]
    L.prio3_accumulate.argtypes = [vp, vp, vp, C.c_uint32, vp, vp]
    L.prio3_helper_prepare_aggregate_batch.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, vp, vp,
                                                       C.c_uint32, vp, vp, vp, vp]
    u32 = C.c_uint32
    L.prio3_helper_aggregate_init_batch.argtypes = [vp, vp, u32, vp, C.c_int, vp, vp, vp, vp, vp,
                                                    vp, u32, vp, vp, vp, u32, vp, vp, vp, vp]
    L.prio3_debug_output_shares.argtypes = [vp, vp]
    L.prio3_batch_free.argtypes = [vp]
    L.prio3_batch_free.restype = None
    L.prio3_device_prepare.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, vp, vp, vp]
    L.prio3_device_accumulate.argtypes = [vp, C.c_uint32, vp, vp, vp, C.c_uint32, vp, vp, vp]
    L.prio3_device_output_shares.argtypes = [vp, C.c_uint32, vp]
    L.prio3_device_combine.argtypes = [vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp, vp]
    L.prio3_client_generate_device.argtypes = [vp, C.c_uint32, C.c_uint64, C.c_uint64, vp, vp,
                                               vp, vp, vp, vp, vp, vp, vp]
    L.prio3_engine_set_option.argtypes = [vp, C.c_char_p, C.c_int64]
    L.prio3_engine_timing.argtypes = [vp, C.c_char_p, C.c_size_t, P(C.c_double),
                                      P(C.c_uint64), C.c_int]
    L.prio3_engine_timing_reset.argtypes = [vp]
    L.prio3_engine_timing_reset.restype = None
    L.prio3_selftest_field.argtypes = [C.c_int, C.c_uint32, vp, vp, vp]
    L.prio3_trace_enabled.argtypes = []
    L.prio3_device_trim.argtypes = [C.c_int]
    L.prio3_device_prepare_aggregate.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, vp, C.c_uint32,
                                                 vp, vp, vp]
    L.prio3_device_aggregate_finish.argtypes = [vp, vp, vp, vp, vp, vp]
    L.prio3_leader_prepare_init_batch.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, vp, P(vp)]
    L.prio3_leader_prepare_next_batch.argtypes = [vp, vp, vp]
    L.prio3_leader_prepare_next_aggregate_batch.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, vp,
                                                            vp]
    L.prio3_device_leader_prepare_init.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, vp, vp]
    L.prio3_device_leader_prepare_next.argtypes = [vp, C.c_uint32, vp, vp, vp]
    L.prio3_device_batch_metadata.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, vp, C.c_uint32, vp,
                                              vp, vp]
    L.prio3_batch_metadata.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, vp, C.c_uint32, vp, vp]
    L.prio3_device_combine_metadata.argtypes = [vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp, vp]
    _lib = L
    return L


def trim_device_pool(device: int = 0) -> None:
    """Free the idle scratch slabs the engine keeps on `device` (prio3_device_trim)."""
    rc = load_library().prio3_device_trim(device)
    if rc:
        raise RuntimeError(f"prio3_device_trim failed (rc={rc})")


def selftest_field(op: int, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Test hook: device Field128 primitive ``op`` over uint8 [m, 16] operands (see header)."""
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    n = a.shape[0] // (16 if op >= 4 else 1)
    out = np.zeros((n, 16), np.uint8)
    rc = load_library().prio3_selftest_field(op, n, _np_ptr(a), _np_ptr(b), _np_ptr(out))
    if rc:
        raise RuntimeError(f"prio3_selftest_field failed (rc={rc})")
    return out


# ------------------------------------------------------------------------------------
# VDAF instances (mirrors of prio's constructors; names follow core/src/vdaf.rs)
# ------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Prio3:
    kind: int
    bits: int = 0
    length: int = 0
    chunk_length: int = 0
    num_proofs: int = 1

    def params(self) -> Prio3Params:
        return Prio3Params(self.kind, self.bits, self.length, self.chunk_length, self.num_proofs)

    def sizes(self) -> Prio3Sizes:
        s = Prio3Sizes()
        rc = load_library().prio3_sizes(C.byref(self.params()), C.byref(s))
        if rc:
            raise ValueError(f"unsupported Prio3 parameters (rc={rc})")
        return s


def Prio3Count() -> Prio3:
    return Prio3(PRIO3_COUNT)


def Prio3Sum(bits: int) -> Prio3:
    return Prio3(PRIO3_SUM, bits=bits)


def Prio3SumVec(bits: int, length: int, chunk_length: int) -> Prio3:
    return Prio3(PRIO3_SUMVEC, bits=bits, length=length, chunk_length=chunk_length)


def Prio3SumVecField64MultiproofHmacSha256Aes128(proofs: int, bits: int, length: int,
                                                 chunk_length: int) -> Prio3:
    """janus_core::vdaf::new_prio3_sum_vec_field64_multiproof_hmacsha256_aes128
    (core/src/vdaf.rs:173-195): 32-byte verify key and seeds, proofs >= 2."""
    if proofs < 2:
        raise ValueError("Must use at least two proofs with Field64")
    return Prio3(PRIO3_SUMVEC_F64_MP, bits, length, chunk_length, proofs)


def Prio3Histogram(length: int, chunk_length: int) -> Prio3:
    return Prio3(PRIO3_HISTOGRAM, length=length, chunk_length=chunk_length)


def Prio3FixedPointBoundedL2VecSum(length: int, bitsize: int = 16) -> Prio3:
    """Prio3::new_fixedpoint_boundedl2_vec_sum_multithreaded(2, length) with FixedI16<U15>
    (bitsize 16) or FixedI32<U31> (bitsize 32) (core/src/vdaf.rs:292-335).  Helper role; the
    circuit is the reconstruction in oracle/fpvec_py.py."""
    if bitsize not in (16, 32):
        raise ValueError("bitsize must be 16 or 32 (Prio3FixedPointBoundedL2VecSumBitSize)")
    return Prio3(PRIO3_FPVEC_BOUNDED_L2, bits=bitsize, length=length)


def _np_ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _tptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(stream, device):
    """Device-resident calls default to torch's current stream on the engine's device, so they
    are ordered after the torch ops that produced their inputs (a handle of 0 is HIP's null
    stream, which the C-ABI takes as such)."""
    if stream:
        return C.c_void_p(stream)
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream or None)


def _seg_accept(n, segment_ids, accept_mask, n_segments):
    """The C ABI reads n segment ids and n accept bytes (janus_prio3.h): a shorter array would be
    a host over-read inside the library, so the length contract is checked here."""
    seg = None if segment_ids is None else np.ascontiguousarray(segment_ids, np.uint32)
    acc = None if accept_mask is None else np.ascontiguousarray(accept_mask, np.uint8)
    if seg is not None and seg.shape != (n,):
        raise ValueError(f"segment_ids must have shape ({n},), got {seg.shape}")
    if acc is not None and acc.shape != (n,):
        raise ValueError(f"accept_mask must have shape ({n},), got {acc.shape}")
    if n_segments < 1:
        raise ValueError("n_segments must be >= 1")
    return seg, acc


class PreparedBatch:
    """Device-resident output shares of one ``prepare_batch`` call (prio3_batch*)."""

    def __init__(self, engine: "HelperEngine", handle: C.c_void_p, n: int):
        self.engine, self.handle, self.n = engine, handle, n

    def accumulate(self, segment_ids=None, accept_mask=None, n_segments: int = 1):
        sz = self.engine.sz
        agg = np.zeros((n_segments, sz.agg_share_len), np.uint8)
        cnt = np.zeros(n_segments, np.uint64)
        seg, acc = _seg_accept(self.n, segment_ids, accept_mask, n_segments)
        rc = load_library().prio3_accumulate(self.handle, _np_ptr(seg), _np_ptr(acc), n_segments,
                                             _np_ptr(agg), _np_ptr(cnt))
        if rc:
            raise RuntimeError(f"prio3_accumulate failed (rc={rc})")
        return agg, cnt

    def leader_prepare_next(self, prep_msgs, status) -> np.ndarray:
        """Leader ``prepare_next`` on the helper's prepare messages (leader_continued,
        aggregation_job_driver.rs:677-691); returns the updated per-report status."""
        st = np.array(status, np.uint8, copy=True)
        msgs = None
        if self.engine.sz.prep_msg_len:
            msgs = np.ascontiguousarray(prep_msgs, np.uint8)
            if msgs.shape != (self.n, self.engine.sz.prep_msg_len):
                raise ValueError("prepare message shape does not match the VDAF instance")
        rc = load_library().prio3_leader_prepare_next_batch(self.handle, _np_ptr(msgs),
                                                            _np_ptr(st))
        if rc:
            raise RuntimeError(f"prio3_leader_prepare_next_batch failed (rc={rc})")
        return st

    def leader_prepare_next_aggregate(self, prep_msgs, status, segment_ids=None,
                                      accept_mask=None, n_segments: int = 1):
        """``leader_prepare_next`` + ``accumulate`` in one launch of the prepare_next executor
        (prio3_leader_prepare_next_aggregate_batch).  Returns (status, agg [S, agg_len],
        counts [S])."""
        st = np.array(status, np.uint8, copy=True)
        msgs = None
        if self.engine.sz.prep_msg_len:
            msgs = np.ascontiguousarray(prep_msgs, np.uint8)
            if msgs.shape != (self.n, self.engine.sz.prep_msg_len):
                raise ValueError("prepare message shape does not match the VDAF instance")
        seg, acc = _seg_accept(self.n, segment_ids, accept_mask, n_segments)
        agg = np.zeros((n_segments, self.engine.sz.agg_share_len), np.uint8)
        cnt = np.zeros(n_segments, np.uint64)
        rc = load_library().prio3_leader_prepare_next_aggregate_batch(
            self.handle, _np_ptr(msgs), _np_ptr(st), _np_ptr(seg), _np_ptr(acc), n_segments,
            _np_ptr(agg), _np_ptr(cnt))
        if rc:
            raise RuntimeError(f"prio3_leader_prepare_next_aggregate_batch failed (rc={rc})")
        return st, agg, cnt

    def output_shares(self) -> np.ndarray:
        out = np.zeros((self.n, self.engine.sz.agg_share_len), np.uint8)
        rc = load_library().prio3_debug_output_shares(self.handle, _np_ptr(out))
        if rc:
            raise RuntimeError(f"prio3_debug_output_shares failed (rc={rc})")
        return out

    def free(self):
        if self.handle:
            load_library().prio3_batch_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HelperEngine:
    """One engine per (Prio3 instance, verify key) -- created where Janus builds ``VdafOps`` for
    a task (aggregator.rs:880-988) -- on one GPU (``device``), on the GPUs of ``device_mask``
    (bit d = GPU d; jobs placed whole on the least-loaded GPU, prio3_engine_create_mask), or on
    an explicit ``devices`` list (a GPU listed k times gets k executors: the one-GPU rehearsal
    of that placement)."""

    def __init__(self, vdaf: Prio3, verify_key: bytes, device: int = 0,
                 allow_unpinned: bool = False, device_mask: Optional[int] = None,
                 devices: Optional[list] = None):
        """allow_unpinned: required for Prio3FixedPointBoundedL2VecSum, whose circuit is a
        reconstruction with parity against prio unpinned (engine option experimental_fpvec)."""
        vk_len = 32 if vdaf.kind == PRIO3_SUMVEC_F64_MP else 16
        if len(verify_key) != vk_len:
            raise ValueError(f"verify key must be {vk_len} bytes (VERIFY_KEY_LENGTH[_HMACSHA256_"
                             "AES128], core/src/vdaf.rs)")
        L = load_library()
        self.sz = vdaf.sizes()
        h = C.c_void_p()
        vk = (C.c_uint8 * vk_len).from_buffer_copy(verify_key)
        if devices is not None:
            arr = (C.c_int * len(devices))(*devices)
            device = devices[0]
            rc = L.prio3_engine_create_devices(C.byref(vdaf.params()), vk, vk_len, arr,
                                               len(devices), C.byref(h))
        elif device_mask is not None:
            device = (device_mask & -device_mask).bit_length() - 1
            rc = L.prio3_engine_create_mask(C.byref(vdaf.params()), vk, vk_len, device_mask,
                                            C.byref(h))
        else:
            rc = L.prio3_engine_create_ex(C.byref(vdaf.params()), vk, vk_len, device, C.byref(h))
        self.vdaf, self.device = vdaf, device
        if rc:
            raise RuntimeError(f"prio3_engine_create failed (rc={rc}); a GPU is required")
        self.handle = h
        if vdaf.kind == PRIO3_FPVEC_BOUNDED_L2 and allow_unpinned:
            self.set_option("experimental_fpvec", 1)

    def close(self):
        if getattr(self, "handle", None):
            load_library().prio3_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, key: str, value: int):
        rc = load_library().prio3_engine_set_option(self.handle, key.encode(), int(value))
        if rc:
            raise ValueError(f"unknown option {key}")

    def members(self) -> list:
        """Per-GPU placement of this engine's host-buffer jobs (prio3_engine_members): one dict
        per member with device, lane, jobs, reports, and its executor's exec_jobs / exec_groups."""
        L = load_library()
        k = L.prio3_engine_members(self.handle, None, 0)
        if k < 0:
            raise RuntimeError(f"prio3_engine_members failed (rc={k})")
        arr = (Prio3MemberInfo * k)()
        L.prio3_engine_members(self.handle, arr, k)
        return [{f: getattr(m, f) for f, _ in Prio3MemberInfo._fields_} for m in arr]

    def executor_stats(self, kind: int = EXEC_PREPARE, member: int = 0) -> dict:
        """Counters of the executor of `kind` that member `member`'s jobs use."""
        st = Prio3ExecutorStats()
        rc = load_library().prio3_executor_stats_get(self.handle, member, kind, C.byref(st))
        if rc:
            raise RuntimeError(f"prio3_executor_stats_get failed (rc={rc})")
        return {f: getattr(st, f) for f, _ in Prio3ExecutorStats._fields_}

    def executor_control(self, key: str, value: int, kind: int = -1):
        """prio3_executor_control on the executors of `kind` (-1: all): "hold" (tests queue jobs
        behind it), "heavy" (load switch)."""
        rc = load_library().prio3_executor_control(self.handle, kind, key.encode(), int(value))
        if rc:
            raise ValueError(f"executor control {key} failed (rc={rc})")

    # ---- host-buffer path -----------------------------------------------------------
    def prepare_batch(self, nonces, public_shares, helper_shares, leader_prep_shares):
        """Batched helper prepare_init -> prepare_shares_to_prepare_message -> prepare_next.

        Arrays are uint8 [n, len].  Returns (prep_msgs [n, prep_msg_len], status [n], batch).
        """
        sz = self.sz
        nonces = np.ascontiguousarray(nonces, np.uint8)
        n = nonces.shape[0]
        helper_shares = np.ascontiguousarray(helper_shares, np.uint8)
        leader_prep_shares = np.ascontiguousarray(leader_prep_shares, np.uint8)
        if helper_shares.shape != (n, sz.helper_share_len) or \
                leader_prep_shares.shape != (n, sz.prep_share_len):
            raise ValueError("input share shapes do not match the VDAF instance")
        pub = None
        if sz.public_share_len:
            pub = np.ascontiguousarray(public_shares, np.uint8)
            if pub.shape != (n, sz.public_share_len):
                raise ValueError("public share shape does not match the VDAF instance")
        msgs = np.zeros((n, max(sz.prep_msg_len, 1)), np.uint8)
        status = np.zeros(n, np.uint8)
        bh = C.c_void_p()
        rc = load_library().prio3_helper_prepare_batch(
            self.handle, n, _np_ptr(nonces), _np_ptr(pub), _np_ptr(helper_shares),
            _np_ptr(leader_prep_shares), _np_ptr(msgs), _np_ptr(status), C.byref(bh))
        if rc:
            raise RuntimeError(f"prio3_helper_prepare_batch failed (rc={rc})")
        return msgs[:, :sz.prep_msg_len], status, PreparedBatch(self, bh, n)

    def prepare_aggregate_batch(self, nonces, public_shares, helper_shares, leader_prep_shares,
                                segment_ids=None, accept_mask=None, n_segments: int = 1):
        """prepare_batch + accumulate of the same reports in one coalesced launch
        (prio3_helper_prepare_aggregate_batch).  Returns (prep_msgs, status, agg [S, agg_len],
        counts [S])."""
        sz = self.sz
        nonces = np.ascontiguousarray(nonces, np.uint8)
        n = nonces.shape[0]
        helper_shares = np.ascontiguousarray(helper_shares, np.uint8)
        leader_prep_shares = np.ascontiguousarray(leader_prep_shares, np.uint8)
        if helper_shares.shape != (n, sz.helper_share_len) or \
                leader_prep_shares.shape != (n, sz.prep_share_len):
            raise ValueError("input share shapes do not match the VDAF instance")
        pub = None
        if sz.public_share_len:
            pub = np.ascontiguousarray(public_shares, np.uint8)
            if pub.shape != (n, sz.public_share_len):
                raise ValueError("public share shape does not match the VDAF instance")
        seg, acc = _seg_accept(n, segment_ids, accept_mask, n_segments)
        msgs = np.zeros((n, max(sz.prep_msg_len, 1)), np.uint8)
        status = np.zeros(n, np.uint8)
        agg = np.zeros((n_segments, sz.agg_share_len), np.uint8)
        cnt = np.zeros(n_segments, np.uint64)
        rc = load_library().prio3_helper_prepare_aggregate_batch(
            self.handle, n, _np_ptr(nonces), _np_ptr(pub), _np_ptr(helper_shares),
            _np_ptr(leader_prep_shares), _np_ptr(seg), _np_ptr(acc), n_segments, _np_ptr(msgs),
            _np_ptr(status), _np_ptr(agg), _np_ptr(cnt))
        if rc:
            raise RuntimeError(f"prio3_helper_prepare_aggregate_batch failed (rc={rc})")
        return msgs[:, :sz.prep_msg_len], status, agg, cnt

    def aggregate_init_batch(self, opener, task_id: bytes, report_ids, times, public_shares,
                             enc, ct, ct_len, leader_prep_shares, segment_ids=None,
                             accept_mask=None, n_segments: int = 1, require_taskprov=False):
        """The helper's whole loop body for one job from the sealed input shares
        (prio3_helper_aggregate_init_batch; aggregator.rs:1794-2096): HPKE open with ``opener``
        (janus_amd.hpke.HpkeOpener), decode, prepare and accumulate in one coalesced launch.
        enc [n, Nenc], ct [n, ct_stride] (stride a multiple of 16), ct_len [n].  Returns
        (prep_msgs, status [merged: STATUS_* or STATUS_HPKE_DECRYPT / STATUS_INVALID_MESSAGE],
        agg [S, agg_len], counts [S])."""
        sz = self.sz
        ids = np.ascontiguousarray(report_ids, np.uint8)
        n = ids.shape[0]
        t = np.ascontiguousarray(times, np.uint64)
        e = np.ascontiguousarray(enc, np.uint8)
        c = np.ascontiguousarray(ct, np.uint8)
        cl = np.ascontiguousarray(ct_len, np.uint32)
        lps = np.ascontiguousarray(leader_prep_shares, np.uint8)
        if ids.shape != (n, 16) or t.shape != (n,) or cl.shape != (n,) or c.ndim != 2 or \
                c.shape[0] != n or e.shape[0] != n or lps.shape != (n, sz.prep_share_len):
            raise ValueError("input shapes do not match the job")
        if len(task_id) != 32:
            raise ValueError("task_id must be 32 bytes")
        pub = None
        if sz.public_share_len:
            pub = np.ascontiguousarray(public_shares, np.uint8)
            if pub.shape != (n, sz.public_share_len):
                raise ValueError("public share shape does not match the VDAF instance")
        seg, acc = _seg_accept(n, segment_ids, accept_mask, n_segments)
        msgs = np.zeros((n, max(sz.prep_msg_len, 1)), np.uint8)
        status = np.zeros(n, np.uint8)
        agg = np.zeros((n_segments, sz.agg_share_len), np.uint8)
        cnt = np.zeros(n_segments, np.uint64)
        tid = (C.c_uint8 * 32).from_buffer_copy(task_id)
        rc = load_library().prio3_helper_aggregate_init_batch(
            self.handle, opener.handle, n, tid, int(bool(require_taskprov)), _np_ptr(ids),
            _np_ptr(t), _np_ptr(pub), _np_ptr(e), _np_ptr(c), _np_ptr(cl), c.shape[1],
            _np_ptr(lps), _np_ptr(seg), _np_ptr(acc), n_segments, _np_ptr(msgs), _np_ptr(status),
            _np_ptr(agg), _np_ptr(cnt))
        if rc:
            raise RuntimeError(f"prio3_helper_aggregate_init_batch failed (rc={rc})")
        return msgs[:, :sz.prep_msg_len], status, agg, cnt

    # ---- leader side (same instance, agg_id 0) -----------------------------------
    def leader_prepare_init_batch(self, nonces, public_shares, leader_input_shares):
        """Batched leader prepare_init (leader_initialized, aggregation_job_driver.rs:397-415).

        Returns (prep_shares [n, prep_share_len], status [n], batch); the batch's
        ``leader_prepare_next`` then takes the helper's prepare messages."""
        sz = self.sz
        nonces = np.ascontiguousarray(nonces, np.uint8)
        n = nonces.shape[0]
        ls = np.ascontiguousarray(leader_input_shares, np.uint8)
        if ls.shape != (n, sz.leader_input_share_len):
            raise ValueError("leader input share shape does not match the VDAF instance")
        pub = None
        if sz.public_share_len:
            pub = np.ascontiguousarray(public_shares, np.uint8)
            if pub.shape != (n, sz.public_share_len):
                raise ValueError("public share shape does not match the VDAF instance")
        ps = np.zeros((n, sz.prep_share_len), np.uint8)
        status = np.zeros(n, np.uint8)
        bh = C.c_void_p()
        rc = load_library().prio3_leader_prepare_init_batch(
            self.handle, n, _np_ptr(nonces), _np_ptr(pub), _np_ptr(ls), _np_ptr(ps),
            _np_ptr(status), C.byref(bh))
        if rc:
            raise RuntimeError(f"prio3_leader_prepare_init_batch failed (rc={rc})")
        return ps, status, PreparedBatch(self, bh, n)

    def leader_prepare_init_device(self, nonces, public_shares, leader_input_shares, prep_shares,
                                   status, stream=None) -> None:
        rc = load_library().prio3_device_leader_prepare_init(
            self.handle, nonces.shape[0], _tptr(nonces), _tptr(public_shares),
            _tptr(leader_input_shares), _tptr(prep_shares), _tptr(status),
            _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_leader_prepare_init failed (rc={rc})")

    def leader_prepare_next_device(self, n, prep_msgs, status, stream=None) -> None:
        rc = load_library().prio3_device_leader_prepare_next(
            self.handle, n, _tptr(prep_msgs), _tptr(status), _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_leader_prepare_next failed (rc={rc})")

    # ---- device-resident path (torch tensors on this engine's GPU) ------------------
    def prepare_device(self, nonces, public_shares, helper_shares, leader_prep_shares,
                       prep_msgs, status, stream=None) -> None:
        rc = load_library().prio3_device_prepare(
            self.handle, nonces.shape[0], _tptr(nonces), _tptr(public_shares),
            _tptr(helper_shares), _tptr(leader_prep_shares), _tptr(prep_msgs), _tptr(status),
            _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_prepare failed (rc={rc})")

    def prepare_aggregate_device(self, nonces, public_shares, helper_shares, leader_prep_shares,
                                 segment_ids, n_segments, prep_msgs, status, stream=None) -> None:
        """Prepare and aggregate in one pass (torch tensors on this engine's GPU)."""
        rc = load_library().prio3_device_prepare_aggregate(
            self.handle, nonces.shape[0], _tptr(nonces), _tptr(public_shares),
            _tptr(helper_shares), _tptr(leader_prep_shares), _tptr(segment_ids), n_segments,
            _tptr(prep_msgs), _tptr(status), _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_prepare_aggregate failed (rc={rc})")

    def aggregate_finish_device(self, status, accept_mask, agg, counts, stream=None) -> None:
        rc = load_library().prio3_device_aggregate_finish(
            self.handle, _tptr(status), _tptr(accept_mask), _tptr(agg), _tptr(counts),
            _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_aggregate_finish failed (rc={rc})")

    def accumulate_device(self, n, status, segment_ids, accept_mask, n_segments, agg, counts,
                          stream=None) -> None:
        rc = load_library().prio3_device_accumulate(
            self.handle, n, _tptr(status), _tptr(segment_ids), _tptr(accept_mask), n_segments,
            _tptr(agg), _tptr(counts), _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_accumulate failed (rc={rc})")

    def combine_device(self, k, n_segments, parts, part_counts, out, out_counts,
                       stream=None) -> None:
        rc = load_library().prio3_device_combine(
            self.handle, k, n_segments, _tptr(parts), _tptr(part_counts), _tptr(out),
            _tptr(out_counts), _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_combine failed (rc={rc})")

    def batch_metadata_device(self, report_ids, times, status, accept_mask, segment_ids,
                              n_segments, checksums, intervals, stream=None) -> None:
        """Per-segment ReportIdChecksum [n_segments, 32] (uint8) and client-timestamp interval
        [n_segments, 2] (int64 start, duration) of the batch (torch tensors on this GPU)."""
        rc = load_library().prio3_device_batch_metadata(
            self.handle, status.shape[0], _tptr(report_ids), _tptr(times), _tptr(status),
            _tptr(accept_mask), _tptr(segment_ids), n_segments, _tptr(checksums),
            _tptr(intervals), _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_batch_metadata failed (rc={rc})")

    def combine_metadata_device(self, k, n_segments, checksums_in, intervals_in, checksums,
                                intervals, stream=None) -> None:
        rc = load_library().prio3_device_combine_metadata(
            self.handle, k, n_segments, _tptr(checksums_in), _tptr(intervals_in),
            _tptr(checksums), _tptr(intervals), _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_device_combine_metadata failed (rc={rc})")

    def batch_metadata(self, report_ids, times, status, accept_mask=None, segment_ids=None,
                       n_segments: int = 1):
        """Host-buffer form: returns (checksums uint8 [S, 32], intervals uint64 [S, 2])."""
        ids = np.ascontiguousarray(report_ids, np.uint8)
        n = ids.shape[0]
        st = np.ascontiguousarray(status, np.uint8)
        if ids.shape != (n, 16) or st.shape != (n,):
            raise ValueError("report_ids must be [n, 16] and status [n]")
        t = None if times is None else np.ascontiguousarray(times, np.uint64)
        m = None if accept_mask is None else np.ascontiguousarray(accept_mask, np.uint8)
        sg = None if segment_ids is None else np.ascontiguousarray(segment_ids, np.uint32)
        ck = np.zeros((n_segments, 32), np.uint8)
        iv = np.zeros((n_segments, 2), np.uint64)
        rc = load_library().prio3_batch_metadata(
            self.handle, n, _np_ptr(ids), _np_ptr(t), _np_ptr(st), _np_ptr(m), _np_ptr(sg),
            n_segments, _np_ptr(ck), _np_ptr(iv))
        if rc:
            raise RuntimeError(f"prio3_batch_metadata failed (rc={rc})")
        return ck, iv

    def device_output_shares(self, n: int) -> np.ndarray:
        out = np.zeros((n, self.sz.agg_share_len), np.uint8)
        rc = load_library().prio3_device_output_shares(self.handle, n, _np_ptr(out))
        if rc:
            raise RuntimeError("prio3_device_output_shares failed")
        return out

    # ---- synthetic client ------------------------------------------------------------
    def generate_reports_device(self, n: int, seed: int = 1, first_index: int = 0,
                                with_checks: bool = False, with_leader_inputs: bool = False,
                                stream=None) -> dict:
        """Honest synthetic reports generated on the GPU (shard + leader prepare_init).

        Returns torch uint8 tensors on this engine's device (plus measurements / leader
        output shares / flags when ``with_checks``).  Every TurboSHAKE instance, including
        FixedPointBoundedL2VecSum (its prover runs on the device too; the engine needs the
        allow_unpinned opt-in), and the HMAC-SHA256/AES-128 multiproof VDAF.  Report i is
        derived from (seed, first_index + i) exactly as oracle's generators derive it."""
        import torch
        sz = self.sz
        dev = torch.device("cuda", self.device)
        u8 = dict(dtype=torch.uint8, device=dev)
        out = dict(nonces=torch.empty((n, 16), **u8),
                   public_shares=torch.empty((n, max(sz.public_share_len, 1)), **u8),
                   helper_shares=torch.empty((n, sz.helper_share_len), **u8),
                   leader_prep_shares=torch.empty((n, sz.prep_share_len), **u8))
        if with_checks:
            # SumVec: the entries; FPVec: the signed fixed-point entries X (x = X / 2^(bits-1))
            mstride = (self.vdaf.length if self.vdaf.kind in (PRIO3_SUMVEC, PRIO3_FPVEC_BOUNDED_L2,
                                                              PRIO3_SUMVEC_F64_MP) else 1)
            out["measurements"] = torch.empty((n, mstride), dtype=torch.int64, device=dev)
            out["leader_out_shares"] = torch.empty((n, sz.agg_share_len), **u8)
            out["flags"] = torch.zeros(n, **u8)
        if with_leader_inputs:
            out["leader_input_shares"] = torch.empty((n, sz.leader_input_share_len), **u8)
        rc = load_library().prio3_client_generate_device(
            self.handle, n, seed, first_index, _tptr(out["nonces"]),
            _tptr(out["public_shares"]) if sz.public_share_len else None,
            _tptr(out["helper_shares"]), _tptr(out["leader_prep_shares"]),
            _tptr(out.get("measurements")), _tptr(out.get("leader_out_shares")),
            _tptr(out.get("flags")), _tptr(out.get("leader_input_shares")),
            _stream(stream, self.device))
        if rc:
            raise RuntimeError(f"prio3_client_generate_device failed (rc={rc})")
        if not sz.public_share_len:
            out["public_shares"] = out["public_shares"][:, :0]
        return out

    # ---- measurement ----------------------------------------------------------------
    def timing(self) -> dict:
        names = C.create_string_buffer(4096)
        ms = (C.c_double * 64)()
        launches = (C.c_uint64 * 64)()
        k = load_library().prio3_engine_timing(self.handle, names, 4096, ms, launches, 64)
        keys = names.value.decode().split(",") if k else []
        return {keys[i]: (ms[i], int(launches[i])) for i in range(min(k, 64))}

    def timing_reset(self):
        load_library().prio3_engine_timing_reset(self.handle)
