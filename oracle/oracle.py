"""ctypes binding of the C restatement (oracle/prio3_oracle.c) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product path (janus_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libprio3_oracle.so")

KINDS = {"count": 0, "sum": 1, "sumvec": 2, "histogram": 3, "fpvec": 4, "sumvec_f64_mp": 5}


class OrcParams(C.Structure):
    _fields_ = [(n, C.c_int if n == "type" else C.c_uint32) for n in [
        "type", "bits", "length", "chunk_length", "num_proofs", "algorithm_id",
        "field_bits", "es", "meas_len", "out_len", "jr_len", "qr_len", "prove_rand_len",
        "arity", "degree", "calls", "wire_len", "proof_len", "verifier_len",
        "helper_share_len", "public_share_len", "leader_share_len", "prep_share_len",
        "prep_msg_len", "out_share_bytes", "fp_C1", "fp_K1", "fp_P1", "seed_size", "xof_hm"]]


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or \
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "prio3_oracle.c")):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.POINTER
        u8p = P(C.c_uint8)
        L.orc_params_init.argtypes = [P(OrcParams), C.c_int, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_uint32]
        L.orc_turboshake128.argtypes = [u8p, C.c_size_t, C.c_uint8, u8p, C.c_size_t]
        L.orc_shake128.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t]
        L.orc_keccak_p1600.argtypes = [P(C.c_uint64), C.c_int]
        L.orc_shard.argtypes = [P(OrcParams), P(C.c_uint64), u8p, u8p, u8p, u8p, u8p]
        L.orc_prepare_init.argtypes = [P(OrcParams), u8p, C.c_int, u8p, u8p, u8p, u8p, u8p]
        L.orc_prep_shares_to_prep_msg.argtypes = [P(OrcParams), u8p, u8p, u8p]
        L.orc_prepare_next.argtypes = [P(OrcParams), u8p, u8p, u8p]
        L.orc_helper_trace.argtypes = [P(OrcParams), u8p, u8p, u8p, u8p] + [u8p] * 7
        L.orc_helper_batch.argtypes = [P(OrcParams), u8p, C.c_uint32, u8p, u8p, u8p, u8p,
                                       P(C.c_uint32), u8p, C.c_uint32, u8p, u8p, u8p,
                                       P(C.c_uint64), C.c_int, C.c_int]
        L.orc_leader_batch.argtypes = [P(OrcParams), u8p, C.c_uint32, u8p, u8p, u8p, u8p, u8p,
                                       u8p, u8p, P(C.c_uint64), C.c_int, C.c_int]
        L.orc_leader_batch_seg.argtypes = [P(OrcParams), u8p, C.c_uint32, u8p, u8p, u8p, u8p,
                                           P(C.c_uint32), C.c_uint32, u8p, u8p, u8p,
                                           P(C.c_uint64), C.c_int, C.c_int]
        L.orc_agg_merge.argtypes = [P(OrcParams), u8p, u8p]
        L.orc_gen_reports.argtypes = [P(OrcParams), u8p, C.c_uint32, C.c_uint64, C.c_int,
                                      u8p, u8p, u8p, u8p, P(C.c_uint64), u8p]
        L.orc_prim_bench.argtypes = [P(C.c_double), P(C.c_double)]
        _lib = L
    return _lib


def _buf(b) -> C.Array:
    return (C.c_uint8 * max(len(b), 1)).from_buffer_copy(bytes(b) if len(b) else b"\0")


def _out(n):
    return (C.c_uint8 * max(n, 1))()


def _ptr(a: np.ndarray, ctype=C.c_uint8):
    return a.ctypes.data_as(C.POINTER(ctype)) if a is not None else None


def turboshake128(msg: bytes, domain: int, n: int) -> bytes:
    o = _out(n)
    lib().orc_turboshake128(_buf(msg), len(msg), domain, o, n)
    return bytes(o)[:n]


def shake128(msg: bytes, n: int) -> bytes:
    o = _out(n)
    lib().orc_shake128(_buf(msg), len(msg), o, n)
    return bytes(o)[:n]


@dataclass
class Oracle:
    """One Prio3 instance (mirrors prio's Prio3 constructors used by core/src/vdaf.rs:198-300)."""
    kind: str
    bits: int = 0
    length: int = 0
    chunk_length: int = 0
    num_proofs: int = 1

    def __post_init__(self):
        self.p = OrcParams()
        rc = lib().orc_params_init(C.byref(self.p), KINDS[self.kind], self.bits, self.length,
                                   self.chunk_length, self.num_proofs)
        if rc:
            raise ValueError("invalid Prio3 parameters")

    def __getattr__(self, name):
        if name != "p" and "p" in self.__dict__ and name in dict(OrcParams._fields_):
            return getattr(self.__dict__["p"], name)
        raise AttributeError(name)

    @property
    def rand_size(self):
        return 16 * (5 if self.p.jr_len else 3)

    def shard(self, measurement, nonce: bytes, rand: bytes):
        m = measurement if isinstance(measurement, (list, tuple)) else [measurement]
        arr = (C.c_uint64 * len(m))(*m)
        pub, ls, hs = _out(self.p.public_share_len), _out(self.p.leader_share_len), \
            _out(self.p.helper_share_len)
        rc = lib().orc_shard(C.byref(self.p), arr, _buf(nonce), _buf(rand), pub, ls, hs)
        if rc:
            raise ValueError("invalid measurement")
        return (bytes(pub)[:self.p.public_share_len], bytes(ls)[:self.p.leader_share_len],
                bytes(hs)[:self.p.helper_share_len])

    def prepare_init(self, vk, agg_id, nonce, public, share):
        st = _out(self.p.meas_len * self.p.es + 16)
        ps = _out(self.p.prep_share_len)
        rc = lib().orc_prepare_init(C.byref(self.p), _buf(vk), agg_id, _buf(nonce), _buf(public),
                                    _buf(share), st, ps)
        return rc, bytes(st), bytes(ps)[:self.p.prep_share_len]

    def prep_shares_to_prep_msg(self, leader_ps, helper_ps):
        m = _out(16)
        rc = lib().orc_prep_shares_to_prep_msg(C.byref(self.p), _buf(leader_ps), _buf(helper_ps),
                                               m)
        return rc, bytes(m)[:self.p.prep_msg_len]

    def prepare_next(self, state, msg):
        o = _out(self.p.out_share_bytes)
        rc = lib().orc_prepare_next(C.byref(self.p), _buf(state), _buf(msg if msg else b"\0" * 16),
                                    o)
        return rc, bytes(o)[:self.p.out_share_bytes]

    def helper_trace(self, vk, nonce, public, helper_share):
        p = self.p
        bufs = dict(meas=_out(p.meas_len * p.es), proofs=_out(p.proof_len * p.num_proofs * p.es),
                    part=_out(16), corrected=_out(16), jr=_out(max(p.jr_len, 1) * 8 * p.es),
                    qr=_out(8 * p.es), verifiers=_out(p.verifier_len * p.num_proofs * p.es))
        rc = lib().orc_helper_trace(C.byref(p), _buf(vk), _buf(nonce), _buf(public),
                                    _buf(helper_share), bufs["meas"], bufs["proofs"],
                                    bufs["part"], bufs["corrected"], bufs["jr"], bufs["qr"],
                                    bufs["verifiers"])
        lens = dict(meas=p.meas_len * p.es, proofs=p.proof_len * p.num_proofs * p.es,
                    part=16 if p.jr_len else 0, corrected=16 if p.jr_len else 0,
                    jr=p.jr_len * p.num_proofs * p.es, qr=p.num_proofs * p.es,
                    verifiers=p.verifier_len * p.num_proofs * p.es)
        return rc, {k: bytes(v)[:lens[k]] for k, v in bufs.items()}

    def helper_batch(self, vk: bytes, nonces: np.ndarray, public_shares, helper_shares,
                     leader_prep_shares, segment_ids=None, accept_mask=None, n_segments=1,
                     n_threads=1, job_size=500):
        """Batched helper prepare+aggregate (Janus job structure); arrays are uint8 [n, len]."""
        p = self.p
        n = nonces.shape[0]
        msgs = np.zeros((n, max(p.prep_msg_len, 1)), np.uint8)
        status = np.zeros(n, np.uint8)
        agg = np.zeros((n_segments, p.out_share_bytes), np.uint8)
        cnt = np.zeros(n_segments, np.uint64)
        seg = None if segment_ids is None else np.ascontiguousarray(segment_ids, np.uint32)
        acc = None if accept_mask is None else np.ascontiguousarray(accept_mask, np.uint8)
        pub = None if p.public_share_len == 0 else np.ascontiguousarray(public_shares)
        lib().orc_helper_batch(C.byref(p), _buf(vk), n, _ptr(np.ascontiguousarray(nonces)),
                               _ptr(pub), _ptr(np.ascontiguousarray(helper_shares)),
                               _ptr(np.ascontiguousarray(leader_prep_shares)),
                               _ptr(seg, C.c_uint32), _ptr(acc), n_segments, _ptr(msgs),
                               _ptr(status), _ptr(agg), _ptr(cnt, C.c_uint64), n_threads,
                               job_size)
        return msgs[:, :p.prep_msg_len], status, agg, cnt

    def leader_batch(self, vk: bytes, nonces, public_shares, leader_shares, prep_msgs,
                     n_threads=1, job_size=500, segment_ids=None, n_segments=1):
        """Batched leader prepare_init (agg_id 0) + prepare_next + aggregate per segment:
        returns (prep_shares, status, agg [S, out], count [S]).  Status 1 = non-canonical leader
        share element (the engine reports it as 6, InputShareDecode), 4 = VdafPrepareNext."""
        p = self.p
        n = nonces.shape[0]
        ps = np.zeros((n, p.prep_share_len), np.uint8)
        status = np.zeros(n, np.uint8)
        agg = np.zeros((n_segments, p.out_share_bytes), np.uint8)
        cnt = np.zeros(n_segments, np.uint64)
        pub = None if p.public_share_len == 0 else np.ascontiguousarray(public_shares)
        msgs = None if p.prep_msg_len == 0 else np.ascontiguousarray(prep_msgs)
        seg = None if segment_ids is None else np.ascontiguousarray(segment_ids, np.uint32)
        lib().orc_leader_batch_seg(C.byref(p), _buf(vk), n, _ptr(np.ascontiguousarray(nonces)),
                                   _ptr(pub), _ptr(np.ascontiguousarray(leader_shares)),
                                   _ptr(msgs), _ptr(seg, C.c_uint32), n_segments, _ptr(ps),
                                   _ptr(status), _ptr(agg), _ptr(cnt, C.c_uint64), n_threads,
                                   job_size)
        return ps, status, agg, cnt

    def gen_reports(self, vk: bytes, n: int, seed: int = 1, n_threads: int = 8):
        """Deterministic honest reports: dict of uint8 arrays + measurements + leader out shares."""
        p = self.p
        mstride = p.length if self.kind == "sumvec" else 1
        d = dict(nonces=np.zeros((n, 16), np.uint8),
                 public_shares=np.zeros((n, max(p.public_share_len, 1)), np.uint8),
                 helper_shares=np.zeros((n, p.helper_share_len), np.uint8),
                 leader_prep_shares=np.zeros((n, p.prep_share_len), np.uint8),
                 measurements=np.zeros((n, mstride), np.uint64),
                 leader_out_shares=np.zeros((n, p.out_share_bytes), np.uint8))
        lib().orc_gen_reports(C.byref(p), _buf(vk), n, seed, n_threads, _ptr(d["nonces"]),
                              _ptr(d["public_shares"]), _ptr(d["helper_shares"]),
                              _ptr(d["leader_prep_shares"]), _ptr(d["measurements"], C.c_uint64),
                              _ptr(d["leader_out_shares"]))
        if p.public_share_len == 0:
            d["public_shares"] = np.zeros((n, 0), np.uint8)
        return d


def prim_bench():
    """(ns per Keccak-p[1600,12] permutation, ns per Field128 multiply) on one core."""
    a, b = C.c_double(), C.c_double()
    lib().orc_prim_bench(C.byref(a), C.byref(b))
    return a.value, b.value


def field_modulus(kind: str) -> int:
    return 2**64 - 2**32 + 1 if kind == "count" else 2**128 - 28 * 2**64 + 1


def decode_elems(buf: np.ndarray, es: int) -> list:
    """uint8 array (..., k*es) -> python ints, LE."""
    b = np.ascontiguousarray(buf, np.uint8).reshape(-1, es)
    return [int.from_bytes(row.tobytes(), "little") for row in b]


def sum_mod(rows: np.ndarray, es: int, p: int) -> list:
    """Element-wise mod-p sum over axis 0 of a [n, out_len*es] uint8 array."""
    n = rows.shape[0]
    k = rows.shape[1] // es
    v = np.ascontiguousarray(rows, np.uint8).reshape(n, k, es)
    acc = [0] * k
    limbs = [v[:, :, 4 * j:4 * j + 4].copy().view(np.uint32).reshape(n, k).astype(np.uint64)
             for j in range(es // 4)]
    sums = [l.sum(axis=0, dtype=np.uint64) for l in limbs]  # n < 2^32 so no overflow
    for e in range(k):
        acc[e] = sum(int(sums[j][e]) << (32 * j) for j in range(es // 4)) % p
    return acc


def batch_metadata(report_ids: np.ndarray, times, status: np.ndarray, accept_mask=None,
                   segment_ids=None, n_segments: int = 1):
    """Per-segment ReportIdChecksum and client-timestamp interval of one batch (TEST ORACLE).

    checksum[s] = XOR of SHA-256(report_id) over the reports counted in segment s (status 0 and
    accept mask non-zero): ReportIdChecksum::for_report_id / combined_with,
    /root/reference/core/src/report_id.rs:18-42, folded per report in
    aggregator/src/aggregator/aggregation_job_writer.rs:637-690.  SHA-256 is ring's
    digest::SHA256 in the reference (FIPS 180-4); hashlib computes the same function.
    interval[s] = (start, duration): Interval::from_time(t) = [t, t + 1) merged over every report
    aggregation of the segment (failed ones included), core/src/time.rs:294-317, starting from
    Interval::EMPTY = (0, 0) (BatchAggregation::new, aggregation_job_writer.rs:606-611).
    """
    import hashlib
    n = len(status)
    ck = np.zeros((n_segments, 32), np.uint8)
    lo = [None] * n_segments
    hi = [None] * n_segments
    for r in range(n):
        s = 0 if segment_ids is None else int(segment_ids[r])
        if s >= n_segments:
            continue
        if times is not None:
            t = int(times[r])
            lo[s] = t if lo[s] is None else min(lo[s], t)
            hi[s] = t + 1 if hi[s] is None else max(hi[s], t + 1)
        if status[r] == 0 and (accept_mask is None or accept_mask[r]):
            d = hashlib.sha256(bytes(report_ids[r])).digest()
            ck[s] ^= np.frombuffer(d, np.uint8)
    iv = np.zeros((n_segments, 2), np.uint64)
    for s in range(n_segments):
        if lo[s] is not None:
            iv[s] = (lo[s], hi[s] - lo[s])
    return ck, iv
