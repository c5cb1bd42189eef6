"""Ping-pong topology framing around the batched helper engine.

Mirrors prio 0.16.2 ``topology::ping_pong`` as Janus drives it on the helper:
``vdaf.helper_initialized(verify_key, &agg_param, nonce, &public_share, &input_share,
prepare_init.message())`` then ``.evaluate(&vdaf)``
(/root/reference/aggregator/src/aggregator.rs:2022-2031).  Wire format of a
``PingPongMessage`` (pinned by /root/reference/messages/src/tests/aggregation.rs:96-268):
    Initialize{prep_share}          = 0x00 || u32be(len) || prep_share
    Continue{prep_msg, prep_share}  = 0x01 || u32be(len) || prep_msg || u32be(len) || prep_share
    Finish{prep_msg}                = 0x02 || u32be(len) || prep_msg
Inside a DAP ``PrepareInit``/``PrepareResp`` the message carries an outer u32be length.

Error precedence follows ``helper_initialized``: prepare_init first (VdafPrepareInit),
then the inbound message type (PeerMessageMismatch), then decoding the leader's prepare
share (CodecPrepShare), then prepare_shares_to_prepare_message, then prepare_next.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import prio3 as P

INITIALIZE, CONTINUE, FINISH = 0, 1, 2


@dataclass(frozen=True)
class PingPongMessage:
    kind: int
    prep_share: bytes = b""
    prep_msg: bytes = b""

    def encode(self) -> bytes:
        if self.kind == INITIALIZE:
            return bytes([0]) + struct.pack(">I", len(self.prep_share)) + self.prep_share
        if self.kind == CONTINUE:
            return (bytes([1]) + struct.pack(">I", len(self.prep_msg)) + self.prep_msg +
                    struct.pack(">I", len(self.prep_share)) + self.prep_share)
        if self.kind == FINISH:
            return bytes([2]) + struct.pack(">I", len(self.prep_msg)) + self.prep_msg
        raise ValueError("unknown ping-pong message type")

    @staticmethod
    def decode(buf: bytes) -> "PingPongMessage":
        def opaque(b, off):
            if off + 4 > len(b):
                raise ValueError("short ping-pong message")
            (n,) = struct.unpack(">I", b[off:off + 4])
            if off + 4 + n > len(b):
                raise ValueError("short ping-pong message")
            return b[off + 4:off + 4 + n], off + 4 + n

        if not buf:
            raise ValueError("empty ping-pong message")
        t = buf[0]
        if t == INITIALIZE:
            ps, off = opaque(buf, 1)
            msg = PingPongMessage(INITIALIZE, prep_share=ps)
        elif t == CONTINUE:
            pm, off = opaque(buf, 1)
            ps, off = opaque(buf, off)
            msg = PingPongMessage(CONTINUE, prep_share=ps, prep_msg=pm)
        elif t == FINISH:
            pm, off = opaque(buf, 1)
            msg = PingPongMessage(FINISH, prep_msg=pm)
        else:
            raise ValueError("unknown ping-pong message type")
        if off != len(buf):
            raise ValueError("trailing bytes after ping-pong message")
        return msg

    @property
    def variant(self) -> str:
        return {INITIALIZE: "initialize", CONTINUE: "continue", FINISH: "finish"}[self.kind]


@dataclass
class HelperResult:
    status: int                       # P.STATUS_*
    outgoing: Optional[bytes]         # encoded PingPongMessage::Finish on success
    error: Optional[str] = None       # PingPongError variant name on failure
    metric_label: Optional[str] = None  # janus_step_failures{type=...}


def helper_initialized_batch(engine: "P.HelperEngine", nonces: np.ndarray,
                             public_shares: np.ndarray, helper_shares: np.ndarray,
                             inbound: Sequence[bytes]):
    """Batched ``helper_initialized(..).evaluate(..)`` for Prio3 (one round).

    ``inbound`` holds each report's encoded PingPongMessage from the leader.  Returns
    (results, batch) where ``batch.accumulate`` merges the finished output shares.
    """
    sz = engine.sz
    n = len(inbound)
    lps = np.zeros((n, sz.prep_share_len), np.uint8)
    host_status = np.zeros(n, np.uint8)
    for i, raw in enumerate(inbound):
        try:
            msg = PingPongMessage.decode(bytes(raw))
        except ValueError:
            host_status[i] = P.STATUS_PEER_MISMATCH
            continue
        if msg.kind != INITIALIZE:
            host_status[i] = P.STATUS_PEER_MISMATCH
        elif len(msg.prep_share) != sz.prep_share_len:
            host_status[i] = P.STATUS_PREP_SHARE_DECODE
        else:
            lps[i] = np.frombuffer(msg.prep_share, np.uint8)
    msgs, dev_status, batch = engine.prepare_batch(nonces, public_shares, helper_shares, lps)
    status = dev_status.copy()
    # prepare_init failures take precedence over the inbound-message checks
    override = (host_status != 0) & (dev_status != P.STATUS_PREP_INIT)
    status[override] = host_status[override]
    results: List[HelperResult] = []
    for i in range(n):
        s = int(status[i])
        if s == P.STATUS_FINISHED:
            out = PingPongMessage(FINISH, prep_msg=msgs[i].tobytes()).encode()
            results.append(HelperResult(s, out))
        else:
            results.append(HelperResult(s, None, P.STATUS_PINGPONG_ERROR[s],
                                        P.STATUS_METRIC_LABEL[s]))
    batch.status_override = status
    return results, batch, status
