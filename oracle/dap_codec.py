"""Pure-Python restatement of the DAP-09 encodings the helper's aggregation-job init reads and
writes -- TEST INFRASTRUCTURE (the checker of janus_amd's device/host codec).

Follows /root/reference/messages/src/lib.rs: ReportMetadata (1257-1300), HpkeCiphertext
(955-1020), ReportShare (1958-2020), PrepareInit (2021-2070), PartialBatchSelector (1652-1680),
AggregationJobInitializeReq (2362-2400), PrepareStepResult / PrepareError (2130-2190),
PrepareResp (2072-2128), AggregationJobResp (2535-2550); PingPongMessage framing per
messages/src/tests/aggregation.rs:96-268 (type 0 Initialize{prep_share}, 1 Continue{prep_msg,
prep_share}, 2 Finish{prep_msg}, each field u32-prefixed).
"""
from __future__ import annotations

import struct


class DecodeError(Exception):
    pass


class _R:
    def __init__(self, b):
        self.b, self.o = b, 0

    def take(self, k):
        if self.o + k > len(self.b):
            raise DecodeError("short")
        v = self.b[self.o:self.o + k]
        self.o += k
        return v

    def u8(self):
        return self.take(1)[0]

    def u16(self):
        return struct.unpack(">H", self.take(2))[0]

    def u32(self):
        return struct.unpack(">I", self.take(4))[0]

    def u64(self):
        return struct.unpack(">Q", self.take(8))[0]


def decode_ping_pong(b: bytes):
    r = _R(b)
    t = r.u8()
    if t == 0:
        m = dict(type="initialize", prep_share=r.take(r.u32()))
    elif t == 1:
        m = dict(type="continue", prep_msg=r.take(r.u32()), prep_share=r.take(r.u32()))
    elif t == 2:
        m = dict(type="finish", prep_msg=r.take(r.u32()))
    else:
        raise DecodeError("ping-pong type")
    if r.o != len(b):
        raise DecodeError("trailing")
    return m


def decode_agg_init_req(b: bytes):
    r = _R(b)
    agg_param = r.take(r.u32())
    qt = r.u8()
    if qt == 1:
        batch_id = None
    elif qt == 2:
        batch_id = r.take(32)
    else:
        raise DecodeError("query type")
    ln = r.u32()
    end = r.o + ln
    if end != len(b):
        raise DecodeError("length")
    inits = []
    while r.o < end:
        rid = r.take(16)
        t = r.u64()
        pub = r.take(r.u32())
        cfg = r.u8()
        enc = r.take(r.u16())
        payload = r.take(r.u32())
        msg = decode_ping_pong(r.take(r.u32()))
        inits.append(dict(report_id=rid, time=t, public_share=pub, config_id=cfg, enc=enc,
                          payload=payload, message=msg))
    if r.o != end:
        raise DecodeError("list")
    return dict(aggregation_parameter=agg_param, query_type=qt, batch_id=batch_id,
                prepare_inits=inits)


def encode_ping_pong(m) -> bytes:
    if m["type"] == "initialize":
        return b"\x00" + struct.pack(">I", len(m["prep_share"])) + m["prep_share"]
    if m["type"] == "continue":
        return (b"\x01" + struct.pack(">I", len(m["prep_msg"])) + m["prep_msg"] +
                struct.pack(">I", len(m["prep_share"])) + m["prep_share"])
    return b"\x02" + struct.pack(">I", len(m["prep_msg"])) + m["prep_msg"]


def encode_prepare_resp(report_id: bytes, result) -> bytes:
    """result: ("continue", message) | ("finished",) | ("reject", code)"""
    if result[0] == "continue":
        msg = encode_ping_pong(result[1])
        return report_id + b"\x00" + struct.pack(">I", len(msg)) + msg
    if result[0] == "finished":
        return report_id + b"\x01"
    return report_id + b"\x02" + bytes([result[1]])


def encode_agg_job_resp(resps) -> bytes:
    body = b"".join(encode_prepare_resp(rid, res) for rid, res in resps)
    return struct.pack(">I", len(body)) + body


def encode_agg_init_req(agg_param: bytes, query_type: int, batch_id, inits) -> bytes:
    out = struct.pack(">I", len(agg_param)) + agg_param + bytes([query_type])
    if query_type == 2:
        out += batch_id
    body = b""
    for p in inits:
        msg = encode_ping_pong(p["message"])
        body += (p["report_id"] + struct.pack(">Q", p["time"]) +
                 struct.pack(">I", len(p["public_share"])) + p["public_share"] +
                 bytes([p["config_id"]]) + struct.pack(">H", len(p["enc"])) + p["enc"] +
                 struct.pack(">I", len(p["payload"])) + p["payload"] +
                 struct.pack(">I", len(msg)) + msg)
    return out + struct.pack(">I", len(body)) + body


def helper_init_resp(report_ids, prepare_error, prio3_status, prep_msgs) -> bytes:
    """The helper's AggregationJobResp for init (aggregator.rs:2044-2069): Continue(Finish) for
    finished reports, Reject(PrepareError) otherwise (VdafPrepError for ping-pong errors)."""
    resps = []
    for i, rid in enumerate(report_ids):
        if prepare_error[i] != 0xFF:
            res = ("reject", int(prepare_error[i]))
        elif prio3_status[i] == 0:
            res = ("continue", dict(type="finish", prep_msg=bytes(prep_msgs[i])))
        else:
            res = ("reject", 5)
        resps.append((bytes(rid), res))
    return encode_agg_job_resp(resps)
