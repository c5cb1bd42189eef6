"""Ping-pong framing bytes, pinned by the reference's codec tests
(/root/reference/messages/src/tests/aggregation.rs:96-268)."""
import pytest

from janus_amd.pingpong import CONTINUE, FINISH, INITIALIZE, PingPongMessage


def test_initialize_bytes():
    # messages/src/tests/aggregation.rs:146-153: "00" type, "00000006" len, "303132333435"
    m = PingPongMessage(INITIALIZE, prep_share=b"012345")
    assert m.encode().hex() == "00" + "00000006" + "303132333435"
    assert len(m.encode()) == 0x0B  # outer "0000000b" length
    assert PingPongMessage.decode(m.encode()) == m


def test_finish_empty_bytes():
    # aggregation.rs:196-204: "00000005" length, "02", "00000000"
    m = PingPongMessage(FINISH, prep_msg=b"")
    assert m.encode().hex() == "02" + "00000000"
    assert len(m.encode()) == 5


def test_continue_bytes():
    # aggregation.rs:219-233: "00000013" length, "01", prep_msg "012345", prep_share "6789"
    m = PingPongMessage(CONTINUE, prep_msg=b"012345", prep_share=b"6789")
    assert m.encode().hex() == "01" + "00000006" + "303132333435" + "00000004" + "36373839"
    assert len(m.encode()) == 0x13
    assert PingPongMessage.decode(m.encode()) == m


@pytest.mark.parametrize("raw", [b"", b"\x03\x00\x00\x00\x00", b"\x00\x00\x00\x00\x05ab",
                                 b"\x02\x00\x00\x00\x00\x00"])
def test_malformed_rejected(raw):
    with pytest.raises(ValueError):
        PingPongMessage.decode(raw)


def test_status_labels_cover_error_rs():
    from janus_amd import prio3 as J
    # error.rs:379-411 helper-role labels
    assert J.STATUS_METRIC_LABEL[J.STATUS_PREP_INIT] == "prepare_init_failure"
    assert J.STATUS_METRIC_LABEL[J.STATUS_PREP_MSG] == "prepare_message_failure"
    assert J.STATUS_METRIC_LABEL[J.STATUS_PREP_NEXT] == "prepare_next_failure"
    assert J.STATUS_METRIC_LABEL[J.STATUS_PREP_SHARE_DECODE] == "leader_prep_share_decode_failure"
