"""Oracle restatement of the token server's wire codec against byte layouts derived from the reference's
own writers and decoders (no Java here, so the vectors are hand-derived from the Java text):

  request  DefaultRequestEntityWriter.writeHead  writeInt(id), writeByte(type)   (cli/codec/DefaultRequestEntityWriter.java:49-51)
           FlowRequestDataWriter.writeTo         writeLong(flowId), writeInt(count), writeBoolean(priority)
  decode   DefaultRequestEntityDecoder.decode    >= 5 bytes, readInt, readByte   (srv/server/codec/DefaultRequestEntityDecoder.java:36-58)
           FlowRequestDataDecoder.decode         >= 12 bytes, readLong, readInt, readBoolean if a byte is left (:31-43)
  response LengthFieldPrepender(2) + DefaultResponseEntityWriter.writeHead (writeInt id, writeByte type, writeByte
           status) + FlowResponseDataWriter.writeTo (writeInt remaining, writeInt waitInMs); the client-side
           FlowResponseDataDecoderTest reads the same two ints back (remaining 12, wait 13).
"""
import struct

import numpy as np

from codec_frames import flow_frame, pack, random_frames
from oracle import binding
from sentinel_amd import abi

FLOW_IDS = np.array([111, 222, 10_000_001, 2**62 + 5], np.int64)


def _decode(frames, flow_ids=FLOW_IDS, t0=1_700_000_000_000):
    payload, offsets = pack(frames)
    ts = t0 + np.arange(len(frames), dtype=np.int64)
    return binding.codec_decode_flow(payload, offsets, ts, flow_ids)


def test_flow_request_fields():
    req, xid, kind = _decode([flow_frame(7, 222, 3, True), flow_frame(-1, 2**62 + 5, 1, False)])
    assert list(kind) == [abi.FRAME_FLOW, abi.FRAME_FLOW]
    assert list(xid) == [7, -1]
    assert req["key"][0] == (1 | abi.KEY_PRIO) and req["acquire"][0] == 3
    assert req["key"][1] == 3 and req["acquire"][1] == 1
    assert list(req["ts_ms"]) == [1_700_000_000_000, 1_700_000_000_001]


def test_byte_layout_is_big_endian():
    frame = flow_frame(0x01020304, 0x0A0B0C0D0E0F1011, 0x7F000001, True)
    assert frame == bytes([1, 2, 3, 4, 1, 0x0A, 0x0B, 0x0C, 0x0D, 0x0E, 0x0F, 0x10, 0x11, 0x7F, 0, 0, 1, 1])
    req, xid, kind = _decode([frame], flow_ids=np.array([0x0A0B0C0D0E0F1011], np.int64))
    assert xid[0] == 0x01020304 and req["key"][0] == (0 | abi.KEY_PRIO) and req["acquire"][0] == 0x7F000001


def test_lookup_and_validation():
    req, _, kind = _decode([flow_frame(1, 999, 1, False),   # unknown flowId → NO_RULE_EXISTS
                            flow_frame(2, 0, 1, False),     # flowId <= 0 → BAD_REQUEST
                            flow_frame(3, -7, 1, True),
                            flow_frame(4, 111, 0, False)])  # count <= 0: the engine's prep answers BAD_REQUEST
    assert list(kind) == [abi.FRAME_FLOW] * 4
    assert req["key"][0] == abi.KEY_NO_RULE
    assert req["key"][1] == abi.KEY_BAD and req["key"][2] == (abi.KEY_BAD | abi.KEY_PRIO)
    assert req["key"][3] == 0 and req["acquire"][3] == 0


def test_malformed_frames():
    frames = [b"", b"\x00\x00\x00", struct.pack(">iB", 5, 1),                 # short; flow without body
              struct.pack(">iB", 6, 1) + bytes(11),                            # 11 body bytes: decoder returns null
              struct.pack(">iB", 7, 0),                                        # ping
              struct.pack(">iB", 8, 2) + bytes(20),                            # param flow
              flow_frame(9, 111, 2, None),                                     # no priority byte → false
              flow_frame(10, 111, 2, True, trailing=b"\xff\xff")]              # trailing bytes ignored
    req, xid, kind = _decode(frames)
    assert list(kind) == [abi.FRAME_SHORT, abi.FRAME_SHORT, abi.FRAME_NO_DATA, abi.FRAME_NO_DATA,
                          abi.FRAME_OTHER, abi.FRAME_OTHER, abi.FRAME_FLOW, abi.FRAME_FLOW]
    assert list(xid) == [0, 0, 5, 6, 7, 8, 9, 10]
    assert all(req["key"][:6] == abi.KEY_BAD) and all(req["acquire"][:6] == 0)
    assert req["key"][6] == 0 and req["key"][7] == abi.KEY_PRIO


def test_response_frames():
    xid = np.array([0x01020304, -2, 5, 6], np.int32)
    kind = np.array([abi.FRAME_FLOW, abi.FRAME_FLOW, abi.FRAME_FLOW, abi.FRAME_OTHER], np.uint8)
    res = np.zeros(4, abi.RES_DTYPE)
    res[0] = (abi.OK, 12, 13)
    res[1] = (abi.BAD_REQUEST, 0, 0)
    res[2] = (abi.SHOULD_WAIT, 0, 100)
    out = binding.codec_encode_flow(xid, kind, res).reshape(4, 16)
    assert bytes(out[0]) == struct.pack(">HiBbii", 14, 0x01020304, 1, 0, 12, 13)
    assert bytes(out[1]) == struct.pack(">HiBbii", 14, -2, 1, -4, 0, 0)   # writeByte(-4) = 0xFC
    assert bytes(out[2]) == struct.pack(">HiBbii", 14, 5, 1, 2, 0, 100)
    assert not out[3].any()
    # the client's FlowResponseDataDecoder reads remaining, wait back (FlowResponseDataDecoderTest: 12, 13)
    assert struct.unpack(">ii", bytes(out[0][8:16])) == (12, 13)


def test_random_frames_against_python_restatement():
    rng = np.random.default_rng(5)
    frames = random_frames(3000, FLOW_IDS, rng, bad_frac=0.2)
    req, xid, kind = _decode(frames)
    index = {int(f): i for i, f in enumerate(FLOW_IDS)}
    for i, f in enumerate(frames):
        if len(f) < 5:
            assert kind[i] == abi.FRAME_SHORT
            continue
        x, t = struct.unpack(">ib", f[:5])
        assert xid[i] == x
        if t != 1:
            assert kind[i] == abi.FRAME_OTHER
        elif len(f) - 5 < 12:
            assert kind[i] == abi.FRAME_NO_DATA
        else:
            fid, cnt = struct.unpack(">qi", f[5:17])
            prio = len(f) > 17 and f[17] != 0
            key = abi.KEY_BAD if fid <= 0 else index.get(fid, abi.KEY_NO_RULE)
            assert kind[i] == abi.FRAME_FLOW and req["acquire"][i] == cnt
            assert req["key"][i] == (key | (abi.KEY_PRIO if prio else 0))
