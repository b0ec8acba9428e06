"""Token-server frame builders for the codec tests: the byte layouts the reference's writers produce.

Request payload (what LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2) hands to NettyRequestDecoder):
  DefaultRequestEntityWriter.writeTo  [i32 xid][u8 type]      (cli/codec/DefaultRequestEntityWriter.java:49-51)
  FlowRequestDataWriter.writeTo       [i64 flowId][i32 count][bool priority]   (cli/codec/data/FlowRequestDataWriter.java)
Big-endian (Netty ByteBuf). The generators below also produce the malformed shapes the server decoder
tolerates (short frames, missing bodies, missing priority byte, trailing bytes, other message types).
"""
import struct

import numpy as np


def flow_frame(xid, flow_id, count, prio=None, type_=1, trailing=b""):
    body = struct.pack(">iBqi", xid, type_, flow_id, count)
    if prio is not None:
        body += struct.pack(">?", bool(prio))
    return body + trailing


def pack(frames):
    """frames (list of bytes) → (payload u8, offsets u32[n + 1])."""
    payload = np.frombuffer(b"".join(frames), np.uint8) if frames else np.zeros(0, np.uint8)
    offsets = np.zeros(len(frames) + 1, np.uint32)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    return payload, offsets


def random_frames(n, flow_ids, rng, bad_frac=0.05):
    """n frames: mostly valid flow requests (known and unknown flowIds, 1% prioritized, 10% acquire 2..4),
    plus bad_frac of every malformed kind."""
    frames = []
    known = np.asarray(flow_ids, np.int64)
    for i in range(n):
        u = rng.random()
        xid = int(rng.integers(-2**31, 2**31))
        if u < bad_frac / 6:
            frames.append(bytes(rng.integers(0, 256, int(rng.integers(0, 5)), dtype=np.uint8)))  # < 5 bytes
        elif u < 2 * bad_frac / 6:
            frames.append(struct.pack(">iB", xid, 1) + bytes(int(rng.integers(0, 12))))       # flow, no body
        elif u < 3 * bad_frac / 6:
            frames.append(struct.pack(">iB", xid, int(rng.choice([0, 2, 3, 4, 7, 200]))) + bytes(8))  # other type
        elif u < 4 * bad_frac / 6:
            frames.append(flow_frame(xid, int(rng.integers(-5, 1)), 1, 0))                    # flowId <= 0
        elif u < 5 * bad_frac / 6:
            frames.append(flow_frame(xid, int(known[rng.integers(len(known))]), int(rng.integers(-3, 1)), 0))
        elif u < bad_frac:
            frames.append(flow_frame(xid, int(known[rng.integers(len(known))]), 1, None,
                                     trailing=b""))                                            # no priority byte
        else:
            fid = int(known[rng.integers(len(known))]) if rng.random() < 0.97 else int(rng.integers(1, 2**62))
            acq = 1 if rng.random() < 0.9 else int(rng.integers(2, 5))
            prio = rng.random() < 0.01
            trailing = bytes(int(rng.integers(1, 4))) if rng.random() < 0.01 else b""
            frames.append(flow_frame(xid, fid, acq, prio, trailing=trailing))
    return frames
