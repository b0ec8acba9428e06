"""Device wire codec (sg_codec_decode_flow / sg_codec_encode_flow, codec.hip) against the oracle codec, and
the whole server step — frames → decode → sg_flow_decide_batch → encode — against the oracle pipeline
(or_codec_decode_flow → ClusterTokenService.decide → or_codec_encode_flow), byte for byte."""
import numpy as np
import pytest

from codec_frames import flow_frame, pack, random_frames
from oracle import binding
from oracle.binding import ClusterTokenService
from sentinel_amd import abi

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


@pytest.fixture(autouse=True, scope="module")
def _torch_first():
    """These tests hand torch device buffers to the library: torch's HIP runtime has to initialise before the
    library's (the order smoke() uses); initialised second it finds no device."""
    import torch
    torch.cuda.init()
    yield


def _rules(n, rng):
    r = np.zeros(n, abi.RULE_DTYPE)
    r["flow_id"] = rng.choice(np.arange(1, 50 * n, dtype=np.int64), n, replace=False) * 7919 + 3
    r["count"] = rng.integers(1, 33, n)
    r["threshold_type"] = abi.THRESHOLD_GLOBAL
    r["sample_count"] = 10
    r["window_interval_ms"] = 1000
    return r


def _ns():
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    return ns


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


def _decode_gpu(eng, payload, offsets, ts):
    import torch
    n = len(offsets) - 1
    p_t = _dev(payload if len(payload) else np.zeros(1, np.uint8))
    o_t, t_t = _dev(offsets), _dev(ts)
    req_t = torch.empty(max(n, 1) * abi.REQ_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    xid_t = torch.empty(max(n, 1) * 4, dtype=torch.uint8, device="cuda")
    kind_t = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    eng.codec_decode(p_t.data_ptr(), o_t.data_ptr(), t_t.data_ptr(), n, req_t.data_ptr(), xid_t.data_ptr(),
                     kind_t.data_ptr(), s)
    torch.cuda.synchronize()
    return req_t, xid_t, kind_t


def _engine(rules, max_batch=1 << 18):
    from sentinel_amd.engine import FlowEngine
    eng = FlowEngine(device=0, max_batch=max_batch)
    eng.set_namespaces(_ns())
    eng.load_rules(rules)
    return eng


@pytest.mark.parametrize("n,bad", [(1, 0.0), (5000, 0.3), (200_000, 0.02)])
def test_decode_matches_oracle(n, bad):
    rng = np.random.default_rng(n)
    rules = _rules(1000, rng)
    frames = random_frames(n, rules["flow_id"], rng, bad_frac=bad)
    payload, offsets = pack(frames)
    ts = T0 + np.sort(rng.integers(0, 3000, n)).astype(np.int64)
    eng = _engine(rules)
    req_t, xid_t, kind_t = _decode_gpu(eng, payload, offsets, ts)
    want_req, want_xid, want_kind = binding.codec_decode_flow(payload, offsets, ts, rules["flow_id"])
    assert np.array_equal(kind_t.cpu().numpy()[:n], want_kind)
    assert np.array_equal(xid_t.cpu().numpy().view(np.int32)[:n], want_xid)
    assert np.array_equal(req_t.cpu().numpy().view(abi.REQ_DTYPE)[:n], want_req)


def test_decode_without_rules_is_no_rule():
    from sentinel_amd.engine import FlowEngine
    eng = FlowEngine(device=0, max_batch=1024)
    payload, offsets = pack([flow_frame(1, 5, 1, False), flow_frame(2, -5, 1, True)])
    req_t, _, kind_t = _decode_gpu(eng, payload, offsets, np.array([T0, T0], np.int64))
    req = req_t.cpu().numpy().view(abi.REQ_DTYPE)
    assert list(req["key"]) == [abi.KEY_NO_RULE, abi.KEY_BAD | abi.KEY_PRIO]
    assert list(kind_t.cpu().numpy()) == [abi.FRAME_FLOW, abi.FRAME_FLOW]


def test_decode_backwards_offsets_are_short_frames():
    """A frame whose end offset lies before its start is decoded as SG_FRAME_SHORT (no read), the rest as usual."""
    rules = _rules(4, np.random.default_rng(2))
    eng = _engine(rules)
    frames = [flow_frame(i + 1, int(rules["flow_id"][i % 4]), 1, False) for i in range(6)]
    payload, offsets = pack(frames)
    offsets = offsets.copy()
    offsets[3] = offsets[2] - 3   # frame 2 runs backwards, frame 3 is then longer
    _, xid_t, kind_t = _decode_gpu(eng, payload, offsets, np.full(6, T0, np.int64))
    kinds = list(kind_t.cpu().numpy()[:6])
    assert kinds[2] == abi.FRAME_SHORT
    assert kinds[:2] == [abi.FRAME_FLOW] * 2 and kinds[4:] == [abi.FRAME_FLOW] * 2


def test_encode_matches_oracle():
    import torch
    rng = np.random.default_rng(9)
    n = 100_001
    xid = rng.integers(-2**31, 2**31, n).astype(np.int32)
    kind = rng.choice(np.array([0, 0, 0, 0, 1, 2, 3], np.uint8), n)
    res = np.zeros(n, abi.RES_DTYPE)
    res["status"] = rng.choice(np.array([abi.OK, abi.BLOCKED, abi.SHOULD_WAIT, abi.NO_RULE_EXISTS,
                                         abi.BAD_REQUEST], np.int32), n)
    res["remaining"] = rng.integers(-2**31, 2**31, n)
    res["wait_ms"] = rng.integers(0, 2000, n)
    eng = _engine(_rules(10, rng))
    out_t = torch.full((n * 16,), 0xAB, dtype=torch.uint8, device="cuda")
    x_t, k_t, r_t = _dev(xid), _dev(kind), _dev(res)  # kept alive until the kernel has run
    eng.codec_encode(x_t.data_ptr(), k_t.data_ptr(), r_t.data_ptr(), n, out_t.data_ptr(),
                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out_t.cpu().numpy(), binding.codec_encode_flow(xid, kind, res))


@pytest.mark.parametrize("seed", [1, 2])
def test_server_step_end_to_end(seed):
    """frames → device decode → device decisions → device encode, over three consecutive 1 s batches."""
    import torch
    rng = np.random.default_rng(seed)
    rules = _rules(2000, rng)
    eng = _engine(rules, max_batch=1 << 17)
    ora = ClusterTokenService()
    ora.set_namespaces(_ns())
    ora.load_rules(rules)
    zipf = 1.0 / np.arange(1, len(rules) + 1)
    zipf /= zipf.sum()
    for b in range(3):
        n = int(rng.integers(20_000, 100_000))
        hot = rules["flow_id"][rng.choice(len(rules), n, p=zipf)]
        frames = random_frames(n, hot, rng, bad_frac=0.02)
        payload, offsets = pack(frames)
        ts = T0 + b * 1000 + np.sort(rng.integers(0, 1000, n)).astype(np.int64)
        req_t, xid_t, kind_t = _decode_gpu(eng, payload, offsets, ts)
        res_t = torch.empty(n * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        eng.decide_device(req_t.data_ptr(), n, res_t.data_ptr(), s)
        out_t = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        eng.codec_encode(xid_t.data_ptr(), kind_t.data_ptr(), res_t.data_ptr(), n, out_t.data_ptr(), s)
        torch.cuda.synchronize()
        want_req, want_xid, want_kind = binding.codec_decode_flow(payload, offsets, ts, rules["flow_id"])
        want = binding.codec_encode_flow(want_xid, want_kind, ora.decide(want_req))
        got = out_t.cpu().numpy()
        if not np.array_equal(got, want):
            bad = np.nonzero((got != want).reshape(n, 16).any(axis=1))[0]
            raise AssertionError(f"batch {b}: {len(bad)} response frames differ; first {bad[0]}: "
                                 f"{got.reshape(n, 16)[bad[0]]} vs {want.reshape(n, 16)[bad[0]]}")
