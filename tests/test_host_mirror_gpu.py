"""The C++ host mirror (sentinel_amd/host/token_service.cpp) over the real library: 16 threads × 20 000
concurrent GpuTokenService.requestToken calls, micro-batched through the asynchronous host pipeline
(sg_flow_submit / sg_flow_poll, pinned buffers); the recorded stream of decided micro-batches must equal the
oracle's sequential replay and every caller must get exactly its batch's answer
(tests/cpp/test_token_service_gpu.cpp, built in-tree by __graft_entry__.build / make -C tests/cpp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "tests", "tsg_gpu")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("threads,per_thread,shards", [(16, 20000, 0), (4, 5000, 0), (16, 10000, 3), (4, 5000, 1)])
def test_mirror_many_threads_against_device(threads, per_thread, shards):
    """shards > 0: the mirror in node mode (GpuTokenService::Options::shardDevices, sg_node_*: the flowIds hashed over
    that many shard handles of device 0, routing inside the library; param and concurrent tokens on the node's front
    handle) — the same replay must hold."""
    assert os.path.exists(EXE), f"{EXE} is missing: run __graft_entry__.build() (make -C tests/cpp)"
    out = subprocess.run([EXE, str(threads), str(per_thread), str(shards)], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-4000:]
    assert out.stdout.startswith("OK"), out.stdout
    n, batches = map(int, out.stdout.split()[1:3])
    assert n == threads * per_thread and batches >= 1
