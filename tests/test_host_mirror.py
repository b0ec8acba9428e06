"""The C++ host mirror of TokenService / ClusterFlowRuleManager (sentinel_amd/host/token_service.cpp),
built with ASan + UBSan against a recording stand-in of the C ABI (tests/cpp/fake_sg.cpp): rule
filtering (FlowRuleUtil.isValidRule, applyClusterFlowRule), flowId → key mapping, DefaultTokenService
validation, FAIL on engine errors, and the multi-threaded micro-batcher."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_mirror_with_recording_abi(tmp_path):
    exe = tmp_path / "tsh"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=undefined", "-pthread", "-o", str(exe),
                           os.path.join(ROOT, "tests/cpp/test_token_service_host.cpp"),
                           os.path.join(ROOT, "tests/cpp/fake_sg.cpp"),
                           os.path.join(ROOT, "sentinel_amd/host/token_service.cpp")])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("OK")
