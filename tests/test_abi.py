"""CPU-side checks of the C ABI: the library loads, exports every symbol include/*.h declares, and the
ctypes mirrors (sentinel_amd/abi.py) match the header's struct layouts. No compute calls (no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from sentinel_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sentinel_gpu.h")


def _declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(sg_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_entry_points():
    names = _declared_functions()
    for n in ["sg_create", "sg_destroy", "sg_flow_decide_batch", "sg_load_flow_rules", "sg_snapshot_metrics"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from sentinel_amd.engine import LIB_PATH, load_library
    assert os.path.exists(LIB_PATH), "build with make -C sentinel_amd/csrc"
    L = load_library()
    for name in _declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (sg_\w+)", out))
    assert set(_declared_functions()) <= exported
    assert b"gfx950" in L.sg_build_info()


def test_library_links_gfx950_code_object():
    from sentinel_amd.engine import LIB_PATH
    blob = open(LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(f'''
#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(sg_config), sizeof(sg_flow_rule), sizeof(sg_namespace),
         sizeof(sg_req), sizeof(sg_result), sizeof(sg_batch_stats));
  printf("%zu %zu %zu %zu\\n", offsetof(sg_req, key), offsetof(sg_req, acquire), offsetof(sg_flow_rule, count),
         offsetof(sg_flow_rule, namespace_id));
  printf("%zu %zu %zu %zu %zu\\n", sizeof(sg_rls_request), offsetof(sg_rls_request, hits_addend),
         offsetof(sg_rls_request, desc_begin), offsetof(sg_rls_request, desc_count), sizeof(sg_rls_status));
  return 0;
}}''')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    lines = subprocess.check_output([str(exe)], text=True).split("\n")
    sizes = [int(x) for x in lines[0].split()]
    assert sizes == [C.sizeof(abi.sg_config), C.sizeof(abi.sg_flow_rule), C.sizeof(abi.sg_namespace),
                     C.sizeof(abi.sg_req), C.sizeof(abi.sg_result), C.sizeof(abi.sg_batch_stats)]
    offs = [int(x) for x in lines[1].split()]
    assert offs == [abi.sg_req.key.offset, abi.sg_req.acquire.offset, abi.sg_flow_rule.count.offset,
                    abi.sg_flow_rule.namespace_id.offset]
    rls = [int(x) for x in lines[2].split()]
    assert rls == [abi.RLS_REQ_DTYPE.itemsize, abi.RLS_REQ_DTYPE.fields["hits_addend"][1],
                   abi.RLS_REQ_DTYPE.fields["desc_begin"][1], abi.RLS_REQ_DTYPE.fields["desc_count"][1],
                   abi.RLS_STATUS_DTYPE.itemsize]


def test_create_fails_cleanly_without_device():
    """On a host without a GPU sg_create must return an error code, not crash."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    from sentinel_amd.engine import EngineError, FlowEngine
    with pytest.raises(EngineError):
        FlowEngine(max_batch=16)
