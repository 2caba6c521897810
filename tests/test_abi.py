"""CPU-side checks of the C-ABI boundary: the library loads and exports every declared symbol."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "sentinel_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sentinel_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("sentinel_engine_create", "sentinel_submit_flow_batch", "sentinel_request_token",
              "sentinel_request_param_token", "sentinel_snapshot"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from sentinel_amd import _lib
    L = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_lib.EXPORTS) == declared_symbols()


def test_no_gpu_fails_loudly_not_silently():
    from sentinel_amd import _lib
    import sentinel_amd as sa
    L = _lib.load()
    if L.sentinel_device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(sa.SentinelError):
        sa.GpuTokenService(0)


def test_struct_layouts_match_header():
    import ctypes as C
    from sentinel_amd import _lib
    assert C.sizeof(_lib.FlowRuleC) == 40
    assert C.sizeof(_lib.ParamRuleC) == 40
    assert C.sizeof(_lib.Namespace) == 16
    assert C.sizeof(_lib.TokenResultC) == 16
    assert C.sizeof(_lib.FlowSnapshotC) == 24
