"""CPU: the C-ABI library loads and exports every symbol include/vcmpc.h declares;
no compute calls (no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "vcmpc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vc_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    syms = _declared_symbols()
    for s in ("vc_create", "vc_destroy", "vc_solve", "vc_rollout", "vc_linearize", "vc_condense",
              "vc_plant_step", "vc_spatial_step", "vc_last_error", "vc_set_stream", "vc_synchronize",
              "vc_track_set", "vc_track_k", "vc_horizon", "vc_drive", "vc_simulate"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from vcmpc import _abi
    lib = _abi.load_library()
    for s in _declared_symbols():
        assert hasattr(lib, s), s
    assert set(_declared_symbols()) == set(_abi.PROTOTYPES)


def test_struct_layout_matches():
    from vcmpc import _abi
    lib = _abi.load_library()
    assert lib.vc_params_sizeof() == ctypes.sizeof(_abi.vc_params)
    assert lib.vc_abi_version() == _abi.ABI_VERSION


def test_library_is_gfx950_code_object():
    from vcmpc import _abi
    blob = open(_abi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_create_fails_loudly_without_device():
    """No silent CPU fallback: creating a context with no GPU raises (or, on a GPU
    box, succeeds on a real device)."""
    import torch
    from vcmpc import Context, _abi
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_abi.VcError, match="no HIP device"):
        Context()


def test_missing_library_raises(tmp_path):
    from vcmpc import _abi
    with pytest.raises(ImportError, match="no CPU fallback"):
        _abi.load_library(str(tmp_path / "libvcmpc.so"))
