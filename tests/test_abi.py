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
    for s in ("vc_create", "vc_destroy", "vc_solve", "vc_solve_from", "vc_rollout", "vc_linearize", "vc_condense",
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


def _integration_stub():
    """The ctypes stub of INTEGRATION.md section 2: the lines from `class vc_params` through
    the ABI assert of its first python block that defines it."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for block in re.findall(r"```python\n(.*?)```", text, flags=re.S):
        if "class vc_params" in block:
            lines = block.splitlines()
            i0 = next(i for i, l in enumerate(lines) if l.startswith("class vc_params"))
            i1 = next(i for i, l in enumerate(lines) if l.startswith("assert lib.vc_abi_version()"))
            return "\n".join(lines[i0:i1 + 1]), "\n".join(lines[i1 + 1:])
    raise AssertionError("INTEGRATION.md has no vc_params stub")


def test_integration_stub_matches_library():
    """INTEGRATION.md's ctypes stub (what a maintainer would paste next to kinematic_mpc.py)
    runs against the built library: its own `vc_abi_version()` / `vc_params_sizeof()` assert
    passes, every field sits at the offset of include/vcmpc.h's struct (via vcmpc._abi), and
    the parameter values it packs are the reference's kinematic.yaml (so the doc cannot drift
    from the header again)."""
    from vcmpc import _abi
    lib = _abi.load_library()
    head, rest = _integration_stub()
    ns = {"C": ctypes, "lib": lib}
    exec(compile(head, "INTEGRATION.md", "exec"), ns)        # defines vc_params, runs the assert
    stub = ns["vc_params"]
    assert ctypes.sizeof(stub) == ctypes.sizeof(_abi.vc_params) == lib.vc_params_sizeof()

    def flat(struct, base=0, prefix=""):
        out = {}
        for name, typ in struct._fields_:
            off = base + getattr(struct, name).offset
            if isinstance(typ, type) and issubclass(typ, ctypes.Structure):
                out.update(flat(typ, off, prefix + name + "."))
            else:
                out[prefix + name] = (off, ctypes.sizeof(typ))
        return out

    ref = {off: size for off, size in flat(_abi.vc_params).values()}
    for name, (off, size) in flat(stub).items():
        if size == 8 or size == 4:
            assert ref.get(off) == size, f"INTEGRATION.md field {name} at offset {off} is not a field of vc_params"
    # the qp block's ABI-9 `elastic` double sits where the header has it
    assert stub.elastic.offset == _abi.vc_params.qp.offset + _abi.vc_qp.elastic.offset
    # the packing line fills the kinematic weights in the header's order
    pack = next(l for l in rest.splitlines() if l.startswith("p.kin_mpc[:]"))
    vals = eval(pack.split("=", 1)[1].split("#")[0], {})
    assert len(vals) == len(_abi.vc_kin_mpc._fields_)
