"""The C-ABI library loads and exports every symbol include/tfhe_aes_gpu.h declares (no GPU needed)."""
import os
import re
import subprocess

import pytest

from tests.conftest import PKG, ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "tfhe_aes_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tae_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    from tfhe_aes import _native
    lib = _native.lib()
    declared = _declared()
    assert len(declared) >= 40
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(_native.EXPORTED) == declared
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (tae_\w+)", out))
    assert set(declared) <= exported


def test_library_is_gfx950_hip():
    """The shared object embeds a gfx950 code object (hipcc --offload-arch=gfx950)."""
    from tfhe_aes import _native
    data = open(_native.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_params_and_errors():
    import tfhe_aes
    with pytest.raises(tfhe_aes.TaeError):
        tfhe_aes.get_params(99)
    assert tfhe_aes.lib().tae_version().decode().startswith("tfhe-aes-2_amd")
