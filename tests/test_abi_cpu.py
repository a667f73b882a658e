"""The C-ABI library loads and exports exactly what include/placement.h declares (no GPU)."""
import ctypes
import os
import subprocess
import re

import pytest

from placement import _abi


def header_functions():
    with open(_abi.HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pe_[a-z_0-9]+)\s*\(", text)) - {"pe_allgather_fn"})


def test_library_built_in_tree():
    assert os.path.exists(_abi.LIB_PATH), "run make -C training-operator_amd/csrc"


def test_every_declared_symbol_is_exported():
    lib = _abi.load()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_abi.SIGNATURES), set(declared) ^ set(_abi.SIGNATURES)


def test_abi_version_and_structs(tmp_path):
    lib = _abi.load()
    assert lib.pe_abi_version() == 7
    # pe_config / pe_stats layouts mirrored in _abi must match the C compiler's (size and offsets)
    src = tmp_path / "sz.c"
    fields = [f for f, _ in _abi.PeConfig._fields_]
    sfields = [f for f, _ in _abi.PeStats._fields_]
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "placement.h"\nint main(void){'
                   'printf("%zu %zu\\n", sizeof(pe_config), sizeof(pe_stats));'
                   + "".join(f'printf("%zu\\n", offsetof(pe_config, {f}));' for f in fields)
                   + "".join(f'printf("%zu\\n", offsetof(pe_stats, {f}));' for f in sfields) + "return 0;}")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(_abi.HEADER), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(_abi.PeConfig) and int(out[1]) == ctypes.sizeof(_abi.PeStats)
    offs = [int(x) for x in out[2:]]
    assert offs[:len(fields)] == [getattr(_abi.PeConfig, f).offset for f in fields]
    assert offs[len(fields):] == [getattr(_abi.PeStats, f).offset for f in sfields]


def test_no_cpu_fallback_without_gpu():
    """On a machine without a GPU the engine refuses to start (PE_ENODEV), it never computes on CPU."""
    if os.path.exists("/dev/kfd"):
        pytest.skip("GPU present")
    from placement import Engine, PlacementError
    with pytest.raises(PlacementError) as e:
        Engine(0)
    assert e.value.code == _abi.PE_ENODEV


def test_error_codes_without_context():
    lib = _abi.load()
    assert lib.pe_get_stats(None, None) == _abi.PE_EINVAL
    assert lib.pe_synchronize(None) == _abi.PE_EINVAL
    assert lib.pe_last_error(None) == b"null context"
